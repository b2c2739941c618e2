#!/bin/bash
# round-4 call 8: kernel + memory-copy traces of four H2D headline runs (the
# bimodal slow mode: ~375-395 vs ~413 M pairs/s on one box, independent of the
# warmup length) for an offline fast/slow comparison
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04h}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for i in 1 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t$i -o run -- python3 $R/bench.py --no-configs --no-cpu-baseline --no-compare --warmup 5 > $O/t$i.json 2> $O/t$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/t$i.json')); print('t$i', d['value'], d['roofline']['kernel_ms'])"
done
echo "done $(date +%T)"
