#!/bin/bash
# the H2D headline leg alone (--no-compare) under a kernel + memory-copy trace, four times:
# a slow and a fast run of the same box to compare
set -o pipefail
TAG=${1:-r03sp}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for i in 1 2 3 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/p$i -o run -- python3 $R/bench.py --no-compare --no-cpu-baseline --no-configs > $O/b$i.json 2> $O/b$i.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]); print($i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
echo "rc=$?"
