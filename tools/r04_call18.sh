#!/bin/bash
# round-4 call 18: H2D device slots (copies issued that far ahead,
# MSM_H2D_SLOTS) 4 (default) vs 8 vs 20 at --warmup 3 and 5, three runs each
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04r}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2 3; do
  for S in 4 8 20; do
    for W in 3 5; do
      L=s${S}_w${W}_$i
      MSM_H2D_SLOTS=$S timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/$L.json 2> $O/$L.err || exit 1
      python3 -c "import json; d=json.load(open('$O/$L.json')); print('$L', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
    done
  done
done
echo "done18 $(date +%T)" && bash tools/r04_call19.sh
