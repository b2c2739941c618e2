#!/bin/bash
# round-4 call 22: MSMs per reduction group (MSM_RED_GROUP) 8 (default: 3
# groups for 20 sets, two tails beside accumulations) vs 10 vs 20 (one group,
# one tail at the end); tools/h2d_ab.py, two processes each, then bench.py
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04v}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2; do
  for G in 8 10 20; do
    MSM_RED_GROUP=$G AB_LABEL=g${G}_$i timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 3 > $O/ab_g${G}_$i.txt 2> $O/ab_g${G}_$i.err || exit 1
    grep "h2d:\|resident:" $O/ab_g${G}_$i.txt
  done
done
for G in 8 20 8 20; do
  MSM_RED_GROUP=$G timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup 3 > $O/b_g$G.json 2> $O/b_g$G.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_g$G.json')); print('bench g$G', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
done
echo "done $(date +%T)"
