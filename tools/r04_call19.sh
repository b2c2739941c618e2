#!/bin/bash
# round-4 call 19: fronts released after the previous MSM's level 0 (start
# beside the next accumulation, MSM_FRONT_AFTER_L0=1) vs after its
# accumulation (beside level 0, the default); bench.py --warmup 3 / 5, three
# runs each, then in-process repetitions (tools/h2d_ab.py)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04s}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2 3; do
  for F in 0 1; do
    for W in 3 5; do
      L=f${F}_w${W}_$i
      MSM_FRONT_AFTER_L0=$F timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/$L.json 2> $O/$L.err || exit 1
      python3 -c "import json; d=json.load(open('$O/$L.json')); print('$L', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
    done
  done
done
for F in 0 1 0 1; do
  MSM_FRONT_AFTER_L0=$F AB_LABEL=f$F timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 4 > $O/ab_f$F.txt 2> $O/ab_f$F.err || exit 1
  grep "h2d:\|resident:" $O/ab_f$F.txt
done
echo "done $(date +%T)"
