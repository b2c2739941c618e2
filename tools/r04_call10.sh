#!/bin/bash
# round-4 call 10: does the profiling (timing events around every accumulation,
# which bench.py turns on) cause the H2D slow mode?  Repeated in-process
# headline batches with profiling off / on, three processes each; G2 2^20 batch
# with one vs two accumulation lanes
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04j}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for P in 0 1 0 1 0 1; do
  AB_LABEL=prof$P timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 4 --profiling $P > $O/ab_p$P.txt 2> $O/ab_p$P.err || exit 1
  grep "rep 0\|h2d:\|resident:" $O/ab_p$P.txt
done
for L in 1 2; do
  MSM_BATCH_LANES=$L timeout -k 10 400 python3 -u bench.py --group 2 --no-configs --no-cpu-baseline > $O/g2_l$L.json 2> $O/g2_l$L.err || exit 1
  python3 -c "import json; d=json.load(open('$O/g2_l$L.json')); print('G2 lanes $L', d['value'], {k: (v.get('value'), v.get('ms_per_step')) for k, v in d['methods'].items()})"
done
echo "done $(date +%T)"
