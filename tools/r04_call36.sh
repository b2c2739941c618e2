#!/bin/bash
# round-4 call 36: accumulation lanes at 2^20 (MSM_BATCH_LANES 1 = default vs
# 2 vs 3) with this round's schedule; tools/h2d_ab.py, two processes each
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ak}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2; do
  for L in 1 2 3; do
    MSM_BATCH_LANES=$L AB_LABEL=l${L}_$i timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 3 > $O/ab_l${L}_$i.txt 2> $O/ab_l${L}_$i.err || exit 1
    grep "h2d:\|resident:" $O/ab_l${L}_$i.txt
  done
done
echo "done $(date +%T)"
