#!/bin/bash
# round-4 call 11: level 0 on the critical path (acc k+1 waits for level 0 of
# k) vs free-running, with the reduction streams at normal / greatest priority;
# level-0 chunk 4 / 6 instead of 8 at 2^20; in-process repetitions (tools/h2d_ab.py), two processes per variant
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04k}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
run() {  # label, env...
  L=$1; shift
  env "$@" AB_LABEL=$L timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 4 > $O/ab_$L.txt 2> $O/ab_$L.err || exit 1
  grep "h2d:\|resident:" $O/ab_$L.txt
}
for i in 1 2; do
  run base$i MSM_ACC_AFTER_L0=1
  run free$i MSM_ACC_AFTER_L0=0
  run freehi$i MSM_ACC_AFTER_L0=0 MSM_TAIL_PRIO=1
  run basehi$i MSM_ACC_AFTER_L0=1 MSM_TAIL_PRIO=1
  run c4_$i MSM_L0_CHUNK=4
  run c6_$i MSM_L0_CHUNK=6
done
echo "done $(date +%T)"
