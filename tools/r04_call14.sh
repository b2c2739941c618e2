#!/bin/bash
# round-4 call 14: level-0 chunk 9 / 10 (one round of the chip's wave slots)
# vs 8, and host scalars read by the front kernels straight from pinned
# memory (MSM_ZERO_COPY_SCALARS=1) vs SDMA copies; tools/h2d_ab.py, two
# processes per variant
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04n}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
run() {  # label, env...
  L=$1; shift
  env "$@" AB_LABEL=$L timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 3 > $O/ab_$L.txt 2> $O/ab_$L.err || exit 1
  grep "h2d:\|resident:" $O/ab_$L.txt
}
for i in 1 2; do
  run c8_$i MSM_L0_CHUNK=8
  run c9_$i MSM_L0_CHUNK=9
  run c10_$i MSM_L0_CHUNK=10
  run zc_$i MSM_ZERO_COPY_SCALARS=1
done
echo "done $(date +%T)"
