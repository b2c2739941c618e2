#!/bin/bash
# round-4 call 13: the slow FIRST H2D batch after a short warm-up -- hardware
# queues per process (GPU_MAX_HW_QUEUES 4 = the box default, vs 8) and a
# warm-up as long as the batch (20 sets) vs 5; six processes per variant,
# two repetitions each (tools/h2d_ab.py)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04m}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T) GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
run() {  # label, warmup, env...
  L=$1; W=$2; shift 2
  env "$@" AB_LABEL=$L timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 2 --warmup $W > $O/ab_$L.txt 2> $O/ab_$L.err || exit 1
  grep "rep " $O/ab_$L.txt
}
for i in 1 2 3 4 5 6; do
  run q4_w5_$i 5
  run q8_w5_$i 5 GPU_MAX_HW_QUEUES=8
  run q4_w20_$i 20
done
echo "done $(date +%T)"
