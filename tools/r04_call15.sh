#!/bin/bash
# round-4 call 15: what the first 20-set H2D batch after a 5-set warm-up
# lacks -- an extra untimed batch of 5 (one reduction group) or 9 sets (two
# groups: both reducer sets and tail streams), resident or H2D, before the
# timed repetitions; three processes per variant (tools/h2d_ab.py)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04o}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
run() {  # label, args...
  L=$1; shift
  AB_LABEL=$L timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 2 "$@" > $O/ab_$L.txt 2> $O/ab_$L.err || exit 1
  grep " rep " $O/ab_$L.txt
}
for i in 1 2 3; do
  run w5_$i
  run pre5r_$i --pre 5
  run pre9r_$i --pre 9
  run pre9h_$i --pre 9 --pre-h2d 1
done
echo "done $(date +%T)"
