#!/bin/bash
# round-4 call 30: front stream priority greatest (default) / normal / least
# with this round's copy schedule; tools/h2d_ab.py, two processes each
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ae}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2; do
  for P in 1 0 -1; do
    MSM_FRONT_PRIO=$P AB_LABEL=p${P}_$i timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 3 > $O/ab_p${P}_$i.txt 2> $O/ab_p${P}_$i.err || exit 1
    grep "h2d:\|resident:" $O/ab_p${P}_$i.txt
  done
done
echo "done $(date +%T)"
