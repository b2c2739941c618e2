#!/bin/bash
# round-4 call 25: front groups (digits + sort of several sets in one pass,
# MSM_FRONT_GROUP) 1 (default at 2^20) vs 2 vs 4 with this round's schedule
# (a device slot per set, one reduction group); tools/h2d_ab.py, two
# processes each
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04y}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2; do
  for F in 1 2 4; do
    MSM_FRONT_GROUP=$F AB_LABEL=fg${F}_$i timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 3 > $O/ab_fg${F}_$i.txt 2> $O/ab_fg${F}_$i.err || exit 1
    grep "h2d:\|resident:" $O/ab_fg${F}_$i.txt
  done
done
for F in 2 4 8; do MSM_FRONT_GROUP=$F timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 > $O/small_fg$F.txt 2>&1 || exit 1; grep -v amdgpu $O/small_fg$F.txt | sed "s/^/fg$F /" | cut -c1-150; done
echo "done $(date +%T)"
