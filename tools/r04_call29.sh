#!/bin/bash
# round-4 call 29: plain-Pippenger batch (configs[1], 2^16) reduction groups
# MSM_PIP_GROUP 8 (default) vs 20, twice each
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ad}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2; do
  for G in 8 20; do
    MSM_PIP_GROUP=$G timeout -k 10 300 python3 -u tools/r04_small_trace.py pb16 pb16c13 > $O/pb_g${G}_$i.txt 2>&1 || exit 1
    grep -v amdgpu $O/pb_g${G}_$i.txt | sed "s/^/g$G /" | cut -c1-150
  done
done
echo "done $(date +%T)"
