#!/bin/bash
# round-4 call 26: small MSMs (the strong-scaling shards 2^17..2^19): front
# groups 2 (lane-mode default) / 4 / 8 and accumulation lanes 2 / 3
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04aa}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for F in 2 4 8; do
  MSM_FRONT_GROUP=$F timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 > $O/small_fg$F.txt 2>&1 || exit 1
  grep -v amdgpu $O/small_fg$F.txt | sed "s/^/fg$F /" | cut -c1-150
done
MSM_BATCH_LANES=3 timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 > $O/small_l3.txt 2>&1 || exit 1
grep -v amdgpu $O/small_l3.txt | sed "s/^/l3 /" | cut -c1-150
echo "done $(date +%T)"
