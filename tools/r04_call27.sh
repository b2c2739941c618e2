#!/bin/bash
# round-4 call 27: small MSMs -- lanes 2 / 3 x front groups 2 / 4, 2^17..2^19,
# twice; then the G2 2^19 and 2^18 batch with 2 / 3 lanes
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ab}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2; do
  for L in 2 3; do
    for F in 2 4; do
      MSM_BATCH_LANES=$L MSM_FRONT_GROUP=$F timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 > $O/small_l${L}_fg${F}_$i.txt 2>&1 || exit 1
      grep -v amdgpu $O/small_l${L}_fg${F}_$i.txt | sed "s/^/l$L fg$F /" | cut -c1-120
    done
  done
done
echo "done $(date +%T)"
