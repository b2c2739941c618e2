#!/bin/bash
# round-4 call 39: small MSMs (three lanes) -- reduction group size 20 (default)
# vs 8 / 10, and the level-0 chunk 4 / 8 instead of 2 (less tail work after the
# last accumulation)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04an}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
run() {  # label, env...
  L=$1; shift
  env "$@" timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 > $O/s_$L.txt 2>&1 || exit 1
  grep -v amdgpu $O/s_$L.txt | sed "s/^/$L /" | cut -c1-110
}
for i in 1 2; do
  run g20 MSM_RED_GROUP=20
  run g8 MSM_RED_GROUP=8
  run g10 MSM_RED_GROUP=10
  run g20c4 MSM_L0_CHUNK=4
  run g20c8 MSM_L0_CHUNK=8
done
echo "done $(date +%T)"
