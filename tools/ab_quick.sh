#!/bin/bash
# Same-box A/B of library variants on the synchronous CHES MSM (per-phase
# times from tools/quick_ches.py): alternates tools/ablib/libmsm_<v>.so into
# the box's tree, one process each, each under its own limit.
# usage (repo root, via gpurun): VARIANTS="a b" bash tools/ab_quick.sh <tag> <rounds> [group log_n]
TAG=$1
N=$2
shift 2
mkdir -p gpurun_out/$TAG
cp msm_blst_amd/libmsm_mi355x.so /tmp/libmsm_orig.so
for i in $(seq 1 $N); do
  for v in $VARIANTS; do
    cp tools/ablib/libmsm_$v.so msm_blst_amd/libmsm_mi355x.so
    timeout -k 10 200 python -u tools/quick_ches.py "$@" > gpurun_out/$TAG/$v$i.txt 2>&1 || { cp /tmp/libmsm_orig.so msm_blst_amd/libmsm_mi355x.so; exit 1; }
  done
done
cp /tmp/libmsm_orig.so msm_blst_amd/libmsm_mi355x.so
echo done
