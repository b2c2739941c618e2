#!/bin/bash
# Same-box A/B of two library builds through bench.py itself (first-batch H2D
# headline): alternates tools/ablib/libmsm_cur.so and libmsm_prev.so into the
# box's copy of the tree, one bench process each, each under its own limit.
# usage (repo root, via gpurun): bash tools/ab_bench.sh <tag> <rounds> [bench args...]
TAG=$1
N=$2
shift 2
mkdir -p gpurun_out/$TAG
for i in $(seq 1 $N); do
  for v in ${VARIANTS:-cur prev}; do
    cp tools/ablib/libmsm_$v.so msm_blst_amd/libmsm_mi355x.so || exit 1
    timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/$TAG/$v$i.json 2> gpurun_out/$TAG/$v$i.err || exit 1
  done
done
cp tools/ablib/libmsm_cur.so msm_blst_amd/libmsm_mi355x.so
echo done
