#!/bin/bash
# Same-box A/B of environment settings through bench.py itself: alternates the
# settings given as ENVS="A=1 A=8" (one bench process each, each under its own
# limit), N rounds.  usage (repo root, via gpurun): ENVS="..." bash tools/ab_env.sh <tag> <rounds> [bench args...]
TAG=$1
N=$2
shift 2
mkdir -p gpurun_out/$TAG
for i in $(seq 1 $N); do
  for e in $ENVS; do
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs "$@" > gpurun_out/$TAG/${e//=/_}_$i.json 2> gpurun_out/$TAG/${e//=/_}_$i.err || exit 1
  done
done
echo done
