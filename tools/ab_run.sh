#!/bin/bash
# Same-box A/B probes of the G1 CHES 2^20 batch (tools/exp_batch.py, K=20, best of 3),
# one fresh process per variant, each under its own time limit.
# usage (repo root, via gpurun): bash tools/ab_run.sh <tag> "<ENV=VAL ...>" ["<ENV=VAL ...>" ...]
TAG=$1
shift
mkdir -p gpurun_out/$TAG
i=0
for v in "$@"; do
  i=$((i + 1))
  echo "== variant $i: $v" > gpurun_out/$TAG/v$i.txt
  env $v EXP_SYNC=1 timeout -k 10 200 python -u tools/exp_batch.py 20 3 >> gpurun_out/$TAG/v$i.txt 2>&1 || exit 1
done
echo done
