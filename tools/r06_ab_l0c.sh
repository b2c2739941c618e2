#!/bin/bash
# Same-box A/B of the batch level-0 chunk (MSM_BATCH_L0_CHUNK 8 vs 4 vs 6) on
# the 2^17 shard batch (tools/shard_leg_probe.py, 4 shards x 3 H2D batches),
# three rounds alternating.  usage (via gpurun): bash tools/r06_ab_l0c.sh
set -o pipefail
O=gpurun_out/l0c; mkdir -p $O
for i in 1 2 3; do
  for v in 8 4 6; do
    echo "== MSM_BATCH_L0_CHUNK=$v round $i" >> $O/out.txt
    MSM_BATCH_L0_CHUNK=$v timeout -k 10 200 python3 tools/shard_leg_probe.py --shards 8 --use 4 >> $O/out.txt 2>> $O/err.txt || exit 1
  done
done
echo done
