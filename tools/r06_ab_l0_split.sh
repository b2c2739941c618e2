#!/bin/bash
# Same-box A/B of the last accumulation group's level 0 on two lanes per chunk
# (MSM_L0_SPLIT, ches.hip run_jobs / pair_kernels.hpp k_segsum_split2) on the
# 2^17 / 2^18 CHES shard batches (tools/shard_leg_probe.py), after the batch
# tail tests; two rounds alternating.  usage (via gpurun): bash tools/r06_ab_l0_split.sh
# (The k_segsum_split2 code measured equal and was removed; profiles/r06_l0_split_ab.txt.)
set -o pipefail
O=gpurun_out/l0split; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch_tails.py tests/test_gpu_ches.py > $O/tests.txt 2>&1 || exit 1
tail -1 $O/tests.txt
for i in 1 2; do
  for v in 0 1; do
    echo "== MSM_L0_SPLIT=$v round $i" >> $O/out.txt
    MSM_L0_SPLIT=$v timeout -k 10 200 python3 tools/shard_leg_probe.py --shards 8 --use 3 >> $O/out.txt 2>> $O/err.txt || exit 1
    MSM_L0_SPLIT=$v timeout -k 10 200 python3 tools/shard_leg_probe.py --shards 4 --use 2 >> $O/out.txt 2>> $O/err.txt || exit 1
  done
done
echo done
