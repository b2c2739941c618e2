#!/bin/bash
# Same-box A/B of the fine-pass workgroup size (bucket_sort.hpp k_bs_fine 1024
# vs 256 threads) in the small-MSM batches: the 2^17 / 2^18 CHES shards
# (MSM_FINE_BT, tools/shard_leg_probe.py) and configs[1]'s plain batch
# (MSM_PIP_FINE_BT, tools/cfg1_window_sweep.py 14), two rounds alternating.
# usage (repo root, via gpurun): bash tools/r06_ab_fine_bt.sh
set -o pipefail
O=gpurun_out/fbt; mkdir -p $O
for i in 1 2; do
  for b in 1024 256; do
    echo "== fine_bt $b round $i" >> $O/out.txt
    MSM_FINE_BT=$b timeout -k 10 200 python3 tools/shard_leg_probe.py --shards 8 --use 3 >> $O/out.txt 2>> $O/err.txt || exit 1
    MSM_FINE_BT=$b timeout -k 10 200 python3 tools/shard_leg_probe.py --shards 4 --use 2 >> $O/out.txt 2>> $O/err.txt || exit 1
    MSM_PIP_FINE_BT=$b timeout -k 10 200 python3 tools/cfg1_window_sweep.py 14 >> $O/out.txt 2>> $O/err.txt || exit 1
  done
done
echo done
