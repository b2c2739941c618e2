#!/bin/bash
# A/B of the front-group taper (MSM_FRONT_TAPER) on the small-MSM batches:
# batch parity tests with the taper on, then shard_study (2^17 q = 2^19 via
# config 17 beta, 2^18 q = 2^20) and pip_study (configs[1], c = 14), alternating.
set -o pipefail
TAG=${1:-r06tp}; N=${2:-2}
O=gpurun_out/$TAG; mkdir -p $O
MSM_FRONT_TAPER=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch_one_lane.py tests/test_gpu_ches.py tests/test_gpu_pippenger_batch.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in $(seq 1 $N); do
  for t in 1 0; do
    echo "# MSM_FRONT_TAPER=$t round $i" >> $O/shard.txt
    MSM_FRONT_TAPER=$t timeout -k 10 200 python3 -u tools/shard_study.py --logs 17 --cfgs 19 --reps 3 --warm 20 >> $O/shard.txt 2>/dev/null || exit 1
    MSM_FRONT_TAPER=$t timeout -k 10 200 python3 -u tools/shard_study.py --logs 18 --cfgs 20 --reps 3 --warm 20 >> $O/shard.txt 2>/dev/null || exit 1
  done
  timeout -k 10 300 python3 -u tools/pip_study.py --windows 14 --envs "MSM_FRONT_TAPER=1;MSM_FRONT_TAPER=0" >> $O/pip.txt 2>&1 || exit 1
done
grep -v "^$" $O/shard.txt $O/pip.txt | grep -v all_configs
