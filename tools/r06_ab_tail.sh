#!/bin/bash
# Round-6 A/B of the batch tails (same box, one library): the last group's bit
# tail (MSM_BIT_TAIL) and the dense stage's per-level coop choice
# (MSM_DENSE_COOP_MAX; 1000000 = every level coop, the round-5 schedule), on
# the 2^17 / 2^18 CHES shards (tools/shard_study.py) and configs[1]
# (tools/pip_study.py), after the batch parity tests.
# usage (repo root, via gpurun): bash tools/r06_ab_tail.sh <tag> [rounds]
set -o pipefail
TAG=${1:-r06ab}
N=${2:-2}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch_one_lane.py tests/test_gpu_ches.py tests/test_gpu_pippenger_batch.py tests/test_gpu_multi.py tests/test_gpu_rccl.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in $(seq 1 $N); do
  for e in "MSM_BIT_TAIL=1" "MSM_BIT_TAIL=0" "MSM_BIT_TAIL=0 MSM_DENSE_COOP_MAX=1000000"; do
    echo "# $e round $i" >> $O/shard.txt
    env $e timeout -k 10 200 python3 -u tools/shard_study.py --logs 17,18 --cfgs 20,19 --reps 3 --warm 20 >> $O/shard.txt 2>/dev/null || exit 1
  done
  timeout -k 10 300 python3 -u tools/pip_study.py --windows 14 --envs "MSM_DENSE_COOP_MAX=16384;MSM_DENSE_COOP_MAX=1000000" >> $O/pip.txt 2>&1 || exit 1
done
grep -v "^$" $O/shard.txt $O/pip.txt
