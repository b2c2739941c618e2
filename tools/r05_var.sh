# last-group tail: coop segment levels (new) + coop dense stage vs none (MSM_TAIL_COOP=0); batch tests first
set -o pipefail
O=gpurun_out/r05tc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ches.py tests/test_gpu_batch_one_lane.py tests/test_gpu_pippenger_batch.py tests/test_gpu_small_reductions.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for tc in 1 0 1 0; do
  echo "## MSM_TAIL_COOP=$tc" >> $O/tc.txt
  MSM_TAIL_COOP=$tc timeout -k 10 300 python -u tools/shard_study.py --logs 17 --cfgs 20 --reps 4 --warm 20 >> $O/tc.txt 2>> $O/tc.err || exit 1
  MSM_TAIL_COOP=$tc timeout -k 10 300 python -u tools/pip_study.py --windows 14 >> $O/tc.txt 2>> $O/tc.err || exit 1
  MSM_TAIL_COOP=$tc AB_LABEL=tc$tc timeout -k 10 300 python -u tools/h2d_ab.py --reps 4 2>> $O/tc.err | grep median >> $O/tc.txt || exit 1
done
cat $O/tc.txt
