# reduction groups: the batch's last m MSMs in a group of their own (MSM_LAST_GROUP); tests first
set -o pipefail
O=gpurun_out/r05lg; mkdir -p $O
MSM_LAST_GROUP=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_ches.py tests/test_gpu_batch_one_lane.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for lg in 0 4 2 6 0 4; do
  echo "## MSM_LAST_GROUP=$lg" >> $O/lg.txt
  MSM_LAST_GROUP=$lg timeout -k 10 300 python -u tools/shard_study.py --logs 17,19 --cfgs 20 --reps 3 --warm 20 2>> $O/lg.err | grep -v agree >> $O/lg.txt || exit 1
  MSM_LAST_GROUP=$lg AB_LABEL=lg$lg timeout -k 10 300 python -u tools/h2d_ab.py --reps 4 --warmup 20 2>> $O/lg.err | grep median >> $O/lg.txt || exit 1
done
cat $O/lg.txt
