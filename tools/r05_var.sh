# first full-length batch: warm-up of 3 vs 20 sets, then 4 timed batches (resident first)
set -o pipefail
O=gpurun_out/r05fw; mkdir -p $O
for w in 3 20 3 20; do
  echo "## warm $w" >> $O/fw.txt
  timeout -k 10 300 python -u tools/shard_study.py --logs 17,19 --cfgs 20 --reps 4 --all --warm $w >> $O/fw.txt 2> $O/fw.err || exit 1
done
cat $O/fw.txt
