# bench.py with --warmup 5 vs 20 (one untimed batch as long as the timed one), same box
set -o pipefail
O=gpurun_out/r05wu; mkdir -p $O
for w in 5 20 5 20; do
  timeout -k 10 400 python -u bench.py --warmup $w --no-configs --no-cpu-baseline > $O/b.json 2> $O/b.err || exit 1
  echo "## warmup $w" >> $O/wu.txt
  python tools/bench_summary.py $O/b.json 2>&1 | grep -E "headline|ches_batch|shards" >> $O/wu.txt
  python -c "import json; d=json.load(open('$O/b.json')); print({k: v['per_shard_ms'] for k, v in d['methods'].items() if k.startswith('shards')})" >> $O/wu.txt
done
cat $O/wu.txt
