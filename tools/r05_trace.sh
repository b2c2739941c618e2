# kernel + memory-copy trace of the headline H2D batch (bench.py, default warm-up), summarised
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r05tr; mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t -o run -- python3 $R/bench.py --no-configs --no-shards --no-cpu-baseline --no-compare > $O/b.json 2> $O/b.err || exit 1
cd $R
python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('headline', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], 'warmup', d['warmup'])" > $O/summary.txt
python3 tools/h2d_trace.py $O/t/run 20 20 >> $O/summary.txt
python3 tools/batch_profile.py $O/t/run_kernel_trace.csv >> $O/summary.txt
cat $O/summary.txt | head -80
