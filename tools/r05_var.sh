# bench.py headline runs after removing the copy stream's cross-stream wait:
# 5 runs under a HIP API trace (before: 3 of 5 and 7 of 8 traced runs slow) + 3 plain
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r05nw; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $O/t$i -o run -- python3 $R/bench.py --no-configs --no-shards --no-cpu-baseline --no-compare > $O/tb$i.json 2> $O/tb$i.err) || exit 1
  python3 -c "import json; d=json.loads(open('$O/tb$i.json').read().strip().splitlines()[-1]); print('traced $i', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" | tee -a $O/runs.txt
done
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline --no-shards > $O/b$i.json 2> $O/b$i.err || exit 1
  python tools/bench_summary.py $O/b$i.json 2>&1 | sed -n 1,3p | tee -a $O/runs.txt
done
