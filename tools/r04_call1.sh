#!/bin/bash
# round-4 call 1: per-MSM fixed-cost traces (small plain / CHES shards) + baseline headline
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 300 python3 -u tools/r04_small_trace.py > $O/small.txt 2>&1 &&
echo "small ok $(date +%T)" && cat $O/small.txt &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/tools/r04_small_trace.py p16 c17 c18 > $O/small_prof.txt 2>&1 &&
echo "prof ok $(date +%T)" && cd $R &&
timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup 3 > $O/bench_w3.json 2> $O/bench_w3.err &&
timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup 5 > $O/bench_w5.json 2> $O/bench_w5.err &&
echo "bench ok $(date +%T)" && python3 -c "
import json
for f in ('w3','w5'):
    d=json.load(open('$O/bench_'+f+'.json')); print(f, d['value'], d['methods']['ches_batch_resident']['value'], d['phases_ms'])"
