#!/bin/bash
# Round-4 final-tree GPU session: parity suite, smoke, the default bench line,
# rocprofv3 kernel trace + stats of the same bench command (roofline check),
# separate FETCH_SIZE / WRITE_SIZE PMC passes over the accumulation.
# usage (repo root, via gpurun): bash tools/r04_final.sh <tag>
set -o pipefail
TAG=${1:-r04z}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
echo "pytest ok $(date +%T) $(tail -1 $O/pytest_gpu.txt)" &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
echo "smoke ok $(date +%T)" &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
echo "bench ok $(date +%T)" && python3 -c "
import json; d=json.load(open('$O/bench.json')); print('headline', d['value'], d['ms_per_step'], d['parity_vs_reference'], d['roofline']['frac'], d['valu_roofline']['mad_frac'])
for k,v in d['methods'].items(): print(' ', k, v.get('value'), v.get('ms_per_step'), v.get('parity_vs_reference'))" &&
cd /tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-configs --no-cpu-baseline > $O/prof.json 2> $O/prof.log &&
echo "rocprof ok $(date +%T)" &&
python3 $R/tools/roofline_check.py $O/prof.json $O/prof/run_kernel_trace.csv $O/roofline_check.json &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_write.log 2>&1 &&
python3 $R/tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv ches 20 $O/pmc_traffic.json $R/profiles/r02_gather_cal.json > /dev/null &&
echo "pmc ok $(date +%T)" && grep accumulate_bytes_per_launch $O/pmc_traffic.json
echo "rc=$?"
