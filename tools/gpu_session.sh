#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprof kernel trace/stats of
# the SAME bench command -> microbenchmarks (Fp-mul peak, gather calibration) ->
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the bench's accumulation and
# the calibration kernels.  Each GPU step has its own time limit; steps are
# chained with && so the first failure ends the session.
# usage (repo root, via gpurun): bash tools/gpu_session.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r02}
shift
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
MB=$R/tools/microbench/bin
echo "start $(date +%T)" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
echo "pytest ok $(date +%T) $(tail -1 $O/pytest_gpu.txt)" &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
echo "smoke ok $(date +%T)" &&
timeout -k 10 600 python -u bench.py "$@" > $O/bench.json 2> $O/bench.err &&
echo "bench ok $(date +%T)" && cat $O/bench.json &&
cd /tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py "$@" > $O/prof.json 2> $O/prof.log &&
echo "rocprof ok $(date +%T)" &&
timeout -k 10 120 $MB/fp_rate > $O/fp_rate.txt 2>&1 &&
timeout -k 10 120 $MB/gather_cal > $O/gather_cal.txt 2>&1 &&
echo "microbench ok $(date +%T)" &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/cal_fetch -o run -- $MB/gather_cal > $O/cal_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/cal_write -o run -- $MB/gather_cal > $O/cal_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_write.log 2>&1 &&
echo "pmc ok $(date +%T)" &&
python3 $R/tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv ches 20 $O/pmc_traffic.json $R/profiles/r02_gather_cal.json > /dev/null &&
grep accumulate_bytes_per_launch $O/pmc_traffic.json
echo "rc=$?"
