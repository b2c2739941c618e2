#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprof kernel stats -> PMC traffic passes.
# Each GPU step runs under its own time limit; steps are chained with && so the
# first failure (fault, abort, timeout) ends the session.
# usage (from the repo root, via gpurun): bash tools/gpu_round.sh <tag> [pytest-args...]
set -o pipefail
TAG=${1:-r01}
shift
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $O/pytest_gpu.txt 2>&1 &&
echo "pytest ok $(date +%T)" &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
echo "smoke ok $(date +%T)" &&
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err &&
echo "bench ok $(date +%T)" && cat $O/bench.json &&
cd /tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-compare > $O/prof.log 2>&1 &&
echo "rocprof ok $(date +%T)" &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_write.log 2>&1 &&
echo "pmc ok $(date +%T)"
echo "rc=$?"
