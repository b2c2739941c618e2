#!/bin/bash
# Round-6 GPU session: parity suite, smoke, the default bench line (summary).
# usage (repo root, via gpurun): bash tools/r06_session.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r06a}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
if [ -z "$2" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
echo "pytest ok $(date +%T) $(tail -1 $O/pytest_gpu.txt)" &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
echo "smoke ok $(date +%T)" || { echo "FAILED $(date +%T)"; tail -30 $O/pytest_gpu.txt; exit 1; }
fi
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
echo "bench ok $(date +%T)" && python3 tools/bench_summary.py $O/bench.json
