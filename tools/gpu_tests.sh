#!/bin/bash
# GPU parity tests (optionally a subset: extra args go to pytest), output under gpurun_out/<tag>/.
# usage (via gpurun): bash tools/gpu_tests.sh <tag> [pytest-args...]
set -o pipefail
TAG=${1:-r02}
shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "${@:-tests}" > gpurun_out/$TAG/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/$TAG/pytest_gpu.txt
exit $rc
