#!/bin/bash
# GPU suite on the fused-front build, then bench A/B fused vs unfused front
set -o pipefail
TAG=${1:-r03f}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.txt 2>&1
rc=$?
tail -3 gpurun_out/$TAG/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
ENVS="MSM_FRONT_FUSED=1 MSM_FRONT_FUSED=0" bash tools/ab_env.sh $TAG 2 --warmup 5 && bash tools/r03_ab_summ.sh $TAG
