#!/bin/bash
# accumulation k after level 0 of MSM k-1 (MSM_ACC_AFTER_L0=1) vs free (=0): batch tests with the knob, then bench A/B
set -o pipefail
TAG=${1:-r03a0}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
MSM_ACC_AFTER_L0=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ches.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.txt 2>&1
rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
ENVS="MSM_ACC_AFTER_L0=1 MSM_ACC_AFTER_L0=0" bash tools/ab_env.sh $TAG 4 --warmup 5 && bash tools/r03_ab_summ.sh $TAG
