#!/bin/bash
# batch GPU tests on the kernel-copy build, then bench A/B: host sets copied by k_copy_h2d vs SDMA
set -o pipefail
TAG=${1:-r03k}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ches.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.txt 2>&1
rc=$?
tail -3 gpurun_out/$TAG/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
ENVS="MSM_H2D_KERNEL=1 MSM_H2D_KERNEL=0" bash tools/ab_env.sh $TAG 3 --warmup 5 && bash tools/r03_ab_summ.sh $TAG
