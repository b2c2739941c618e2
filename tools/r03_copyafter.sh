#!/bin/bash
# host-set copies issued after the previous accumulation (MSM_COPY_AFTER_ACC=1) vs beside it:
# batch tests with the knob, then bench A/B, then the 8-shard multi-context rehearsal
set -o pipefail
TAG=${1:-r03ca}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
MSM_COPY_AFTER_ACC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ches.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.txt 2>&1
rc=$?
tail -2 gpurun_out/$TAG/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
ENVS="MSM_COPY_AFTER_ACC=1 MSM_COPY_AFTER_ACC=0" bash tools/ab_env.sh $TAG 3 --warmup 5 && bash tools/r03_ab_summ.sh $TAG &&
timeout -k 10 300 python -u bench.py --multi-context 8 --one-device --steps 10 --warmup 2 --no-cpu-baseline --no-configs > gpurun_out/$TAG/mc8.json 2> gpurun_out/$TAG/mc8.err &&
python3 -c "import json; d=json.loads(open('gpurun_out/$TAG/mc8.json').read().strip().splitlines()[-1]); print('mc8', {k: (v.get('value'), v.get('parity_vs_reference')) for k, v in d['methods'].items() if 'cfg3' in k})"
echo "rc=$?"
