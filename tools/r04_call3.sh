#!/bin/bash
# round-4 call 3: lanes 2 vs 3 at 2^17..2^20 and the 2^20 H2D headline per lane count
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04c}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine_cache.py tests/test_gpu_pointer_gather.py tests/test_gpu_table_rows.py tests/test_gpu_ches.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 &&
echo "pytest ok $(date +%T) $(tail -1 $O/pytest.txt)" &&
MSM_BATCH_LANES=3 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ches.py -m gpu -x -v --timeout 200 --timeout-method thread -k batch > $O/pytest_l3.txt 2>&1 &&
echo "pytest l3 ok $(tail -1 $O/pytest_l3.txt)" &&
for L in 2 3; do MSM_BATCH_LANES=$L timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 c20 > $O/small_l$L.txt 2>&1 || exit 1; grep -v amdgpu $O/small_l$L.txt | sed "s/^/L$L /" | cut -c1-150; done &&
for L in 1 2 3; do for W in 3 5; do
  MSM_BATCH_LANES=$L timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/bench_l${L}_w$W.json 2> $O/bench_l${L}_w$W.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_l${L}_w$W.json')); print('L$L W$W', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
done; done
echo "done $(date +%T)"
