#!/bin/bash
# round-4 call 33: the batch's host combine on the worker threads -- batch
# tests, small MSMs, bench.py twice
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ah}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ches.py tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc $(date +%T) $(tail -1 $O/pytest.txt)"; grep -E "FAILED|^E " $O/pytest.txt | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 c20b > $O/small.txt 2>&1 && grep -v amdgpu $O/small.txt | cut -c1-150 &&
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup 3 > $O/b$i.json 2> $O/b$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b$i.json')); print('bench', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
done
echo "done $(date +%T)"
