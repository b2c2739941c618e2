#!/bin/bash
# round-4 call 20: the new default (a device slot per set) through bench.py at
# --warmup 3 / 5, four runs each, the batch tests, and G2 / small-MSM batches
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04t}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ches.py tests/test_gpu_multi.py tests/test_gpu_pippenger_batch.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc $(date +%T) $(tail -1 $O/pytest.txt)"; grep -E "FAILED|^E " $O/pytest.txt | head -20
[ $rc -eq 0 ] || exit 1
for i in 1 2 3 4; do
  for W in 3 5; do
    L=w${W}_$i
    timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/$L.json 2> $O/$L.err || exit 1
    python3 -c "import json; d=json.load(open('$O/$L.json')); print('$L', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
  done
done
timeout -k 10 400 python3 -u bench.py --group 2 --no-configs --no-cpu-baseline > $O/g2.json 2> $O/g2.err &&
python3 -c "import json; d=json.load(open('$O/g2.json')); print('G2', d['value'], d['ms_per_step'], {k: v.get('value') for k, v in d['methods'].items()}, d['valu_roofline']['mad_frac'])" &&
timeout -k 10 300 python3 -u tools/r04_small_trace.py pb16 c17 c18 c19 > $O/small.txt 2>&1 && grep -v amdgpu $O/small.txt | cut -c1-200
echo "done $(date +%T)"
