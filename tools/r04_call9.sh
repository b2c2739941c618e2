#!/bin/bash
# round-4 call 9: the 256-thread batch fine pass (fits beside three accumulation
# waves per SIMD) and the lean k_sched_scatter -- batch tests, then repeated
# in-process H2D / resident headline batches, fine 256 vs 1024
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04i}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ches.py tests/test_gpu_pippenger_batch.py tests/test_gpu_multi.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc $(date +%T) $(tail -1 $O/pytest.txt)"; grep -E "FAILED|^E " $O/pytest.txt | head -20
[ $rc -eq 0 ] || exit 1
for BT in 256 1024 256 1024; do
  MSM_FINE_BT=$BT AB_LABEL=bt$BT timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 5 > $O/ab_bt$BT.txt 2> $O/ab_bt$BT.err || exit 1
  grep "h2d:\|resident:" $O/ab_bt$BT.txt
done
for MM in 1 0; do MSM_MULTI_MERGE=$MM timeout -k 10 400 python3 -u bench.py --multi-context 8 --one-device --steps 10 --warmup 2 --no-cpu-baseline --no-configs > $O/mc8_m$MM.json 2> $O/mc8_m$MM.err || exit 1
python3 -c "import json; d=json.load(open('$O/mc8_m$MM.json')); print('mc8 merge=$MM', d['value'], {k: (v.get('value'), v.get('ms_per_step'), v.get('parity_vs_reference')) for k, v in d['methods'].items() if 'cfg3' in k})"; done
timeout -k 10 300 python3 -u tools/r04_small_trace.py c17b c18 c19 > $O/small.txt 2>&1 && grep -v amdgpu $O/small.txt | cut -c1-200
echo "done $(date +%T)"
