#!/bin/bash
# round-4 call 23: reduction groups of up to 20 (default now) -- batch tests,
# bench.py --warmup 3 / 5 twice, G2
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04w}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ches.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_small_reductions.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc $(date +%T) $(tail -1 $O/pytest.txt)"; grep -E "FAILED|^E " $O/pytest.txt | head -20
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  for W in 3 5; do
    L=w${W}_$i
    timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/$L.json 2> $O/$L.err || exit 1
    python3 -c "import json; d=json.load(open('$O/$L.json')); print('$L', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'], d['valu_roofline']['mad_frac'])"
  done
done
timeout -k 10 400 python3 -u bench.py --group 2 --no-configs --no-cpu-baseline > $O/g2.json 2> $O/g2.err &&
python3 -c "import json; d=json.load(open('$O/g2.json')); print('G2', d['value'], d['ms_per_step'], {k: v.get('value') for k, v in d['methods'].items()}, d['valu_roofline']['mad_frac'])"
echo "done $(date +%T)"
