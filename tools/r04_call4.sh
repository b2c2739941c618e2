#!/bin/bash
# round-4 call 4: new GPU tests, plain-Pippenger batch, small-MSM timings, lanes A/B through bench.py, batch trace at 2^17
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04d}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_engine_cache.py tests/test_gpu_pointer_gather.py tests/test_gpu_table_rows.py tests/test_gpu_pippenger_batch.py tests/test_gpu_ches.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
echo "pytest rc=$? $(date +%T) $(tail -1 $O/pytest.txt)"; grep -E "FAILED|Error" $O/pytest.txt | head -20
timeout -k 10 300 python3 -u tools/r04_small_trace.py p16 pb16 pb16c13 pb16c12 c17 c18 c19 c20 > $O/small.txt 2>&1 &&
grep -v amdgpu $O/small.txt | cut -c1-200 &&
for L in 1 2 3; do for W in 3 5; do
  MSM_BATCH_LANES=$L timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/bench_l${L}_w$W.json 2> $O/bench_l${L}_w$W.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_l${L}_w$W.json')); print('L$L W$W', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'], d['valu_roofline']['mad_frac'], d['valu_roofline']['mad_frac_alone'])"
done; done &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof17 -o run -- python3 $R/tools/r04_small_trace.py c17 > $O/prof17.txt 2>&1 &&
echo "done $(date +%T)"
