#!/bin/bash
# round-4 call 6: full GPU suite on the new tree, lean-doubling study build vs the
# table-row test, small-MSM timings, warmup 3/5 (+ preheat) A/B, one full default bench
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04f}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc $(date +%T) $(tail -1 $O/pytest_gpu.txt)"; grep -E "FAILED|^E " $O/pytest_gpu.txt | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python3 -u tools/r04_small_trace.py pb16 c17 c18 c19 > $O/small.txt 2>&1 && grep -v amdgpu $O/small.txt | cut -c1-200 &&
for W in 3 5 3; do
  timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/bench_w$W.json 2> $O/bench_w$W.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_w$W.json')); print('W$W', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
  BENCH_PREHEAT_MS=300 timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --warmup $W > $O/bench_pre_w$W.json 2> $O/bench_pre_w$W.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_pre_w$W.json')); print('pre W$W', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
done &&
for L in 1 2 3; do MSM_BATCH_LANES=$L timeout -k 10 300 python3 -u tools/r04_small_trace.py c20b > $O/small_c20b_l$L.txt 2>&1 || exit 1; grep -v amdgpu $O/small_c20b_l$L.txt | sed "s/^/L$L /" | cut -c1-170; done &&
for L in 2 3; do
  MSM_BATCH_LANES=$L timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --beta 1 --warmup 5 > $O/bench_beta_l$L.json 2> $O/bench_beta_l$L.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench_beta_l$L.json')); print('beta L$L', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
done &&
timeout -k 10 600 python3 -u bench.py > $O/bench_full.json 2> $O/bench_full.err &&
python3 -c "
import json; d=json.load(open('$O/bench_full.json')); print('full', d['value'], d['parity_vs_reference'])
for k,v in d['methods'].items(): print(' ', k, v.get('value'), v.get('ms_per_step'), v.get('parity_vs_reference'), v.get('ratio_vs_ctx_sync',''))
print(d['cpu_baseline'])" &&
for MP in 1 0; do MSM_MULTI_PIPELINE=$MP timeout -k 10 400 python3 -u bench.py --multi-context 8 --one-device --steps 10 --warmup 2 --no-cpu-baseline --no-configs > $O/mc8_p$MP.json 2> $O/mc8_p$MP.err || exit 1
python3 -c "import json; d=json.load(open('$O/mc8_p$MP.json')); print('mc8 pipeline=$MP', d['value'], {k: (v.get('value'), v.get('ms_per_step'), v.get('parity_vs_reference')) for k, v in d['methods'].items() if 'cfg3' in k})"; done &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29538 bench.py --gpus 8 --dist-backend gloo --one-device --steps 10 --warmup 2 --no-cpu-baseline > $O/n8.json 2> $O/n8.err &&
python3 -c "import json; d=json.loads(open('$O/n8.json').read().strip().splitlines()[-1]); print('N=8', d['value'], d['scaling'], d['config']['n_total'], d['parity_vs_reference'])" &&
cp tools/ablib/libmsm_lean.so msm_blst_amd/libmsm_mi355x.so &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_table_rows.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_lean_rows.txt 2>&1
echo "lean rows rc=$?"; grep -E "PASSED|FAILED|rows differ" $O/pytest_lean_rows.txt | head -20
echo "done $(date +%T)"
