#!/bin/bash
# round-4 call 2: two-lane batch schedule -- batch parity tests, small-MSM timings
# (lanes auto vs 1), strong-scaling rehearsal N = 2, 4, 8 (gloo, one device)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04b}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ches.py tests/test_gpu_multi.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_batch.txt 2>&1 &&
echo "pytest ok $(date +%T) $(tail -1 $O/pytest_batch.txt)" &&
timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 c20 > $O/small_auto.txt 2>&1 &&
MSM_BATCH_LANES=1 timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 > $O/small_l1.txt 2>&1 &&
MSM_BATCH_LANES=2 timeout -k 10 300 python3 -u tools/r04_small_trace.py c20 > $O/small_l2_c20.txt 2>&1 &&
cat $O/small_auto.txt $O/small_l1.txt $O/small_l2_c20.txt | grep -v amdgpu.ids &&
for N in 2 4 8; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2953$N \
    bench.py --gpus $N --dist-backend gloo --one-device --steps 10 --warmup 2 --no-cpu-baseline > $O/n$N.json 2> $O/n$N.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/n$N.json').read().strip().splitlines()[-1]); print('N=$N', d['value'], d['scaling'], d['config']['n_total'], d['parity_vs_reference'], {k: (v.get('value'), v.get('parity_vs_reference')) for k, v in d['methods'].items()})"
done
echo "done $(date +%T)"
