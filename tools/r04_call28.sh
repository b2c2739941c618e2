#!/bin/bash
# round-4 call 28: three lanes + front groups of 4 as the small-G1 default --
# batch / multi / parity tests, small-MSM timings, N = 8 strong rehearsal
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ac}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ches.py tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_gpu_small_reductions.py tests/test_gpu_blst_ches_abi.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc $(date +%T) $(tail -1 $O/pytest.txt)"; grep -E "FAILED|^E " $O/pytest.txt | head -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 c19 > $O/small.txt 2>&1 && grep -v amdgpu $O/small.txt | cut -c1-150 &&
for N in 8 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29570 + N)) bench.py --gpus $N --dist-backend gloo --one-device --steps 10 --warmup 2 --no-cpu-baseline > $O/n$N.json 2> $O/n$N.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/n$N.json').read().strip().splitlines()[-1]); print('N=$N', d['value'], d['scaling'], d['config']['n_total'], d['parity_vs_reference'])"
done
echo "done $(date +%T)"
