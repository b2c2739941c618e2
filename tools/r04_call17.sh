#!/bin/bash
# round-4 call 17: bench.py headline at --warmup 3 / 5 with 4 (box default) vs
# 8 vs 16 hardware queues per process (GPU_MAX_HW_QUEUES), three runs each
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04q}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T) GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
for i in 1 2 3; do
  for Q in 4 8 16; do
    for W in 3 5; do
      L=q${Q}_w${W}_$i
      GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --setup-batch 0 --warmup $W > $O/$L.json 2> $O/$L.err || exit 1
      python3 -c "import json; d=json.load(open('$O/$L.json')); print('$L', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
    done
  done
done
echo "done $(date +%T)"
