#!/bin/bash
# round-4 call 16: the bench's setup batch (one untimed resident batch of the K
# sets when the context is set up) vs none, at --warmup 3 and 5, three runs
# each, through bench.py itself
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04p}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2 3; do
  for SB in 0 1; do
    for W in 3 5; do
      L=sb${SB}_w${W}_$i
      timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline --setup-batch $SB --warmup $W > $O/$L.json 2> $O/$L.err || exit 1
      python3 -c "import json; d=json.load(open('$O/$L.json')); print('$L', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
    done
  done
done
echo "done $(date +%T)"
