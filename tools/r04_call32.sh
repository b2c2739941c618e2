#!/bin/bash
# round-4 call 32: G2 2^20 batch with accumulation k+1 waiting for level 0 of
# k (MSM_ACC_AFTER_L0=1, the G1 default) vs free-running (G2 default), three
# runs each, H2D headline + resident
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ag}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for i in 1 2 3; do
  for A in 0 1; do
    MSM_ACC_AFTER_L0=$A timeout -k 10 400 python3 -u bench.py --group 2 --no-configs --no-cpu-baseline > $O/g2_a${A}_$i.json 2> $O/g2_a${A}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('$O/g2_a${A}_$i.json')); print('G2 wait=$A', d['value'], d['methods']['ches_batch_resident']['value'], d['roofline']['kernel_ms'])"
  done
done
echo "done $(date +%T)"
