#!/bin/bash
# A/B of the batch front placement (MSM_FRONT_SERIAL) through bench.py, alternating runs on one box
set -o pipefail
TAG=${1:-r03s2}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B="--no-configs --no-cpu-baseline"
summ() { python3 -c "import json,sys; d=json.load(open('$O/$1.json')); m=d['methods']; print('$1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], m['ches_batch_resident']['value'], m['ches_batch_resident']['ms_per_step'], m['ches_batch_resident']['kernel_ms'], d['phases_ms']['accumulate'], d['parity_vs_reference'])"; }
for i in 1 2; do
  timeout -k 10 180 python -u bench.py $B --warmup 5 > $O/def$i.json 2> $O/def$i.err && summ def$i &&
  MSM_FRONT_SERIAL=1 timeout -k 10 180 python -u bench.py $B --warmup 5 > $O/ser$i.json 2> $O/ser$i.err && summ ser$i || exit 1
done
echo "rc=$?"
