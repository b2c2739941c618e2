#!/bin/bash
# Why does the H2D headline sit 0.1-0.4 ms per MSM behind the resident batch?
# (1) resident batch alone / beside unrelated H2D and D2D copies
# (2) bench.py headline: default, zero-copy scalar reads, default again, --warmup 20
# usage (repo root, via gpurun): bash tools/r03_h2d_probe.sh <tag>
set -o pipefail
TAG=${1:-r03h}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
B="--no-configs --no-cpu-baseline"
timeout -k 10 180 python -u tools/copy_interference.py > $O/copy_interference.json 2> $O/copy_interference.err &&
echo "interference: $(cat $O/copy_interference.json)" &&
timeout -k 10 180 python -u bench.py $B > $O/def1.json 2> $O/def1.err &&
MSM_ZERO_COPY_SCALARS=1 timeout -k 10 180 python -u bench.py $B > $O/zc.json 2> $O/zc.err &&
timeout -k 10 180 python -u bench.py $B > $O/def2.json 2> $O/def2.err &&
timeout -k 10 180 python -u bench.py $B --warmup 20 > $O/warm20.json 2> $O/warm20.err &&
for f in def1 zc def2 warm20; do
  python3 -c "import json,sys; d=json.load(open('$O/$f.json')); m=d['methods']; print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], m['ches_batch_resident']['value'], m['ches_batch_resident']['kernel_ms'])"
done
echo "rc=$?"
