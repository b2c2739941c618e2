#!/bin/bash
# round-4 call 24: host worker threads for the drop-in staging and the
# pointer-array gather (MSM_HOST_THREADS, default 8 = 7 workers + caller) vs
# 16 (the box's CPU share per GPU); full bench.py twice each
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04x}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
for T in 8 16 8 16; do
  MSM_HOST_THREADS=$T timeout -k 10 600 python3 -u bench.py --no-cpu-baseline > $O/b_t$T.json 2> $O/b_t$T.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/b_t$T.json')); m=d['methods']
print('threads $T', d['value'], {k: (m[k]['ms_per_step'], m[k].get('ratio_vs_ctx_sync'), m[k].get('parity_vs_reference')) for k in m if 'blst' in k or 'tile' in k})"
done
echo "done $(date +%T)"
