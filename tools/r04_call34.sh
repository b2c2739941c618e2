#!/bin/bash
# round-4 call 34: kernel + memory-copy trace of the 2^20 blst_p1s_mult_pippenger
# drop-in (tools/dropin_timing.py 20), for the per-call timeline
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04ai}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/dropin_timing.py 20 > $O/plain.json 2> $O/plain.err && cat $O/plain.json &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t -o run -- python3 $R/tools/dropin_timing.py 20 > $O/t.json 2> $O/t.err && cat $O/t.json
echo "done $(date +%T)"
