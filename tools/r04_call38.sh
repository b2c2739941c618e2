#!/bin/bash
# round-4 call 38 (round-5 planning data, no code change): kernel trace of the
# 2^17 strong-scaling shard batch (three lanes, front groups of 4) and a kernel
# summary of where its GPU time goes
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04am}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p17 -o run -- python3 $R/tools/r04_small_trace.py c17 > $O/p17.txt 2>&1 &&
cd $R && grep -v amdgpu $O/p17.txt | cut -c1-150 && python3 tools/trace_seq.py $O/p17/run_kernel_trace.csv k_accumulate 40 60 > $O/p17_seq.txt && head -70 $O/p17_seq.txt
echo "done $(date +%T)"
