#!/bin/bash
# kernel trace of the small-MSM batches (tools/r06_small_trace.py), split and
# summarised by tools/batch_profile.py; tools/tail_listing.py lists each
# batch's exposed tail.  usage (via gpurun): bash tools/r06_trace.sh <tag> [cases]
set -o pipefail
TAG=${1:-r06tr}
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- python3 $R/tools/r06_small_trace.py ${2:-pip16 ches17} > $O/run.txt 2> $O/run.err || exit 1
cd $R && python3 tools/batch_profile.py $O/t/run_kernel_trace.csv > $O/summary.txt && python3 tools/tail_listing.py $O/t/run_kernel_trace.csv > $O/tails.txt && cat $O/run.txt $O/summary.txt | head -150
