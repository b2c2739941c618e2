#!/bin/bash
# kernel + memory-copy trace of the headline H2D batch (bench.py, no other legs)
# usage (repo root, via gpurun): bash tools/trace_h2d.sh <tag> [bench args]
TAG=$1
shift
R=$(pwd)
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/bench.py --no-configs --no-cpu-baseline --no-compare "$@" > $R/gpurun_out/$TAG/bench.json 2> $R/gpurun_out/$TAG/bench.err
