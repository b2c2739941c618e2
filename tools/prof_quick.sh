#!/bin/bash
# rocprofv3 kernel trace + stats of tools/quick_ches.py <group> <log_n> into gpurun_out/<tag>/
# usage (repo root, via gpurun): bash tools/prof_quick.sh <tag> <group> <log_n>
TAG=$1
R=$(pwd)
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python3 $R/tools/quick_ches.py $2 $3 > $R/gpurun_out/$TAG/log.txt 2>&1
