#!/bin/bash
# kernel + memory-copy trace of tools/warm_probe.py (resident / H2D legs alternating)
set -o pipefail
TAG=${1:-r03ct}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/prof -o run -- python3 $R/tools/warm_probe.py 3 > $O/probe.json 2> $O/probe.err &&
cat $O/probe.json && ls $O/prof
echo "rc=$?"
