#!/bin/bash
# cold-GPU probe: tools/warm_probe.py with warm-up batches of 3 and 0, plus a kernel trace of the first
set -o pipefail
TAG=${1:-r03w}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/warm_probe.py 3 > $O/w3.json 2> $O/w3.err &&
cat $O/w3.json &&
timeout -k 10 180 python -u tools/warm_probe.py 1 > $O/w1.json 2> $O/w1.err &&
cat $O/w1.json &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/tools/warm_probe.py 3 > $O/prof.json 2> $O/prof.err &&
cat $O/prof.json
echo "rc=$?"
