#!/bin/bash
# kernel-trace of a short CHES batch bench (timeline analysis: tools/timeline.py)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-t}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-compare > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-compare > $O/log.txt 2>&1
echo rc=$?
