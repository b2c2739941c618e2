#!/bin/bash
# smoke -> bench -> rocprof kernel-trace stats; each GPU step time-limited, chained with &&
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench_r01.json 2> gpurun_out/bench_r01.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r01 -o run -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_r01.log 2>&1
echo "rc=$?"
