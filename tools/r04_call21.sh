#!/bin/bash
# round-4 call 21: kernel + memory-copy trace of the bench's H2D headline and
# resident batches with the slot-per-set copy schedule (tools/h2d_trace.py)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04u}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t1 -o run -- python3 $R/bench.py --no-configs --no-cpu-baseline --warmup 5 > $O/t1.json 2> $O/t1.err &&
python3 -c "import json; d=json.load(open('$O/t1.json')); print('t1', d['value'], d['methods']['ches_batch_resident']['value'])" &&
cd $R && python3 tools/h2d_trace.py $O/t1/run 5 20 > $O/t1_h2d.txt && python3 tools/h2d_trace.py $O/t1/run 25 20 > $O/t1_res.txt && tail -3 $O/t1_h2d.txt $O/t1_res.txt
echo "done $(date +%T)"
