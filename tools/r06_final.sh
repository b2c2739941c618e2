#!/bin/bash
# Round-6 final-tree GPU session: parity suite, smoke, the default bench line,
# rocprofv3 kernel trace + stats of the same bench command (roofline check),
# separate FETCH_SIZE / WRITE_SIZE PMC passes over the accumulation, a
# VALU-busy PMC pass, the G2 line, the one-process configs[3] line and gloo
# rehearsals of --gpus 2 / 8 on the one GPU.
# usage (repo root, via gpurun): bash tools/r06_final.sh <tag>
set -o pipefail
TAG=${1:-r06z}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 &&
echo "pytest ok $(date +%T) $(tail -1 $O/pytest_gpu.txt)" &&
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
echo "smoke ok $(date +%T)" &&
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
echo "bench ok $(date +%T)" && python3 tools/bench_summary.py $O/bench.json &&
cd /tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-configs --no-cpu-baseline --no-shards > $O/prof.json 2> $O/prof.log &&
echo "rocprof ok $(date +%T)" &&
python3 $R/tools/roofline_check.py $O/prof.json $O/prof/run_kernel_trace.csv $O/roofline_check.json &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_write.log 2>&1 &&
python3 $R/tools/pmc_traffic.py $O/pmc_fetch/run_counter_collection.csv $O/pmc_write/run_counter_collection.csv ches 20 $O/pmc_traffic.json $R/profiles/r02_gather_cal.json > /dev/null &&
echo "pmc ok $(date +%T)" && grep accumulate_bytes_per_launch $O/pmc_traffic.json &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES --output-format csv -d $O/pmc_valu -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch > $O/pmc_valu.log 2>&1 &&
echo "pmc valu ok $(date +%T)" &&
cd $R &&
timeout -k 10 400 python3 -u bench.py --group 2 --no-configs --no-cpu-baseline --no-shards > $O/bench_g2.json 2> $O/bench_g2.err &&
python3 tools/bench_summary.py $O/bench_g2.json &&
timeout -k 10 400 python3 -u bench.py --multi-context 8 --one-device --steps 10 --warmup 2 --no-cpu-baseline --no-configs --no-compare --no-shards > $O/mc8.json 2> $O/mc8.err &&
python3 -c "import json; d=json.loads(open('$O/mc8.json').read().strip().splitlines()[-1]); print('mc8', d['legs'].get('cfg3_multi_ctx'))" &&
for N in 2 8; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29560 + N)) bench.py --gpus $N --dist-backend gloo --one-device --steps 10 --warmup 2 --no-cpu-baseline --no-shards > $O/n$N.json 2> $O/n$N.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/n$N.json').read().strip().splitlines()[-1]); print('N=$N', d['value'], d['scaling'], d['config']['n_total'], d['config'].get('config_file'), d['parity_vs_reference'], {k: (v.get('M'), v.get('ok')) for k, v in d['legs'].items()})"
done
echo "rc=$?"
