#!/bin/bash
# Round-5 GPU session steps, chained with && (each GPU step under its own limit).
# usage (repo root, via gpurun): bash tools/r05_session.sh <tag> <step>...
#   steps: new (one-lane batch tests) | suite (pytest -m gpu) | smoke | bench | shards (tools/shard_study.py)
#          | g2 (bench --group 2) | prof (rocprofv3 kernel trace + stats of the default bench)
set -o pipefail
TAG=$1; shift
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  echo "[$step] start $(date +%T)"
  case $step in
    new) timeout -k 10 500 python -u -m pytest tests/test_gpu_batch_one_lane.py -x -v --timeout 300 --timeout-method thread > $O/pytest_new.txt 2>&1; rc=$?; tail -3 $O/pytest_new.txt ;;
    suite) timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?; tail -2 $O/pytest_gpu.txt ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?; tail -2 $O/smoke.txt ;;
    bench) timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
           python3 tools/bench_summary.py $O/bench.json ;;
    shards) timeout -k 10 400 python -u tools/shard_study.py > $O/shards.txt 2> $O/shards.err; rc=$?; cat $O/shards.txt ;;
    pip) timeout -k 10 500 python -u tools/pip_study.py --windows 13,14 --envs "MSM_FRONT_PHASE=0;MSM_FRONT_PHASE=1;MSM_FRONT_PHASE=1 MSM_PIP_FRONT_GROUP=8;MSM_FRONT_PHASE=1 MSM_PIP_FRONT_GROUP=2" > $O/pip.txt 2> $O/pip.err; rc=$?; cat $O/pip.txt ;;
    piptests) timeout -k 10 300 python -u -m pytest tests/test_gpu_pippenger_batch.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/pytest_pip.txt 2>&1; rc=$?; tail -3 $O/pytest_pip.txt ;;
    shards_ab) timeout -k 10 500 python -u tools/shard_study.py --cfgs 20,19 > $O/shards_ab.txt 2> $O/shards_ab.err && MSM_BATCH_L0_CHUNK=0 MSM_TAIL_COOP=0 timeout -k 10 500 python -u tools/shard_study.py --cfgs 20,19 >> $O/shards_ab.txt 2>> $O/shards_ab.err; rc=$?; cat $O/shards_ab.txt ;;
    ptrace) cd /tmp && MSM_PIP_L0_CHUNK=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ptrace -o run -- python3 $R/tools/r04_small_trace.py pb16 > $O/ptrace.txt 2> $O/ptrace.err; rc=$?; cd $R
           cat $O/ptrace.txt; python3 tools/batch_profile.py $O/ptrace/run_kernel_trace.csv > $O/ptrace_profile.txt; cat $O/ptrace_profile.txt ;;
    trace) cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/r04_small_trace.py pb16 c17 > $O/trace.txt 2> $O/trace.err; rc=$?; cd $R
           cat $O/trace.txt; python3 tools/batch_profile.py $O/trace/run_kernel_trace.csv > $O/trace_profile.txt; cat $O/trace_profile.txt ;;
    shards_acc) timeout -k 10 300 python -u tools/shard_study.py --cfgs 20,19 > $O/shards_acc.txt 2> $O/shards_acc.err && MSM_FRONT_PHASE=0 timeout -k 10 300 python -u tools/shard_study.py --cfgs 20 >> $O/shards_acc.txt 2>> $O/shards_acc.err && MSM_FRONT_GROUP=8 timeout -k 10 300 python -u tools/shard_study.py --cfgs 20,19 >> $O/shards_acc.txt 2>> $O/shards_acc.err; rc=$?; cat $O/shards_acc.txt ;;
    abitests) timeout -k 10 400 python -u -m pytest tests/test_gpu_blst_ches_abi.py tests/test_gpu_tile_grid.py tests/test_gpu_dropin.py tests/test_gpu_pointer_gather.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/pytest_abi.txt 2>&1; rc=$?; tail -3 $O/pytest_abi.txt ;;
    rccltests) timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multi.py -x -v --timeout 300 --timeout-method thread > $O/pytest_rccl.txt 2>&1; rc=$?; tail -5 $O/pytest_rccl.txt ;;
    batchtests) timeout -k 10 500 python -u -m pytest tests/test_gpu_ches.py tests/test_gpu_batch_one_lane.py tests/test_gpu_multi.py -x -v --timeout 300 --timeout-method thread > $O/pytest_batch.txt 2>&1; rc=$?; tail -3 $O/pytest_batch.txt ;;
    tile) timeout -k 10 300 python -u tools/tile_timing.py > $O/tile.txt 2> $O/tile.err; rc=$?; cat $O/tile.txt; grep "\[tile\]" $O/tile.err ;;
    rehearse) for N in 2 4 8; do
        timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29560 + N)) bench.py --gpus $N --dist-backend gloo --one-device --steps 10 --warmup 2 --no-cpu-baseline > $O/n$N.json 2> $O/n$N.err || { rc=1; break; }
        python3 -c "import json; d=json.loads(open('$O/n$N.json').read().strip().splitlines()[-1]); print('N=$N', d['value'], d['scaling'], d['config']['n_total'], d['parity_vs_reference'], {k: (v.get('value'), v.get('parity_vs_reference')) for k, v in d['methods'].items()})"
        rc=0
      done ;;
    accrate) timeout -k 10 300 python -u tools/acc_rate.py 16,17,18,19,20 > $O/accrate.txt 2> $O/accrate.err; rc=$?; cat $O/accrate.txt; tail -3 $O/accrate.err ;;
    headab) for fg in 1 2 4 2 1; do
        MSM_FRONT_GROUP=$fg timeout -k 10 300 python -u bench.py --no-configs --no-cpu-baseline --no-shards > $O/head_fg$fg.json 2> $O/head_fg$fg.err || { rc=1; break; }
        echo "FG=$fg $(python3 tools/bench_summary.py $O/head_fg$fg.json | head -4 | tr '\n' ' ')"; rc=0
      done ;;
    g2ab) for fg in 1 2; do
        MSM_FRONT_GROUP=$fg timeout -k 10 300 python -u bench.py --group 2 --no-configs --no-cpu-baseline > $O/g2_fg$fg.json 2> $O/g2_fg$fg.err || { rc=1; break; }
        echo "G2 FG=$fg $(python3 tools/bench_summary.py $O/g2_fg$fg.json | head -3 | tr '\n' ' ')"; rc=0
      done ;;
    g2) timeout -k 10 400 python -u bench.py --group 2 --no-configs --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err; rc=$?
        python3 tools/bench_summary.py $O/bench_g2.json ;;
    prof) cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-configs --no-cpu-baseline > $O/prof.json 2> $O/prof.log; rc=$?; cd $R ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "[$step] rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
