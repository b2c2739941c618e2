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
    g2) timeout -k 10 400 python -u bench.py --group 2 --no-configs --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err; rc=$?
        python3 tools/bench_summary.py $O/bench_g2.json ;;
    prof) cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-configs --no-cpu-baseline > $O/prof.json 2> $O/prof.log; rc=$?; cd $R ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "[$step] rc=$rc $(date +%T)"
  [ $rc -eq 0 ] || exit $rc
done
