#!/bin/bash
# Round-3 session: schedule-ordered bucket metadata + payload window.
# GPU parity subset, same-box A/B of cur vs prev, then PMC FETCH/WRITE passes (separate runs).
R=$(pwd)
O=$R/gpurun_out/${1:-r03s}
mkdir -p $O
cp tools/ablib/libmsm_cur.so msm_blst_amd/libmsm_mi355x.so || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
VARIANTS="${VARIANTS:-cur prev}" bash tools/ab_bench.sh ${1:-r03s}/ab 2 --steps 20 --warmup 3 --no-configs || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 20 --no-configs > $O/warm20.json 2> $O/warm20.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch --no-configs > $O/pmc_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-compare --no-batch --no-configs > $O/pmc_write.log 2>&1 &&
echo "pmc ok"
cd $R
[ -n "$G2PROF" ] && bash tools/prof_quick.sh ${1:-r03s}/g2prof 2 20 && echo "g2prof ok"
true
