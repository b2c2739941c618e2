#!/bin/bash
# round-4 call 7: GPU suite with the lean doubling default; warmup-length study
# (W 3/4/5, slot touch); G2 batch regression check; small-n front groups / lanes
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04g}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc $(date +%T) $(tail -1 $O/pytest_gpu.txt)"; grep -E "FAILED|^E " $O/pytest_gpu.txt | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
b() { # tag, env..., then bench args after --
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --no-configs --no-cpu-baseline $BARGS > $O/bench_$tag.json 2> $O/bench_$tag.err || return 1
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); m=d['methods']; print('$tag', d['value'], m.get('ches_batch_resident',{}).get('value'), d['roofline']['kernel_ms'], d['phases_ms']['accumulate'], d['parity_vs_reference'])"
}
BARGS="--warmup 3" b w3 A=1 && BARGS="--warmup 4" b w4 A=1 && BARGS="--warmup 5" b w5 A=1 &&
BARGS="--warmup 3" b w3touch MSM_TOUCH_SLOTS=1 && BARGS="--warmup 5" b w5touch MSM_TOUCH_SLOTS=1 && BARGS="--warmup 3" b w3touchb MSM_TOUCH_SLOTS=1 &&
BARGS="--group 2 --steps 10" b g2 A=1 && BARGS="--group 2 --steps 10" b g2l0 MSM_ACC_AFTER_L0=1 && BARGS="--group 2 --steps 10" b g2lanes2 MSM_BATCH_LANES=2 &&
for FG in 2 4; do MSM_FRONT_GROUP=$FG timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 > $O/small_fg$FG.txt 2>&1 || exit 1; grep -v amdgpu $O/small_fg$FG.txt | sed "s/^/fg$FG /" | cut -c1-140; done &&
MSM_BATCH_LANES=3 timeout -k 10 300 python3 -u tools/r04_small_trace.py c17 c18 > $O/small_l3.txt 2>&1 && grep -v amdgpu $O/small_l3.txt | sed "s/^/l3 /" | cut -c1-140 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/profg2 -o run -- python3 $R/bench.py --group 2 --no-configs --no-cpu-baseline --no-compare --steps 10 --warmup 2 > $O/profg2.txt 2>&1 &&
echo "done $(date +%T)"
