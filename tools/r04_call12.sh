#!/bin/bash
# round-4 call 12: level 0 inside the next accumulation's grid (MSM_L0_FUSE=1:
# level-0 workgroups first, =2: last) vs the separate level-0 launch; batch
# tests under the fused schedule first
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04l}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
MSM_L0_FUSE=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ches.py tests/test_gpu_multi.py tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_fuse1.txt 2>&1
rc=$?; echo "pytest fuse1 rc=$rc $(date +%T) $(tail -1 $O/pytest_fuse1.txt)"; grep -E "FAILED|^E " $O/pytest_fuse1.txt | head -20
[ $rc -eq 0 ] || exit 1
run() {  # label, env...
  L=$1; shift
  env "$@" AB_LABEL=$L timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 4 > $O/ab_$L.txt 2> $O/ab_$L.err || exit 1
  grep "h2d:\|resident:" $O/ab_$L.txt
}
for i in 1 2; do
  run base$i MSM_L0_FUSE=0
  run fuse1_$i MSM_L0_FUSE=1
  run fuse2_$i MSM_L0_FUSE=2
  run freehi$i MSM_L0_FUSE=0 MSM_ACC_AFTER_L0=0 MSM_TAIL_PRIO=1
done
for F in 0 1; do
  MSM_L0_FUSE=$F timeout -k 10 400 python3 -u bench.py --group 2 --no-configs --no-cpu-baseline --no-compare > $O/g2_f$F.json 2> $O/g2_f$F.err || exit 1
  python3 -c "import json; d=json.load(open('$O/g2_f$F.json')); print('G2 fuse $F', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity_vs_reference'])"
done
echo "done $(date +%T)"
