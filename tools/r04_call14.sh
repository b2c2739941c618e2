#!/bin/bash
# round-4 call 14: level-0 chunk 9 / 10 (one round of the chip's wave slots)
# vs 8, and host scalars read by the front kernels straight from pinned
# memory (MSM_ZERO_COPY_SCALARS=1) vs SDMA copies; tools/h2d_ab.py, two
# processes per variant; G2 level 0 at 3 waves per SIMD (variant library)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${1:-r04n}
mkdir -p $O
export TMPDIR=/tmp
echo "start $(date +%T)"
run() {  # label, env...
  L=$1; shift
  env "$@" AB_LABEL=$L timeout -k 10 300 python3 -u tools/h2d_ab.py --reps 3 > $O/ab_$L.txt 2> $O/ab_$L.err || exit 1
  grep "h2d:\|resident:" $O/ab_$L.txt
}
for i in 1 2; do
  run c8_$i MSM_L0_CHUNK=8
  run c9_$i MSM_L0_CHUNK=9
  run c10_$i MSM_L0_CHUNK=10
  run zc_$i MSM_ZERO_COPY_SCALARS=1
done
# G2 level 0 (k_segsum2p) at 3 waves per SIMD (168 VGPRs + 448 B scratch) vs 2 (227 VGPRs)
for V in base s2w3 base2 s2w3b; do
  case $V in s2w3*) cp tools/ablib/libmsm_s2w3.so msm_blst_amd/libmsm_mi355x.so ;; esac
  timeout -k 10 400 python3 -u bench.py --group 2 --no-configs --no-cpu-baseline > $O/g2_$V.json 2> $O/g2_$V.err || exit 1
  python3 -c "import json; d=json.load(open('$O/g2_$V.json')); print('G2 $V', d['value'], d['ms_per_step'], {k: v.get('value') for k, v in d['methods'].items()}, d['phases_ms'])"
  case $V in s2w3) cp /tmp/lib_base_$$.so msm_blst_amd/libmsm_mi355x.so ;; base) cp msm_blst_amd/libmsm_mi355x.so /tmp/lib_base_$$.so ;; esac
done
rm -f /tmp/lib_base_$$.so
echo "done $(date +%T)"
