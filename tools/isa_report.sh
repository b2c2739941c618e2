#!/bin/bash
# Instruction counts of the device code (CPU only: hipcc -S for gfx950):
# one Montgomery product / square / two-product sum, one xyzz madd (G1, G2 lane
# pair) and the accumulation kernels as built.  usage: bash tools/isa_report.sh > profiles/<round>_isa_counts.txt
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
HIPCC="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -I$R/include"
$HIPCC -o $T/ops.s $R/tools/microbench/isa_ops.hip
$HIPCC -DMSM_GROUP=1 -o $T/ches1.s $R/msm_blst_amd/csrc/ches.hip
$HIPCC -DMSM_GROUP=2 -o $T/ches2.s $R/msm_blst_amd/csrc/ches.hip
echo "# gfx950 ISA instruction counts ($(date -u +%F), $(git -C $R rev-parse --short HEAD))"
echo "# per-op kernels: tools/microbench/isa_ops.hip (one op between a load and a store)"
for k in _Z11k_op_fp_mulP k_op_fp_sqr k_op_fp_mul2 k_op_g2l_mul_bs k_op_g2l_sqr k_op_g2l_mul_sub k_op_g1_madd k_op_g2l_madd; do python3 $R/tools/isa_count.py $T/ops.s $k; done
echo "# accumulation kernels as built (ches.hip, MSM_GROUP=1 / 2)"
python3 $R/tools/isa_count.py $T/ches1.s k_accumulate
python3 $R/tools/isa_count.py $T/ches2.s k_accumulate2p
rm -rf $T
