// One field / curve operation per kernel, for instruction counts of the
// device code (tools/isa_report.sh): hipcc -S --cuda-device-only, then
// tools/isa_count.py on each kernel.
#include "../../msm_blst_amd/csrc/ec.hpp"
#include "../../msm_blst_amd/csrc/fp2l.hpp"

using namespace msm;

__global__ void k_op_fp_mul(const Fp *a, const Fp *b, Fp *r) {
  const int t = threadIdx.x;
  Fp x = a[t], y = b[t], z;
  fp_mul(z, x, y);
  r[t] = z;
}
__global__ void k_op_fp_sqr(const Fp *a, Fp *r) {
  const int t = threadIdx.x;
  Fp x = a[t], z;
  fp_sqr(z, x);
  r[t] = z;
}
__global__ void k_op_fp_mul2(const Fp *a, const Fp *b, Fp *r) {
  const int t = threadIdx.x;
  Fp x = a[t], y = b[t], u = a[t + 64], v = b[t + 64], z;
  fp_mul2(z, x, y, u, v);
  r[t] = z;
}
// G2 on lane pairs (fp2l.hpp): the three products of the lane-pair madd, per lane
__global__ void k_op_g2l_mul_bs(const Fp2L *a, const Fp2L *b, Fp2L *r) {
  const int t = threadIdx.x;
  Fp2L x = a[t], y = b[t], z;
  f_mul_bs(z, x, y);
  r[t] = z;
}
__global__ void k_op_g2l_sqr(const Fp2L *a, Fp2L *r) {
  const int t = threadIdx.x;
  Fp2L x = a[t], z;
  f_sqr(z, x);
  r[t] = z;
}
__global__ void k_op_g2l_mul_sub(const Fp2L *a, const Fp2L *b, Fp2L *r) {
  const int t = threadIdx.x;
  Fp2L x = a[t], y = b[t], u = a[t + 64], v = b[t + 64], z;
  f_mul_sub(z, x, y, u, v);
  r[t] = z;
}
__global__ void __launch_bounds__(256, 3) k_op_g1_madd(const Xyzz<Fp> *acc, const Aff<Fp> *p, Xyzz<Fp> *r) {
  const int t = threadIdx.x;
  Xyzz<Fp> q = acc[t];
  xyzz_madd(q, p[t], (t & 1) != 0);
  r[t] = q;
}
__global__ void __launch_bounds__(256) k_op_g2l_madd(const Xyzz<Fp2L> *acc, const Aff<Fp2L> *p, Xyzz<Fp2L> *r) {
  const int t = threadIdx.x;
  Xyzz<Fp2L> q = acc[t];
  xyzz_madd(q, p[t], (t & 2) != 0);
  r[t] = q;
}
