// Does a Montgomery product issue faster as ONE dependent mad chain?
// fp.hpp fp_mul (as compiled: each column's a*b sum is an independent chain
// merged with the carry by one v_lshl_add_u64 -- 26 merges per product) vs
// fp_mul_serial below (the same terms in the same order, each v_mad_u64_u32 in
// inline asm so the compiler cannot split the chain: the carry is the addend of
// the next column's first mad; 26 fewer VALU ops, a 392-long dependency chain).
// fp_mul_col (serial_col.inc, tools/microbench/gen_serial_col.py): the same
// chain with one asm block per column half (fewer compiler-inserted s_nops).
// Register-resident loop of two independent products per lane (the probe's
// k_probe_fpmul), at 2 / 3 / 4 waves per SIMD; prints Fp-mul/s and checks the
// two versions agree bit for bit.
// hipcc -O3 --offload-arch=gfx950 -I msm_blst_amd/csrc tools/microbench/serial_chain.hip -o serial_chain
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "fp.hpp"

using namespace msm;

__device__ __forceinline__ uint64_t mad_v(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c), "=&s"(cc) : "v"(a), "v"(b));
  return c;
}
__device__ __forceinline__ uint64_t mad_s(uint32_t a, uint32_t b, uint64_t c) {  // b uniform (p's limbs)
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c), "=&s"(cc) : "v"(a), "s"(b));
  return c;
}

__device__ __forceinline__ void fp_mul_serial(Fp &r, const Fp &a, const Fp &b) {
  uint32_t m[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) acc = mad_v(a.v[i], b.v[k - i], acc);
#pragma unroll
    for (int i = 0; i < k; ++i) acc = mad_s(m[i], P28[k - i], acc);
    m[k] = ((uint32_t)acc * N0P) & MASK;
    acc = mad_s(m[k], P28[0], acc);
    acc >>= 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; ++k) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad_v(a.v[i], b.v[k - i], acc);
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad_s(m[i], P28[k - i], acc);
    r.v[k - NL] = (uint32_t)acc & MASK;
    acc >>= 28;
  }
  r.v[NL - 1] = (uint32_t)acc;
}

#include "serial_col.inc"

// one-level Karatsuba on the product half: a = a_lo +
// a_hi X, X = 2^196 (7 + 7 limbs); a b = P0 + (P1 - P0 - P2) X + P2 X^2 with
// P0 = a_lo b_lo, P2 = a_hi b_hi, P1 = (a_lo + a_hi)(b_lo + b_hi): 147 mads
// instead of 196, then the same FIPS reduction over the 27 columns.  Needs
// normalized inputs (limbs < 2^28: limb sums < 2^29, a P1 column of 7 terms
// < 2^61); every column of P1 - P0 - P2 is a sum of cross products, >= 0.
__device__ __forceinline__ void fp_mul_kara(Fp &r, const Fp &a, const Fp &b) {
  constexpr int H = NL / 2;
  uint32_t sa[H], sb[H];
#pragma unroll
  for (int i = 0; i < H; ++i) sa[i] = a.v[i] + a.v[i + H], sb[i] = b.v[i] + b.v[i + H];
  uint64_t p0[2 * H - 1], p1[2 * H - 1], p2[2 * H - 1];
#pragma unroll
  for (int k = 0; k < 2 * H - 1; ++k) {
    const int lo = k < H ? 0 : k - H + 1, hi = k < H ? k : H - 1;
    uint64_t x = 0, y = 0, z = 0;
#pragma unroll
    for (int i = lo; i <= hi; ++i) {
      x = mad64(a.v[i], b.v[k - i], x);
      y = mad64(sa[i], sb[k - i], y);
      z = mad64(a.v[i + H], b.v[k - i + H], z);
    }
    p0[k] = x, p1[k] = y - x - z, p2[k] = z;
  }
  uint32_t m[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; ++k) {
    uint64_t c = 0;
    if (k <= 2 * H - 2) c += p0[k];
    if (k >= H && k - H <= 2 * H - 2) c += p1[k - H];
    if (k >= 2 * H) c += p2[k - 2 * H];
    acc += c;
    if (k < NL) {
#pragma unroll
      for (int i = 0; i < k; ++i) acc = mad64(m[i], P28[k - i], acc);
      m[k] = ((uint32_t)acc * N0P) & MASK;
      acc = mad64(m[k], P28[0], acc);
    } else {
#pragma unroll
      for (int i = k - NL + 1; i < NL; ++i) acc = mad64(m[i], P28[k - i], acc);
      r.v[k - NL] = (uint32_t)acc & MASK;
    }
    acc >>= 28;
  }
  r.v[NL - 1] = (uint32_t)acc;
}

template <int SERIAL, int W>
__global__ void __launch_bounds__(256, W) k_rate(uint32_t *out, int iters) {
  const uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  Fp a, b, c, d;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    a.v[i] = (t * 0x9e3779b9u + i) & MASK;
    b.v[i] = (t * 0x85ebca6bu + 3 * i) & MASK;
    c.v[i] = (t * 0xc2b2ae35u + 7 * i) & MASK;
  }
  a.v[NL - 1] &= 0xffff;
  b.v[NL - 1] &= 0xffff;
  c.v[NL - 1] &= 0xffff;
  for (int it = 0; it < iters; ++it) {
    if (SERIAL == 3) {
      fp_mul_kara(d, a, b);
      fp_mul_kara(a, c, b);
    } else if (SERIAL == 2) {
      fp_mul_col(d, a, b);
      fp_mul_col(a, c, b);
    } else if (SERIAL) {
      fp_mul_serial(d, a, b);
      fp_mul_serial(a, c, b);
    } else {
      fp_mul(d, a, b);
      fp_mul(a, c, b);
    }
    c = d;
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) s ^= a.v[i] * (i + 1) ^ c.v[i] * (i + 7);
  out[t] = s;
}

template <int SERIAL, int W>
static double rate(uint32_t *out, int cus, std::vector<uint32_t> &host) {
  const int blocks = cus * W, iters = 512;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((k_rate<SERIAL, W>), dim3(blocks), dim3(256), 0, 0, out, iters);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_rate<SERIAL, W>), dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = best < ms ? best : ms;
  }
  host.resize((size_t)blocks * 256);
  (void)hipMemcpy(host.data(), out, host.size() * 4, hipMemcpyDeviceToHost);
  return (double)blocks * 256 * iters * 2 / (best * 1e-3);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t *out;
  if (hipMalloc(&out, (size_t)cus * 8 * 256 * 4) != hipSuccess) return 1;
  std::vector<uint32_t> h0, h1;
  for (int rep = 0; rep < 2; ++rep) {
    std::vector<uint32_t> h2, h3;
    double b2 = rate<0, 2>(out, cus, h0), s2 = rate<1, 2>(out, cus, h1), c2 = rate<2, 2>(out, cus, h2),
           k2 = rate<3, 2>(out, cus, h3);
    bool same2 = h0 == h1 && h0 == h2 && h0 == h3;
    double b3 = rate<0, 3>(out, cus, h0), s3 = rate<1, 3>(out, cus, h1), c3 = rate<2, 3>(out, cus, h2),
           k3 = rate<3, 3>(out, cus, h3);
    bool same3 = h0 == h1 && h0 == h2 && h0 == h3;
    double b4 = rate<0, 4>(out, cus, h0), s4 = rate<1, 4>(out, cus, h1), c4 = rate<2, 4>(out, cus, h2),
           k4 = rate<3, 4>(out, cus, h3);
    bool same4 = h0 == h1 && h0 == h2 && h0 == h3;
    printf("waves/SIMD 2: split %.2f G  serial %.2f G  column-asm %.2f G  karatsuba %.2f G  same %d\n", b2 / 1e9, s2 / 1e9, c2 / 1e9, k2 / 1e9, same2);
    printf("waves/SIMD 3: split %.2f G  serial %.2f G  column-asm %.2f G  karatsuba %.2f G  same %d\n", b3 / 1e9, s3 / 1e9, c3 / 1e9, k3 / 1e9, same3);
    printf("waves/SIMD 4: split %.2f G  serial %.2f G  column-asm %.2f G  karatsuba %.2f G  same %d\n", b4 / 1e9, s4 / 1e9, c4 / 1e9, k4 / 1e9, same4);
  }
  (void)hipFree(out);
  return 0;
}
