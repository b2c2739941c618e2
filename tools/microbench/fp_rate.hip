// Fp381 / xyzz throughput microbenchmark for gfx950 (register-resident, no
// memory traffic in the loop).  Gives the "measured peak" the bench's VALU
// roofline is priced against, and the dependent-chain latency of
// v_mad_u64_u32 (which decides whether one FIPS column chain per lane can
// keep a SIMD busy).
//
//   hipcc -O3 --offload-arch=gfx950 -I msm_blst_amd/csrc tools/microbench/fp_rate.hip -o fp_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "kernels.hpp"

using namespace msm;

template <int CH>
__global__ __launch_bounds__(256) void k_mad_chain(uint64_t *out, uint32_t seed, int iters) {
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  uint64_t acc[CH];
  uint32_t a = t | 1, b = seed | 3;
#pragma unroll
  for (int k = 0; k < CH; ++k) acc[k] = t + k;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < CH; ++k) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < CH; ++k) s += acc[k];
  if (s == 0x123456789ull) out[t] = s;
}

__global__ __launch_bounds__(256) void k_fpmul(uint32_t *out, int iters) {
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
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
    fp_mul(d, a, b);  // two independent products per iteration
    fp_mul(a, c, b);
    c = d;
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) s ^= a.v[i] ^ c.v[i];
  out[t] = s;
}

template <int G>
__global__ __launch_bounds__(256) void k_madd(uint32_t *out, const Aff<typename FieldOf<G>::F> *pts, int iters) {
  typedef typename FieldOf<G>::F F;
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  Xyzz<F> acc;
  Aff<F> p = pts[0], q = pts[1];
  xyzz_from_aff(acc, pts[2 + (t & 1)], false);
  for (int it = 0; it < iters; ++it) {
    xyzz_madd(acc, p, (it & 1) != 0);
    xyzz_madd(acc, q, (it & 2) != 0);
  }
  uint32_t s = 0;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(&acc);
  for (int i = 0; i < (int)(sizeof(acc) / 4); ++i) s ^= w[i];
  out[t] = s;
}

template <int G>
__global__ __launch_bounds__(256) void k_add(uint32_t *out, const Aff<typename FieldOf<G>::F> *pts, int iters) {
  typedef typename FieldOf<G>::F F;
  uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  Xyzz<F> acc, b;
  xyzz_from_aff(acc, pts[2 + (t & 1)], false);
  xyzz_from_aff(b, pts[0], false);
  xyzz_madd(b, pts[1], false);
  for (int it = 0; it < iters; ++it) {
    xyzz_add(acc, b);
  }
  uint32_t s = 0;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(&acc);
  for (int i = 0; i < (int)(sizeof(acc) / 4); ++i) s ^= w[i];
  out[t] = s;
}

template <class K>
float timeit(K launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipError_t err = hipDeviceSynchronize();
  if (err == hipSuccess) err = hipGetLastError();
  if (err != hipSuccess) printf("  launch error: %s\n", hipGetErrorString(err));
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    hipEventRecord(e0);
    launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

// pseudo-random valid-looking affine points: madd's rare branches never trigger on them
template <int G>
void fill_pts(Aff<typename FieldOf<G>::F> *h) {
  uint32_t x = 12345;
  uint32_t *w = reinterpret_cast<uint32_t *>(h);
  for (size_t i = 0; i < 4 * sizeof(h[0]) / 4; ++i) {
    x = x * 1664525u + 1013904223u;
    w[i] = (x >> 4) & MASK;
    if ((i % NL) == NL - 1) w[i] &= 0xffff;
  }
}

int main() {
  uint64_t *d_out;
  hipMalloc(&d_out, 1 << 26);
  // dependent-chain latency: one lane-chain per lane, waves/SIMD = blocks*4 / 1024
  for (int bpc : {1, 2, 4, 8}) {  // blocks of 256 per CU -> waves per SIMD = bpc
    int blocks = 256 * bpc;
    int iters = 4096;
    float ms1 = timeit([&] { hipLaunchKernelGGL(k_mad_chain<1>, dim3(blocks), dim3(256), 0, 0, d_out, 7u, iters); });
    float ms8 = timeit([&] { hipLaunchKernelGGL(k_mad_chain<8>, dim3(blocks), dim3(256), 0, 0, d_out, 7u, iters); });
    // cycles per instruction per wave on its SIMD
    double clk = 2.4e9;
    printf("mad64 waves/SIMD=%d: 1 chain %.2f cyc/instr/wave, 8 chains %.2f cyc/instr/wave  (%.1f / %.1f T lane-ops/s)\n", bpc,
           ms1 * 1e-3 * clk / iters, ms8 * 1e-3 * clk / (iters * 8.0), (double)blocks * 256 * iters / ms1 / 1e9,
           (double)blocks * 256 * iters * 8 / ms8 / 1e9);
  }
  for (int bpc : {1, 2, 3, 4, 8}) {
    int blocks = 256 * bpc, iters = 256;
    float ms = timeit([&] { hipLaunchKernelGGL(k_fpmul, dim3(blocks), dim3(256), 0, 0, (uint32_t *)d_out, iters); });
    double muls = (double)blocks * 256 * iters * 2;
    printf("fp_mul waves/SIMD<=%d: %.3f ms  %.2f G Fp-mul/s\n", bpc, ms, muls / ms / 1e6);
  }
  Aff<Fp> h1[4];
  Aff<Fp2> h2[4];
  fill_pts<1>(h1);
  fill_pts<2>(h2);
  void *dp1, *dp2;
  hipMalloc(&dp1, sizeof h1);
  hipMalloc(&dp2, sizeof h2);
  hipMemcpy(dp1, h1, sizeof h1, hipMemcpyHostToDevice);
  hipMemcpy(dp2, h2, sizeof h2, hipMemcpyHostToDevice);
  for (int bpc : {1, 2, 4, 8}) {
    int blocks = 256 * bpc, iters = 64;
    float ms = timeit([&] { hipLaunchKernelGGL(k_madd<1>, dim3(blocks), dim3(256), 0, 0, (uint32_t *)d_out, (const Aff<Fp> *)dp1, iters); });
    double ops = (double)blocks * 256 * iters * 2;
    printf("G1 xyzz_madd blocks/CU=%d: %.3f ms  %.3f G madd/s\n", bpc, ms, ops / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(k_add<1>, dim3(blocks), dim3(256), 0, 0, (uint32_t *)d_out, (const Aff<Fp> *)dp1, iters); });
    ops = (double)blocks * 256 * iters;
    printf("G1 xyzz_add  blocks/CU=%d: %.3f ms  %.3f G add/s\n", bpc, ms, ops / ms / 1e6);
  }
  for (int bpc : {1, 2}) {
    int blocks = 256 * bpc, iters = 32;
    float ms = timeit([&] { hipLaunchKernelGGL(k_madd<2>, dim3(blocks), dim3(256), 0, 0, (uint32_t *)d_out, (const Aff<Fp2> *)dp2, iters); });
    double ops = (double)blocks * 256 * iters * 2;
    printf("G2 xyzz_madd blocks/CU=%d: %.3f ms  %.3f G madd/s\n", bpc, ms, ops / ms / 1e6);
  }
  return 0;
}
