// Single-wave latency of one Montgomery product (FIPS fp_mul vs fp_mul_lat)
// and of one xyzz_add, on an otherwise idle GPU: the regime of the reduction
// tails.  hipcc -O3 --offload-arch=gfx950 -I msm_blst_amd/csrc tools/microbench/lat.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "kernels.hpp"

using namespace msm;

// same product, a*b column sums formed as independent chains first
__device__ __forceinline__ void fp_mont_lat(Fp &r, const Fp &a, const Fp &b) {
  uint64_t s[2 * NL - 1];
#pragma unroll
  for (int k = 0; k < 2 * NL - 1; ++k) {
    const int lo = k < NL ? 0 : k - NL + 1, hi = k < NL ? k : NL - 1;
    uint64_t t = 0;
#pragma unroll
    for (int i = lo; i <= hi; ++i) t = mad64(a.v[i], b.v[k - i], t);
    s[k] = t;
  }
  uint32_t m[NL];
  uint64_t carry = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    uint64_t t = s[k] + carry;
#pragma unroll
    for (int i = 0; i < k; ++i) t = mad64(m[i], P28[k - i], t);
    m[k] = ((uint32_t)t * N0P) & MASK;
    t = mad64(m[k], P28[0], t);
    carry = t >> 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; ++k) {
    uint64_t t = 0;
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) t = mad64(m[i], P28[k - i], t);
    t += s[k] + carry;
    r.v[k - NL] = (uint32_t)t & MASK;
    carry = t >> 28;
  }
  r.v[NL - 1] = (uint32_t)carry;
}

template <int KIND>
__global__ __launch_bounds__(64) void k_chain(uint32_t *out, int iters, long long *cycles) {
  Fp a, b;
  for (int i = 0; i < NL; ++i) {
    a.v[i] = (threadIdx.x * 0x9e3779b9u + i) & MASK;
    b.v[i] = (threadIdx.x * 0x85ebca6bu + 3 * i) & MASK;
  }
  a.v[NL - 1] &= 0xffff;
  b.v[NL - 1] &= 0xffff;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (KIND == 0) fp_mul(a, a, b);
    else fp_mont_lat(a, a, b);
  }
  long long t1 = clock64();
  uint32_t s = 0;
  for (int i = 0; i < NL; ++i) s ^= a.v[i];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cycles = t1 - t0;
}

__global__ void k_check(uint32_t *out) {
  Fp a, b, r1, r2;
  uint32_t x = threadIdx.x * 2654435761u + 1;
  for (int i = 0; i < NL; ++i) {
    x = x * 1664525u + 1013904223u; a.v[i] = (x >> 3) & 0x1fffffff;
    x = x * 1664525u + 1013904223u; b.v[i] = (x >> 3) & 0x1fffffff;
  }
  a.v[NL - 1] &= 0x3ffff;
  b.v[NL - 1] &= 0x3ffff;
  fp_mul(r1, a, b);
  fp_mont_lat(r2, a, b);
  uint32_t bad = 0;
  for (int i = 0; i < NL; ++i) bad |= r1.v[i] ^ r2.v[i];
  out[threadIdx.x] = bad;
}

template <int KIND>
__global__ __launch_bounds__(64) void k_add_chain(const Xyzz<Fp> *pts, uint32_t *out, int iters, long long *cycles) {
  Xyzz<Fp> acc = pts[(threadIdx.x & 31) * 2], b = pts[(threadIdx.x & 31) * 2 + 1];
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    xyzz_add(acc, b);
  }
  long long t1 = clock64();
  out[threadIdx.x] = acc.x.v[0] ^ acc.y.v[1];
  if (threadIdx.x == 0) *cycles = t1 - t0;
}

// one kernel = one add of two points loaded from memory (a reduction tail level)
template <int KIND>
__global__ __launch_bounds__(64) void k_one_add(const Xyzz<Fp> *pts, Xyzz<Fp> *outp) {
  size_t t = KIND == 0 ? threadIdx.x : threadIdx.x >> 2;
  Xyzz<Fp> a = ld16(&pts[2 * t]), b = ld16(&pts[2 * t + 1]);
  xyzz_add(a, b);
  if (KIND == 0 || (threadIdx.x & 3) == 0) st16(&outp[t], a);
}

int main() {
  uint32_t *d_out;
  long long *d_cyc;
  hipMalloc(&d_out, 1 << 20);
  hipMalloc(&d_cyc, 64);
  hipLaunchKernelGGL(k_check, dim3(64), dim3(256), 0, 0, d_out);
  uint32_t h[256 * 64];
  hipMemcpy(h, d_out, sizeof h, hipMemcpyDeviceToHost);
  uint32_t bad = 0;
  for (uint32_t v : h) bad |= v;
  printf("fp_mont_lat == fp_mul on 16384 random lazy inputs: %s\n", bad ? "MISMATCH" : "ok");
  const int iters = 200;
  for (int kind = 0; kind < 2; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (kind == 0) hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, d_out, iters, d_cyc);
      else hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, d_out, iters, d_cyc);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      long long cyc;
      hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%s: %.0f cycles per dependent product (clock64), %.2f us per product (wall)\n",
                      kind ? "fp_mont_lat" : "fp_mul     ", (double)cyc / iters, ms * 1e3 / iters);
    }
  }
  // two valid-looking xyzz points with ZZ = ZZZ = 1 (never infinity, never equal)
  Xyzz<Fp> hp[128];
  uint32_t x = 7;
  for (int k = 0; k < 128; ++k) {
    for (int i = 0; i < NL; ++i) {
      x = x * 1664525u + 1013904223u; hp[k].x.v[i] = (x >> 4) & MASK;
      x = x * 1664525u + 1013904223u; hp[k].y.v[i] = (x >> 4) & MASK;
      hp[k].zz.v[i] = hp[k].zzz.v[i] = 0;
    }
    hp[k].x.v[NL - 1] &= 0xffff; hp[k].y.v[NL - 1] &= 0xffff;
    hp[k].zz.v[0] = hp[k].zzz.v[0] = 1;
  }
  Xyzz<Fp> *dp, *dq;
  hipMalloc(&dp, sizeof hp);
  hipMalloc(&dq, sizeof hp);
  hipMemcpy(dp, hp, sizeof hp, hipMemcpyHostToDevice);
  for (int kind = 0; kind < 1; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      if (kind == 0) hipLaunchKernelGGL(k_add_chain<0>, dim3(1), dim3(64), 0, 0, dp, d_out, 50, d_cyc);
      else hipLaunchKernelGGL(k_add_chain<1>, dim3(1), dim3(64), 0, 0, dp, d_out, 50, d_cyc);
      hipDeviceSynchronize();
      long long cyc;
      hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%s: %.0f cycles per dependent xyzz add\n", "xyzz_add", (double)cyc / 50);
    }
  }
  for (int kind = 0; kind < 1; ++kind) {
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (kind == 0) hipLaunchKernelGGL(k_one_add<0>, dim3(1), dim3(64), 0, 0, dp, dq);
      else hipLaunchKernelGGL(k_one_add<1>, dim3(1), dim3(64), 0, 0, dp, dq);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("one-add kernel (%s, 1 wave): %.2f us (event wall)\n", kind ? "quad" : "serial", best * 1e3);
  }
  return 0;
}
