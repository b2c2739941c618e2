// probe.hip -- the VALU ceilings the bench prices the accumulation against,
// measured on the device and in the process that runs the bench (round 6:
// the round-2 constants of tools/microbench/fp_rate.hip were measured on
// another box, and boxes differ by up to 12 % in the clock they hold).
//
//   k_probe_mad    16 independent v_mad_u64_u32 chains per lane, 1-4 waves
//                  per SIMD: the chip's integer mad issue rate (lane-ops/s)
//   k_probe_fpmul  two independent register-resident Fp products per lane
//                  (fp.hpp fp_mul, 392 mads each): Fp-mul/s
//   k_probe_madd   G1 xyzz madd chains (ec.hpp xyzz_madd, the accumulation's
//                  loop body) over four points that stay in cache, compiled
//                  with the accumulation's launch bound: madd/s -- what
//                  k_accumulate<1> would reach with free memory
// Each rate is the best of 3 timed launches per occupancy tried, after one
// untimed launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "kernels.hpp"
#include "engine.hpp"

namespace msm {
namespace {

__global__ void __launch_bounds__(256) k_probe_mad(uint64_t *out, uint32_t seed, int iters) {
  const uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  uint64_t acc[16];
  const uint32_t a = t | 1, b = seed | 3;
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = t + k;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += acc[k];
  if (s == 0x123456789ull) out[t] = s;  // never true in practice; keeps the chains live
}

__global__ void __launch_bounds__(256) k_probe_fpmul(uint32_t *out, int iters) {
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
    fp_mul(d, a, b);
    fp_mul(a, c, b);
    c = d;
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) s ^= a.v[i] ^ c.v[i];
  out[t] = s;
}

__global__ void __launch_bounds__(256, MSM_ACC_WAVES) k_probe_madd(uint32_t *out, const Aff<Fp> *pts, int iters) {
  const uint32_t t = threadIdx.x + blockIdx.x * blockDim.x;
  Xyzz<Fp> acc;
  xyzz_from_aff(acc, pts[2 + (t & 1)], false);
  for (int it = 0; it < 2 * iters; ++it) {  // one point load per madd, as in the accumulation (cache hits here)
    const Aff<Fp> p = pts[it & 3];
    xyzz_madd(acc, p, (it & 2) != 0);
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) s ^= acc.x.v[i] ^ acc.y.v[i] ^ acc.zzz.v[i] ^ acc.zz.v[i];
  out[t] = s;
}

template <class L>
float best_ms(L launch) {
  hipEvent_t e0, e1;
  MSM_HIP_CHECK(hipEventCreate(&e0));
  MSM_HIP_CHECK(hipEventCreate(&e1));
  launch();
  MSM_HIP_CHECK(hipGetLastError());
  MSM_HIP_CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    MSM_HIP_CHECK(hipEventRecord(e0, 0));
    launch();
    MSM_HIP_CHECK(hipEventRecord(e1, 0));
    MSM_HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    MSM_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

}  // namespace

// out = {mad lane-ops/s, Fp-mul/s, G1 madd/s, ms of device time spent}
void valu_probe(int device, double out[4]) {
  {
    DeviceGuard g(device);
    int cus = 0;
    MSM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    DevBuf obuf, pbuf;
    obuf.ensure((size_t)cus * 8 * 256 * 8);
    // four pseudo-random limb vectors in range (madd's doubling / infinity branches never trigger)
    Aff<Fp> h[4];
    uint32_t x = 12345;
    uint32_t *w = reinterpret_cast<uint32_t *>(h);
    for (size_t i = 0; i < sizeof(h) / 4; ++i) {
      x = x * 1664525u + 1013904223u;
      w[i] = (x >> 4) & MASK;
      if ((i % NL) == NL - 1) w[i] &= 0xffff;
    }
    pbuf.ensure(sizeof(h));
    MSM_HIP_CHECK(hipMemcpy(pbuf.p, h, sizeof(h), hipMemcpyHostToDevice));
    double mad = 0, fpm = 0, madd = 0;
    float total = 0;
    for (int bpc : {4, 8, 16}) {  // 256-thread blocks per CU = waves per SIMD
      const int blocks = cus * bpc, iters = 16384 / bpc;
      const float ms = best_ms([&] {
        hipLaunchKernelGGL(k_probe_mad, dim3(blocks), dim3(256), 0, 0, obuf.as<uint64_t>(), 7u, iters);
      });
      total += 4 * ms;
      mad = std::max(mad, (double)blocks * 256 * iters * 16 / (ms * 1e-3));
    }
    for (int bpc : {3, 4, 8}) {
      const int blocks = cus * bpc, iters = 256;
      const float ms = best_ms([&] {
        hipLaunchKernelGGL(k_probe_fpmul, dim3(blocks), dim3(256), 0, 0, obuf.as<uint32_t>(), iters);
      });
      total += 4 * ms;
      fpm = std::max(fpm, (double)blocks * 256 * iters * 2 / (ms * 1e-3));
    }
    for (int bpc : {3, 6}) {  // one / two rounds of the 3-wave launch bound
      const int blocks = cus * bpc, iters = 64;
      const float ms = best_ms([&] {
        hipLaunchKernelGGL(k_probe_madd, dim3(blocks), dim3(256), 0, 0, obuf.as<uint32_t>(), pbuf.as<Aff<Fp>>(),
                           iters);
      });
      total += 4 * ms;
      madd = std::max(madd, (double)blocks * 256 * iters * 2 / (ms * 1e-3));
    }
    out[0] = mad;
    out[1] = fpm;
    out[2] = madd;
    out[3] = total;
  }
}

}  // namespace msm
