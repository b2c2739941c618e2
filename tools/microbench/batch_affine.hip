// Batch-affine accumulation (ref src/bulk_addition.c:51-143: affine additions
// with one field inversion per batch, Montgomery's trick) measured on gfx950
// against the xyzz mixed addition the bucket accumulation uses (SURVEY row A19,
// DESIGN section 8).  Three numbers decide whether the technique can replace
// k_accumulate:
//   1. k_inv_chain: latency of ONE field inversion (Fermat a^(p-2), the
//      engine's f_inv) on one lane -- a batch-affine level cannot start before
//      the previous level's inversion finished;
//   2. k_ba: throughput of affine additions with the Montgomery trick across
//      K independent pairs per lane (prefix products in HBM, pairs gathered
//      from a 4-GiB table like the accumulation's rows), one inversion per
//      lane, i.e. the inversion amortised over K (the best case: no cross-lane
//      tree, no dependency between the K additions);
//   3. k_madd_gather: the xyzz madd throughput with the same gathers.
//
//   hipcc -O3 --offload-arch=gfx950 -I msm_blst_amd/csrc tools/microbench/batch_affine.hip -o batch_affine
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "ches_kernels.hpp"

using namespace msm;

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                  \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__global__ void k_inv_chain(Fp *io, int reps) {
  if (threadIdx.x || blockIdx.x) return;
  Fp a = io[0];
  for (int r = 0; r < reps; ++r) {
    Fp b;
    fp_inv(b, a);
    a = b;
    a.v[0] ^= 1;  // keep the chain dependent and non-trivial
  }
  io[0] = a;
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

// K independent affine additions per lane: pair k = rows (h(t,k,0), h(t,k,1))
__global__ void __launch_bounds__(256) k_ba(const AffP<Fp> *__restrict__ T, uint32_t rows, int K,
                                            Fp *__restrict__ pref, AffP<Fp> *__restrict__ out, size_t L) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  Fp c;
  fp_one(c);
  for (int k = 0; k < K; ++k) {
    Aff<Fp> p1 = ld_point(&T[mix((uint32_t)(t * 2 * K + 2 * k)) % rows]);
    Aff<Fp> p2 = ld_point(&T[mix((uint32_t)(t * 2 * K + 2 * k + 1)) % rows]);
    Fp d;
    fp_sub<4>(d, p2.x, p1.x);
    fp_nred(d);
    fp_mul(c, c, d);
    pref[(size_t)k * L + t] = c;
  }
  Fp inv;
  fp_inv(inv, c);
  for (int k = K - 1; k >= 0; --k) {
    Aff<Fp> p1 = ld_point(&T[mix((uint32_t)(t * 2 * K + 2 * k)) % rows]);
    Aff<Fp> p2 = ld_point(&T[mix((uint32_t)(t * 2 * K + 2 * k + 1)) % rows]);
    Fp d, ik, lam, x3, y3, tmp;
    fp_sub<4>(d, p2.x, p1.x);
    fp_nred(d);
    if (k > 0) {
      Fp pk = pref[(size_t)(k - 1) * L + t];
      fp_mul(ik, inv, pk);
      fp_mul(inv, inv, d);
    } else {
      ik = inv;
    }
    fp_sub<4>(tmp, p2.y, p1.y);  // lambda = (y2 - y1) / (x2 - x1)
    fp_mul(lam, tmp, ik);
    fp_sqr(x3, lam);             // x3 = lambda^2 - x1 - x2
    fp_sub<4>(x3, x3, p1.x);
    fp_norm(x3);
    fp_sub<4>(x3, x3, p2.x);
    fp_nred(x3);
    fp_sub<4>(tmp, p1.x, x3);    // y3 = lambda (x1 - x3) - y1
    fp_mul(y3, lam, tmp);
    fp_sub<4>(y3, y3, p1.y);
    fp_nred(y3);
    Aff<Fp> r;
    r.x = x3;
    r.y = y3;
    st_point(&out[(size_t)k * L + t], r);
  }
}

// the accumulation's operation with the same gathers: K madds per lane
__global__ void __launch_bounds__(256) k_madd_gather(const AffP<Fp> *__restrict__ T, uint32_t rows, int K,
                                                     Xyzz<Fp> *__restrict__ out, size_t L) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= L) return;
  Xyzz<Fp> acc;
  xyzz_set_inf(acc);
  for (int k = 0; k < K; ++k) {
    Aff<Fp> p = ld_point(&T[mix((uint32_t)(t * K + k)) % rows]);
    xyzz_madd(acc, p, (k & 1) != 0);
  }
  st16(&out[t], acc);
}

// random-looking but valid field elements (x, y < p); the curve equation is
// irrelevant to the cost of the formulas
static void fill(std::vector<AffP<Fp>> &h) {
  uint64_t s = 88172645463325252ull;
  for (auto &r : h) {
    uint32_t *w = reinterpret_cast<uint32_t *>(&r);
    for (size_t i = 0; i < sizeof(r) / 4; ++i) {
      s ^= s << 13, s ^= s >> 7, s ^= s << 17;
      w[i] = (uint32_t)s & MASK;
    }
    r.x.v[NL - 1] &= 0xffff;
    r.y.v[NL - 1] &= 0xffff;
  }
}

int main() {
  const uint32_t rows = 1u << 25;  // 32 M rows x 128 B = 4 GiB (the CHES table is 4.5 GiB)
  std::vector<AffP<Fp>> h(1 << 20);
  fill(h);
  AffP<Fp> *T;
  CK(hipMalloc(&T, (size_t)rows * sizeof(AffP<Fp>)));
  for (uint32_t r0 = 0; r0 < rows; r0 += (uint32_t)h.size())
    CK(hipMemcpy(T + r0, h.data(), h.size() * sizeof(AffP<Fp>), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  // 1. inversion latency
  Fp *io;
  CK(hipMalloc(&io, sizeof(Fp)));
  CK(hipMemcpy(io, &h[0].x, sizeof(Fp), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_inv_chain, dim3(1), dim3(64), 0, 0, io, 1);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_inv_chain, dim3(1), dim3(64), 0, 0, io, 16);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  printf("fp_inv (Fermat) latency, one lane: %.1f us per inversion\n", ms * 1e3 / 16);
  // 2./3. throughput, 12.58 M additions (one CHES 2^20 accumulation's count)
  const size_t total = 12582912;
  for (int K : {4, 16, 64, 256}) {
    const size_t L = total / K;
    Fp *pref;
    AffP<Fp> *out;
    CK(hipMalloc(&pref, (size_t)K * L * sizeof(Fp)));
    CK(hipMalloc(&out, (size_t)K * L * sizeof(AffP<Fp>)));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_ba, dim3((L + 255) / 256), dim3(256), 0, 0, T, rows, K, pref, out, L);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("batch-affine, K=%3d pairs/lane (1 inversion per lane): %.3f ms for %zu additions = %.2f G add/s\n", K, ms,
           K * L, K * L / ms / 1e6);
    CK(hipFree(pref));
    CK(hipFree(out));
  }
  for (int K : {13, 64}) {
    const size_t L = total / K;
    Xyzz<Fp> *out;
    CK(hipMalloc(&out, L * sizeof(Xyzz<Fp>)));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a));
      hipLaunchKernelGGL(k_madd_gather, dim3((L + 255) / 256), dim3(256), 0, 0, T, rows, K, out, L);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    printf("xyzz madd, K=%3d per lane: %.3f ms for %zu additions = %.2f G add/s\n", K, ms, K * L, K * L / ms / 1e6);
    CK(hipFree(out));
  }
  return 0;
}
