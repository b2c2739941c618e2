// heavy.hpp -- bucket accumulation with heavy buckets split over several lanes,
// for the blst-level tile entry points (compat.hip).
//
// The tiles receive the caller's entries as they are.  The CHES driver's top
// digit (<= a_h + 1) sends n entries into the few buckets of value <= a_h + 1
// (the device contexts spread those over bucket copies, Ches::plan_buckets),
// and one lane per bucket then runs a serial chain of several hundred mixed
// additions at ~9 us each when its wave is alone: the 2^16 tile's GPU phase was
// 10.2 ms against 1.06 ms for the context (MSM_TILE_TIMING, profiles/r05_tile_timing.txt).
//
// Here, after the sort (schedule positions by descending entry count):
//   k_heavy_plan     one workgroup: T = max(T0, ceil(count[0] / 16)) entries per
//                    chunk; hp = the positions with count > T, rounded up to a
//                    wave group (<= kHeavyMax); per position its chunk range
//   k_accumulate_skip  the ordinary one-lane-per-bucket accumulation of
//                    positions >= hp
//   k_heavy_chunks   one lane per chunk of <= T entries of a heavy position
//   k_heavy_fold     one lane per heavy position: the sum of its <= 16 chunk
//                    partials -> its bucket
// Same group element per bucket (xyzz sums in another association order), so
// the weighted reduction and the exported buckets are unchanged.
#pragma once
#include <algorithm>

#include "engine.hpp"
#include "pair_kernels.hpp"

namespace msm {

constexpr uint32_t kHeavyMax = 8192;   // heavy schedule positions considered
constexpr uint32_t kHeavySplit = 16;   // chunks per heavy bucket (at most)
constexpr uint32_t kHeavyChunks = kHeavyMax * (kHeavySplit + 1);  // chunk bound

struct HeavyPlan {
  uint32_t hp, nchunks, T, pad;
};

// counts: per schedule position, descending.  One workgroup of 1024 threads.
static __global__ void __launch_bounds__(1024)
    k_heavy_plan(const uint32_t *__restrict__ counts, uint32_t nb, uint32_t T0, HeavyPlan *__restrict__ plan,
                 uint32_t *__restrict__ pos_chunk0, uint32_t *__restrict__ chunk_pos) {
  __shared__ uint32_t s_hp, s_T, part[1024];
  const uint32_t tid = threadIdx.x;
  if (tid == 0) {
    const uint32_t c0 = nb ? counts[0] : 0u;
    const uint32_t T = max(T0, (c0 + kHeavySplit - 1) / kHeavySplit);
    // first position with count <= T (counts descending), within kHeavyMax
    uint32_t lo = 0, hi = min(nb, kHeavyMax);
    while (lo < hi) {
      const uint32_t mid = (lo + hi) / 2;
      if (counts[mid] > T) lo = mid + 1;
      else hi = mid;
    }
    s_hp = lo == 0 ? 0u : min(min(nb, kHeavyMax), (lo + 63) & ~63u);  // whole wave groups
    s_T = T;
  }
  __syncthreads();
  const uint32_t hp = s_hp, T = s_T;
  // chunks of position t: ceil(count / T) (>= 1); each thread scans a run of positions
  const uint32_t per = (hp + 1023) / 1024, a = min(hp, tid * per), b = min(hp, a + per);
  uint32_t sum = 0;
  for (uint32_t t = a; t < b; ++t) sum += max(1u, (counts[t] + T - 1) / T);
  part[tid] = sum;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive scan of the per-thread sums
    const uint32_t v = tid >= d ? part[tid - d] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t c = part[tid] - sum;
  for (uint32_t t = a; t < b; ++t) {
    pos_chunk0[t] = c;
    const uint32_t nc = max(1u, (counts[t] + T - 1) / T);
    for (uint32_t j = 0; j < nc; ++j) chunk_pos[c + j] = t;
    c += nc;
  }
  if (tid == 1023) {
    pos_chunk0[hp] = part[1023];
    plan->hp = hp;
    plan->nchunks = part[1023];
    plan->T = T;
    plan->pad = 0;
  }
}

// ---- G1: one lane per bucket / chunk ----
template <class PT>
static __global__ void __launch_bounds__(256, MSM_ACC_WAVES)
    k_accumulate_skip(const AccSched S, const PT *__restrict__ pts, Xyzz<Fp> *__restrict__ buckets, size_t nbuckets,
                      const HeavyPlan *__restrict__ plan) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nbuckets && t >= plan->hp) accumulate_bucket<1>(S, pts, buckets, t);
}
template <class PT>
static __global__ void __launch_bounds__(256, MSM_ACC_WAVES)
    k_heavy_chunks(const AccSched S, const PT *__restrict__ pts, const HeavyPlan *__restrict__ plan,
                   const uint32_t *__restrict__ pos_chunk0, const uint32_t *__restrict__ chunk_pos,
                   Xyzz<Fp> *__restrict__ cpart) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= plan->nchunks) return;
  const uint32_t t = chunk_pos[i], T = plan->T, cnt = S.counts[t];
  const uint32_t k0 = (i - pos_chunk0[t]) * T, k1 = min(cnt, k0 + T);
  const PayloadStream ps(S, t);
  Xyzz<Fp> acc;
  xyzz_set_inf(acc);
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t e = ps.at(k);
    Aff<Fp> p = ld_point(&pts[e & 0x7fffffffu]);
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;  // affine infinity (ec_ops.h:717)
    xyzz_madd(acc, p, (e >> 31) != 0);
  }
  st16(&cpart[i], acc);
}
static __global__ void __launch_bounds__(64)
    k_heavy_fold(const AccSched S, const HeavyPlan *__restrict__ plan, const uint32_t *__restrict__ pos_chunk0,
                 const Xyzz<Fp> *__restrict__ cpart, Xyzz<Fp> *__restrict__ buckets) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= plan->hp) return;
  const uint32_t c0 = pos_chunk0[t], c1 = pos_chunk0[t + 1];
  Xyzz<Fp> acc = ld16(&cpart[c0]);
  for (uint32_t c = c0 + 1; c < c1; ++c) {
    Xyzz<Fp> b = ld16(&cpart[c]);
    xyzz_add(acc, b);
  }
  st16(&buckets[S.order[t]], acc);
}

// ---- G2: the same on lane pairs (fp2l.hpp) ----
template <class PT>
static __global__ void __launch_bounds__(256)
    k_accumulate_skip2p(const AccSched S, const PT *__restrict__ pts, Xyzz<Fp2> *__restrict__ buckets, size_t nbuckets,
                        const HeavyPlan *__restrict__ plan) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 2 * nbuckets && (t >> 1) >= plan->hp) accumulate_pair(S, pts, buckets, t);
}
template <class PT>
static __global__ void __launch_bounds__(256)
    k_heavy_chunks2p(const AccSched S, const PT *__restrict__ pts, const HeavyPlan *__restrict__ plan,
                     const uint32_t *__restrict__ pos_chunk0, const uint32_t *__restrict__ chunk_pos,
                     Xyzz<Fp2> *__restrict__ cpart) {
  const uint32_t tt = blockIdx.x * blockDim.x + threadIdx.x, i = tt >> 1;
  const int comp = (int)(tt & 1);
  if (i >= plan->nchunks) return;  // whole pairs
  const uint32_t t = chunk_pos[i], T = plan->T, cnt = S.counts[t];
  const uint32_t k0 = (i - pos_chunk0[t]) * T, k1 = min(cnt, k0 + T);
  const PayloadStream ps(S, t);
  Xyzz<Fp2L> acc;
  xyzz_set_inf(acc);
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t e = ps.at(k);
    Aff<Fp2L> p;
    ld_point2l(p, &pts[e & 0x7fffffffu], comp);
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;
    xyzz_madd(acc, p, (e >> 31) != 0);
  }
  st_xyzz2l(&cpart[i], acc, comp);
}
static __global__ void __launch_bounds__(64)
    k_heavy_fold2p(const AccSched S, const HeavyPlan *__restrict__ plan, const uint32_t *__restrict__ pos_chunk0,
                   const Xyzz<Fp2> *__restrict__ cpart, Xyzz<Fp2> *__restrict__ buckets) {
  const uint32_t tt = blockIdx.x * blockDim.x + threadIdx.x, t = tt >> 1;
  const int comp = (int)(tt & 1);
  if (t >= plan->hp) return;
  const uint32_t c0 = pos_chunk0[t], c1 = pos_chunk0[t + 1];
  Xyzz<Fp2L> acc;
  ld_xyzz2l(acc, &cpart[c0], comp);
  for (uint32_t c = c0 + 1; c < c1; ++c) {
    Xyzz<Fp2L> b;
    ld_xyzz2l(b, &cpart[c], comp);
    xyzz_add(acc, b);
  }
  st_xyzz2l(&buckets[S.order[t]], acc, comp);
}

// device scratch of the split (owned by the caller's state)
struct HeavyScratch {
  DevBuf plan, pos_chunk0, chunk_pos, cpart;
  size_t device_bytes() const { return plan.bytes + pos_chunk0.bytes + chunk_pos.bytes + cpart.bytes; }
};

// the accumulation of nb buckets (schedule S) with heavy buckets split; T0:
// smallest chunk length
template <int G, class PT>
inline void launch_accumulate_heavy(hipStream_t s, const AccSched &S, const PT *pts,
                                    Xyzz<typename FieldOf<G>::F> *buckets, size_t nb, HeavyScratch &H,
                                    uint32_t T0 = 32) {
  typedef typename FieldOf<G>::F F;
  if (!nb) return;
  H.plan.ensure(sizeof(HeavyPlan));
  H.pos_chunk0.ensure((kHeavyMax + 1) * 4);
  H.chunk_pos.ensure((size_t)kHeavyChunks * 4);
  H.cpart.ensure((size_t)kHeavyChunks * sizeof(Xyzz<F>));
  HeavyPlan *plan = H.plan.as<HeavyPlan>();
  hipLaunchKernelGGL(k_heavy_plan, dim3(1), dim3(1024), 0, s, S.counts, (uint32_t)nb, T0, plan,
                     H.pos_chunk0.as<uint32_t>(), H.chunk_pos.as<uint32_t>());
  // chunk lanes: at most kHeavySplit + 1 per heavy position (launch bound; the
  // lanes past plan->nchunks exit at once)
  const size_t hmax = std::min<size_t>(nb, kHeavyMax), cmax = hmax * (kHeavySplit + 1);
  if constexpr (G == 1) {
    hipLaunchKernelGGL((k_heavy_chunks<PT>), dim3(nblk(cmax, 256)), dim3(256), 0, s, S, pts, plan,
                       H.pos_chunk0.as<uint32_t>(), H.chunk_pos.as<uint32_t>(), H.cpart.as<Xyzz<Fp>>());
    hipLaunchKernelGGL((k_accumulate_skip<PT>), dim3(nblk(nb, 256)), dim3(256), 0, s, S, pts, buckets, nb, plan);
    hipLaunchKernelGGL(k_heavy_fold, dim3(nblk(hmax, 64)), dim3(64), 0, s, S, plan, H.pos_chunk0.as<uint32_t>(),
                       H.cpart.as<Xyzz<Fp>>(), buckets);
  } else {
    hipLaunchKernelGGL((k_heavy_chunks2p<PT>), dim3(nblk(2 * cmax, 256)), dim3(256), 0, s, S, pts, plan,
                       H.pos_chunk0.as<uint32_t>(), H.chunk_pos.as<uint32_t>(), H.cpart.as<Xyzz<Fp2>>());
    hipLaunchKernelGGL((k_accumulate_skip2p<PT>), dim3(nblk(2 * nb, 256)), dim3(256), 0, s, S, pts, buckets, nb,
                       plan);
    hipLaunchKernelGGL(k_heavy_fold2p, dim3(nblk(2 * hmax, 64)), dim3(64), 0, s, S, plan,
                       H.pos_chunk0.as<uint32_t>(), H.cpart.as<Xyzz<Fp2>>(), buckets);
  }
}

}  // namespace msm
