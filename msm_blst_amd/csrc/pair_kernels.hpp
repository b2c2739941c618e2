// pair_kernels.hpp -- G2 bucket kernels on lane pairs (fp2l.hpp) and the
// launchers every pipeline uses for the bucket accumulation and the level
// segment sums: G1 keeps one lane per bucket / output; G2 runs two lanes per
// bucket / output, one Fp2 component each (half the registers per lane, so
// several waves per SIMD instead of one).
#pragma once
#include "ches_kernels.hpp"
#include "fp2l.hpp"

namespace msm {

// component `comp` of an Fp2 stored at p (14 limbs, 8-B aligned: 56-B components)
__device__ __forceinline__ void ld_comp(Fp &r, const Fp2 *p, int comp) {
  const uint2 *s = reinterpret_cast<const uint2 *>(reinterpret_cast<const uint8_t *>(p) + comp * sizeof(Fp));
#pragma unroll
  for (int i = 0; i < NL / 2; ++i) {
    uint2 v = s[i];
    r.v[2 * i] = v.x;
    r.v[2 * i + 1] = v.y;
  }
}
__device__ __forceinline__ void st_comp(Fp2 *p, const Fp &a, int comp) {
  uint2 *d = reinterpret_cast<uint2 *>(reinterpret_cast<uint8_t *>(p) + comp * sizeof(Fp));
#pragma unroll
  for (int i = 0; i < NL / 2; ++i) d[i] = make_uint2(a.v[2 * i], a.v[2 * i + 1]);
}
template <class PT>
__device__ __forceinline__ void ld_point2l(Aff<Fp2L> &r, const PT *p, int comp) {
  const Aff<Fp2> *q = reinterpret_cast<const Aff<Fp2> *>(p);
  ld_comp(r.x.c, &q->x, comp);
  ld_comp(r.y.c, &q->y, comp);
}
__device__ __forceinline__ void ld_xyzz2l(Xyzz<Fp2L> &r, const Xyzz<Fp2> *p, int comp) {
  ld_comp(r.x.c, &p->x, comp);
  ld_comp(r.y.c, &p->y, comp);
  ld_comp(r.zzz.c, &p->zzz, comp);
  ld_comp(r.zz.c, &p->zz, comp);
}
__device__ __forceinline__ void st_xyzz2l(Xyzz<Fp2> *p, const Xyzz<Fp2L> &a, int comp) {
  st_comp(&p->x, a.x.c, comp);
  st_comp(&p->y, a.y.c, comp);
  st_comp(&p->zzz, a.zzz.c, comp);
  st_comp(&p->zz, a.zz.c, comp);
}

// 1 / (a0 + a1 i) = (a0 - a1 i) / (a0^2 + a1^2) on a lane pair: both lanes form
// the norm a0^2 + a1^2 (own square + partner's square) and invert it (the same
// instructions on both lanes), then scale their own (negated on odd lanes)
// component.  a in S.
__device__ __forceinline__ void f_inv(Fp2L &r, const Fp2L &a) {
  Fp own = a.c, sq, psq, d, neg, x;
  fp_norm(own);
  fp_sqr(sq, own);
  pair_swap(psq, sq);
  fp_add(d, sq, psq);  // < 4p lazy
  fp_inv(d, d);
  fp_neg<4>(neg, own);
  pair_sel(x, pair_odd(), neg, own);
  fp_mul(r.c, x, d);
}
__device__ __forceinline__ void f_csub(Fp2L &a) { fp_csub_p(a.c); }

// k_ches_table (ches_kernels.hpp) for G2 on lane pairs: lanes 2t, 2t + 1 build
// the rows of base point i0 + t, one Fp2 component each.  The one-lane G2
// table kernel needed 256 VGPRs + 256 AGPRs + 1.5 KB/lane of scratch (and a
// call); its device results changed with a source-equivalent reordering of
// xyzz_dbl (tests/test_gpu_table_rows.py).  Here a lane holds one
// component: the register use of the G1 kernel, no spills.
template <int M>
static __global__ void __launch_bounds__(128)
    k_ches_table2p(const Aff<Fp2> *__restrict__ P, size_t i0, size_t cnt, int q_exp, int h,
                   Xyzz<Fp2> *__restrict__ scratch, Fp2 *__restrict__ pref, AffP<Fp2> *__restrict__ T) {
  const size_t tt = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tt >= 2 * cnt) return;  // whole pairs only
  const int comp = (int)(tt & 1);
  const size_t t = tt >> 1, i = i0 + t;
  static_assert(M == 1 || M == 3, "M");
  const int K = M * h;
  Aff<Fp2L> p;
  ld_point2l(p, &P[i], comp);
  AffP<Fp2> *out = T + (size_t)K * i;
  static_assert(sizeof(AffP<Fp2>) == 256, "one G2 row per 256 B");
  if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) {  // infinity: every multiple is infinity (uniform per pair)
    Fp z;
    fp_zero(z);
    for (int k = 0; k < K; ++k) {
      Aff<Fp2> *o = reinterpret_cast<Aff<Fp2> *>(out + k);
      st_comp(&o->x, z, comp);
      st_comp(&o->y, z, comp);
    }
    return;
  }
  Xyzz<Fp2L> Q;
  xyzz_from_aff(Q, p, false);
  for (int j = 0; j < h; ++j) {
    st_xyzz2l(&scratch[(size_t)(M * j) * cnt + t], Q, comp);
    if (M == 3) {  // 2 Q, then 3 Q = 2 Q + Q in place (one point fewer live)
      Xyzz<Fp2L> R;
      xyzz_dbl(R, Q);
      st_xyzz2l(&scratch[(size_t)(3 * j + 1) * cnt + t], R, comp);
      xyzz_add(R, Q);
      st_xyzz2l(&scratch[(size_t)(3 * j + 2) * cnt + t], R, comp);
    }
    if (j + 1 < h)
      for (int e = 0; e < q_exp; ++e) {
        Xyzz<Fp2L> tmp = Q;
        xyzz_dbl(Q, tmp);
      }
  }
  // Montgomery batch inversion of u_k = ZZ_k ZZZ_k (1/ZZ = ZZZ/u, 1/ZZZ = ZZ/u)
  Fp2L c;
  f_one(c);
  for (int k = 0; k < K; ++k) {
    Xyzz<Fp2L> a;
    ld_xyzz2l(a, &scratch[(size_t)k * cnt + t], comp);
    Fp2L u;
    f_mul(u, a.zz, a.zzz);
    f_mul(c, c, u);
    st_comp(&pref[(size_t)k * cnt + t], c.c, comp);
  }
  Fp2L inv;
  f_inv(inv, c);
  for (int k = K - 1; k >= 0; --k) {
    Xyzz<Fp2L> a;
    ld_xyzz2l(a, &scratch[(size_t)k * cnt + t], comp);
    Fp2L ik;
    if (k > 0) {
      Fp2L pk;
      ld_comp(pk.c, &pref[(size_t)(k - 1) * cnt + t], comp);
      f_mul(ik, inv, pk);
      Fp2L u;
      f_mul(u, a.zz, a.zzz);
      f_mul(inv, inv, u);
    } else {
      ik = inv;
    }
    Fp2L izz, izzz, x, y;
    f_mul(izz, ik, a.zzz);
    f_mul(izzz, ik, a.zz);
    f_mul(x, a.x, izz);
    f_mul(y, a.y, izzz);
    f_csub(x);
    f_csub(y);
    Aff<Fp2> *o = reinterpret_cast<Aff<Fp2> *>(out + k);
    st_comp(&o->x, x.c, comp);
    st_comp(&o->y, y.c, comp);
  }
}

// k_accumulate (kernels.hpp) for G2 with two lanes per bucket
template <class PT>
__device__ __forceinline__ void accumulate_pair(const AccSched &S, const PT *__restrict__ pts,
                                                Xyzz<Fp2> *__restrict__ buckets, size_t t) {
  const int comp = (int)(t & 1);
  const uint32_t pos = (uint32_t)(t >> 1);  // schedule position (k_accumulate)
  const uint32_t cnt = S.counts[pos];
  const PayloadStream ps(S, pos);
  Xyzz<Fp2L> acc;
  xyzz_set_inf(acc);
#if MSM_ACC2P_PREFETCH
  // the next entry's row is loaded before this entry's madd (28 VGPRs of the
  // 256 a 2-wave kernel has), so its HBM latency hides behind the madd's issue
  uint32_t e = cnt ? ps.at(0) : 0u;
  Aff<Fp2L> nxt;
  if (cnt) ld_point2l(nxt, &pts[e & 0x7fffffffu], comp);
  for (uint32_t k = 0; k < cnt; ++k) {
    const Aff<Fp2L> p = nxt;
    const uint32_t ce = e;
    if (k + 1 < cnt) {
      e = ps.at(k + 1);
      ld_point2l(nxt, &pts[e & 0x7fffffffu], comp);
    }
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;  // affine infinity (ec_ops.h:717)
    xyzz_madd(acc, p, (ce >> 31) != 0);
  }
#else
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint32_t e = ps.at(k);
    Aff<Fp2L> p;
    ld_point2l(p, &pts[e & 0x7fffffffu], comp);
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;  // affine infinity (ec_ops.h:717)
    xyzz_madd(acc, p, (e >> 31) != 0);
  }
#endif
  st_xyzz2l(&buckets[S.order[pos]], acc, comp);
}
// MSM_ACC2P_PREFETCH=1 (build-time A/B knob): the next entry's row is loaded
// during the current madd (247 VGPRs, no scratch).  Measured equal, so the G2
// accumulation is not row-latency-bound: configs[4] 168.2 / 167.5 vs 167.1 /
// 166.8 M pairs/s, accumulation 5.71-5.72 vs 5.70 ms (profiles/r06_g2_prefetch_ab.txt)
#ifndef MSM_ACC2P_PREFETCH
#define MSM_ACC2P_PREFETCH 0
#endif
// waves per SIMD the G2 accumulation is compiled for (0: no occupancy bound)
#ifndef MSM_ACC2P_WAVES
#define MSM_ACC2P_WAVES 0
#endif
#if MSM_ACC2P_WAVES
#define MSM_ACC2P_BOUNDS __launch_bounds__(256, MSM_ACC2P_WAVES)
#else
#define MSM_ACC2P_BOUNDS __launch_bounds__(256)
#endif
template <class PT>
__global__ void MSM_ACC2P_BOUNDS
    k_accumulate2p(const AccSched S, const PT *__restrict__ pts, Xyzz<Fp2> *__restrict__ buckets, size_t nbuckets) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 2 * nbuckets) accumulate_pair(S, pts, buckets, t);  // whole pairs only: 2 nbuckets lanes
}

// k_accumulate_sets (kernels.hpp) for G2: R sets in one grid, lane pairs
template <class PT>
__global__ void MSM_ACC2P_BOUNDS
    k_accumulate2p_sets(const AccSched S, const AccStride st, const PT *__restrict__ pts, Xyzz<Fp2> *__restrict__ buckets,
                        size_t nbuckets) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 2 * nbuckets) accumulate_pair(acc_set(S, st, blockIdx.y), pts, buckets + blockIdx.y * nbuckets, t);
}

// k_segsum (ches_kernels.hpp) for G2 with two lanes per output
__device__ __forceinline__ void segsum_pair(const Xyzz<Fp2> *__restrict__ src, const uint32_t *__restrict__ idx,
                                            const uint32_t *__restrict__ starts, Xyzz<Fp2> *__restrict__ dst,
                                            size_t t) {
  const int comp = (int)(t & 1);
  const size_t o = t >> 1;
  const uint32_t lo = starts[o], hi = starts[o + 1];
  Xyzz<Fp2L> acc;
  if (lo == hi) {
    xyzz_set_inf(acc);
  } else {
    ld_xyzz2l(acc, &src[idx ? idx[lo] : lo], comp);
#if MSM_SEGSUM_PREFETCH
    Xyzz<Fp2L> nxt;  // next operand loaded before the current add (k_segsum)
    if (lo + 1 < hi) ld_xyzz2l(nxt, &src[idx ? idx[lo + 1] : lo + 1], comp);
    for (uint32_t k = lo + 1; k < hi; ++k) {
      Xyzz<Fp2L> a = nxt;
      if (k + 1 < hi) ld_xyzz2l(nxt, &src[idx ? idx[k + 1] : k + 1], comp);
      xyzz_add(acc, a);
    }
#else
    for (uint32_t k = lo + 1; k < hi; ++k) {
      Xyzz<Fp2L> a;
      ld_xyzz2l(a, &src[idx ? idx[k] : k], comp);
      xyzz_add(acc, a);
    }
#endif
  }
  st_xyzz2l(&dst[o], acc, comp);
}
#ifndef MSM_SEGSUM2P_WAVES
#define MSM_SEGSUM2P_WAVES 2
#endif
static __global__ void __launch_bounds__(256, MSM_SEGSUM2P_WAVES)
    k_segsum2p(const Xyzz<Fp2> *__restrict__ src, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ starts,
               Xyzz<Fp2> *__restrict__ dst, size_t nout, size_t src_stride, size_t dst_stride) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * nout) return;
  // MSM blockIdx.y of a batch group (k_segsum)
  segsum_pair(src + blockIdx.y * src_stride, idx, starts, dst + blockIdx.y * dst_stride, t);
}
// k_accumulate_l0 (ches_kernels.hpp) for G2: level 0 of the previous MSM and
// this MSM's accumulation in one grid, both on lane pairs
template <class PT>
__global__ void __launch_bounds__(256)
    k_accumulate2p_l0(const AccSched S, const PT *__restrict__ pts, Xyzz<Fp2> *__restrict__ buckets, size_t nbuckets,
                      const Xyzz<Fp2> *__restrict__ l0src, const uint32_t *__restrict__ l0idx,
                      const uint32_t *__restrict__ l0starts, Xyzz<Fp2> *__restrict__ l0dst, size_t l0out,
                      uint32_t l0blocks, int l0_last) {
  const uint32_t nacc = gridDim.x - l0blocks;
  const bool l0 = l0_last ? blockIdx.x >= nacc : blockIdx.x < l0blocks;
  const uint32_t b = l0 ? (l0_last ? blockIdx.x - nacc : blockIdx.x) : (l0_last ? blockIdx.x : blockIdx.x - l0blocks);
  const size_t t = (size_t)b * blockDim.x + threadIdx.x;
  if (l0) {
    if (t < 2 * l0out) segsum_pair(l0src, l0idx, l0starts, l0dst, t);
  } else if (t < 2 * nbuckets) {
    accumulate_pair(S, pts, buckets, t);
  }
}

// k_suffix_step / k_pair_step (ches_kernels.hpp) for G2 with two lanes per output
static __global__ void __launch_bounds__(64)
    k_suffix_step2p(const Xyzz<Fp2> *__restrict__ in, Xyzz<Fp2> *__restrict__ out, int S, int d, int W) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * (size_t)W * S) return;
  const int comp = (int)(t & 1);
  const size_t o = t >> 1;
  const int k = (int)(o % (size_t)S);
  Xyzz<Fp2L> a;
  ld_xyzz2l(a, &in[o], comp);
  if (k + d < S) {
    Xyzz<Fp2L> b;
    ld_xyzz2l(b, &in[o + d], comp);
    xyzz_add(a, b);
  }
  st_xyzz2l(&out[o], a, comp);
}
static __global__ void __launch_bounds__(64)
    k_pair_step2p(const Xyzz<Fp2> *__restrict__ in, Xyzz<Fp2> *__restrict__ out, size_t nout) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * nout) return;
  const int comp = (int)(t & 1);
  const size_t o = t >> 1;
  Xyzz<Fp2L> a, b;
  ld_xyzz2l(a, &in[2 * o], comp);
  ld_xyzz2l(b, &in[2 * o + 1], comp);
  xyzz_add(a, b);
  st_xyzz2l(&out[o], a, comp);
}

// ---- launchers (host) ----
template <int G, class PT>
inline void launch_accumulate(hipStream_t s, const AccSched &S, const PT *pts, Xyzz<typename FieldOf<G>::F> *buckets,
                              size_t nb) {
  if (!nb) return;
  if constexpr (G == 1)
    hipLaunchKernelGGL((k_accumulate<G, PT>), dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, S, pts, buckets, nb);
  else
    hipLaunchKernelGGL((k_accumulate2p<PT>), dim3((unsigned)((2 * nb + 255) / 256)), dim3(256), 0, s, S, pts, buckets, nb);
}
// R sets of one front group (schedules S + r st, buckets at r nb), one launch
template <int G, class PT>
inline void launch_accumulate_sets(hipStream_t s, const AccSched &S, const AccStride &st, const PT *pts,
                                   Xyzz<typename FieldOf<G>::F> *buckets, size_t nb, int R) {
  if (!nb || R < 1) return;
  if constexpr (G == 1)
    hipLaunchKernelGGL((k_accumulate_sets<G, PT>), dim3((unsigned)((nb + 255) / 256), (unsigned)R), dim3(256), 0, s, S,
                       st, pts, buckets, nb);
  else
    hipLaunchKernelGGL((k_accumulate2p_sets<PT>), dim3((unsigned)((2 * nb + 255) / 256), (unsigned)R), dim3(256), 0, s,
                       S, st, pts, buckets, nb);
}
// nmsm > 1: the same segment sums for nmsm MSMs of a batch group in one launch
template <int G>
inline void launch_segsum(hipStream_t s, const Xyzz<typename FieldOf<G>::F> *src, const uint32_t *idx,
                          const uint32_t *starts, Xyzz<typename FieldOf<G>::F> *dst, size_t nout, int nmsm = 1,
                          size_t src_stride = 0, size_t dst_stride = 0) {
  if (!nout || nmsm < 1) return;
  if constexpr (G == 1)
    hipLaunchKernelGGL(k_segsum<G>, dim3((unsigned)((nout + 63) / 64), (unsigned)nmsm), dim3(64), 0, s, src, idx, starts,
                       dst, nout, src_stride, dst_stride);
  else
    hipLaunchKernelGGL(k_segsum2p, dim3((unsigned)((2 * nout + 63) / 64), (unsigned)nmsm), dim3(64), 0, s, src, idx,
                       starts, dst, nout, src_stride, dst_stride);
}

}  // namespace msm
