// coop.hpp -- one xyzz addition split across the 4 waves (= 4 SIMDs) of a
// workgroup, for the latency-bound tail levels of the bucket reductions.
//
// Measured (tools/microbench/lat.hip): a single wave spends ~12.7 us issuing the
// ~14 Montgomery products of one xyzz add (1.05 us each; one wave is issue-
// bound, not latency-bound), so a tail level with a few thousand lanes costs a
// whole add of one SIMD's issue time no matter how few lanes are active.  Here
// wave w of the workgroup computes ~1/4 of the products of the same 64 adds
// (lane i of every wave = add i), exchanging operands through LDS between the
// four dependency levels of add-2008-s:
//   L1  U1 = X1 ZZ2 | S1 = Y1 ZZZ2 | U2 = X2 ZZ1 | S2 = Y2 ZZZ1
//   L2  PP = P^2    | RR = R^2     | ZZ1 ZZ2    | ZZZ1 ZZZ2        (P = U2 - U1, R = S2 - S1)
//   L3  PPP = PP P  | Q = U1 PP    | ZZ3 = ZZ1 ZZ2 PP
//   L4  ZZZ3        | X3, Y3 = R (Q - X3) - S1 PPP
// Same formulas and range classes as xyzz_add (ec.hpp); the rare branches
// (an input at infinity, P == +-bucket) take the serial formulas.
// G2 runs the same split on lane pairs (fp2l.hpp): F = Fp2L, lanes 2i / 2i+1 of
// every wave hold the two components of add i, so a 256-thread workgroup does
// 32 G2 adds with 8 lanes each (the *_c2p kernels below).
#pragma once
#include "fp2l.hpp"
#include "kernels.hpp"

namespace msm {

template <class F>
struct CoopLds {
  uint32_t v[8][sizeof(F) / 4][64];  // [value slot][32-bit word][lane]: conflict-free
};

// 32-bit word k of a field element (by member access: no address-taken locals)
__device__ __forceinline__ uint32_t &fw(Fp &x, int k) { return x.v[k]; }
__device__ __forceinline__ uint32_t fw(const Fp &x, int k) { return x.v[k]; }
__device__ __forceinline__ uint32_t &fw(Fp2 &x, int k) { return k < NL ? x.c0.v[k] : x.c1.v[k - NL]; }
__device__ __forceinline__ uint32_t fw(const Fp2 &x, int k) { return k < NL ? x.c0.v[k] : x.c1.v[k - NL]; }
__device__ __forceinline__ uint32_t &fw(Fp2L &x, int k) { return x.c.v[k]; }
__device__ __forceinline__ uint32_t fw(const Fp2L &x, int k) { return x.c.v[k]; }

template <class F>
__device__ __forceinline__ void coop_put(CoopLds<F> &L, int slot, int lane, const F &x) {
#pragma unroll
  for (int k = 0; k < (int)(sizeof(F) / 4); ++k) L.v[slot][k][lane] = fw(x, k);
}
template <class F>
__device__ __forceinline__ F coop_get(const CoopLds<F> &L, int slot, int lane) {
  F x;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(F) / 4); ++k) fw(x, k) = L.v[slot][k][lane];
  return x;
}
// coordinate c of an xyzz point in memory: 0 x, 1 y, 2 zzz, 3 zz
template <class F>
__device__ __forceinline__ void coop_st(Xyzz<F> *dst, int c, const F &v) {
  F *p = c == 0 ? &dst->x : c == 1 ? &dst->y : c == 2 ? &dst->zzz : &dst->zz;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(F) / 4); ++k) fw(*p, k) = fw(v, k);
}
// value select of a field element by masks (and/or on the limbs: keeps the
// four candidates in registers; a select chain here becomes a select of
// pointers to stack copies)
template <class F>
__device__ __forceinline__ F fsel4(int w, const F &x0, const F &x1, const F &x2, const F &x3) {
  const uint32_t m0 = 0u - (uint32_t)(w == 0), m1 = 0u - (uint32_t)(w == 1), m2 = 0u - (uint32_t)(w == 2),
                 m3 = 0u - (uint32_t)(w == 3);
  F r;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(F) / 4); ++k)
    fw(r, k) = (fw(x0, k) & m0) | (fw(x1, k) & m1) | (fw(x2, k) & m2) | (fw(x3, k) & m3);
  return r;
}

// a + b -> st(coordinate, value) (coordinate: 0 x, 1 y, 2 zzz, 3 zz).  Every
// thread of the 256-thread workgroup calls this with the (a, b, active) of its
// lane (the 4 waves pass the same values); it contains three __syncthreads.
// The operands of each level are selected by value per wave so that every wave
// runs the same product code.
template <class F, class Store>
__device__ __forceinline__ void coop_xyzz_add(const Xyzz<F> &a, const Xyzz<F> &b, Store st, bool active,
                                              CoopLds<F> &L) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  F r;
  // L1: U1 = X1 ZZ2 | S1 = Y1 ZZZ2 | U2 = X2 ZZ1 | S2 = Y2 ZZZ1
  f_mul(r, fsel4(w, a.x, a.y, b.x, b.y), fsel4(w, b.zz, b.zzz, a.zz, a.zzz));
  coop_put(L, w, lane, r);
  __syncthreads();
  // L2: PP = P^2 | RR = R^2 | ZZ1 ZZ2 | ZZZ1 ZZZ2
  const F u1 = coop_get(L, 0, lane), s1 = coop_get(L, 1, lane);
  F P = coop_get(L, 2, lane), R = coop_get(L, 3, lane);
  f_sub4(P, P, u1);  // < 6p
  f_sub4(R, R, s1);  // < 6p
  f_mul(r, fsel4(w, P, R, a.zz, a.zzz), fsel4(w, P, R, b.zz, b.zzz));
  coop_put(L, 4 + w, lane, r);
  __syncthreads();
  // L3: PPP = PP P | Q = U1 PP | ZZ3 = ZZ1 ZZ2 PP   (slots 2, 3 -- U2, S2 -- are free again)
  const F PP = coop_get(L, 4, lane);
  f_mul(r, fsel4(w, P, u1, coop_get(L, 6, lane), P), PP);
  if (w < 2) coop_put(L, 2 + w, lane, r);  // PPP, Q
  const F zz3 = r;                          // (wave 2)
  __syncthreads();
  if (!active) return;
  // L4 -- owned outputs: wave 0 ZZZ3, wave 1 X3 and Y3, wave 2 ZZ3
  F o0, o1;
  if (w == 0) {
    f_mul(o0, coop_get(L, 7, lane), coop_get(L, 2, lane));  // ZZZ1 ZZZ2 PPP
  } else if (w == 1) {
    const F PPP = coop_get(L, 2, lane), Q = coop_get(L, 3, lane);
    F X3 = coop_get(L, 5, lane), t;  // RR
    f_sub_2x(X3, X3, PPP, Q);  // R^2 + 8p - PPP - 2Q   < 10p
    f_norm(X3);         // X3 = R^2 - PPP - 2Q   X (normalized, < 10p)
    f_sub16(t, Q, X3);  // < 18p
    f_mul_sub(o1, t, R, s1, PPP);  // Y3 = R (Q - X3) - S1 PPP   S
    o0 = X3;
  } else {
    o0 = zz3;
    o1 = zz3;
  }
  // rare lanes: an input at infinity, or X1 == X2 (double a, or a == -b -> infinity)
  const bool binf = xyzz_is_inf(b), ainf = xyzz_is_inf(a);
  if (__builtin_expect(!binf && !ainf && f_is_zero_S(PP), 0)) {
    Xyzz<F> d;
    if (f_is_zero_S(coop_get(L, 5, lane))) xyzz_dbl(d, a);
    else xyzz_set_inf(d);
    o0 = fsel4(w, d.zzz, d.x, d.zz, d.zz);
    o1 = d.y;
  }
  if (binf) {
    o0 = fsel4(w, a.zzz, a.x, a.zz, a.zz);
    o1 = a.y;
  } else if (ainf) {
    o0 = fsel4(w, b.zzz, b.x, b.zz, b.zz);
    o1 = b.y;
  }
  if (w < 3) st(w == 0 ? 2 : w == 1 ? 0 : 3, o0);
  if (w == 1) st(1, o1);
}
template <class F>
__device__ __forceinline__ void coop_xyzz_add(const Xyzz<F> &a, const Xyzz<F> &b, Xyzz<F> *dst, bool active,
                                              CoopLds<F> &L) {
  coop_xyzz_add(a, b, [&](int c, const F &v) { coop_st(dst, c, v); }, active, L);
}
// G2 lane pairs: this lane's component of coordinate c goes to dst
__device__ __forceinline__ void coop_st2l(Xyzz<Fp2> *dst, int c, const Fp2L &v) {
  Fp2 *p = c == 0 ? &dst->x : c == 1 ? &dst->y : c == 2 ? &dst->zzz : &dst->zz;
  const int comp = (int)(threadIdx.x & 1);
  uint2 *d = reinterpret_cast<uint2 *>(reinterpret_cast<uint8_t *>(p) + comp * sizeof(Fp));
#pragma unroll
  for (int i = 0; i < NL / 2; ++i) d[i] = make_uint2(v.c.v[2 * i], v.c.v[2 * i + 1]);
}
__device__ __forceinline__ void coop_ld2l(Xyzz<Fp2L> &r, const Xyzz<Fp2> *p) {
  const int comp = (int)(threadIdx.x & 1);
  const Fp2 *f[4] = {&p->x, &p->y, &p->zzz, &p->zz};
  Fp *o[4] = {&r.x.c, &r.y.c, &r.zzz.c, &r.zz.c};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint2 *s = reinterpret_cast<const uint2 *>(reinterpret_cast<const uint8_t *>(f[c]) + comp * sizeof(Fp));
#pragma unroll
    for (int i = 0; i < NL / 2; ++i) {
      const uint2 v = s[i];
      o[c]->v[2 * i] = v.x;
      o[c]->v[2 * i + 1] = v.y;
    }
  }
}

// ---- tail-level kernels: 256 threads = 4 waves per 64 outputs ----
template <class F>
__device__ __forceinline__ Xyzz<F> coop_inf() {
  Xyzz<F> z;
  xyzz_set_inf(z);
  return z;
}

// pairwise tree step: out[t] = in[2t] + in[2t + 1]
template <int G>
static __global__ void __launch_bounds__(256)
    k_pair_step_c(const Xyzz<typename FieldOf<G>::F> *__restrict__ in, Xyzz<typename FieldOf<G>::F> *__restrict__ out,
                  size_t nout) {
  typedef typename FieldOf<G>::F F;
  __shared__ CoopLds<F> L;
  const size_t t = (size_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const bool active = t < nout;
  const Xyzz<F> a = active ? ld16(&in[2 * t]) : coop_inf<F>();
  const Xyzz<F> b = active ? ld16(&in[2 * t + 1]) : coop_inf<F>();
  coop_xyzz_add(a, b, &out[active ? t : 0], active, L);
}

// suffix-scan step within each window of S: out[t] = in[t] + in[t + d] (k + d < S)
template <int G>
static __global__ void __launch_bounds__(256)
    k_suffix_step_c(const Xyzz<typename FieldOf<G>::F> *__restrict__ in, Xyzz<typename FieldOf<G>::F> *__restrict__ out,
                    int S, int d, int W) {
  typedef typename FieldOf<G>::F F;
  __shared__ CoopLds<F> L;
  const size_t t = (size_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const bool active = t < (size_t)W * S;
  const int k = active ? (int)(t % (size_t)S) : 0;
  const Xyzz<F> a = active ? ld16(&in[t]) : coop_inf<F>();
  const Xyzz<F> b = active && k + d < S ? ld16(&in[t + d]) : coop_inf<F>();
  coop_xyzz_add(a, b, &out[active ? t : 0], active, L);
}

// segment sums of <= 2 items (the reduction levels after level 0):
// dst[t] = sum_{k in [starts[t], starts[t+1])} src[idx ? idx[k] : k]; longer
// segments fold their leading items serially first.  grid.y: the MSMs of a
// batch group (src / dst advanced by their strides, one plan for all)
template <int G>
static __global__ void __launch_bounds__(256)
    k_segsum_c(const Xyzz<typename FieldOf<G>::F> *__restrict__ src, const uint32_t *__restrict__ idx,
               const uint32_t *__restrict__ starts, Xyzz<typename FieldOf<G>::F> *__restrict__ dst, size_t nout,
               size_t src_stride, size_t dst_stride) {
  typedef typename FieldOf<G>::F F;
  __shared__ CoopLds<F> L;
  src += blockIdx.y * src_stride;
  dst += blockIdx.y * dst_stride;
  const size_t t = (size_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const bool active = t < nout;
  Xyzz<F> a = coop_inf<F>(), b = coop_inf<F>();
  if (active) {
    const uint32_t lo = starts[t], hi = starts[t + 1];
    if (hi > lo) {
      a = ld16(&src[idx ? idx[lo] : lo]);
      for (uint32_t k = lo + 1; k + 1 < hi; ++k) {
        const Xyzz<F> c = ld16(&src[idx ? idx[k] : k]);
        xyzz_add(a, c);
      }
      if (hi - lo >= 2) b = ld16(&src[idx ? idx[hi - 1] : hi - 1]);
    }
  }
  coop_xyzz_add(a, b, &dst[active ? t : 0], active, L);
}

// ---- G2: the same kernels on lane pairs, 256 threads = 4 waves per 32 outputs ----
__device__ __forceinline__ Xyzz<Fp2L> coop_inf2l() {
  Xyzz<Fp2L> z;
  xyzz_set_inf(z);
  return z;
}

static __global__ void __launch_bounds__(256)
    k_pair_step_c2p(const Xyzz<Fp2> *__restrict__ in, Xyzz<Fp2> *__restrict__ out, size_t nout) {
  __shared__ CoopLds<Fp2L> L;
  const size_t t = (size_t)blockIdx.x * 32 + ((threadIdx.x & 63) >> 1);
  const bool active = t < nout;
  Xyzz<Fp2L> a = coop_inf2l(), b = coop_inf2l();
  if (active) {
    coop_ld2l(a, &in[2 * t]);
    coop_ld2l(b, &in[2 * t + 1]);
  }
  Xyzz<Fp2> *d = &out[active ? t : 0];
  coop_xyzz_add(a, b, [&](int c, const Fp2L &v) { coop_st2l(d, c, v); }, active, L);
}

static __global__ void __launch_bounds__(256)
    k_suffix_step_c2p(const Xyzz<Fp2> *__restrict__ in, Xyzz<Fp2> *__restrict__ out, int S, int dd, int W) {
  __shared__ CoopLds<Fp2L> L;
  const size_t t = (size_t)blockIdx.x * 32 + ((threadIdx.x & 63) >> 1);
  const bool active = t < (size_t)W * S;
  const int k = active ? (int)(t % (size_t)S) : 0;
  Xyzz<Fp2L> a = coop_inf2l(), b = coop_inf2l();
  if (active) coop_ld2l(a, &in[t]);
  if (active && k + dd < S) coop_ld2l(b, &in[t + dd]);
  Xyzz<Fp2> *d = &out[active ? t : 0];
  coop_xyzz_add(a, b, [&](int c, const Fp2L &v) { coop_st2l(d, c, v); }, active, L);
}

// segment sums as k_segsum_c, for G2 on lane pairs
static __global__ void __launch_bounds__(256)
    k_segsum_c2p(const Xyzz<Fp2> *__restrict__ src, const uint32_t *__restrict__ idx,
                 const uint32_t *__restrict__ starts, Xyzz<Fp2> *__restrict__ dst, size_t nout, size_t src_stride,
                 size_t dst_stride) {
  __shared__ CoopLds<Fp2L> L;
  src += blockIdx.y * src_stride;
  dst += blockIdx.y * dst_stride;
  const size_t t = (size_t)blockIdx.x * 32 + ((threadIdx.x & 63) >> 1);
  const bool active = t < nout;
  Xyzz<Fp2L> a = coop_inf2l(), b = coop_inf2l();
  if (active) {
    const uint32_t lo = starts[t], hi = starts[t + 1];
    if (hi > lo) {
      coop_ld2l(a, &src[idx ? idx[lo] : lo]);
      for (uint32_t k = lo + 1; k + 1 < hi; ++k) {
        Xyzz<Fp2L> c;
        coop_ld2l(c, &src[idx ? idx[k] : k]);
        xyzz_add(a, c);
      }
      if (hi - lo >= 2) coop_ld2l(b, &src[idx ? idx[hi - 1] : hi - 1]);
    }
  }
  Xyzz<Fp2> *d = &dst[active ? t : 0];
  coop_xyzz_add(a, b, [&](int c, const Fp2L &v) { coop_st2l(d, c, v); }, active, L);
}

}  // namespace msm
