// kernels.hpp -- HIP kernels of the MSM engine (gfx950).  Templated on the
// group: G1 (F = Fp) and G2 (F = Fp2).
//
// Plain Pippenger pipeline (replaces ref src/multi_scalar.c:383-419 tile /
// :281-297 integrate / :549-576 window loop):
//   k_digits      signed c-bit window digits of every scalar -> one (bucket,
//                 point | sign) entry per window
//   BucketSort    two-level LDS counting sort by bucket (bucket_sort.hpp);
//                 bucket schedule = ids sorted by count, descending, so a
//                 wavefront's 64 buckets are equally long
//   k_accumulate  one lane per bucket: xyzz += +-P over its sorted points
//   reduction     WeightedReducer (ches.hip): segment sums by weight bits,
//                 dense suffix-scan stage (sum_b b*B_b)
//   k_finalize    window totals -> blst Jacobian (R=2^384 Montgomery)
// CHES pipeline: see ches.hpp.
#pragma once
#include "acc_sched.hpp"
#include "ec.hpp"

namespace msm {

template <int G>
struct FieldOf;
template <>
struct FieldOf<1> {
  typedef Fp F;
};
template <>
struct FieldOf<2> {
  typedef Fp2 F;
};

// ---- wide (16 B) loads/stores of POD structs whose size is a multiple of 16 ----
template <class T>
__device__ __forceinline__ T ld16(const T *p) {
  static_assert(sizeof(T) % 16 == 0, "16B multiple");
  T r;
  const uint4 *s = reinterpret_cast<const uint4 *>(p);
  uint4 tmp[sizeof(T) / 16];
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); ++i) tmp[i] = s[i];
  __builtin_memcpy(&r, tmp, sizeof(T));
  return r;
}
template <class T>
__device__ __forceinline__ void st16(T *p, const T &v) {
  static_assert(sizeof(T) % 16 == 0, "16B multiple");
  uint4 tmp[sizeof(T) / 16];
  __builtin_memcpy(tmp, &v, sizeof(T));
  uint4 *d = reinterpret_cast<uint4 *>(p);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); ++i) d[i] = tmp[i];
}

// Affine point padded to a multiple of 128 B: one row of the CHES table per
// 128-B cache line (G1: 112 -> 128 B, G2: 224 -> 256 B), so a random gather
// touches the minimum number of lines.
template <class F>
struct AffP {
  F x, y;
  uint32_t pad[((128 - (2 * sizeof(F)) % 128) % 128) / 4];
};
template <class F>
__device__ __forceinline__ Aff<F> ld_point(const Aff<F> *p) {
  return ld16(p);
}
template <class F>
__device__ __forceinline__ Aff<F> ld_point(const AffP<F> *p) {
  return ld16(reinterpret_cast<const Aff<F> *>(p));
}
// one coordinate (0: x, 1: y) of a G1 table row, 8-B loads
__device__ __forceinline__ Fp ld_coord(const AffP<Fp> *p, int c) {
  const uint2 *s = reinterpret_cast<const uint2 *>(reinterpret_cast<const uint8_t *>(p) + c * sizeof(Fp));
  Fp r;
#pragma unroll
  for (int i = 0; i < NL / 2; ++i) {
    const uint2 v = s[i];
    r.v[2 * i] = v.x;
    r.v[2 * i + 1] = v.y;
  }
  return r;
}
__device__ __forceinline__ Fp ld_coord(const Aff<Fp> *p, int c) {
  return ld_coord(reinterpret_cast<const AffP<Fp> *>(p), c);
}
template <class F>
__device__ __forceinline__ void st_point(Aff<F> *p, const Aff<F> &a) {
  st16(p, a);
}
template <class F>
__device__ __forceinline__ void st_point(AffP<F> *p, const Aff<F> &a) {
  st16(reinterpret_cast<Aff<F> *>(p), a);
}

// ---- blst 6x64 LE  <->  14 x 28-bit limbs ----
__device__ __forceinline__ void unpack384(Fp &r, const uint64_t *l) {
  uint32_t w[12];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    w[2 * i] = (uint32_t)l[i];
    w[2 * i + 1] = (uint32_t)(l[i] >> 32);
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int bit = 28 * k, wi = bit / 32, sh = bit % 32;
    uint32_t lo = wi < 12 ? w[wi] : 0u;
    uint32_t hi = wi + 1 < 12 ? w[wi + 1] : 0u;
    uint64_t v = ((uint64_t)hi << 32) | lo;
    r.v[k] = (uint32_t)(v >> sh) & MASK;
  }
}
__device__ __forceinline__ void pack384(uint64_t *l, const Fp &a) {  // a normalized, < 2^384
  uint32_t w[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) w[i] = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int bit = 28 * k, wi = bit / 32, sh = bit % 32;
    uint64_t v = (uint64_t)a.v[k] << sh;
    if (wi < 12) w[wi] |= (uint32_t)v;
    if (wi + 1 < 12) w[wi + 1] |= (uint32_t)(v >> 32);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) l[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}
// blst Montgomery (R=2^384, canonical) -> internal (R=2^392, canonical)
__device__ __forceinline__ void fp_from_blst(Fp &r, const uint64_t *l) {
  Fp a, k;
  unpack384(a, l);
  fp_set(k, TOINT28);
  fp_mul(r, a, k);
  fp_csub_p(r);
}
// internal (any class-S / lazy value) -> blst Montgomery canonical
__device__ __forceinline__ void fp_to_blst(uint64_t *l, const Fp &a) {
  Fp k, r;
  fp_set(k, FROMINT28);
  fp_mul(r, a, k);
  fp_csub_p(r);
  pack384(l, r);
}
__device__ __forceinline__ void f_from_blst(Fp &r, const uint64_t *l) { fp_from_blst(r, l); }
__device__ __forceinline__ void f_from_blst(Fp2 &r, const uint64_t *l) {
  fp_from_blst(r.c0, l);
  fp_from_blst(r.c1, l + 6);
}
__device__ __forceinline__ void f_to_blst(uint64_t *l, const Fp &a) { fp_to_blst(l, a); }
__device__ __forceinline__ void f_to_blst(uint64_t *l, const Fp2 &a) {
  fp_to_blst(l, a.c0);
  fp_to_blst(l + 6, a.c1);
}

// ---------------------------------------------------------------------------
// point conversion: blst affine (Montgomery R=2^384) -> internal affine limbs
// ---------------------------------------------------------------------------
template <int G, class PT = Aff<typename FieldOf<G>::F>>
__global__ void k_convert_points(const uint64_t *__restrict__ in, PT *__restrict__ out, size_t n) {
  typedef typename FieldOf<G>::F F;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t *p = in + i * 12 * G;
  Aff<F> a;
  f_from_blst(a.x, p);
  f_from_blst(a.y, p + 6 * G);
  st_point(&out[i], a);
}

// ---------------------------------------------------------------------------
// signed window digits (ref ec_mult.h:23-55 booth encoding, generalised):
// window w covers bits [w*c, w*c+c); raw = bits + carry; raw > 2^(c-1) ->
// digit raw - 2^c with carry 1.  The top window never carries because
// W*c >= nbits + 1.  Entry key = (bucket-1) | sign<<31, or ~0 for digit 0.
// ---------------------------------------------------------------------------
constexpr uint32_t KEY_NONE = 0xffffffffu;

__device__ __forceinline__ uint32_t scalar_bits(const uint32_t s[10], int off, int c) {
  int wi = off >> 5, sh = off & 31;
  uint64_t v = (uint64_t)s[wi] | ((uint64_t)s[wi + 1] << 32);
  return (uint32_t)(v >> sh) & ((1u << c) - 1u);
}

// neg (optional): entry i's point enters negated (blst tile digits, k_tile_booth)
// Top window: its digits take only 2^topbits values (topbits = nbits - (W-1) C
// <= C - 1; e.g. 3 for C = 12, nbits = 255), so one lane per bucket would run
// n / 2^topbits sequential madds there.  Its NB slots instead hold 2^tcl copies
// of its 2^topbits buckets (entry i -> copy i mod 2^tcl), each copy weighted
// like its bucket in the reduction plan (Pippenger<G>::back).
// blockIdx.y = scalar set r of a front group (scalars + r set_stride; entries
// at keys / vals + r W n)
template <int C>
__global__ void k_digits(const uint8_t *__restrict__ scalars, size_t stride, size_t n, int nbits, int W,
                         uint32_t *__restrict__ keys, uint32_t *__restrict__ vals, const uint8_t *__restrict__ neg,
                         int tcl, size_t set_stride) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t flip = neg ? (uint32_t)(neg[i] != 0) : 0u;
  constexpr uint32_t NB = 1u << (C - 1);
  const uint8_t *sp = scalars + blockIdx.y * set_stride + i * stride;
  keys += (size_t)blockIdx.y * W * n;
  vals += (size_t)blockIdx.y * W * n;
  int nbytes = (nbits + 7) / 8;
  uint32_t s[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) s[k] = 0;
  if (stride % 4 == 0 && nbytes == 32) {
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(sp);
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = s32[k];
  } else {
    for (int b = 0; b < nbytes; ++b) s[b >> 2] |= (uint32_t)sp[b] << (8 * (b & 3));
  }
  // keep only the low nbits bits (ref multi_scalar.c:396 wmask semantics)
  if (nbits < 256) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      int lo = 32 * k;
      if (nbits <= lo) s[k] = 0;
      else if (nbits < lo + 32) s[k] &= (1u << (nbits - lo)) - 1u;
    }
  }
  uint32_t carry = 0;
  constexpr int WMAX = (257 + C - 1) / C;
#pragma unroll
  for (int w = 0; w < WMAX; ++w) {
    if (w < W) {
      uint32_t raw = scalar_bits(s, w * C, C) + carry;
      uint32_t b, sign;
      if (w < W - 1 && raw > NB) {
        b = (1u << C) - raw;
        sign = 1;
        carry = 1;
      } else {
        b = raw;
        sign = 0;
        carry = 0;
      }
      size_t e = (size_t)w * n + i;
      if (b) {
        const uint32_t copy = w == W - 1 ? ((uint32_t)i & ((1u << tcl) - 1u)) << (C - 1 - tcl) : 0u;
        keys[e] = (uint32_t)w * NB + (b - 1) + copy;
        vals[e] = (uint32_t)i | ((sign ^ flip) << 31);
      } else {
        keys[e] = KEY_NONE;
      }
    }
  }
}

// One blst window tile (ref multi_scalar.c:383-419 with ec_mult.h:23-55): the
// Booth digit of scalar i over bits [bit0 - 1, bit0 + wbits) (lookback bit
// bit0 - 1; bits >= nbits read as 0), split into |d| (a 4-byte "scalar" the
// plain pipeline multiplies with) and the sign (neg[i], applied by k_digits).
static __global__ void k_tile_booth(const uint8_t *__restrict__ scalars, size_t stride, size_t n, int nbits, int bit0,
                             int wbits, int cbits, uint32_t *__restrict__ mag, uint8_t *__restrict__ neg) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *sp = scalars + i * stride;
  uint32_t v = 0;
  for (int k = 0; k <= wbits; ++k) {
    const int b = bit0 - 1 + k;
    if (b < 0 || b >= nbits) continue;
    v |= (uint32_t)((sp[b >> 3] >> (b & 7)) & 1) << k;
  }
  const uint32_t sign = (v >> cbits) & 1;
  int d = (int)((v + 1) >> 1);
  if (sign) d -= 1 << cbits;
  mag[i] = (uint32_t)(d < 0 ? -d : d);
  neg[i] = (uint8_t)(d < 0);
}

static __global__ void k_iota(uint32_t *a, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = (uint32_t)i;
}

// MSM_ACC_PREFETCH (build-time A/B knob): 1 loads the next entry's row during
// the current madd (168 VGPRs + 44 B scratch, not run), 2 only its x (162
// VGPRs): 2 measured slower in the batch (accumulation 1.81 vs 1.78 ms, H2D
// headline 420-429 vs 432-433 M pairs/s; profiles/r06_taper_prefetch_ab.txt)
#ifndef MSM_ACC_PREFETCH
#define MSM_ACC_PREFETCH 0
#endif
// waves per SIMD the G1 accumulation is compiled for (VGPR budget 512 / waves)
#ifndef MSM_ACC_WAVES
#define MSM_ACC_WAVES 3
#endif
// The entry stream of schedule position t (AccSched): row k of its wave
// group's interleaved block (stride 64: one coalesced read per wave step), or,
// for a group left in bucket order, its run in `sorted` (stride 1).
struct PayloadStream {
  const uint32_t *p;
  uint32_t stride;
  MSM_FN PayloadStream(const AccSched &S, uint32_t t) {
    const uint32_t b = S.wbase[t >> 6];
    if (b != ~0u) {
      p = S.ipay + (size_t)b * 64 + (t & 63);
      stride = 64;
    } else {
      p = S.sorted + S.offsets[t];
      stride = 1;
    }
  }
  MSM_FN uint32_t at(uint32_t k) const { return p[(size_t)k * stride]; }
};

// One lane per bucket, buckets visited in the schedule `order` (descending
// entry count, BucketSort) so the 64 lanes of a wave run loops of nearly equal
// length and the longest buckets start first.  Everything is read by schedule
// position (AccSched: coalesced); S.order[t] is the bucket the sum is stored to.
template <int G, class PT>
__device__ __forceinline__ void accumulate_bucket(const AccSched &S, const PT *__restrict__ pts,
                                                  Xyzz<typename FieldOf<G>::F> *__restrict__ buckets, size_t t) {
  typedef typename FieldOf<G>::F F;
  const uint32_t cnt = S.counts[t];
  const PayloadStream ps(S, (uint32_t)t);
  Xyzz<F> acc;
  xyzz_set_inf(acc);
#if MSM_ACC_PREFETCH == 2
  // A/B knob (build time): the next entry's x loaded before this entry's madd,
  // this entry's y at the top of its iteration (first used by the madd's second
  // product); x == 0 exactly is the only way into the infinity test
  uint32_t e = cnt ? ps.at(0) : 0u;
  F nx;
  if (cnt) nx = ld_coord(&pts[e & 0x7fffffffu], 0);
  for (uint32_t k = 0; k < cnt; ++k) {
    Aff<F> p;
    p.x = nx;
    const uint32_t ce = e;
    p.y = ld_coord(&pts[ce & 0x7fffffffu], 1);
    if (k + 1 < cnt) {
      e = ps.at(k + 1);
      nx = ld_coord(&pts[e & 0x7fffffffu], 0);
    }
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;  // affine infinity (ec_ops.h:717)
    xyzz_madd(acc, p, (ce >> 31) != 0);
  }
#elif MSM_ACC_PREFETCH
  // A/B knob (build time): the next entry's row loaded before this entry's madd
  uint32_t e = cnt ? ps.at(0) : 0u;
  Aff<F> nxt;
  if (cnt) nxt = ld_point(&pts[e & 0x7fffffffu]);
  for (uint32_t k = 0; k < cnt; ++k) {
    const Aff<F> p = nxt;
    const uint32_t ce = e;
    if (k + 1 < cnt) {
      e = ps.at(k + 1);
      nxt = ld_point(&pts[e & 0x7fffffffu]);
    }
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;  // affine infinity (ec_ops.h:717)
    xyzz_madd(acc, p, (ce >> 31) != 0);
  }
#else
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint32_t e = ps.at(k);
    Aff<F> p = ld_point(&pts[e & 0x7fffffffu]);
    if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) continue;  // affine infinity (ec_ops.h:717)
    xyzz_madd(acc, p, (e >> 31) != 0);
  }
#endif
  st16(&buckets[S.order[t]], acc);
}
template <int G, class PT = Aff<typename FieldOf<G>::F>>
__global__ void __launch_bounds__(256, MSM_ACC_WAVES)
    k_accumulate(const AccSched S, const PT *__restrict__ pts, Xyzz<typename FieldOf<G>::F> *__restrict__ buckets,
                 size_t nbuckets) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nbuckets) accumulate_bucket<G>(S, pts, buckets, t);
}
// The accumulations of a front group's R sets in ONE grid (blockIdx.y = set r,
// buckets of set r at r nbuckets): a small MSM's one-lane-per-bucket grid fills
// the chip's wave slots only ~1 round deep and its last, shortest waves run
// with the chip half idle; R sets in one dispatch keep it full until the
// group's last round (Ches::run_jobs, accumulation groups).
template <int G, class PT>
__global__ void __launch_bounds__(256, MSM_ACC_WAVES)
    k_accumulate_sets(const AccSched S, const AccStride st, const PT *__restrict__ pts,
                      Xyzz<typename FieldOf<G>::F> *__restrict__ buckets, size_t nbuckets) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nbuckets) accumulate_bucket<G>(acc_set(S, st, blockIdx.y), pts, buckets + blockIdx.y * nbuckets, t);
}

// xyzz -> blst Jacobian (X*ZZ, Y*ZZZ, ZZ)  (ref ec_ops.h:771-777), canonical blst Montgomery
// (one lane per window, 64-thread blocks: the bound lets G2 keep every operand
// in registers -- the default 1024-thread bound capped it at 128 VGPRs and
// spilled 236 B, tests/test_kernel_resources.py)
template <int G>
__global__ void __launch_bounds__(64) k_finalize(const Xyzz<typename FieldOf<G>::F> *__restrict__ T, uint64_t *__restrict__ out, int W) {
  typedef typename FieldOf<G>::F F;
  int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  Xyzz<F> a = ld16(&T[w]);
  F X, Y;
  f_mul(X, a.x, a.zz);
  f_mul(Y, a.y, a.zzz);
  uint64_t *o = out + (size_t)w * 18 * G;
  if (xyzz_is_inf(a)) {
    for (int k = 0; k < 18 * G; ++k) o[k] = 0;
    return;
  }
  f_to_blst(o, X);
  f_to_blst(o + 6 * G, Y);
  f_to_blst(o + 12 * G, a.zz);
}

}  // namespace msm
