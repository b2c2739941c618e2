// fp.hpp -- BLS12-381 base-field arithmetic for gfx950, kept in registers.
//
// Replaces the reference's Fp384 Montgomery routines (src/asm/mulx_mont_384-
// x86_64.pl:1613-1828, add_mod_384-x86_64.pl:32-1000; portable spec
// src/no_asm.h:29-291) and the Fp2 tower ops (no_asm.h:566-688).
//
// Design (measured on MI355X, tools/microbench/instr_rate.hip): one
// v_mad_u64_u32 (32x32+64 -> 64) issues at the same rate as one
// v_add_co_u32, so the cost of a multi-precision product is set by how many
// carry instructions surround each mad.  We therefore use 14 limbs of 28
// bits (392 bits, radix 2^28, Montgomery R = 2^392) instead of the 6x64-bit
// layout of blst: every 28x28 product is < 2^56 and a whole product-scanning
// column (<= 28 terms, limbs < 2^30) fits in one 64-bit accumulator, so each
// limb product is exactly ONE v_mad_u64_u32 with no carry handling (FIPS
// Montgomery: 392 mads + ~4 ops per column).
//
// Values are kept lazily reduced: a Montgomery product of inputs < 2^386 is
// < 2p, adds do no carry propagation (limbs < 2^30 stay legal mul inputs),
// subtraction adds a limb-wise "borrow-adjusted" multiple of p (every limb
// >= 2^28-1) so no limb goes negative.  Range invariants are documented at
// each use in ec.hpp.  Canonical values (< p) are produced only at the
// boundary (fp_canon).  The 6x64-bit blst layout is used in HBM at the C-ABI
// boundary and converted once per point on upload.
#pragma once
#include <stdint.h>

// MSM_FP_HOST_TEST: a host (g++) build of this header and ec.hpp for the
// lazy-reduction bound tests (tests/test_fp_bounds.py);
// the engine itself always compiles them as device code for gfx950.
// The host build checks every range assumption the device code relies on
// (MSM_CHECK: a 64-bit column or 32-bit limb that would wrap, a negative limb
// or a negative reduced value sets msm_fp_overflow); on the device the checks
// compile to nothing.
#ifdef MSM_FP_HOST_TEST
#define MSM_FN inline
#define MSM_CONST constexpr
extern "C" int msm_fp_overflow;
#define MSM_CHECK(c)                                                    \
  do {                                                                  \
    if (!(c)) __atomic_store_n(&msm_fp_overflow, 1, __ATOMIC_RELAXED);  \
  } while (0)
#else
#include <hip/hip_runtime.h>
#define MSM_FN __device__ __forceinline__
#define MSM_CONST __device__ constexpr
#define MSM_CHECK(c) ((void)0)
#endif

namespace msm {

constexpr int NL = 14;            // limbs
constexpr uint32_t MASK = 0x0fffffffu;
constexpr uint32_t N0P = 0x0ffcfffdu;  // -p^-1 mod 2^28

// p in radix 2^28
MSM_CONST uint32_t P28[NL] = {0xfffaaab, 0xfefffff, 0x3ffffb9, 0xfffeb15, 0x6241eab, 0xa0f6b0f, 0xf6730d2,
                                         0xf38512b, 0x4774b84, 0x4bacd76, 0xba7b643, 0xe69a4b1, 0x1ea397f, 0x001a011};
// k*p with limbs borrow-adjusted so limbs 0..12 are >= 2^28-1 (subtrahend headroom)
MSM_CONST uint32_t SUB4P[NL] = {0x1ffeaaac, 0x1fbffffe, 0x1ffffee6, 0x1fffac53, 0x18907aae,
                                           0x183dac3c, 0x1d9cc349, 0x1ce144ae, 0x11dd2e12, 0x12eb35d8,
                                           0x1e9ed90c, 0x19a692c5, 0x17a8e5fe, 0x0068043};
MSM_CONST uint32_t SUB8P[NL] = {0x1ffd5558, 0x1f7ffffe, 0x1ffffdce, 0x1fff58a8, 0x1120f55e,
                                           0x107b587a, 0x1b398694, 0x19c2895e, 0x13ba5c26, 0x15d66bb1,
                                           0x1d3db219, 0x134d258c, 0x1f51cbfe, 0x00d0087};
MSM_CONST uint32_t SUB16P[NL] = {0x1ffaaab0, 0x1efffffe, 0x1ffffb9e, 0x1ffeb152, 0x1241eabe,
                                            0x10f6b0f5, 0x16730d29, 0x138512be, 0x1774b84e, 0x1bacd763,
                                            0x1a7b6433, 0x169a4b1a, 0x1ea397fd, 0x01a0110};
MSM_CONST uint32_t SUB32P[NL] = {0x1ff55560, 0x1dfffffe, 0x1ffff73e, 0x1ffd62a6, 0x1483d57e,
                                            0x11ed61eb, 0x1ce61a53, 0x170a257d, 0x1ee9709d, 0x1759aec7,
                                            0x14f6c868, 0x1d349636, 0x1d472ffb, 0x0340222};
// 8p borrow-adjusted so limbs 0..12 are >= 3(2^28-1): the minuend of fp_sub_2x
MSM_CONST uint32_t SUB8P3[NL] = {0x3ffd5558, 0x3f7ffffc, 0x3ffffdcc, 0x3fff58a6, 0x3120f55c,
                                            0x307b5878, 0x3b398692, 0x39c2895c, 0x33ba5c24, 0x35d66baf,
                                            0x3d3db217, 0x334d258a, 0x3f51cbfc, 0x00d0085};
// 2^392 mod p (one), 2^400 mod p (blst -> internal), 2^384 mod p (internal -> blst)
MSM_CONST uint32_t ONE28[NL] = {0x347fcb8, 0xd800000, 0x002b119, 0x0cde6d2, 0xc7212e0, 0x83a2090, 0x037669f,
                                           0xda0f73e, 0x9b09b42, 0x1297bb0, 0x515d98f, 0x012ca7c, 0x659fcfa, 0x000577a};
MSM_CONST uint32_t TOINT28[NL] = {0x80e6299, 0x3500034, 0xeb12856, 0xdeb2699, 0xc988670,
                                             0x4ef6697, 0x70983e8, 0xa4e6fe9, 0x3e8a053, 0xecf271e,
                                             0xc20d323, 0x6eb6385, 0x47f1286, 0x00156da};
MSM_CONST uint32_t FROMINT28[NL] = {0x002fffd, 0x0900000, 0xc000276, 0x000bc40, 0x8baebf4,
                                               0x5753c75, 0x55f4898, 0x7052574, 0x7ce5853, 0x56ec6d7,
                                               0x71a97a2, 0xe4935c0, 0xec3fa80, 0x0015f65};

struct Fp {
  uint32_t v[NL];
};

MSM_FN uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  MSM_CHECK((uint64_t)a * (uint64_t)b <= ~c);  // the column accumulator never wraps
  return (uint64_t)a * (uint64_t)b + c;  // -> v_mad_u64_u32
}
// final (top) limb of a Montgomery product: the accumulator must fit 32 bits
MSM_FN uint32_t top32(uint64_t acc) {
  MSM_CHECK(acc <= 0xffffffffull);
  return (uint32_t)acc;
}

// Montgomery product, FIPS (finely integrated product scanning).
// Inputs: limbs < 2^30, values with a*b < 2^392 * p (e.g. both < 2^386).
// Output: normalized limbs (< 2^28), value < 2p.
MSM_FN void fp_mul(Fp &r, const Fp &a, const Fp &b) {
  uint32_t m[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) acc = mad64(a.v[i], b.v[k - i], acc);
#pragma unroll
    for (int i = 0; i < k; ++i) acc = mad64(m[i], P28[k - i], acc);
    m[k] = ((uint32_t)acc * N0P) & MASK;
    acc = mad64(m[k], P28[0], acc);
    acc >>= 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; ++k) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad64(a.v[i], b.v[k - i], acc);
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad64(m[i], P28[k - i], acc);
    r.v[k - NL] = (uint32_t)acc & MASK;
    acc >>= 28;
  }
  r.v[NL - 1] = top32(acc);
}

// Sum of two products with ONE Montgomery reduction: (a b + c d) / R mod p.
// Column bound (FIPS accumulator): 14 a_i b_j < 2^59.2 (limbs < 2^29.6) +
// 14 c_i d_j < 2^57.6 (c limbs < 2^28.6, d limbs < 2^29) + 14 m p < 2^56 +
// carry < 2^63.4.  Used as a b - c d with d := 4p - d (lazy reduction of the
// Y3 = R (Q - X3) - Y1 PPP line of the xyzz formulas): 588 mads instead of 784.
// Output: normalized, < 1.1 p for the callers' ranges (a b + c d < 63 p^2).
MSM_FN void fp_mul2(Fp &r, const Fp &a, const Fp &b, const Fp &c, const Fp &d) {
  uint32_t m[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) acc = mad64(a.v[i], b.v[k - i], acc);
#pragma unroll
    for (int i = 0; i <= k; ++i) acc = mad64(c.v[i], d.v[k - i], acc);
#pragma unroll
    for (int i = 0; i < k; ++i) acc = mad64(m[i], P28[k - i], acc);
    m[k] = ((uint32_t)acc * N0P) & MASK;
    acc = mad64(m[k], P28[0], acc);
    acc >>= 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; ++k) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad64(a.v[i], b.v[k - i], acc);
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad64(c.v[i], d.v[k - i], acc);
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad64(m[i], P28[k - i], acc);
    r.v[k - NL] = (uint32_t)acc & MASK;
    acc >>= 28;
  }
  r.v[NL - 1] = top32(acc);
}

// Four products with ONE Montgomery reduction: (a b + c d + e f + g h) / R mod p.
// The caller keeps every column < 2^64: 14 (a_i b_j + c_i d_j + e_i f_j + g_i h_j)
// + 14 m p + carry (see the Fp2 f_mul_sub below for the ranges it uses).
MSM_FN void fp_mul4(Fp &r, const Fp &a, const Fp &b, const Fp &c, const Fp &d, const Fp &e,
                                        const Fp &f, const Fp &g, const Fp &h) {
  uint32_t m[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) {
      acc = mad64(a.v[i], b.v[k - i], acc);
      acc = mad64(c.v[i], d.v[k - i], acc);
      acc = mad64(e.v[i], f.v[k - i], acc);
      acc = mad64(g.v[i], h.v[k - i], acc);
    }
#pragma unroll
    for (int i = 0; i < k; ++i) acc = mad64(m[i], P28[k - i], acc);
    m[k] = ((uint32_t)acc * N0P) & MASK;
    acc = mad64(m[k], P28[0], acc);
    acc >>= 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; ++k) {
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) {
      acc = mad64(a.v[i], b.v[k - i], acc);
      acc = mad64(c.v[i], d.v[k - i], acc);
      acc = mad64(e.v[i], f.v[k - i], acc);
      acc = mad64(g.v[i], h.v[k - i], acc);
    }
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad64(m[i], P28[k - i], acc);
    r.v[k - NL] = (uint32_t)acc & MASK;
    acc >>= 28;
  }
  r.v[NL - 1] = top32(acc);
}

// doubled cross sum of a square column folded into the accumulator: acc + 2x
// in one v_lshl_add_u64 (x is its own mad chain, so the column keeps two
// independent chains without a doubled copy of the operand)
MSM_FN uint64_t add_dbl(uint64_t x, uint64_t acc) {
  MSM_CHECK(x < (1ull << 63) && (x << 1) <= ~acc);
  return (x << 1) + acc;
}
// Montgomery square: each cross product once, per column x = sum_{i<j} a_i a_j
// on its own chain and acc += 2x (no doubled operand copy: 14 fewer live
// VGPRs and 14 fewer shifts than squaring against a << 1).
MSM_FN void fp_sqr(Fp &r, const Fp &a) {
  uint32_t m[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    if (k > 0) {
      uint64_t x = 0;
#pragma unroll
      for (int i = 0; 2 * i < k; ++i) x = mad64(a.v[i], a.v[k - i], x);
      acc = add_dbl(x, acc);
    }
    if ((k & 1) == 0) acc = mad64(a.v[k / 2], a.v[k / 2], acc);
#pragma unroll
    for (int i = 0; i < k; ++i) acc = mad64(m[i], P28[k - i], acc);
    m[k] = ((uint32_t)acc * N0P) & MASK;
    acc = mad64(m[k], P28[0], acc);
    acc >>= 28;
  }
#pragma unroll
  for (int k = NL; k < 2 * NL - 1; ++k) {
    if (k < 2 * NL - 2) {
      uint64_t x = 0;
#pragma unroll
      for (int i = k - NL + 1; 2 * i < k; ++i) x = mad64(a.v[i], a.v[k - i], x);
      acc = add_dbl(x, acc);
    }
    if ((k & 1) == 0) acc = mad64(a.v[k / 2], a.v[k / 2], acc);
#pragma unroll
    for (int i = k - NL + 1; i < NL; ++i) acc = mad64(m[i], P28[k - i], acc);
    r.v[k - NL] = (uint32_t)acc & MASK;
    acc >>= 28;
  }
  r.v[NL - 1] = top32(acc);
}

// lazy add: no carry propagation
MSM_FN void fp_add(Fp &r, const Fp &a, const Fp &b) {
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    MSM_CHECK((uint64_t)a.v[i] + b.v[i] <= 0xffffffffull);
    r.v[i] = a.v[i] + b.v[i];
  }
}
// carry propagation -> limbs < 2^28 (value unchanged, non-negative limbs assumed)
MSM_FN void fp_norm(Fp &a) {
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    MSM_CHECK((uint64_t)a.v[i + 1] + (a.v[i] >> 28) <= 0xffffffffull);
    a.v[i + 1] += a.v[i] >> 28;
    a.v[i] &= MASK;
  }
}
// r = a + K*p - b, K in {4,8,16,32}; b must be normalized (limbs < 2^28) with b < K*p/2-ish
// (precisely: b's top limb below the adjusted top limb of K*p).
template <int K>
MSM_FN void fp_sub(Fp &r, const Fp &a, const Fp &b) {
  const uint32_t *C = K == 4 ? SUB4P : K == 8 ? SUB8P : K == 16 ? SUB16P : SUB32P;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    MSM_CHECK((uint64_t)a.v[i] + C[i] <= 0xffffffffull && a.v[i] + C[i] >= b.v[i]);  // no wrap, limb >= 0
    r.v[i] = a.v[i] + C[i] - b.v[i];
  }
}
// r = a + 8p - b - 2c for b, c normalized (limbs < 2^28) with b + 2c <= 8p:
// three VALU ops per limb (v_lshl_add_u32, v_sub, v_add) instead of three
// fp_sub<4> + two fp_norm -- the X3 = R^2 - PPP - 2Q line of the xyzz formulas.
MSM_FN void fp_sub_2x(Fp &r, const Fp &a, const Fp &b, const Fp &c) {
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint32_t t = b.v[i] + (c.v[i] << 1);
    MSM_CHECK((uint64_t)b.v[i] + 2ull * c.v[i] <= SUB8P3[i]);           // limb >= 0
    MSM_CHECK((uint64_t)a.v[i] + SUB8P3[i] - t <= 0xffffffffull);       // no wrap
    r.v[i] = a.v[i] + (SUB8P3[i] - t);
  }
}
// r = K*p - a (negation), a normalized
template <int K>
MSM_FN void fp_neg(Fp &r, const Fp &a) {
  const uint32_t *C = K == 4 ? SUB4P : K == 8 ? SUB8P : K == 16 ? SUB16P : SUB32P;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    MSM_CHECK(C[i] >= a.v[i]);
    r.v[i] = C[i] - a.v[i];
  }
}
MSM_FN void fp_cneg4(Fp &r, const Fp &a, bool neg) {
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    MSM_CHECK(!neg || SUB4P[i] >= a.v[i]);
    r.v[i] = neg ? SUB4P[i] - a.v[i] : a.v[i];
  }
}
MSM_FN void fp_set(Fp &r, const uint32_t *c) {
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = c[i];
}
MSM_FN void fp_zero(Fp &r) {
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = 0;
}
MSM_FN void fp_one(Fp &r) { fp_set(r, ONE28); }
MSM_FN bool fp_is_zero_exact(const Fp &a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) o |= a.v[i];
  return o == 0;
}
// a normalized with a < 2p: a == 0 mod p  <=>  a == 0 or a == p
MSM_FN bool fp_is_zero_lt2p(const Fp &a) {
  uint32_t o = 0, x = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    o |= a.v[i];
    x |= a.v[i] ^ P28[i];
  }
  return o == 0 || x == 0;
}
// conditional subtract p for normalized a < 2p -> canonical [0,p)
MSM_FN void fp_csub_p(Fp &a) {
  uint32_t t[NL];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    int32_t d = (int32_t)a.v[i] - (int32_t)P28[i] + br;
    br = d >> 28;          // arithmetic shift: 0 or -1
    t[i] = (uint32_t)d & MASK;
  }
  bool ge = br == 0;       // no final borrow -> a >= p
#pragma unroll
  for (int i = 0; i < NL; ++i) a.v[i] = ge ? t[i] : a.v[i];
}
// canonical representative of any lazy value (< 2^386, limbs < 2^30):
// multiply by one (=2^392 mod p, Montgomery one) keeps the value, result < 2p normalized.
MSM_FN void fp_canon(Fp &r, const Fp &a) {
  Fp one;
  fp_one(one);
  fp_mul(r, a, one);
  fp_csub_p(r);
}

// Reduce a normalized value v < 32p to [0, 2p) (class S): quotient estimate
// from the top limb, q = floor(v13 * floor(2^32/(p13+1)) / 2^32) <= floor(v/p);
// v - q*p < 1.0003p (checked exhaustively over the top limb: tests/fp_bounds.py red()).
constexpr uint32_t RED_MAG = 0x9d83;  // floor(2^32 / (p13 + 1)), p13 = 0x1a011
MSM_FN void fp_red(Fp &a) {
  uint32_t q = (uint32_t)(((uint64_t)a.v[NL - 1] * RED_MAG) >> 32);
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    int64_t t = (int64_t)a.v[i] - (int64_t)((uint64_t)q * P28[i]) + c;
    a.v[i] = (uint32_t)t & MASK;
    c = t >> 28;
  }
  MSM_CHECK(c == 0);  // v - q p >= 0 and < 2^392: nothing left over
}
// normalize then reduce: lazy value (< 32p, limbs < 2^31, non-negative) -> class S
MSM_FN void fp_nred(Fp &a) {
  fp_norm(a);
  fp_red(a);
}

// ------------------------------------------------------------ generic API ---
// Range classes used by ec.hpp (all values non-negative):
//   S : normalized limbs (< 2^28), value < 2p.  Every f_mul/f_sqr output, every
//       f_nred output, every stored coordinate.
//   X : normalized limbs, value < 10p: the x coordinate of a stored xyzz point
//       (X3 = R^2 - PPP - 2Q is normalized but not reduced; x only ever enters
//       products and the subtrahend of f_sub16).
//   lazy : limbs < 2^30, value < 40p.  Legal f_mul/f_sqr input.
//   f_add(S,S) < 4p lazy; f_sub4(x,S) = x + 4p - S (x S -> < 6p lazy);
//   f_sub subtrahend MUST be S.
MSM_FN void f_mul(Fp &r, const Fp &a, const Fp &b) { fp_mul(r, a, b); }
MSM_FN void f_sqr(Fp &r, const Fp &a) { fp_sqr(r, a); }
MSM_FN void f_add(Fp &r, const Fp &a, const Fp &b) { fp_add(r, a, b); }
MSM_FN void f_sub4(Fp &r, const Fp &a, const Fp &b) { fp_sub<4>(r, a, b); }
// a + 8p - b - 2c, b and c in S (b + 2c < 6p) -> lazy (< a + 8p, limbs < 2^31)
MSM_FN void f_sub_2x(Fp &r, const Fp &a, const Fp &b, const Fp &c) { fp_sub_2x(r, a, b, c); }
// a + 16p - b for b normalized < 16p (class X: the lazily reduced x coordinate)
MSM_FN void f_sub16(Fp &r, const Fp &a, const Fp &b) { fp_sub<16>(r, a, b); }
MSM_FN void f_nred(Fp &a) { fp_nred(a); }
MSM_FN void f_norm(Fp &a) { fp_norm(a); }
MSM_FN void f_neg4(Fp &r, const Fp &a) { fp_neg<4>(r, a); }
MSM_FN void f_one(Fp &r) { fp_one(r); }
MSM_FN void f_zero(Fp &r) { fp_zero(r); }
MSM_FN bool f_is_zero_exact(const Fp &a) { return fp_is_zero_exact(a); }
MSM_FN bool f_is_zero_S(const Fp &a) { return fp_is_zero_lt2p(a); }
// a b - c d for a, b lazy (< 6p, limbs < 2^29.6), c, d in S -> S
MSM_FN void f_mul_sub(Fp &r, const Fp &a, const Fp &b, const Fp &c, const Fp &d) {
  Fp nd;
  fp_neg<4>(nd, d);  // 4p - d, limbs < 2^29
  fp_mul2(r, a, b, c, nd);
}
// 3a for a in S -> lazy (< 6p, limbs < 2^30)
MSM_FN void f_mul3(Fp &r, const Fp &a) {
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    MSM_CHECK(a.v[i] <= 0x55555555u);
    r.v[i] = a.v[i] * 3u;
  }
}

// ---------------------------------------------------------------- Fp2 ----
struct Fp2 {
  Fp c0, c1;
};

// (a0 + a1 i)(b0 + b1 i) as two sums of products with one Montgomery reduction
// each (fp_mul2), instead of Karatsuba's three products (ref no_asm.h:566-579):
//   c0 = a0 b0 + a1 (8p - b1),   c1 = a0 b1 + a1 b0.
// Same 1176 mads, but no add/sub/reduce fix-ups and two live temporaries
// instead of five -- the G2 bucket accumulation is register-bound.
// Ranges: a lazy (< 6p, limbs < 2^30); b lazy, normalized here (limbs < 2^28
// below the top limb) so every column stays < 2^63.5 (14 a_i b_j < 2^61.8,
// 14 a_i (8p - b1)_j < 2^62.8, 14 m p < 2^59.8); a b + a1 (8p - b1) < 84 p^2 ->
// output normalized, < 1.1 p (class S).  r may alias a or b.
MSM_FN void f_mul(Fp2 &r, const Fp2 &a, const Fp2 &b) {
  Fp b0 = b.c0, b1 = b.c1, nb1, t0, t1;
  fp_norm(b0);
  fp_norm(b1);
  fp_neg<8>(nb1, b1);
  fp_mul2(t0, a.c0, b0, a.c1, nb1);
  fp_mul2(t1, a.c0, b1, a.c1, b0);
  r.c0 = t0;
  r.c1 = t1;
}
// f_mul for a b already normalized (class S, or any normalized value < 8p):
// no normalized copies of b, one temporary (fp_mul2 writes limb j only after
// its last read of limb j of any input, so r.c1 may be produced in place).
MSM_FN void f_mul_bs(Fp2 &r, const Fp2 &a, const Fp2 &b) {
  Fp nb1, t0;
  fp_neg<8>(nb1, b.c1);
  fp_mul2(t0, a.c0, b.c0, a.c1, nb1);
  fp_mul2(r.c1, a.c0, b.c1, a.c1, b.c0);
  r.c0 = t0;
}
MSM_FN void f_mul_bs(Fp &r, const Fp &a, const Fp &b) { fp_mul(r, a, b); }

// (a0 + a1 i)^2 = (a0+a1)(a0-a1) + 2 a0 a1 i   (ref no_asm.h:638-688)
// Both components are normalized first: with lazy inputs (limbs < 3 2^28) the
// product s d would reach 14 (6 2^28)(5 2^28) > 2^64 in a column (DESIGN 4a,
// tests/fp_bounds.py); normalized, s limbs < 2^29 and d limbs < 2^30.
// Callers pass values < 18p (P = U2 - X1, X1 in class X), so 32p - a1 > 0 and
// s d < 36p 50p < 2^392 p.
MSM_FN void f_sqr(Fp2 &r, const Fp2 &a) {
  Fp s, d, m, a0 = a.c0, a1 = a.c1;
  fp_norm(a0);
  fp_norm(a1);
  fp_add(s, a0, a1);
  fp_sub<32>(d, a0, a1);
  fp_mul(m, a0, a1);
  fp_mul(r.c0, s, d);
  fp_add(r.c1, m, m);
  fp_red(r.c1);  // m + m < 4p with limbs < 2^29: red handles non-normalized limbs via signed carry
  fp_norm(r.c1);
}
MSM_FN void f_add(Fp2 &r, const Fp2 &a, const Fp2 &b) {
  fp_add(r.c0, a.c0, b.c0);
  fp_add(r.c1, a.c1, b.c1);
}
MSM_FN void f_sub4(Fp2 &r, const Fp2 &a, const Fp2 &b) {
  fp_sub<4>(r.c0, a.c0, b.c0);
  fp_sub<4>(r.c1, a.c1, b.c1);
}
MSM_FN void f_sub16(Fp2 &r, const Fp2 &a, const Fp2 &b) {
  fp_sub<16>(r.c0, a.c0, b.c0);
  fp_sub<16>(r.c1, a.c1, b.c1);
}
MSM_FN void f_sub_2x(Fp2 &r, const Fp2 &a, const Fp2 &b, const Fp2 &c) {
  fp_sub_2x(r.c0, a.c0, b.c0, c.c0);
  fp_sub_2x(r.c1, a.c1, b.c1, c.c1);
}
MSM_FN void f_nred(Fp2 &a) { fp_nred(a.c0); fp_nred(a.c1); }
MSM_FN void f_norm(Fp2 &a) { fp_norm(a.c0); fp_norm(a.c1); }
MSM_FN void f_neg4(Fp2 &r, const Fp2 &a) { fp_neg<4>(r.c0, a.c0); fp_neg<4>(r.c1, a.c1); }
MSM_FN void f_one(Fp2 &r) { fp_one(r.c0); fp_zero(r.c1); }
MSM_FN void f_zero(Fp2 &r) { fp_zero(r.c0); fp_zero(r.c1); }
MSM_FN bool f_is_zero_exact(const Fp2 &a) { return fp_is_zero_exact(a.c0) && fp_is_zero_exact(a.c1); }
MSM_FN bool f_is_zero_S(const Fp2 &a) { return fp_is_zero_lt2p(a.c0) && fp_is_zero_lt2p(a.c1); }
MSM_FN void f_mul3(Fp2 &r, const Fp2 &a) { f_mul3(r.c0, a.c0); f_mul3(r.c1, a.c1); }
// a b - c d over Fp2, each component one four-product reduction (fp_mul4):
//   r0 = a0 b0 + a1 (8p - b1) + c0 (8p - d0) + c1 d1
//   r1 = a0 b1 + a1 b0 + c0 (8p - d1) + c1 (8p - d0)
// Ranges (every caller: xyzz Y3 lines): a lazy (< 6p, limbs < 2^29.6), b lazy
// (normalized here), c, d in S.  Column < 14 (2^57.6 + 2^58.6 + 2^57 + 2^57)
// + 14 m p < 2^63.6; value < 104 p^2 -> output normalized, < 1.1 p (S).
// r may alias any input.
MSM_FN void f_mul_sub(Fp2 &r, const Fp2 &a, const Fp2 &b, const Fp2 &c, const Fp2 &d) {
  Fp b0 = b.c0, b1 = b.c1, nb1, nd0, nd1, t0, t1;
  fp_norm(b0);
  fp_norm(b1);
  fp_neg<8>(nb1, b1);
  fp_neg<8>(nd0, d.c0);
  fp_neg<8>(nd1, d.c1);
  fp_mul4(t0, a.c0, b0, a.c1, nb1, c.c0, nd0, c.c1, d.c1);
  fp_mul4(t1, a.c0, b1, a.c1, b0, c.c0, nd1, c.c1, nd0);
  r.c0 = t0;
  r.c1 = t1;
}

}  // namespace msm
