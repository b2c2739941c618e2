// ches_kernels.hpp -- device kernels of the CHES "nh + q/5" bucket-set MSM
// (LuoGuiwen/MSM_blst) for gfx950, templated on the group (G1: Fp, G2: Fp2).
//
//   k_ches_table    T[3(i h + j) + m - 1] = m q^j P_i, affine, built on the GPU
//                   (replaces the 470 s CPU loop of ref main_p1.cpp:155-172):
//                   xyzz doublings per lane + one Montgomery batch inversion
//                   per lane over its 3h points
//   k_ches_digits   MB radix-q digits of every scalar, on device
//                   (ref auxiliaryfunc.h:92-118 + main_p1.cpp:208-228): std
//                   q-ary digit + carry -> digit-hash lookup -> (bucket index,
//                   m, alpha); entries with bucket value 0 are dropped (the
//                   reference's `if (booth_idx)` guard, multi_scalar.c:440)
//                   -> one (bucket, table slot | sign << 31) entry per digit,
//                   sorted by BucketSort (bucket_sort.hpp)
//   k_segsum        segment sums of xyzz points over an index list (the two
//                   regroupings of the bucket reduction, see ches.hip)
// Bucket accumulation and the dense window reduction reuse k_accumulate /
// k_reduce of kernels.hpp.
#pragma once
#include "bucket_sort.hpp"
#include "kernels.hpp"

namespace msm {

// packed digit-hash entry (device): bits 0..23 bucket index in B (0 = value 0,
// skipped), bits 24..25 m - 1, bit 31 alpha (negative digit, carry +1)
constexpr uint32_t CH_IDX_MASK = 0x00ffffffu;

// ---------------------------------------------------------------- inversion --
// a^(p-2) mod p (Fermat), fixed 2-bit windows, input any lazy value, output S.
// Inlined and register-lean (a, a^2, a^3 and the accumulator: ~60 VGPRs): the
// earlier 4-bit version kept a 16-entry table in scratch (912 B/lane) and was
// a call -- the table kernels that use it are now scratch-free.
// One inversion per lane amortises over the lane's 3h table rows, so its ~570
// products (vs ~490 with 4-bit windows) do not matter.
__device__ constexpr uint64_t PM2[6] = {0xb9feffffffffaaa9ull, 0x1eabfffeb153ffffull, 0x6730d2a0f6b0f624ull,
                                        0x64774b84f38512bfull, 0x4b1ba7b6434bacd7ull, 0x1a0111ea397fe69aull};
__device__ __forceinline__ void fp_inv(Fp &r, const Fp &a) {
  Fp a1 = a, a2, a3, acc;
  fp_norm(a1);
  fp_sqr(a2, a1);
  fp_mul(a3, a2, a1);
  fp_one(acc);
  for (int k = 190; k >= 0; --k) {  // 2-bit windows of p - 2 (381 bits), from the top
    if (k != 190) {
      fp_sqr(acc, acc);
      fp_sqr(acc, acc);
    }
    const uint32_t w = (uint32_t)(PM2[k >> 5] >> ((k & 31) * 2)) & 3u;  // uniform: the exponent is a constant
    if (w) {
      const uint32_t m1 = 0u - (uint32_t)(w == 1), m2 = 0u - (uint32_t)(w == 2), m3 = 0u - (uint32_t)(w == 3);
      Fp t;
#pragma unroll
      for (int i = 0; i < NL; ++i) t.v[i] = (a1.v[i] & m1) | (a2.v[i] & m2) | (a3.v[i] & m3);
      fp_mul(acc, acc, t);
    }
  }
  r = acc;
}
__device__ __forceinline__ void f_inv(Fp &r, const Fp &a) { fp_inv(r, a); }
// 1/(a0 + a1 i) = (a0 - a1 i) / (a0^2 + a1^2)
__device__ __forceinline__ void f_inv(Fp2 &r, const Fp2 &a) {
  Fp t0, t1, d;
  fp_sqr(t0, a.c0);
  fp_sqr(t1, a.c1);
  fp_add(d, t0, t1);
  fp_inv(d, d);
  fp_mul(r.c0, a.c0, d);
  Fp n1;
  Fp a1 = a.c1;
  fp_norm(a1);
  fp_neg<4>(n1, a1);
  fp_mul(r.c1, n1, d);
}
__device__ __forceinline__ void f_csub(Fp &a) { fp_csub_p(a); }
__device__ __forceinline__ void f_csub(Fp2 &a) {
  fp_csub_p(a.c0);
  fp_csub_p(a.c1);
}

// ------------------------------------------------------------ table build --
// One lane per base point i in [i0, i0+cnt).  scratch holds the lane's M h
// xyzz points and prefix products, interleaved by lane for coalescing.
// M = 3: CHES table T[3(i h + j) + m - 1] = m q^j P_i (ref main_p1.cpp:155-172);
// M = 1: BGMW95 table T[i h + j] = q^j P_i (ref main_p1.cpp:94-122).
template <int G, int M = 3>
static __global__ void __launch_bounds__(256)
    k_ches_table(const Aff<typename FieldOf<G>::F> *__restrict__ P, size_t i0, size_t cnt, int q_exp, int h,
                 Xyzz<typename FieldOf<G>::F> *__restrict__ scratch, typename FieldOf<G>::F *__restrict__ pref,
                 AffP<typename FieldOf<G>::F> *__restrict__ T) {
  typedef typename FieldOf<G>::F F;
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cnt) return;
  const size_t i = i0 + t;
  static_assert(M == 1 || M == 3, "M");
  const int K = M * h;
  Aff<F> p = ld16(&P[i]);
  AffP<F> *out = T + (size_t)K * i;
  if (f_is_zero_exact(p.x) && f_is_zero_exact(p.y)) {  // infinity: every multiple is infinity
    Aff<F> z;
    f_zero(z.x);
    f_zero(z.y);
    for (int k = 0; k < K; ++k) st_point(&out[k], z);
    return;
  }
  Xyzz<F> Q;
  xyzz_from_aff(Q, p, false);
  for (int j = 0; j < h; ++j) {
    st16(&scratch[(size_t)(M * j) * cnt + t], Q);
    if (M == 3) {  // 2 Q, then 3 Q = 2 Q + Q in place (one point fewer live)
      Xyzz<F> R;
      xyzz_dbl(R, Q);
      st16(&scratch[(size_t)(3 * j + 1) * cnt + t], R);
      xyzz_add(R, Q);
      st16(&scratch[(size_t)(3 * j + 2) * cnt + t], R);
    }
    if (j + 1 < h)
      for (int e = 0; e < q_exp; ++e) {
        Xyzz<F> tmp = Q;
        xyzz_dbl(Q, tmp);
      }
  }
  // Montgomery batch inversion of u_k = ZZ_k * ZZZ_k  (1/ZZ = ZZZ/u, 1/ZZZ = ZZ/u)
  F c;
  f_one(c);
  for (int k = 0; k < K; ++k) {
    Xyzz<F> a = ld16(&scratch[(size_t)k * cnt + t]);
    F u;
    f_mul(u, a.zz, a.zzz);
    f_mul(c, c, u);
    pref[(size_t)k * cnt + t] = c;
  }
  F inv;
  f_inv(inv, c);
  for (int k = K - 1; k >= 0; --k) {
    Xyzz<F> a = ld16(&scratch[(size_t)k * cnt + t]);
    F ik;
    if (k > 0) {
      F pk = pref[(size_t)(k - 1) * cnt + t];
      f_mul(ik, inv, pk);
      F u;
      f_mul(u, a.zz, a.zzz);
      f_mul(inv, inv, u);
    } else {
      ik = inv;
    }
    F izz, izzz;
    f_mul(izz, ik, a.zzz);
    f_mul(izzz, ik, a.zz);
    Aff<F> r;
    f_mul(r.x, a.x, izz);
    f_mul(r.y, a.y, izzz);
    f_csub(r.x);
    f_csub(r.y);
    st_point(&out[k], r);
  }
}

// internal affine -> blst affine (canonical Montgomery, R = 2^384)
template <int G, class PT>
__global__ void k_export_affine(const PT *__restrict__ in, uint64_t *__restrict__ out, size_t n) {
  typedef typename FieldOf<G>::F F;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Aff<F> a = ld_point(&in[i]);
  uint64_t *o = out + i * 12 * G;
  if (f_is_zero_exact(a.x) && f_is_zero_exact(a.y)) {
    for (int k = 0; k < 12 * G; ++k) o[k] = 0;
    return;
  }
  f_to_blst(o, a.x);
  f_to_blst(o + 6 * G, a.y);
}

// ------------------------------------------------------------------ digits --
// r (BLS12-381 group order), little-endian 32-bit words
__device__ constexpr uint32_t FR_R32[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                           0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};

// s >= r ? s - r : s   (on 8 x 32-bit words)
__device__ __forceinline__ void sub_r_if_ge(uint32_t s[8]) {
  uint32_t t[8];
  int64_t br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    int64_t d = (int64_t)s[k] - (int64_t)FR_R32[k] + br;
    t[k] = (uint32_t)d;
    br = d >> 32;
  }
  bool ge = br == 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = ge ? t[k] : s[k];
}

// One lane per scalar.  Scalars >= r are reduced mod r first (the reference
// requires s < r for this method, SURVEY 8b "Errors"; reducing keeps the result
// equal to sum s_i P_i for points of order r).
// Top-digit entries whose bucket index k is <= small go to copy i % copies of
// bucket k (copy 0 = k itself, copy c >= 1 = nb0 + (c-1) small + k - 1).
// HT = compile-time digit count (fully unrolled: every code lookup, for both
// carry states, is issued before the carry chain resolves, then every rank
// lookup); HT = 0 handles any h with a runtime loop.
//
// Digit code (replaces a gather from the (q+1)-entry, 16 MiB hash H of ref
// main_p1.cpp:140-152, whose random 4-B reads missed L2 and cost 0.17 ms at
// 2^20): H[d] = (m, b, alpha) always has b = (alpha ? q - d : d) / m
// (ches_digit_code checks this on the host), so the device keeps only
//   code[d]: 4 bits, (m - 1) | alpha << 2 | (b == 0) << 3, 8 per word (2 MiB)
//   rank[v >> 5] = {bit v & 31 set iff v in B, #B below 32 (v >> 5)} (512 KiB)
// and computes idx(b) = prefix + popcount(bits below b): both tables stay in
// each XCD's 4 MiB L2.
template <int HT>
static __global__ void __launch_bounds__(256)
    k_ches_digits(const uint8_t *__restrict__ scalars, size_t stride, size_t n, int q_exp, int h_rt,
                  const uint32_t *__restrict__ code, const uint2 *__restrict__ rank, uint32_t *__restrict__ keys, uint32_t *__restrict__ vals,
                  uint32_t nb0, uint32_t small, uint32_t copies, size_t set_stride) {
  const int h = HT ? HT : h_rt;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // blockIdx.y: scalar set of a batch front group (set_stride bytes apart), its
  // n h entries at keys / vals + set n h (BucketSort's per-set inputs)
  scalars += (size_t)blockIdx.y * set_stride;
  keys += (size_t)blockIdx.y * n * h;
  vals += (size_t)blockIdx.y * n * h;
  const uint8_t *sp = scalars + i * stride;
  uint32_t s[10];
  if ((stride & 3) == 0) {
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(sp);
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = s32[k];
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      s[k] = (uint32_t)sp[4 * k] | ((uint32_t)sp[4 * k + 1] << 8) | ((uint32_t)sp[4 * k + 2] << 16) |
             ((uint32_t)sp[4 * k + 3] << 24);
  }
  sub_r_if_ge(s);
  sub_r_if_ge(s);
  s[8] = s[9] = 0;
  const uint32_t qmask = (1u << q_exp) - 1u;
  auto digit = [&](int j) -> uint32_t {
    int off = j * q_exp;
    int wi = off >> 5, sh = off & 31;
    uint32_t lo = wi < 10 ? s[wi] : 0u, hi = wi + 1 < 10 ? s[wi + 1] : 0u;
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & qmask;
  };
  auto emit = [&](int j, uint32_t e) {
    const size_t slot = i * (size_t)h + j;  // (i, j) of the table index 3(i h + j) + m - 1
    const size_t k = (size_t)j * n + i;     // entry position: digit-major, coalesced stores
    uint32_t b = e & CH_IDX_MASK;
    if (j == h - 1 && b != 0 && b <= small) {
      uint32_t c = (uint32_t)(i % copies);
      if (c) b = nb0 + (c - 1) * small + b - 1;
    }
    if (b) {
      keys[k] = b;
      vals[k] = (uint32_t)(3 * slot + ((e >> 24) & 3u)) | (e & 0x80000000u);
    } else {
      keys[k] = KEY_NONE;
    }
  };
  const uint32_t q = 1u << q_exp;
  // code pair (d, d + 1) -> the carry-resolved (m - 1 | alpha << 2 | zero << 3, b)
  auto pair = [&](uint32_t d) -> uint64_t {
    const uint2 w = *reinterpret_cast<const uint2 *>(code + (d >> 3));  // 4-B aligned 8-B load
    return ((((uint64_t)w.y << 32) | w.x) >> (4 * (d & 7))) & 0xffu;
  };
  auto resolve = [&](uint32_t d, uint32_t c, uint32_t &b) {
    const uint32_t m1 = c & 3u, alpha = (c >> 2) & 1u;
    uint32_t v = alpha ? q - d : d;
    b = m1 == 0 ? v : (m1 == 1 ? v >> 1 : v / 3u);
  };
  auto entry = [&](uint32_t c, uint32_t b) -> uint32_t {
    if (c & 8u) return 0u;
    const uint2 r = rank[b >> 5];
    const uint32_t idx = r.y + (uint32_t)__popc(r.x & ((1u << (b & 31)) - 1u));
    return idx | ((c & 3u) << 24) | ((c & 4u) << 29);
  };
  if constexpr (HT > 0) {
    uint32_t dj[HT], cj[HT], bj[HT];
#pragma unroll
    for (int j = 0; j < HT; ++j) {
      dj[j] = digit(j);
      cj[j] = (uint32_t)pair(dj[j]);  // low nibble: code[d], high: code[d + 1]
    }
    uint32_t carry = 0;
#pragma unroll
    for (int j = 0; j < HT; ++j) {
      const uint32_t c = carry ? cj[j] >> 4 : cj[j] & 15u;
      resolve(dj[j] + carry, c, bj[j]);
      cj[j] = c;
      carry = (c >> 2) & 1u;
    }
#pragma unroll
    for (int j = 0; j < HT; ++j) emit(j, entry(cj[j], bj[j]));
  } else {
    uint32_t carry = 0;
    for (int j = 0; j < h; ++j) {
      const uint32_t d = digit(j) + carry;
      const uint32_t c = (uint32_t)pair(d) & 15u;
      uint32_t b;
      resolve(d, c, b);
      carry = (c >> 2) & 1u;
      emit(j, entry(c, b));
    }
  }
}

// ------------------------------------------------ fused CHES front (HT > 0) --
// The h entries of scalar i as k_ches_digits computes them (key = bucket or
// KEY_NONE, val = table slot | sign << 31), kept in registers.
template <int HT>
__device__ __forceinline__ void ches_entries(const uint8_t *__restrict__ sp, size_t stride, size_t i, int q_exp,
                                             const uint32_t *__restrict__ code, const uint2 *__restrict__ rank,
                                             uint32_t nb0, uint32_t small, uint32_t copies, uint32_t (&key)[HT],
                                             uint32_t (&val)[HT]) {
  uint32_t s[10];
  if ((stride & 3) == 0) {
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(sp);
#pragma unroll
    for (int k = 0; k < 8; ++k) s[k] = s32[k];
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      s[k] = (uint32_t)sp[4 * k] | ((uint32_t)sp[4 * k + 1] << 8) | ((uint32_t)sp[4 * k + 2] << 16) |
             ((uint32_t)sp[4 * k + 3] << 24);
  }
  sub_r_if_ge(s);
  sub_r_if_ge(s);
  s[8] = s[9] = 0;
  const uint32_t qmask = (1u << q_exp) - 1u, q = 1u << q_exp;
  uint32_t dj[HT], cj[HT];
#pragma unroll
  for (int j = 0; j < HT; ++j) {
    const int off = j * q_exp, wi = off >> 5, sh = off & 31;
    const uint32_t lo = wi < 10 ? s[wi] : 0u, hi = wi + 1 < 10 ? s[wi + 1] : 0u;
    dj[j] = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & qmask;
    const uint2 w = *reinterpret_cast<const uint2 *>(code + (dj[j] >> 3));  // code pair (d, d + 1)
    cj[j] = (uint32_t)(((((uint64_t)w.y << 32) | w.x) >> (4 * (dj[j] & 7))) & 0xffu);
  }
  uint32_t carry = 0;
#pragma unroll
  for (int j = 0; j < HT; ++j) {
    const uint32_t c = carry ? cj[j] >> 4 : cj[j] & 15u, d = dj[j] + carry;
    const uint32_t m1 = c & 3u, v = (c & 4u) ? q - d : d;
    dj[j] = m1 == 0 ? v : (m1 == 1 ? v >> 1 : v / 3u);  // bucket value b
    cj[j] = c;
    carry = (c >> 2) & 1u;
  }
#pragma unroll
  for (int j = 0; j < HT; ++j) {
    const uint32_t c = cj[j];
    uint32_t b = 0;
    if (!(c & 8u)) {
      const uint2 r = rank[dj[j] >> 5];
      b = r.y + (uint32_t)__popc(r.x & ((1u << (dj[j] & 31)) - 1u));
    }
    if (j == HT - 1 && b != 0 && b <= small) {
      const uint32_t cp = (uint32_t)(i % copies);
      if (cp) b = nb0 + (cp - 1) * small + b - 1;
    }
    key[j] = b ? b : KEY_NONE;
    val[j] = (uint32_t)(3 * (i * (size_t)HT + j) + (c & 3u)) | ((c & 4u) << 29);
  }
}

// Front pass A: the digits of a tile of 256 scalars (256 HT entries) counted
// per coarse bin in LDS -> ghist[set][bin][tile] (bucket_sort.hpp k_bs_hist
// without the keys array: nothing is written per entry).  Block 0 clears the
// schedule's class counters.
template <int HT>
static __global__ void __launch_bounds__(256)
    k_ches_front_hist(const uint8_t *__restrict__ scalars, size_t stride, size_t n, int q_exp,
                      const uint32_t *__restrict__ code, const uint2 *__restrict__ rank, uint32_t nb0, uint32_t small,
                      uint32_t copies, size_t set_stride, int fb_bits, int ncb, int ntiles, uint32_t *__restrict__ ghist,
                      uint32_t *__restrict__ classes) {
  __shared__ uint32_t h[BS_MAX_CB];
  scalars += (size_t)blockIdx.y * set_stride;
  ghist += (size_t)blockIdx.y * ncb * ntiles;
  if (blockIdx.x == 0)
    for (int c = threadIdx.x; c < 512; c += blockDim.x) classes[(size_t)blockIdx.y * 512 + c] = 0;
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) h[b] = 0;
  __syncthreads();
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t key[HT], val[HT];
    ches_entries<HT>(scalars + i * stride, stride, i, q_exp, code, rank, nb0, small, copies, key, val);
#pragma unroll
    for (int j = 0; j < HT; ++j)
      if (key[j] != KEY_NONE) atomicAdd(&h[key[j] >> fb_bits], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) ghist[(size_t)b * ntiles + blockIdx.x] = h[b];
}

// Front pass B: the same digits recomputed, ranked per coarse bin in LDS and
// staged bin-sorted in LDS, then streamed to the tile's run of each bin
// (k_bs_coarse with the entries taken from registers instead of keys / vals
// arrays: the digit kernel's 8-B-per-entry write and the sort's two reads of
// it are gone).  gbase: exclusive scan of ghist.  Dynamic LDS: 2 ncb + 2 * 256 HT words.
template <int HT>
static __global__ void __launch_bounds__(256)
    k_ches_front_coarse(const uint8_t *__restrict__ scalars, size_t stride, size_t n, int q_exp,
                        const uint32_t *__restrict__ code, const uint2 *__restrict__ rank, uint32_t nb0,
                        uint32_t small, uint32_t copies, size_t set_stride, int fb_bits, int ncb, int ntiles,
                        const uint32_t *__restrict__ gbase, uint32_t *__restrict__ okeys,
                        uint32_t *__restrict__ ovals) {
  extern __shared__ uint32_t sm[];
  __shared__ uint32_t wsum[4];
  uint32_t *loff = sm, *gb = sm + ncb, *sk = sm + 2 * ncb, *sv = sk + 256 * HT;
  scalars += (size_t)blockIdx.y * set_stride;
  gbase += (size_t)blockIdx.y * ncb * ntiles;
  for (int b = threadIdx.x; b < ncb; b += blockDim.x) {
    loff[b] = 0;
    gb[b] = gbase[(size_t)b * ntiles + blockIdx.x];
  }
  __syncthreads();
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t key[HT], val[HT], rk[HT];
  if (i < n) {
    ches_entries<HT>(scalars + i * stride, stride, i, q_exp, code, rank, nb0, small, copies, key, val);
  } else {
#pragma unroll
    for (int j = 0; j < HT; ++j) key[j] = KEY_NONE, val[j] = 0;
  }
#pragma unroll
  for (int j = 0; j < HT; ++j) rk[j] = key[j] != KEY_NONE ? atomicAdd(&loff[key[j] >> fb_bits], 1u) : 0u;
  __syncthreads();
  const uint32_t total = block_exclusive_scan_256(loff, ncb, wsum);
#pragma unroll
  for (int j = 0; j < HT; ++j) {
    if (key[j] == KEY_NONE) continue;
    const uint32_t pos = loff[key[j] >> fb_bits] + rk[j];
    sk[pos] = key[j];
    sv[pos] = val[j];
  }
  __syncthreads();
  for (uint32_t e = threadIdx.x; e < total; e += 256) {
    const uint32_t k = sk[e], b = k >> fb_bits;
    const uint32_t g = gb[b] + (e - loff[b]);
    okeys[g] = k;
    ovals[g] = sv[e];
  }
}

// ----------------------------------------------------------- BGMW95 digits --
// Signed radix-q digits in (-q/2, q/2] (ref auxiliaryfunc.h:130-145
// trans_uint256_t_to_qhalf_expr): d_j = bits [j q_exp, (j+1) q_exp) plus the
// carry; d_j > q/2 -> d_j - q, carry 1.  When the top digit would exceed q/2
// the scalar is replaced by r - s and every digit negated (the reference's
// "a > 0.5 q q^(h-1)" branch, main_p1.cpp:311-357, applied whenever it is
// needed).  One entry per nonzero digit: key = |d| - 1 (bucket of value |d|),
// val = table slot i h + j | sign << 31 (table T[i h + j] = q^j P_i).  Top-
// digit entries with bucket < small go to copy i % copies of their bucket
// (copy c >= 1 = nb0 + (c - 1) small + bucket), as in k_ches_digits.
__device__ __forceinline__ void r_minus(uint32_t s[8]) {
  int64_t br = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    int64_t d = (int64_t)FR_R32[k] - (int64_t)s[k] + br;
    s[k] = (uint32_t)d;
    br = d >> 32;
  }
}
static __global__ void __launch_bounds__(256)
    k_bgmw_digits(const uint8_t *__restrict__ scalars, size_t stride, size_t n, int q_exp, int h,
                  uint32_t *__restrict__ keys, uint32_t *__restrict__ vals, uint32_t nb0, uint32_t small,
                  uint32_t copies) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t *sp = scalars + i * stride;
  uint32_t s[10];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    s[k] = (stride & 3) == 0 ? reinterpret_cast<const uint32_t *>(sp)[k]
                             : (uint32_t)sp[4 * k] | ((uint32_t)sp[4 * k + 1] << 8) |
                                   ((uint32_t)sp[4 * k + 2] << 16) | ((uint32_t)sp[4 * k + 3] << 24);
  sub_r_if_ge(s);
  sub_r_if_ge(s);
  s[8] = s[9] = 0;
  const int32_t q = 1 << q_exp, qh = q >> 1;
  const uint32_t qmask = (uint32_t)q - 1u;
  auto digit = [&](int j) -> int32_t {
    int off = j * q_exp;
    int wi = off >> 5, sh = off & 31;
    uint32_t lo = wi < 10 ? s[wi] : 0u, hi = wi + 1 < 10 ? s[wi + 1] : 0u;
    return (int32_t)((uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & qmask);
  };
  // top digit after carries: > q/2 exactly when the carry-propagated value of
  // the top digit is; run the carry chain once to decide, then emit
  int32_t carry = 0;
  for (int j = 0; j < h - 1; ++j) carry = digit(j) + carry > qh ? 1 : 0;
  uint32_t neg = 0;
  if (digit(h - 1) + carry > qh) {
    r_minus(s);
    neg = 1u;
  }
  carry = 0;
  for (int j = 0; j < h; ++j) {
    int32_t d = digit(j) + carry;
    carry = 0;
    if (j < h - 1 && d > qh) {
      d -= q;
      carry = 1;
    }
    const size_t k = (size_t)j * n + i;
    if (d == 0) {
      keys[k] = KEY_NONE;
      continue;
    }
    uint32_t sign = (d < 0 ? 1u : 0u) ^ neg;
    uint32_t b = (uint32_t)(d < 0 ? -d : d) - 1u;
    if (j == h - 1 && b < small) {
      uint32_t c = (uint32_t)(i % copies);
      if (c) b = nb0 + (c - 1) * small + b;
    }
    keys[k] = b;
    vals[k] = (uint32_t)(i * (size_t)h + j) | (sign << 31);
  }
}

// ------------------------------------------------------------ segment sums --
// MSM_SEGSUM_PREFETCH=1 (A/B build knob): load the next operand before the
// current add (G1: 149 -> 218 VGPRs, 3 -> 2 waves per SIMD)
#ifndef MSM_SEGSUM_PREFETCH
#define MSM_SEGSUM_PREFETCH 0
#endif
// dst[t] = sum_{k in [starts[t], starts[t+1])} src[idx ? idx[k] : k]   (xyzz)
// for each of gridDim.y MSMs of a batch group: MSM blockIdx.y reads src +
// y src_stride and writes dst + y dst_stride (the same plan for every MSM)
template <int G>
__device__ __forceinline__ void segsum_one(const Xyzz<typename FieldOf<G>::F> *__restrict__ src,
                                           const uint32_t *__restrict__ idx, const uint32_t *__restrict__ starts,
                                           Xyzz<typename FieldOf<G>::F> *__restrict__ dst, size_t t) {
  typedef typename FieldOf<G>::F F;
  uint32_t lo = starts[t], hi = starts[t + 1];
  Xyzz<F> acc;
  if (lo == hi) {
    xyzz_set_inf(acc);
  } else {
    acc = ld16(&src[idx ? idx[lo] : lo]);
    // the next operand is loaded before the current add: its (random, L2-missing)
    // load overlaps ~3.5 k instructions of the add instead of stalling the lane
#if MSM_SEGSUM_PREFETCH
    Xyzz<F> nxt;
    if (lo + 1 < hi) nxt = ld16(&src[idx ? idx[lo + 1] : lo + 1]);
    for (uint32_t k = lo + 1; k < hi; ++k) {
      Xyzz<F> a = nxt;
      if (k + 1 < hi) nxt = ld16(&src[idx ? idx[k + 1] : k + 1]);
      xyzz_add(acc, a);
    }
#else
    for (uint32_t k = lo + 1; k < hi; ++k) {
      Xyzz<F> a = ld16(&src[idx ? idx[k] : k]);
      xyzz_add(acc, a);
    }
#endif
  }
  st16(&dst[t], acc);
}
template <int G>
static __global__ void __launch_bounds__(256)
    k_segsum(const Xyzz<typename FieldOf<G>::F> *__restrict__ src, const uint32_t *__restrict__ idx,
             const uint32_t *__restrict__ starts, Xyzz<typename FieldOf<G>::F> *__restrict__ dst, size_t nout,
             size_t src_stride, size_t dst_stride) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nout) return;
  segsum_one<G>(src + blockIdx.y * src_stride, idx, starts, dst + blockIdx.y * dst_stride, t);
}

// Accumulation of MSM k and level 0 of MSM k - 1 in ONE grid (the G1 batch,
// Ches::run_jobs): the first l0_blocks workgroups are level-0 segment sums of
// the previous MSM's buckets (k_segsum), the rest the accumulation of this
// one (k_accumulate).  Level 0 alone (~3.7 k waves at 2^20) fills the chip's
// 3 x 1024 wave slots 1.2 rounds deep and ran at ~0.7 of the issue rate on the
// batch's critical path; inside the accumulation's grid its waves share the
// dispatch with ~15 k accumulation waves and the last round's idle slots fill
// with accumulation work.  Registers: the larger of the two bodies (149), still
// 3 waves per SIMD.
template <class PT>
static __global__ void __launch_bounds__(256, MSM_ACC_WAVES)
    k_accumulate_l0(const AccSched S, const PT *__restrict__ pts, Xyzz<Fp> *__restrict__ buckets, size_t nbuckets,
                    const Xyzz<Fp> *__restrict__ l0src, const uint32_t *__restrict__ l0idx,
                    const uint32_t *__restrict__ l0starts, Xyzz<Fp> *__restrict__ l0dst, size_t l0out,
                    uint32_t l0blocks, int l0_last) {
  // l0_last: level-0 workgroups after the accumulation's instead of before
  const uint32_t nacc = gridDim.x - l0blocks;
  const bool l0 = l0_last ? blockIdx.x >= nacc : blockIdx.x < l0blocks;
  const uint32_t b = l0 ? (l0_last ? blockIdx.x - nacc : blockIdx.x) : (l0_last ? blockIdx.x : blockIdx.x - l0blocks);
  const size_t t = (size_t)b * blockDim.x + threadIdx.x;
  if (l0) {
    if (t < l0out) segsum_one<1>(l0src, l0idx, l0starts, l0dst, t);
  } else if (t < nbuckets) {
    accumulate_bucket<1>(S, pts, buckets, t);
  }
}

// ------------------------------------------------------- dense scan reduce --
// suffix-scan step within each window of S: out[k] = in[k] + in[k + d] (k + d < S)
template <int G>
static __global__ void __launch_bounds__(64)
    k_suffix_step(const Xyzz<typename FieldOf<G>::F> *__restrict__ in, Xyzz<typename FieldOf<G>::F> *__restrict__ out,
                  int S, int d, int W) {
  typedef typename FieldOf<G>::F F;
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (size_t)W * S) return;
  int k = (int)(t % (size_t)S);
  Xyzz<F> a = ld16(&in[t]);
  if (k + d < S) {
    Xyzz<F> b = ld16(&in[t + d]);
    xyzz_add(a, b);
  }
  st16(&out[t], a);
}
// pairwise tree step: out[w*(S/2) + k] = in[w*S + 2k] + in[w*S + 2k + 1]
template <int G>
static __global__ void __launch_bounds__(64)
    k_pair_step(const Xyzz<typename FieldOf<G>::F> *__restrict__ in, Xyzz<typename FieldOf<G>::F> *__restrict__ out,
                size_t nout) {
  typedef typename FieldOf<G>::F F;
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nout) return;
  Xyzz<F> a = ld16(&in[2 * t]);
  Xyzz<F> b = ld16(&in[2 * t + 1]);
  xyzz_add(a, b);
  st16(&out[t], a);
}

// 4-waves-per-add forms of the tail steps (latency): coop.hpp

// blst xyzz {x, y, zzz, zz} (Montgomery R=2^384) -> internal xyzz
template <int G>
__global__ void __launch_bounds__(256) k_import_xyzz(const uint64_t *__restrict__ in, Xyzz<typename FieldOf<G>::F> *__restrict__ out,
                              size_t n) {
  typedef typename FieldOf<G>::F F;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t *p = in + i * 24 * G;
  Xyzz<F> a;
  f_from_blst(a.x, p);
  f_from_blst(a.y, p + 6 * G);
  f_from_blst(a.zzz, p + 12 * G);
  f_from_blst(a.zz, p + 18 * G);
  st16(&out[i], a);
}

}  // namespace msm

namespace msm {
// internal xyzz -> blst xyzz {x, y, zzz, zz} (Montgomery R=2^384, canonical);
// infinity -> all zero
template <int G>
__global__ void __launch_bounds__(256) k_export_xyzz(const Xyzz<typename FieldOf<G>::F> *__restrict__ in, uint64_t *__restrict__ out,
                              size_t n) {
  typedef typename FieldOf<G>::F F;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Xyzz<F> a = ld16(&in[i]);
  uint64_t *o = out + i * 24 * G;
  if (xyzz_is_inf(a)) {
    for (int k = 0; k < 24 * G; ++k) o[k] = 0;
    return;
  }
  f_to_blst(o, a.x);
  f_to_blst(o + 6 * G, a.y);
  f_to_blst(o + 12 * G, a.zzz);
  f_to_blst(o + 18 * G, a.zz);
}
}  // namespace msm
