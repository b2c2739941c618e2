// host_fp.hpp -- host-side BLS12-381 field/curve helpers for the engine's
// boundary work only: blst-layout (6x64 LE, Montgomery R=2^384) values,
// the one inversion per MSM (to_affine, ref e1.c:60-92 / recip.c:58-92),
// ZCash compression (ref e1.c:190-234, e2.c:228-260), the Horner combine of
// the per-window sums (ref multi_scalar.c:565-575: window doublings), and
// generation of the fixed input points P_i = 2^(i+1) G (main_p1.cpp:52-66).
// The MSM itself never runs here.
#pragma once
#include <stdint.h>
#include <string.h>

#include <vector>

namespace hfp {

typedef unsigned __int128 u128;

struct Fp {
  uint64_t l[6];
};
struct Fp2 {
  Fp c[2];
};

static const uint64_t P[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                              0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const uint64_t N0 = 0x89f3fffcfffcfffdULL;

inline bool geq_p(const uint64_t a[6]) {
  for (int i = 5; i >= 0; --i) {
    if (a[i] != P[i]) return a[i] > P[i];
  }
  return true;
}
inline void sub_p(uint64_t a[6]) {
  uint64_t br = 0;
  for (int i = 0; i < 6; ++i) {
    u128 x = (u128)a[i] - P[i] - br;
    a[i] = (uint64_t)x;
    br = (uint64_t)(x >> 64) & 1;
  }
}
inline Fp mul(const Fp &a, const Fp &b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 6; ++i) {
    u128 c = 0;
    for (int j = 0; j < 6; ++j) {
      c = (u128)a.l[j] * b.l[i] + t[j] + (uint64_t)(c >> 64);
      t[j] = (uint64_t)c;
    }
    u128 s = (u128)t[6] + (uint64_t)(c >> 64);
    t[6] = (uint64_t)s;
    t[7] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * N0;
    c = (u128)m * P[0] + t[0];
    for (int j = 1; j < 6; ++j) {
      c = (u128)m * P[j] + t[j] + (uint64_t)(c >> 64);
      t[j - 1] = (uint64_t)c;
    }
    s = (u128)t[6] + (uint64_t)(c >> 64);
    t[5] = (uint64_t)s;
    t[6] = t[7] + (uint64_t)(s >> 64);
  }
  if (t[6] || geq_p(t)) sub_p(t);
  Fp r;
  memcpy(r.l, t, 48);
  return r;
}
inline Fp add(const Fp &a, const Fp &b) {
  Fp r;
  uint64_t c = 0;
  for (int i = 0; i < 6; ++i) {
    u128 x = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (uint64_t)x;
    c = (uint64_t)(x >> 64);
  }
  if (c || geq_p(r.l)) sub_p(r.l);
  return r;
}
inline Fp sub(const Fp &a, const Fp &b) {
  Fp r;
  uint64_t br = 0;
  for (int i = 0; i < 6; ++i) {
    u128 x = (u128)a.l[i] - b.l[i] - br;
    r.l[i] = (uint64_t)x;
    br = (uint64_t)(x >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; ++i) {
      u128 x = (u128)r.l[i] + P[i] + c;
      r.l[i] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
  }
  return r;
}
inline bool is_zero(const Fp &a) {
  uint64_t o = 0;
  for (int i = 0; i < 6; ++i) o |= a.l[i];
  return o == 0;
}
inline Fp zero() {
  Fp r;
  memset(&r, 0, sizeof r);
  return r;
}
inline Fp one() {  // 2^384 mod p
  static Fp o = [] {
    Fp t = zero();
    t.l[0] = 1;
    for (int i = 0; i < 384; ++i) t = add(t, t);
    return t;
  }();
  return o;
}
inline Fp rr() {  // 2^768 mod p
  static Fp o = [] {
    Fp t = one();
    for (int i = 0; i < 384; ++i) t = add(t, t);
    return t;
  }();
  return o;
}
inline Fp to_mont(const Fp &a) { return mul(a, rr()); }
inline Fp from_mont(const Fp &a) {
  Fp o = zero();
  o.l[0] = 1;
  return mul(a, o);
}
inline Fp neg(const Fp &a) { return is_zero(a) ? a : sub(zero(), a); }
inline Fp inv(const Fp &a) {  // Fermat a^(p-2)
  uint64_t e[6];
  memcpy(e, P, 48);
  e[0] -= 2;
  Fp acc = one();
  for (int i = 5; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      acc = mul(acc, acc);
      if ((e[i] >> b) & 1) acc = mul(acc, a);
    }
  return acc;
}

// ---- Fp2 ----
inline Fp2 add(const Fp2 &a, const Fp2 &b) { return Fp2{{add(a.c[0], b.c[0]), add(a.c[1], b.c[1])}}; }
inline Fp2 sub(const Fp2 &a, const Fp2 &b) { return Fp2{{sub(a.c[0], b.c[0]), sub(a.c[1], b.c[1])}}; }
inline Fp2 mul(const Fp2 &a, const Fp2 &b) {
  Fp t0 = mul(a.c[0], b.c[0]), t1 = mul(a.c[1], b.c[1]);
  Fp t2 = mul(add(a.c[0], a.c[1]), add(b.c[0], b.c[1]));
  return Fp2{{sub(t0, t1), sub(sub(t2, t0), t1)}};
}
inline bool is_zero(const Fp2 &a) { return is_zero(a.c[0]) && is_zero(a.c[1]); }
inline Fp2 inv(const Fp2 &a) {
  Fp n = add(mul(a.c[0], a.c[0]), mul(a.c[1], a.c[1]));
  Fp ni = inv(n);
  return Fp2{{mul(a.c[0], ni), neg(mul(a.c[1], ni))}};
}
inline Fp2 zero2() { return Fp2{{zero(), zero()}}; }
inline Fp2 one2() { return Fp2{{one(), zero()}}; }
inline Fp2 neg(const Fp2 &a) { return Fp2{{neg(a.c[0]), neg(a.c[1])}}; }

inline Fp fzero(Fp) { return zero(); }
inline Fp2 fzero(Fp2) { return zero2(); }
inline Fp fone(Fp) { return one(); }
inline Fp2 fone(Fp2) { return one2(); }

// ---- Jacobian points (layout of blst_p1 / blst_p2) ----
template <class F>
struct Jac {
  F x, y, z;
};
template <class F>
struct Aff {
  F x, y;
};

template <class F>
Jac<F> dbl(const Jac<F> &a) {  // dbl-2009-l (ref ec_ops.h:299-327)
  if (is_zero(a.z)) return a;
  F A = mul(a.x, a.x), B = mul(a.y, a.y), C = mul(B, B);
  F t = add(a.x, B);
  t = sub(sub(mul(t, t), A), C);
  F D = add(t, t);
  F E = add(add(A, A), A);
  F Fv = mul(E, E);
  Jac<F> o;
  o.x = sub(sub(Fv, D), D);
  o.z = mul(add(a.z, a.z), a.y);
  F C8 = add(C, C);
  C8 = add(C8, C8);
  C8 = add(C8, C8);
  o.y = sub(mul(sub(D, o.x), E), C8);
  return o;
}
template <class F>
Jac<F> addj(const Jac<F> &a, const Jac<F> &b) {  // general add, doubling/infinity aware
  if (is_zero(a.z)) return b;
  if (is_zero(b.z)) return a;
  F z1z1 = mul(a.z, a.z), z2z2 = mul(b.z, b.z);
  F u1 = mul(a.x, z2z2), u2 = mul(b.x, z1z1);
  F s1 = mul(mul(a.y, b.z), z2z2), s2 = mul(mul(b.y, a.z), z1z1);
  F h = sub(u2, u1), r = sub(s2, s1);
  if (is_zero(h)) {
    if (is_zero(r)) return dbl(a);
    Jac<F> o;
    o.x = fzero(F());
    o.y = fzero(F());
    o.z = fzero(F());
    return o;
  }
  F hh = mul(h, h), hhh = mul(hh, h), v = mul(u1, hh);
  Jac<F> o;
  o.x = sub(sub(sub(mul(r, r), hhh), v), v);
  o.y = sub(mul(sub(v, o.x), r), mul(s1, hhh));
  o.z = mul(mul(a.z, b.z), h);
  return o;
}
template <class F>
Aff<F> to_affine(const Jac<F> &a) {
  Aff<F> r;
  if (is_zero(a.z)) {
    r.x = fzero(F());
    r.y = fzero(F());
    return r;
  }
  F zi = inv(a.z), zi2 = mul(zi, zi), zi3 = mul(zi2, zi);
  r.x = mul(a.x, zi2);
  r.y = mul(a.y, zi3);
  return r;
}
// batch affine with one inversion
template <class F>
void to_affine_batch(Aff<F> *out, const Jac<F> *in, size_t n) {
  std::vector<F> pre(n);
  F acc = fone(F());
  for (size_t i = 0; i < n; ++i) {
    pre[i] = acc;
    if (!is_zero(in[i].z)) acc = mul(acc, in[i].z);
  }
  F iv = inv(acc);
  for (size_t i = n; i-- > 0;) {
    if (is_zero(in[i].z)) {
      out[i].x = fzero(F());
      out[i].y = fzero(F());
      continue;
    }
    F zi = mul(iv, pre[i]);
    iv = mul(iv, in[i].z);
    F zi2 = mul(zi, zi), zi3 = mul(zi2, zi);
    out[i].x = mul(in[i].x, zi2);
    out[i].y = mul(in[i].y, zi3);
  }
}

// ---- xyzz points (layout of blst_p1xyzz / blst_p2xyzz: x, y, zzz, zz) ----
// Host restatements of the single-point bucket helpers the reference exports
// (ref src/ec_ops.h:642-785, multi_scalar.c:609-641).  They serve the per-point
// blst_p*xyzz_* boundary functions only; bucket accumulation runs on the GPU.
template <class F>
struct Xyzz {
  F x, y, zzz, zz;
};
template <class F>
bool xyzz_is_inf(const Xyzz<F> &a) {
  return is_zero(a.zzz) && is_zero(a.zz);
}
// mdbl-2008-s-1 of the affine point (x, y)
template <class F>
Xyzz<F> xyzz_dbl_aff(const F &x, const F &y) {
  Xyzz<F> r;
  F U = add(y, y);
  r.zz = mul(U, U);
  r.zzz = mul(r.zz, U);
  F S = mul(x, r.zz);
  F M = mul(x, x);
  M = add(add(M, M), M);
  r.x = sub(sub(mul(M, M), S), S);
  r.y = sub(mul(sub(S, r.x), M), mul(r.zzz, y));
  return r;
}
// p1 + (subtract ? -p2 : p2)   (ref ec_ops.h:710-769, madd-2008-s with twists)
template <class F>
Xyzz<F> xyzz_madd(const Xyzz<F> &p1, const Aff<F> &p2, bool subtract) {
  if (is_zero(p2.x) && is_zero(p2.y)) return p1;
  const F one = fone(F());
  if (xyzz_is_inf(p1)) {
    Xyzz<F> r{p2.x, p2.y, subtract ? neg(one) : one, one};
    return r;
  }
  F P = sub(mul(p2.x, p1.zz), p1.x);
  F R = mul(p2.y, p1.zzz);
  if (subtract) R = neg(R);
  R = sub(R, p1.y);
  Xyzz<F> r;
  if (!is_zero(P)) {
    F PP = mul(P, P), PPP = mul(PP, P), Q = mul(p1.x, PP);
    r.x = sub(sub(mul(R, R), PPP), add(Q, Q));
    r.y = sub(mul(sub(Q, r.x), R), mul(p1.y, PPP));
    r.zz = mul(p1.zz, PP);
    r.zzz = mul(p1.zzz, PPP);
  } else if (is_zero(R)) {
    r = xyzz_dbl_aff(p2.x, p2.y);
    if (subtract) r.zzz = neg(r.zzz);
  } else {
    r = Xyzz<F>{p1.x, p1.y, fzero(F()), fzero(F())};
  }
  return r;
}
// p1 + p2   (ref ec_ops.h:642-702, add-2008-s / dbl-2008-s-1)
template <class F>
Xyzz<F> xyzz_add(const Xyzz<F> &p1, const Xyzz<F> &p2) {
  if (xyzz_is_inf(p2)) return p1;
  if (xyzz_is_inf(p1)) return p2;
  F U1 = mul(p1.x, p2.zz), S1 = mul(p1.y, p2.zzz);
  F P = sub(mul(p2.x, p1.zz), U1), R = sub(mul(p2.y, p1.zzz), S1);
  Xyzz<F> r;
  if (!is_zero(P)) {
    F PP = mul(P, P), PPP = mul(PP, P), Q = mul(U1, PP);
    r.x = sub(sub(mul(R, R), PPP), add(Q, Q));
    r.y = sub(mul(sub(Q, r.x), R), mul(S1, PPP));
    r.zz = mul(mul(p1.zz, p2.zz), PP);
    r.zzz = mul(mul(p1.zzz, p2.zzz), PPP);
  } else if (is_zero(R)) {  // p1 == p2: dbl-2008-s-1
    F U = add(p1.y, p1.y), V = mul(U, U), W = mul(U, V), S = mul(p1.x, V);
    F M = mul(p1.x, p1.x);
    M = add(add(M, M), M);
    r.x = sub(sub(mul(M, M), S), S);
    r.y = sub(mul(sub(S, r.x), M), mul(W, p1.y));
    r.zz = mul(V, p1.zz);
    r.zzz = mul(W, p1.zzz);
  } else {
    r = Xyzz<F>{p1.x, p1.y, fzero(F()), fzero(F())};
  }
  return r;
}
template <class F>
Jac<F> xyzz_to_jac(const Xyzz<F> &a) {  // ref ec_ops.h:771-777
  return Jac<F>{mul(a.x, a.zz), mul(a.y, a.zzz), a.zz};
}
template <class F>
Xyzz<F> jac_to_xyzz(const Jac<F> &a) {  // ref ec_ops.h:779-785
  F zz = mul(a.z, a.z);
  return Xyzz<F>{a.x, a.y, mul(zz, a.z), zz};
}

inline void be48(uint8_t out[48], const Fp &n) {
  for (int i = 0; i < 48; ++i) out[i] = (uint8_t)(n.l[(47 - i) / 8] >> (8 * ((47 - i) % 8)));
}
inline bool lexi_large(const Fp &n) {  // n > (p-1)/2 for canonical non-Montgomery n
  uint64_t t[6], c = 0;
  for (int i = 0; i < 6; ++i) {
    t[i] = (n.l[i] << 1) | c;
    c = n.l[i] >> 63;
  }
  return c || geq_p(t);
}
inline void compress(uint8_t out[48], const Aff<Fp> &a) {
  if (is_zero(a.x) && is_zero(a.y)) {
    memset(out, 0, 48);
    out[0] = 0xc0;
    return;
  }
  be48(out, from_mont(a.x));
  out[0] |= (uint8_t)(0x80 | (lexi_large(from_mont(a.y)) ? 0x20 : 0));
}
inline void compress(uint8_t out[96], const Aff<Fp2> &a) {
  if (is_zero(a.x) && is_zero(a.y)) {
    memset(out, 0, 96);
    out[0] = 0xc0;
    return;
  }
  be48(out, from_mont(a.x.c[1]));
  be48(out + 48, from_mont(a.x.c[0]));
  Fp y0 = from_mont(a.y.c[0]), y1 = from_mont(a.y.c[1]);
  bool s = is_zero(y1) ? lexi_large(y0) : lexi_large(y1);
  out[0] |= (uint8_t)(0x80 | (s ? 0x20 : 0));
}

inline Fp from_hex(const char *hex) {
  Fp r = zero();
  size_t L = strlen(hex);
  for (size_t k = 0; k < L; ++k) {
    char c = hex[L - 1 - k];
    uint64_t v = (c >= '0' && c <= '9') ? (uint64_t)(c - '0') : (uint64_t)((c | 32) - 'a' + 10);
    r.l[k / 16] |= v << (4 * (k % 16));
  }
  return r;
}
inline Jac<Fp> g1_generator() {
  Jac<Fp> g;
  g.x = to_mont(from_hex("17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb"));
  g.y = to_mont(from_hex("08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1"));
  g.z = one();
  return g;
}
inline Jac<Fp2> g2_generator() {
  Jac<Fp2> g;
  g.x.c[0] = to_mont(from_hex("024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8"));
  g.x.c[1] = to_mont(from_hex("13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"));
  g.y.c[0] = to_mont(from_hex("0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801"));
  g.y.c[1] = to_mont(from_hex("0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be"));
  g.z = one2();
  return g;
}

}  // namespace hfp
