/*
 * msm_oracle.c -- plain-C restatement of the reference MSM hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see msm_oracle.h).  Written from the
 * reference's algorithm descriptions; every function cites the reference
 * file:line whose behaviour it restates.  Not constant-time, not optimised
 * beyond what keeps the CPU baseline honest (single-thread + a
 * points x windows threaded grid).
 */
#include "msm_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ */
/* Fp: BLS12-381 base field, 6 x 64-bit LE limbs, Montgomery R=2^384   */
/* (ref src/consts.c:10-15 p, consts.h:12 p0; src/no_asm.h:29-291)     */
/* ------------------------------------------------------------------ */

static const uint64_t FP_P[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                                 0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static const uint64_t FP_N0 = 0x89f3fffcfffcfffdULL; /* -p^-1 mod 2^64 */
/* group order r (ref src/consts.c:28-31, auxiliaryfunc.h:5-7) */
static const uint64_t FR_R[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                                 0x73eda753299d7d48ULL};

static or_fp FP_ONE;  /* R mod p */
static or_fp FP_RR;   /* R^2 mod p */
static int g_inited = 0;

static int geq_p(const uint64_t a[6]) {
  for (int i = 5; i >= 0; --i) {
    if (a[i] > FP_P[i]) return 1;
    if (a[i] < FP_P[i]) return 0;
  }
  return 1;
}
static void sub_p(uint64_t a[6]) {
  uint64_t br = 0;
  for (int i = 0; i < 6; ++i) {
    u128 x = (u128)a[i] - FP_P[i] - br;
    a[i] = (uint64_t)x;
    br = (uint64_t)(x >> 64) & 1;
  }
}
/* 2a mod p on canonical a */
static void dbl_mod(uint64_t a[6]) {
  uint64_t c = 0;
  for (int i = 0; i < 6; ++i) {
    uint64_t t = a[i];
    a[i] = (t << 1) | c;
    c = t >> 63;
  }
  if (c || geq_p(a)) sub_p(a);
}

static void init_consts(void) {
  if (g_inited) return;
  uint64_t t[6] = {1, 0, 0, 0, 0, 0};
  for (int i = 0; i < 768; ++i) {
    dbl_mod(t);
    if (i == 383) memcpy(FP_ONE.l, t, 48);
  }
  memcpy(FP_RR.l, t, 48);
  g_inited = 1;
}

/* CIOS Montgomery product; canonical output (no_asm.h:29-82 semantics) */
void or_fp_mul(or_fp *r, const or_fp *a, const or_fp *b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 6; ++i) {
    u128 c = 0;
    for (int j = 0; j < 6; ++j) {
      c = (u128)a->l[j] * b->l[i] + t[j] + (uint64_t)(c >> 64);
      t[j] = (uint64_t)c;
    }
    u128 s = (u128)t[6] + (uint64_t)(c >> 64);
    t[6] = (uint64_t)s;
    t[7] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * FP_N0;
    c = (u128)m * FP_P[0] + t[0];
    for (int j = 1; j < 6; ++j) {
      c = (u128)m * FP_P[j] + t[j] + (uint64_t)(c >> 64);
      t[j - 1] = (uint64_t)c;
    }
    s = (u128)t[6] + (uint64_t)(c >> 64);
    t[5] = (uint64_t)s;
    t[6] = t[7] + (uint64_t)(s >> 64);
  }
  if (t[6] || geq_p(t)) sub_p(t);
  memcpy(r->l, t, 48);
}
static void fp_sqr(or_fp *r, const or_fp *a) { or_fp_mul(r, a, a); }

void or_fp_add(or_fp *r, const or_fp *a, const or_fp *b) { /* no_asm.h:104-135 */
  uint64_t t[6], c = 0;
  for (int i = 0; i < 6; ++i) {
    u128 x = (u128)a->l[i] + b->l[i] + c;
    t[i] = (uint64_t)x;
    c = (uint64_t)(x >> 64);
  }
  if (c || geq_p(t)) sub_p(t);
  memcpy(r->l, t, 48);
}
void or_fp_sub(or_fp *r, const or_fp *a, const or_fp *b) { /* no_asm.h:137-169 */
  uint64_t t[6], br = 0;
  for (int i = 0; i < 6; ++i) {
    u128 x = (u128)a->l[i] - b->l[i] - br;
    t[i] = (uint64_t)x;
    br = (uint64_t)(x >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 6; ++i) {
      u128 x = (u128)t[i] + FP_P[i] + c;
      t[i] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
  }
  memcpy(r->l, t, 48);
}
static int fp_is_zero(const or_fp *a) {
  uint64_t o = 0;
  for (int i = 0; i < 6; ++i) o |= a->l[i];
  return o == 0;
}
static void fp_neg(or_fp *r, const or_fp *a) { /* cneg, no_asm.h:264-291 */
  if (fp_is_zero(a)) { memset(r, 0, 48); return; }
  or_fp z; memset(&z, 0, 48);
  or_fp_sub(r, &z, a);
}
static void fp_cneg(or_fp *r, const or_fp *a, int flag) {
  if (flag) fp_neg(r, a); else if (r != a) *r = *a;
}
static void fp_mul3(or_fp *r, const or_fp *a) { or_fp t; or_fp_add(&t, a, a); or_fp_add(r, &t, a); }
static void fp_set_one(or_fp *r) { init_consts(); *r = FP_ONE; }
static void fp_set_zero(or_fp *r) { memset(r, 0, 48); }

void or_fp_to_mont(or_fp *r, const or_fp *a) { init_consts(); or_fp_mul(r, a, &FP_RR); }
void or_fp_from_mont(or_fp *r, const or_fp *a) { or_fp one = {{1, 0, 0, 0, 0, 0}}; or_fp_mul(r, a, &one); }

/* a^(p-2) by left-to-right square-and-multiply (Fermat; ref recip.c:58-92 computes the same inverse) */
void or_fp_inv(or_fp *r, const or_fp *a) {
  uint64_t e[6];
  memcpy(e, FP_P, 48);
  e[0] -= 2;
  or_fp acc; fp_set_one(&acc);
  for (int i = 5; i >= 0; --i)
    for (int b = 63; b >= 0; --b) {
      fp_sqr(&acc, &acc);
      if ((e[i] >> b) & 1) or_fp_mul(&acc, &acc, a);
    }
  *r = acc;
}

/* ------------------------------------------------------------------ */
/* Fp2 = Fp[i]/(i^2+1)  (ref no_asm.h:566-579 Karatsuba, :638-688 sqr) */
/* ------------------------------------------------------------------ */
void or_fp2_mul(or_fp2 *r, const or_fp2 *a, const or_fp2 *b) {
  or_fp t0, t1, sa, sb, t2;
  or_fp_mul(&t0, &a->fp[0], &b->fp[0]);
  or_fp_mul(&t1, &a->fp[1], &b->fp[1]);
  or_fp_add(&sa, &a->fp[0], &a->fp[1]);
  or_fp_add(&sb, &b->fp[0], &b->fp[1]);
  or_fp_mul(&t2, &sa, &sb);
  or_fp_sub(&r->fp[0], &t0, &t1);
  or_fp_sub(&t2, &t2, &t0);
  or_fp_sub(&r->fp[1], &t2, &t1);
}
void or_fp2_sqr(or_fp2 *r, const or_fp2 *a) {
  or_fp s, d, m;
  or_fp_add(&s, &a->fp[0], &a->fp[1]);
  or_fp_sub(&d, &a->fp[0], &a->fp[1]);
  or_fp_mul(&m, &a->fp[0], &a->fp[1]);
  or_fp_mul(&r->fp[0], &s, &d);
  or_fp_add(&r->fp[1], &m, &m);
}
static void fp2_add(or_fp2 *r, const or_fp2 *a, const or_fp2 *b) {
  or_fp_add(&r->fp[0], &a->fp[0], &b->fp[0]); or_fp_add(&r->fp[1], &a->fp[1], &b->fp[1]);
}
static void fp2_sub(or_fp2 *r, const or_fp2 *a, const or_fp2 *b) {
  or_fp_sub(&r->fp[0], &a->fp[0], &b->fp[0]); or_fp_sub(&r->fp[1], &a->fp[1], &b->fp[1]);
}
static int fp2_is_zero(const or_fp2 *a) { return fp_is_zero(&a->fp[0]) && fp_is_zero(&a->fp[1]); }
static void fp2_cneg(or_fp2 *r, const or_fp2 *a, int flag) {
  fp_cneg(&r->fp[0], &a->fp[0], flag); fp_cneg(&r->fp[1], &a->fp[1], flag);
}
static void fp2_mul3(or_fp2 *r, const or_fp2 *a) { fp_mul3(&r->fp[0], &a->fp[0]); fp_mul3(&r->fp[1], &a->fp[1]); }
static void fp2_set_one(or_fp2 *r) { fp_set_one(&r->fp[0]); fp_set_zero(&r->fp[1]); }
static void fp2_set_zero(or_fp2 *r) { memset(r, 0, 96); }
static void fp2_inv(or_fp2 *r, const or_fp2 *a) {  /* (a0 - a1 i)/(a0^2 + a1^2) */
  or_fp n0, n1, n, ni;
  or_fp_mul(&n0, &a->fp[0], &a->fp[0]);
  or_fp_mul(&n1, &a->fp[1], &a->fp[1]);
  or_fp_add(&n, &n0, &n1);
  or_fp_inv(&ni, &n);
  or_fp_mul(&r->fp[0], &a->fp[0], &ni);
  or_fp t; or_fp_mul(&t, &a->fp[1], &ni);
  fp_neg(&r->fp[1], &t);
}
#define fp_mul or_fp_mul
#define fp_add or_fp_add
#define fp_sub or_fp_sub
#define fp_inv or_fp_inv
#define fp2_mul or_fp2_mul
#define fp2_sqr or_fp2_sqr

/* sign of a canonical (non-Montgomery) value: a > (p-1)/2  (ref no_asm.h:501-524) */
static int fp_lexi_large(const or_fp *a_norm) {
  uint64_t t[6], c = 0;
  for (int i = 0; i < 6; ++i) { t[i] = (a_norm->l[i] << 1) | c; c = a_norm->l[i] >> 63; }
  if (c) return 1;
  return geq_p(t);
}
static void be48(uint8_t out[48], const or_fp *a_norm) {
  for (int i = 0; i < 48; ++i) out[i] = (uint8_t)(a_norm->l[(47 - i) / 8] >> (8 * ((47 - i) % 8)));
}

/* ------------------------------------------------------------------ */
/* curve formulas, templated over the field (G1: Fp, G2: Fp2)          */
/* ------------------------------------------------------------------ */
#define DEFINE_CURVE(PT, F, FT)                                                                          \
  /* Jacobian doubling dbl-2009-l (ref ec_ops.h:299-327) */                                             \
  static void PT##_dbl(or_##PT *r, const or_##PT *a) {                                                  \
    FT A, B, C, D, E, Fv, t;                                                                             \
    if (F##_is_zero(&a->z)) { *r = *a; return; }                                                         \
    F##_sqr_(&A, &a->x); F##_sqr_(&B, &a->y); F##_sqr_(&C, &B);                                          \
    F##_add(&t, &a->x, &B); F##_sqr_(&t, &t); F##_sub(&t, &t, &A); F##_sub(&t, &t, &C);                 \
    F##_add(&D, &t, &t);                                                                                 \
    F##_mul3(&E, &A); F##_sqr_(&Fv, &E);                                                                 \
    or_##PT o;                                                                                           \
    F##_sub(&o.x, &Fv, &D); F##_sub(&o.x, &o.x, &D);                                                    \
    F##_add(&t, &a->z, &a->z); F##_mul(&o.z, &t, &a->y);                                                \
    F##_add(&C, &C, &C); F##_add(&C, &C, &C); F##_add(&C, &C, &C);                                      \
    F##_sub(&t, &D, &o.x); F##_mul(&t, &t, &E); F##_sub(&o.y, &t, &C);                                  \
    *r = o;                                                                                              \
  }                                                                                                      \
  /* general Jacobian addition, doubling/infinity aware (ref ec_ops.h:40-100 semantics) */               \
  static void PT##_add_j(or_##PT *r, const or_##PT *a, const or_##PT *b) {                              \
    if (F##_is_zero(&a->z)) { *r = *b; return; }                                                         \
    if (F##_is_zero(&b->z)) { *r = *a; return; }                                                         \
    FT z1z1, z2z2, u1, u2, s1, s2, h, rr, hh, hhh, v, t;                                                 \
    F##_sqr_(&z1z1, &a->z); F##_sqr_(&z2z2, &b->z);                                                      \
    F##_mul(&u1, &a->x, &z2z2); F##_mul(&u2, &b->x, &z1z1);                                              \
    F##_mul(&s1, &a->y, &b->z); F##_mul(&s1, &s1, &z2z2);                                                \
    F##_mul(&s2, &b->y, &a->z); F##_mul(&s2, &s2, &z1z1);                                                \
    F##_sub(&h, &u2, &u1); F##_sub(&rr, &s2, &s1);                                                       \
    if (F##_is_zero(&h)) {                                                                               \
      if (F##_is_zero(&rr)) { PT##_dbl(r, a); return; }                                                  \
      memset(r, 0, sizeof(*r)); return;                                                                  \
    }                                                                                                    \
    or_##PT o;                                                                                           \
    F##_sqr_(&hh, &h); F##_mul(&hhh, &hh, &h); F##_mul(&v, &u1, &hh);                                    \
    F##_sqr_(&o.x, &rr); F##_sub(&o.x, &o.x, &hhh); F##_sub(&o.x, &o.x, &v); F##_sub(&o.x, &o.x, &v);   \
    F##_sub(&t, &v, &o.x); F##_mul(&t, &t, &rr); F##_mul(&s1, &s1, &hhh); F##_sub(&o.y, &t, &s1);       \
    F##_mul(&o.z, &a->z, &b->z); F##_mul(&o.z, &o.z, &h);                                                \
    *r = o;                                                                                              \
  }                                                                                                      \
  /* xyzz + affine with sign (ref ec_ops.h:710-769, madd-2008-s / mdbl-2008-s-1) */                      \
  static void PT##xyzz_madd(or_##PT##xyzz *r, const or_##PT##xyzz *a, const or_##PT##_affine *p,        \
                            int subtract) {                                                              \
    if (F##_is_zero(&p->x) && F##_is_zero(&p->y)) { *r = *a; return; }                                   \
    if (F##_is_zero(&a->zzz) && F##_is_zero(&a->zz)) {                                                   \
      r->x = p->x; r->y = p->y; F##_set_one(&r->zzz); F##_cneg(&r->zzz, &r->zzz, subtract);              \
      F##_set_one(&r->zz); return;                                                                       \
    }                                                                                                    \
    FT P, R, y2;                                                                                         \
    F##_mul(&P, &p->x, &a->zz);                                                                          \
    F##_cneg(&y2, &p->y, subtract);                                                                      \
    F##_mul(&R, &y2, &a->zzz);                                                                           \
    F##_sub(&P, &P, &a->x); F##_sub(&R, &R, &a->y);                                                      \
    if (!F##_is_zero(&P)) {                                                                              \
      FT PP, PPP, Q, t; or_##PT##xyzz o;                                                                 \
      F##_sqr_(&PP, &P); F##_mul(&PPP, &PP, &P); F##_mul(&Q, &a->x, &PP);                                \
      F##_sqr_(&o.x, &R); F##_sub(&o.x, &o.x, &PPP); F##_add(&t, &Q, &Q); F##_sub(&o.x, &o.x, &t);       \
      F##_sub(&Q, &Q, &o.x); F##_mul(&Q, &Q, &R); F##_mul(&t, &a->y, &PPP); F##_sub(&o.y, &Q, &t);       \
      F##_mul(&o.zz, &a->zz, &PP); F##_mul(&o.zzz, &a->zzz, &PPP);                                       \
      *r = o;                                                                                            \
    } else if (F##_is_zero(&R)) {                                                                        \
      FT U, V, W, S, M, t; or_##PT##xyzz o;                                                              \
      F##_add(&U, &y2, &y2); F##_sqr_(&V, &U); F##_mul(&W, &V, &U); F##_mul(&S, &p->x, &V);              \
      F##_sqr_(&M, &p->x); F##_mul3(&M, &M); F##_sqr_(&o.x, &M); F##_add(&t, &S, &S);                    \
      F##_sub(&o.x, &o.x, &t); F##_mul(&t, &W, &y2); F##_sub(&S, &S, &o.x); F##_mul(&S, &S, &M);        \
      F##_sub(&o.y, &S, &t); o.zz = V; o.zzz = W;                                                        \
      *r = o;                                                                                            \
    } else {                                                                                             \
      *r = *a; F##_set_zero(&r->zzz); F##_set_zero(&r->zz);                                              \
    }                                                                                                    \
  }                                                                                                      \
  /* xyzz + xyzz (ref ec_ops.h:642-702, add-2008-s / dbl-2008-s-1) */                                    \
  static void PT##xyzz_add(or_##PT##xyzz *r, const or_##PT##xyzz *a, const or_##PT##xyzz *b) {          \
    if (F##_is_zero(&b->zzz) && F##_is_zero(&b->zz)) { *r = *a; return; }                                \
    if (F##_is_zero(&a->zzz) && F##_is_zero(&a->zz)) { *r = *b; return; }                                \
    FT U, S, P, R;                                                                                       \
    F##_mul(&U, &a->x, &b->zz); F##_mul(&S, &a->y, &b->zzz);                                             \
    F##_mul(&P, &b->x, &a->zz); F##_mul(&R, &b->y, &a->zzz);                                             \
    F##_sub(&P, &P, &U); F##_sub(&R, &R, &S);                                                            \
    if (!F##_is_zero(&P)) {                                                                              \
      FT PP, PPP, Q, t; or_##PT##xyzz o;                                                                 \
      F##_sqr_(&PP, &P); F##_mul(&PPP, &PP, &P); F##_mul(&Q, &U, &PP);                                   \
      F##_sqr_(&o.x, &R); F##_sub(&o.x, &o.x, &PPP); F##_add(&t, &Q, &Q); F##_sub(&o.x, &o.x, &t);       \
      F##_sub(&Q, &Q, &o.x); F##_mul(&Q, &Q, &R); F##_mul(&t, &S, &PPP); F##_sub(&o.y, &Q, &t);          \
      F##_mul(&o.zz, &a->zz, &b->zz); F##_mul(&o.zz, &o.zz, &PP);                                        \
      F##_mul(&o.zzz, &a->zzz, &b->zzz); F##_mul(&o.zzz, &o.zzz, &PPP);                                  \
      *r = o;                                                                                            \
    } else if (F##_is_zero(&R)) {                                                                        \
      FT V, W, M, t; or_##PT##xyzz o;                                                                    \
      F##_add(&U, &a->y, &a->y); F##_sqr_(&V, &U); F##_mul(&W, &V, &U); F##_mul(&S, &a->x, &V);          \
      F##_sqr_(&M, &a->x); F##_mul3(&M, &M); F##_sqr_(&o.x, &M); F##_add(&t, &S, &S);                    \
      F##_sub(&o.x, &o.x, &t); F##_mul(&t, &W, &a->y); F##_sub(&S, &S, &o.x); F##_mul(&S, &S, &M);      \
      F##_sub(&o.y, &S, &t); F##_mul(&o.zz, &a->zz, &V); F##_mul(&o.zzz, &a->zzz, &W);                   \
      *r = o;                                                                                            \
    } else {                                                                                             \
      *r = *a; F##_set_zero(&r->zzz); F##_set_zero(&r->zz);                                              \
    }                                                                                                    \
  }                                                                                                      \
  /* ref ec_ops.h:771-777 */                                                                             \
  static void PT##xyzz_to_j(or_##PT *r, const or_##PT##xyzz *a) {                                       \
    or_##PT o;                                                                                           \
    F##_mul(&o.x, &a->x, &a->zz); F##_mul(&o.y, &a->y, &a->zzz); o.z = a->zz;                           \
    *r = o;                                                                                              \
  }                                                                                                      \
  static void PT##_from_affine(or_##PT *r, const or_##PT##_affine *a) {                                 \
    r->x = a->x; r->y = a->y;                                                                            \
    if (F##_is_zero(&a->x) && F##_is_zero(&a->y)) F##_set_zero(&r->z); else F##_set_one(&r->z);          \
  }                                                                                                      \
  /* ref e1.c:60-92 */                                                                                   \
  static void PT##_to_aff(or_##PT##_affine *r, const or_##PT *a) {                                      \
    if (F##_is_zero(&a->z)) { memset(r, 0, sizeof(*r)); return; }                                        \
    FT zi, zi2, zi3;                                                                                     \
    F##_inv_(&zi, &a->z); F##_sqr_(&zi2, &zi); F##_mul(&zi3, &zi2, &zi);                                 \
    F##_mul(&r->x, &a->x, &zi2); F##_mul(&r->y, &a->y, &zi3);                                            \
  }                                                                                                      \
  /* batch affine with one inversion (Montgomery trick) */                                               \
  static void PT##s_to_aff(or_##PT##_affine *r, const or_##PT *a, size_t n) {                           \
    FT *pre = (FT *)malloc(sizeof(FT) * (n + 1));                                                        \
    FT acc; F##_set_one(&acc);                                                                           \
    for (size_t i = 0; i < n; ++i) {                                                                     \
      pre[i] = acc;                                                                                      \
      if (!F##_is_zero(&a[i].z)) F##_mul(&acc, &acc, &a[i].z);                                           \
    }                                                                                                    \
    FT inv; F##_inv_(&inv, &acc);                                                                        \
    for (size_t i = n; i-- > 0;) {                                                                       \
      if (F##_is_zero(&a[i].z)) { memset(&r[i], 0, sizeof(r[i])); continue; }                           \
      FT zi, zi2, zi3; F##_mul(&zi, &inv, &pre[i]); F##_mul(&inv, &inv, &a[i].z);                        \
      F##_sqr_(&zi2, &zi); F##_mul(&zi3, &zi2, &zi);                                                     \
      FT x, y; F##_mul(&x, &a[i].x, &zi2); F##_mul(&y, &a[i].y, &zi3); r[i].x = x; r[i].y = y;           \
    }                                                                                                    \
    free(pre);                                                                                           \
  }                                                                                                      \
  /* double-and-add over a LE byte scalar (used for naive MSM and tables) */                             \
  static void PT##_mult_(or_##PT *r, const or_##PT##_affine *p, const uint8_t *s, size_t nbits) {       \
    or_##PT acc, pj; memset(&acc, 0, sizeof(acc)); PT##_from_affine(&pj, p);                             \
    for (size_t b = nbits; b-- > 0;) {                                                                   \
      PT##_dbl(&acc, &acc);                                                                              \
      if ((s[b / 8] >> (b % 8)) & 1) PT##_add_j(&acc, &acc, &pj);                                        \
    }                                                                                                    \
    *r = acc;                                                                                            \
  }

#define fp_sqr_ fp_sqr
#define fp_inv_ or_fp_inv
#define fp2_sqr_ or_fp2_sqr
#define fp2_inv_ fp2_inv

DEFINE_CURVE(p1, fp, or_fp)
DEFINE_CURVE(p2, fp2, or_fp2)

/* exported wrappers */
void or_p1_to_affine(or_p1_affine *o, const or_p1 *i) { p1_to_aff(o, i); }
void or_p2_to_affine(or_p2_affine *o, const or_p2 *i) { p2_to_aff(o, i); }
void or_p1_add(or_p1 *r, const or_p1 *a, const or_p1 *b) { p1_add_j(r, a, b); }
void or_p2_add(or_p2 *r, const or_p2 *a, const or_p2 *b) { p2_add_j(r, a, b); }
void or_p1_double(or_p1 *r, const or_p1 *a) { p1_dbl(r, a); }
void or_p1_mult(or_p1 *r, const or_p1_affine *p, const uint8_t *s, size_t nbits) { p1_mult_(r, p, s, nbits); }
void or_p2_mult(or_p2 *r, const or_p2_affine *p, const uint8_t *s, size_t nbits) { p2_mult_(r, p, s, nbits); }
void or_p1xyzz_dadd_affine(or_p1xyzz *r, const or_p1xyzz *a, const or_p1_affine *p, int s) { p1xyzz_madd(r, a, p, s); }
void or_p1xyzz_dadd(or_p1xyzz *r, const or_p1xyzz *a, const or_p1xyzz *b) { p1xyzz_add(r, a, b); }
void or_p1xyzz_to_jacobian(or_p1 *r, const or_p1xyzz *a) { p1xyzz_to_j(r, a); }
void or_p2xyzz_dadd_affine(or_p2xyzz *r, const or_p2xyzz *a, const or_p2_affine *p, int s) { p2xyzz_madd(r, a, p, s); }
void or_p2xyzz_dadd(or_p2xyzz *r, const or_p2xyzz *a, const or_p2xyzz *b) { p2xyzz_add(r, a, b); }
void or_p2xyzz_to_jacobian(or_p2 *r, const or_p2xyzz *a) { p2xyzz_to_j(r, a); }

/* compressed ZCash encoding (ref e1.c:190-234, e2.c:228-260) */
void or_p1_affine_compress(uint8_t out[48], const or_p1_affine *a) {
  if (fp_is_zero(&a->x) && fp_is_zero(&a->y)) { memset(out, 0, 48); out[0] = 0xc0; return; }
  or_fp x, y;
  or_fp_from_mont(&x, &a->x); or_fp_from_mont(&y, &a->y);
  be48(out, &x);
  out[0] |= (uint8_t)(0x80 | (fp_lexi_large(&y) ? 0x20 : 0));
}
void or_p1_compress(uint8_t out[48], const or_p1 *p) {
  or_p1_affine a; p1_to_aff(&a, p);
  or_p1_affine_compress(out, &a);
}
void or_p2_affine_compress(uint8_t out[96], const or_p2_affine *a) {
  if (fp2_is_zero(&a->x) && fp2_is_zero(&a->y)) { memset(out, 0, 96); out[0] = 0xc0; return; }
  or_fp x0, x1, y0, y1;
  or_fp_from_mont(&x0, &a->x.fp[0]); or_fp_from_mont(&x1, &a->x.fp[1]);
  or_fp_from_mont(&y0, &a->y.fp[0]); or_fp_from_mont(&y1, &a->y.fp[1]);
  be48(out, &x1); be48(out + 48, &x0);
  int s = fp_is_zero(&y1) ? fp_lexi_large(&y0) : fp_lexi_large(&y1);
  out[0] |= (uint8_t)(0x80 | (s ? 0x20 : 0));
}
void or_p2_compress(uint8_t out[96], const or_p2 *p) {
  or_p2_affine a; p2_to_aff(&a, p);
  or_p2_affine_compress(out, &a);
}

/* ------------------------------------------------------------------ */
/* inputs                                                               */
/* ------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static int lt_r(const uint64_t a[4]) {
  for (int i = 3; i >= 0; --i) {
    if (a[i] < FR_R[i]) return 1;
    if (a[i] > FR_R[i]) return 0;
  }
  return 0;
}
/* 255-bit uniform scalars < r; distribution of auxiliaryfunc.h:178-207, seeded RNG per BASELINE.md */
void or_gen_scalars(uint8_t *out, size_t n, uint64_t seed) {
  uint64_t st = seed;
  for (size_t i = 0; i < n; ++i) {
    uint64_t a[4];
    do {
      for (int k = 0; k < 4; ++k) a[k] = splitmix64(&st);
      a[3] >>= 1;
    } while (!lt_r(a));
    for (int k = 0; k < 32; ++k) out[32 * i + k] = (uint8_t)(a[k / 8] >> (8 * (k % 8)));  /* exports.c:356-378 */
  }
}

static void hex_to_fp(or_fp *r, const char *hex) { /* big-endian hex, 96 chars */
  memset(r, 0, 48);
  size_t L = strlen(hex);
  for (size_t k = 0; k < L; ++k) {
    char c = hex[L - 1 - k];
    uint64_t v = (c >= '0' && c <= '9') ? (uint64_t)(c - '0') : (uint64_t)((c | 32) - 'a' + 10);
    r->l[k / 16] |= v << (4 * (k % 16));
  }
}
/* standard generators (the IETF/ZCash constants; ref e1.c:20-32, e2.c:23-47 hold them in Montgomery form) */
void or_p1_generator(or_p1 *g) {
  or_fp x, y;
  hex_to_fp(&x, "17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb");
  hex_to_fp(&y, "08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1");
  or_fp_to_mont(&g->x, &x); or_fp_to_mont(&g->y, &y); fp_set_one(&g->z);
}
void or_p2_generator(or_p2 *g) {
  or_fp t;
  hex_to_fp(&t, "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8");
  or_fp_to_mont(&g->x.fp[0], &t);
  hex_to_fp(&t, "13e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e");
  or_fp_to_mont(&g->x.fp[1], &t);
  hex_to_fp(&t, "0ce5d527727d6e118cc9cdc6da2e351aadfd9baa8cbdd3a76d429a695160d12c923ac9cc3baca289e193548608b82801");
  or_fp_to_mont(&g->y.fp[0], &t);
  hex_to_fp(&t, "0606c4a02ea734cc32acd2b02bc28b99cb3e287e85a763af267492ab572e99ab3f370d275cec1da1aaa9075ff05f79be");
  or_fp_to_mont(&g->y.fp[1], &t);
  fp2_set_one(&g->z);
}
/* P_i = 2^(i+1) G (ref main_p1.cpp:52-66) */
void or_p1_fixed_points(or_p1_affine *out, size_t n) {
  or_p1 *j = (or_p1 *)malloc(sizeof(or_p1) * n);
  or_p1 cur; or_p1_generator(&cur);
  for (size_t i = 0; i < n; ++i) { p1_dbl(&cur, &cur); j[i] = cur; }
  p1s_to_aff(out, j, n);
  free(j);
}
void or_p2_fixed_points(or_p2_affine *out, size_t n) {
  or_p2 *j = (or_p2 *)malloc(sizeof(or_p2) * n);
  or_p2 cur; or_p2_generator(&cur);
  for (size_t i = 0; i < n; ++i) { p2_dbl(&cur, &cur); j[i] = cur; }
  p2s_to_aff(out, j, n);
  free(j);
}

/* ------------------------------------------------------------------ */
/* MSM: naive, and the blst Pippenger schedule                          */
/* ------------------------------------------------------------------ */
void or_p1s_mult_naive(or_p1 *r, const or_p1_affine *pts, size_t n, const uint8_t *sc, size_t nbits) {
  size_t nb = (nbits + 7) / 8;
  or_p1 acc, t; memset(&acc, 0, sizeof(acc));
  for (size_t i = 0; i < n; ++i) { p1_mult_(&t, &pts[i], sc + nb * i, nbits); p1_add_j(&acc, &acc, &t); }
  *r = acc;
}
void or_p2s_mult_naive(or_p2 *r, const or_p2_affine *pts, size_t n, const uint8_t *sc, size_t nbits) {
  size_t nb = (nbits + 7) / 8;
  or_p2 acc, t; memset(&acc, 0, sizeof(acc));
  for (size_t i = 0; i < n; ++i) { p2_mult_(&t, &pts[i], sc + nb * i, nbits); p2_add_j(&acc, &acc, &t); }
  *r = acc;
}

/* window rule (ref multi_scalar.c:268-275) */
size_t or_pippenger_window(size_t n) {
  size_t w = 0;
  while (n >>= 1) ++w;
  return w > 12 ? w - 3 : (w > 4 ? w - 2 : (w ? 2 : 1));
}

/* bits [off, off+len) of a LE byte string of nbytes (bits past the string read 0) */
static uint32_t get_bits(const uint8_t *s, size_t nbytes, long off, size_t len) {
  uint32_t v = 0;
  for (size_t k = 0; k < len; ++k) {
    long b = off + (long)k;
    if (b < 0 || (size_t)(b / 8) >= nbytes) continue;
    v |= (uint32_t)((s[b / 8] >> (b % 8)) & 1) << k;
  }
  return v;
}

/* Signed Booth digit of the window [bit0, bit0+wbits) with lookback bit bit0-1
 * (ref ec_mult.h:23-55 get_wval_limb/booth_encode + multi_scalar.c:390-402);
 * the value is masked to wbits+1 bits, the sign bit sits at position cbits. */
static int booth_digit(const uint8_t *s, size_t nbytes, size_t bit0, size_t wbits, size_t cbits) {
  uint32_t v = get_bits(s, nbytes, (long)bit0 - 1, wbits + 1);
  uint32_t sign = (v >> cbits) & 1;
  int d = (int)((v + 1) >> 1);
  return sign ? d - (1 << cbits) : d;
}

#define DEFINE_PIPPENGER(PT)                                                                             \
  /* one window over all points + bucket integration (ref multi_scalar.c:281-297,347-356,383-419) */   \
  static void PT##_tile(or_##PT *ret, const or_##PT##_affine *pts, size_t n, const uint8_t *sc,         \
                        size_t nbits, or_##PT##xyzz *bk, size_t bit0, size_t wbits, size_t cbits) {     \
    size_t nb = (nbits + 7) / 8, nbk = (size_t)1 << (cbits - 1);                                        \
    memset(bk, 0, sizeof(*bk) * nbk);                                                                    \
    for (size_t i = 0; i < n; ++i) {                                                                     \
      int d = booth_digit(sc + nb * i, nb, bit0, wbits, cbits);                                          \
      if (d > 0) PT##xyzz_madd(&bk[d - 1], &bk[d - 1], &pts[i], 0);                                     \
      else if (d < 0) PT##xyzz_madd(&bk[-d - 1], &bk[-d - 1], &pts[i], 1);                              \
    }                                                                                                    \
    or_##PT##xyzz acc = bk[nbk - 1], sum = bk[nbk - 1];                                                  \
    for (size_t k = nbk - 1; k-- > 0;) { PT##xyzz_add(&acc, &acc, &bk[k]); PT##xyzz_add(&sum, &sum, &acc); } \
    PT##xyzz_to_j(ret, &sum);                                                                            \
  }                                                                                                      \
  /* full MSM, windows top-down (ref multi_scalar.c:549-576) */                                          \
  void or_##PT##s_mult_pippenger(or_##PT *r, const or_##PT##_affine *pts, size_t n, const uint8_t *sc,  \
                                 size_t nbits) {                                                         \
    size_t window = or_pippenger_window(n), bit0 = nbits, wbits, cbits;                                  \
    or_##PT##xyzz *bk = (or_##PT##xyzz *)malloc(sizeof(or_##PT##xyzz) << (window - 1));                 \
    or_##PT ret, tile; memset(&ret, 0, sizeof(ret));                                                     \
    wbits = nbits % window; cbits = wbits + 1;                                                           \
    while (bit0 -= wbits) {                                                                              \
      PT##_tile(&tile, pts, n, sc, nbits, bk, bit0, wbits, cbits);                                       \
      PT##_add_j(&ret, &ret, &tile);                                                                     \
      for (size_t i = 0; i < window; ++i) PT##_dbl(&ret, &ret);                                          \
      cbits = wbits = window;                                                                            \
    }                                                                                                    \
    PT##_tile(&tile, pts, n, sc, nbits, bk, 0, wbits, cbits);                                            \
    PT##_add_j(&ret, &ret, &tile);                                                                       \
    free(bk);                                                                                            \
    *r = ret;                                                                                            \
  }

DEFINE_PIPPENGER(p1)
DEFINE_PIPPENGER(p2)

/* threaded grid: tiles of (point range x window), combined per window row
 * (the decomposition of ref bindings/go/blst.go:1959-2198) */
typedef struct {
  const or_p1_affine *pts; const uint8_t *sc; size_t n0, n1, nbits, bit0, wbits, cbits; or_p1 out;
} p1_job;
typedef struct { p1_job *jobs; size_t njobs; size_t next; pthread_mutex_t mu; } p1_pool;
static void *p1_worker(void *arg) {
  p1_pool *pool = (p1_pool *)arg;
  or_p1xyzz *bk = NULL; size_t bk_cap = 0;
  for (;;) {
    pthread_mutex_lock(&pool->mu);
    size_t k = pool->next++;
    pthread_mutex_unlock(&pool->mu);
    if (k >= pool->njobs) break;
    p1_job *j = &pool->jobs[k];
    size_t need = (size_t)1 << (j->cbits - 1);
    if (need > bk_cap) { free(bk); bk = (or_p1xyzz *)malloc(sizeof(or_p1xyzz) * need); bk_cap = need; }
    size_t nb = (j->nbits + 7) / 8;
    p1_tile(&j->out, j->pts + j->n0, j->n1 - j->n0, j->sc + nb * j->n0, j->nbits, bk, j->bit0, j->wbits, j->cbits);
  }
  free(bk);
  return NULL;
}
void or_p1s_mult_pippenger_mt(or_p1 *r, const or_p1_affine *pts, size_t n, const uint8_t *sc, size_t nbits,
                              int nthreads) {
  if (nthreads < 1) nthreads = 1;
  size_t window = or_pippenger_window(n);
  size_t nwin = 0, wb = nbits % window, b0 = nbits;
  size_t wins_bit0[64], wins_wbits[64], wins_cbits[64];
  { size_t wbits = wb, cbits = wb + 1, bit0 = b0;
    while (bit0 -= wbits) { wins_bit0[nwin] = bit0; wins_wbits[nwin] = wbits; wins_cbits[nwin] = cbits; ++nwin; cbits = wbits = window; }
    wins_bit0[nwin] = 0; wins_wbits[nwin] = wbits; wins_cbits[nwin] = cbits; ++nwin; }
  size_t nx = ((size_t)nthreads + nwin - 1) / nwin;   /* point ranges per window row */
  if (nx > n) nx = n;
  if (nx < 1) nx = 1;
  size_t njobs = nx * nwin;
  p1_job *jobs = (p1_job *)calloc(njobs, sizeof(p1_job));
  for (size_t w = 0; w < nwin; ++w)
    for (size_t x = 0; x < nx; ++x) {
      p1_job *j = &jobs[w * nx + x];
      j->pts = pts; j->sc = sc; j->nbits = nbits;
      j->n0 = n * x / nx; j->n1 = n * (x + 1) / nx;
      j->bit0 = wins_bit0[w]; j->wbits = wins_wbits[w]; j->cbits = wins_cbits[w];
    }
  p1_pool pool = {jobs, njobs, 0, PTHREAD_MUTEX_INITIALIZER};
  pthread_t th[256];
  int nt = nthreads > 256 ? 256 : nthreads;
  for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, p1_worker, &pool);
  for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
  or_p1 ret; memset(&ret, 0, sizeof(ret));
  for (size_t w = 0; w < nwin; ++w) {
    or_p1 row; memset(&row, 0, sizeof(row));
    for (size_t x = 0; x < nx; ++x) p1_add_j(&row, &row, &jobs[w * nx + x].out);
    p1_add_j(&ret, &ret, &row);
    if (w + 1 < nwin) for (size_t i = 0; i < window; ++i) p1_dbl(&ret, &ret);
  }
  free(jobs);
  *r = ret;
}

/* ------------------------------------------------------------------ */
/* CHES "nh + q/5" (ref auxiliaryfunc.h, main_p1.cpp, multi_scalar.c)  */
/* ------------------------------------------------------------------ */
/* the 17 parameter files ches_config_files/config_file_n_exp_{8..21,16_beta,17_beta,20_beta}.h (values only) */
static const or_ches_params CHES_TABLE[] = {
  /* n_exp beta q_exp  h   a_h   d   |B|   q_bgmw h_bgmw */
  {8, 0, 12, 22, 7, 6, 857, 10, 26},         {9, 0, 13, 20, 231, 6, 1725, 11, 24},
  {10, 0, 13, 20, 231, 6, 1725, 12, 22},     {11, 0, 14, 19, 7, 6, 3417, 13, 20},
  {12, 0, 14, 19, 7, 6, 3417, 13, 20},       {13, 0, 16, 16, 29677, 6, 18343, 15, 17},
  {14, 0, 16, 16, 29677, 6, 18343, 15, 17},  {15, 0, 16, 16, 29677, 6, 18343, 16, 16},
  {16, 0, 19, 14, 231, 6, 109244, 17, 15},   {16, 1, 18, 15, 7, 6, 54618, 17, 15},
  {17, 0, 20, 13, 29677, 6, 220931, 17, 15}, {17, 1, 19, 14, 231, 6, 109244, 17, 15},
  {18, 0, 20, 13, 29677, 6, 220931, 19, 14}, {19, 0, 20, 13, 29677, 6, 220931, 20, 13},
  {20, 0, 22, 12, 7419, 6, 874437, 20, 13},  {20, 1, 20, 13, 29677, 6, 220931, 20, 13},
  {21, 0, 22, 12, 7419, 6, 874437, 22, 12},
};
int or_ches_params_for(int n_exp, int beta, or_ches_params *out) {
  for (size_t i = 0; i < sizeof(CHES_TABLE) / sizeof(CHES_TABLE[0]); ++i)
    if (CHES_TABLE[i].n_exp == n_exp && CHES_TABLE[i].beta == beta) { *out = CHES_TABLE[i]; return 0; }
  return -1;
}

static int omega2(int v) { int e = 0; while (v % 2 == 0) { v /= 2; ++e; } return e; }
static int omega3(int v) { int e = 0; while (v % 3 == 0) { v /= 3; ++e; } return e; }
static int even23(int v) { return ((omega2(v) + omega3(v)) % 2) == 0; }

/* ref auxiliaryfunc.h:257-288 (sequential erase semantics preserved) */
size_t or_ches_bucket_set(int *out, int q, int a_h) {
  size_t lim = (size_t)(q / 2) + 1;
  if ((size_t)a_h + 2 > lim) lim = (size_t)a_h + 2;
  uint8_t *in = (uint8_t *)calloc(lim, 1);
  in[0] = 1; in[1] = 1;
  for (int i = 2; i <= q / 2; ++i) if (even23(i)) in[i] = 1;
  for (int i = q / 4; i < q / 2; ++i) {
    int t = q - 2 * i;
    if (in[i] && t >= 0 && (size_t)t < lim && in[t]) in[t] = 0;
  }
  for (int i = q / 6; i < q / 4; ++i) {
    int t = q - 3 * i;
    if (in[i] && t >= 0 && (size_t)t < lim && in[t]) in[t] = 0;
  }
  for (int i = 1; i <= a_h + 1; ++i) if (even23(i)) in[i] = 1;
  size_t k = 0;
  for (size_t v = 0; v < lim; ++v) if (in[v]) { if (out) out[k] = (int)v; ++k; }
  free(in);
  return k;
}

/* ref main_p1.cpp:134-152: alpha=1 pass then alpha=0 pass, later writes win */
void or_ches_digit_table(or_digit *H, int *v2i, const int *B, size_t bsize, int q) {
  for (size_t i = 0; i < bsize; ++i) v2i[B[i]] = (int)i;
  for (int m = 1; m <= 3; ++m)
    for (size_t i = 0; i < bsize; ++i) {
      long mb = (long)m * B[i];
      if (mb <= q) { H[q - mb].m = m; H[q - mb].b = B[i]; H[q - mb].alpha = 1; }
    }
  for (int m = 1; m <= 3; ++m)
    for (size_t i = 0; i < bsize; ++i) {
      long mb = (long)m * B[i];
      if (mb <= q) { H[mb].m = m; H[mb].b = B[i]; H[mb].alpha = 0; }
    }
}

/* ref auxiliaryfunc.h:92-118 (std q-ary digits, then hash with carry) */
void or_ches_mb_digits(int *b, uint8_t *sign, int *m, const uint8_t *s32, const or_digit *H, int q_exp, int h) {
  int d[64];
  for (int j = 0; j < h; ++j) d[j] = (int)get_bits(s32, 32, (long)j * q_exp, (size_t)q_exp);
  d[h] = 0;
  for (int j = 0; j < h; ++j) {
    or_digit t = H[d[j]];
    b[j] = t.b; m[j] = t.m; sign[j] = (uint8_t)t.alpha;
    if (t.alpha) d[j + 1] += 1;
  }
}

#define DEFINE_CHES(PT, FT)                                                                              \
  /* T[3(i*h+j)+m-1] = m*q^j*P_i (ref main_p1.cpp:155-172) */                                            \
  void or_##PT##_ches_table(or_##PT##_affine *T, const or_##PT##_affine *P, size_t n, int q_exp, int h) { \
    size_t tot = 3 * n * (size_t)h;                                                                      \
    or_##PT *J = (or_##PT *)malloc(sizeof(or_##PT) * tot);                                               \
    for (size_t i = 0; i < n; ++i) {                                                                     \
      or_##PT Q; PT##_from_affine(&Q, &P[i]);                                                            \
      for (int j = 0; j < h; ++j) {                                                                      \
        size_t k = 3 * (i * (size_t)h + j);                                                              \
        J[k] = Q; PT##_dbl(&J[k + 1], &Q); PT##_add_j(&J[k + 2], &J[k + 1], &Q);                        \
        for (int e = 0; e < q_exp; ++e) PT##_dbl(&Q, &Q);                                                \
      }                                                                                                  \
    }                                                                                                    \
    PT##s_to_aff(T, J, tot);                                                                             \
    free(J);                                                                                             \
  }                                                                                                      \
  /* ref multi_scalar.c:301-321 */                                                                       \
  static void PT##_ches_reduce_(or_##PT *r, const or_##PT##xyzz *S, const int *B, size_t bsize, int d_max) { \
    or_##PT##xyzz tmp, tmp1, td[64];                                                                     \
    memset(&tmp, 0, sizeof(tmp)); memset(td, 0, sizeof(td[0]) * (size_t)(d_max + 1));                   \
    for (size_t i = bsize - 1; i > 0; --i) {                                                             \
      PT##xyzz_add(&tmp, &tmp, &S[i]);                                                                   \
      int df = B[i] - B[i - 1];                                                                          \
      PT##xyzz_add(&td[df], &td[df], &tmp);                                                              \
    }                                                                                                    \
    memset(&tmp, 0, sizeof(tmp)); memset(&tmp1, 0, sizeof(tmp1));                                       \
    for (int i = d_max; i > 0; --i) { PT##xyzz_add(&tmp, &tmp, &td[i]); PT##xyzz_add(&tmp1, &tmp1, &tmp); } \
    PT##xyzz_to_j(r, &tmp1);                                                                             \
  }                                                                                                      \
  /* digit conversion + accumulation (ref main_p1.cpp:192-246, multi_scalar.c:421-463; the  */           \
  /* last-element guard defect of :461 is NOT reproduced: this computes the true sum)        */           \
  void or_##PT##_ches_msm(or_##PT *r, const or_##PT##_affine *T, size_t n, const uint8_t *s32,           \
                          const or_digit *H, const int *v2i, const int *B, size_t bsize, int q_exp, int h, \
                          int d_max) {                                                                   \
    or_##PT##xyzz *bk = (or_##PT##xyzz *)calloc(bsize, sizeof(or_##PT##xyzz));                          \
    int bv[64], mv[64]; uint8_t sg[64];                                                                  \
    for (size_t i = 0; i < n; ++i) {                                                                     \
      or_ches_mb_digits(bv, sg, mv, s32 + 32 * i, H, q_exp, h);                                          \
      for (int j = 0; j < h; ++j) {                                                                      \
        int idx = v2i[bv[j]];                                                                            \
        if (idx) PT##xyzz_madd(&bk[idx], &bk[idx], &T[3 * (i * (size_t)h + j) + mv[j] - 1], sg[j]);     \
      }                                                                                                  \
    }                                                                                                    \
    PT##_ches_reduce_(r, bk, B, bsize, d_max);                                                           \
    free(bk);                                                                                            \
  }

DEFINE_CHES(p1, or_fp)
DEFINE_CHES(p2, or_fp2)

void or_p1_ches_reduce(or_p1 *r, const or_p1xyzz *S, const int *B, size_t bsize, int d_max) {
  p1_ches_reduce_(r, S, B, bsize, d_max);
}

/* ------------------------------------------------------------------ */
/* BGMW95 (ref auxiliaryfunc.h:130-145, main_p1.cpp:294-398)            */
/* ------------------------------------------------------------------ */
static void sub_from_r(uint8_t out[32], const uint8_t s[32]) {
  uint64_t a[4] = {0}, br = 0;
  for (int k = 0; k < 32; ++k) a[k / 8] |= (uint64_t)s[k] << (8 * (k % 8));
  for (int i = 0; i < 4; ++i) {
    u128 x = (u128)FR_R[i] - a[i] - br;
    a[i] = (uint64_t)x; br = (uint64_t)(x >> 64) & 1;
  }
  for (int k = 0; k < 32; ++k) out[k] = (uint8_t)(a[k / 8] >> (8 * (k % 8)));
}
static int qhalf_digits(int *d, const uint8_t *s, int q_exp, int h) {
  int q = 1 << q_exp;
  for (int j = 0; j < h; ++j) d[j] = (int)get_bits(s, 32, (long)j * q_exp, (size_t)q_exp);
  for (int j = 0; j < h - 1; ++j)
    if (d[j] > q / 2) { d[j] -= q; d[j + 1] += 1; }
  return d[h - 1] <= q / 2;
}
/* signed digits in (-q/2, q/2]; when the top digit would exceed q/2 the r-s
 * representation is used with every digit negated (main_p1.cpp:311-357) */
void or_bgmw_digits(int *d, const uint8_t *s32, int q_exp, int h) {
  if (qhalf_digits(d, s32, q_exp, h)) return;
  uint8_t t[32];
  sub_from_r(t, s32);
  qhalf_digits(d, t, q_exp, h);
  for (int j = 0; j < h; ++j) d[j] = -d[j];
}
#define DEFINE_BGMW(PT)                                                                                   \
  /* T[i*h+j] = q^j*P_i (ref main_p1.cpp:94-122) */                                                      \
  void or_##PT##_bgmw_table(or_##PT##_affine *T, const or_##PT##_affine *P, size_t n, int q_exp, int h) { \
    size_t tot = n * (size_t)h;                                                                          \
    or_##PT *J = (or_##PT *)malloc(sizeof(or_##PT) * tot);                                               \
    for (size_t i = 0; i < n; ++i) {                                                                     \
      or_##PT Q; PT##_from_affine(&Q, &P[i]);                                                            \
      for (int j = 0; j < h; ++j) {                                                                      \
        J[i * (size_t)h + j] = Q;                                                                        \
        for (int e = 0; e < q_exp; ++e) PT##_dbl(&Q, &Q);                                                \
      }                                                                                                  \
    }                                                                                                    \
    PT##s_to_aff(T, J, tot);                                                                             \
    free(J);                                                                                             \
  }                                                                                                      \
  /* ref multi_scalar.c:506-547 + integrate_buckets :281-297 */                                          \
  void or_##PT##_bgmw_msm(or_##PT *r, const or_##PT##_affine *T, size_t n, const uint8_t *s32, int q_exp, int h) { \
    size_t nbk = (size_t)1 << (q_exp - 1);                                                               \
    or_##PT##xyzz *bk = (or_##PT##xyzz *)calloc(nbk, sizeof(or_##PT##xyzz));                             \
    int d[64];                                                                                           \
    for (size_t i = 0; i < n; ++i) {                                                                     \
      or_bgmw_digits(d, s32 + 32 * i, q_exp, h);                                                         \
      for (int j = 0; j < h; ++j) {                                                                      \
        if (d[j] > 0) PT##xyzz_madd(&bk[d[j] - 1], &bk[d[j] - 1], &T[i * (size_t)h + j], 0);            \
        else if (d[j] < 0) PT##xyzz_madd(&bk[-d[j] - 1], &bk[-d[j] - 1], &T[i * (size_t)h + j], 1);     \
      }                                                                                                  \
    }                                                                                                    \
    or_##PT##xyzz acc = bk[nbk - 1], sum = bk[nbk - 1];                                                  \
    for (size_t k = nbk - 1; k-- > 0;) { PT##xyzz_add(&acc, &acc, &bk[k]); PT##xyzz_add(&sum, &sum, &acc); } \
    PT##xyzz_to_j(r, &sum);                                                                              \
    free(bk);                                                                                            \
  }

DEFINE_BGMW(p1)
DEFINE_BGMW(p2)
