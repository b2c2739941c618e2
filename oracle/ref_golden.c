/*
 * ref_golden.c -- golden-vector generator that links the REFERENCE library
 * (libblst built from /root/reference/src/server.c + build/assembly.S by
 * oracle/Makefile into oracle/_ref/).  Runs only in the build container;
 * its output is committed as tests/golden/*.json by
 * tests/golden/make_golden.py.  This file is our own harness code; it only
 * calls the reference's public C ABI (bindings/blst.h).
 *
 * Usage: ref_golden <mode> [args]
 *   msm  <group 1|2> <n> <seed> <nbits> [case]   -> compressed MSM result (hex)
 *   fpkat <count> <seed>                         -> Fp mul/add/sub vectors
 *   xyzz <count>                                 -> xyzz madd/add sequences (raw limbs)
 * case: "rand" (default), "zero" (all-zero scalars), "ones" (2^nbits-1),
 *       "rminus1" (r-1), "equal" (all points P_0, equal scalars),
 *       "negpairs" (P_0,-P_0,P_1,-P_1,... equal scalars), "ptr" (pointer arrays)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "blst.h"

static uint64_t sm_next(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static const uint64_t R_[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                               0x73eda753299d7d48ULL};
static int lt_r(const uint64_t a[4]) {
  for (int i = 3; i >= 0; --i) {
    if (a[i] < R_[i]) return 1;
    if (a[i] > R_[i]) return 0;
  }
  return 0;
}
/* same generator as BASELINE.md section 3 / oracle or_gen_scalars */
static void gen_scalars(blst_scalar *out, size_t n, uint64_t seed) {
  uint64_t st = seed;
  for (size_t i = 0; i < n; ++i) {
    uint64_t a[4];
    do {
      for (int k = 0; k < 4; ++k) a[k] = sm_next(&st);
      a[3] >>= 1;
    } while (!lt_r(a));
    blst_scalar_from_uint64(&out[i], a);
  }
}
static void hex(const uint8_t *b, size_t n) {
  for (size_t i = 0; i < n; ++i) printf("%02x", b[i]);
}
static void hex_limbs(const uint64_t *l, size_t n) { /* little-endian limbs as 16-hex each, limb 0 first */
  for (size_t i = 0; i < n; ++i) printf("%016llx", (unsigned long long)l[i]);
}

static int do_msm(int group, size_t n, uint64_t seed, size_t nbits, const char *cas) {
  size_t nbytes = (nbits + 7) / 8;
  blst_scalar *sc32 = (blst_scalar *)calloc(n, sizeof(blst_scalar));
  gen_scalars(sc32, n, seed);
  uint8_t *sc = (uint8_t *)calloc(n, nbytes);
  for (size_t i = 0; i < n; ++i) {
    if (!strcmp(cas, "zero")) memset(sc32[i].b, 0, 32);
    if (!strcmp(cas, "ones")) { memset(sc32[i].b, 0xff, 32); if (nbits % 8) sc32[i].b[nbits / 8] &= (uint8_t)((1u << (nbits % 8)) - 1); }
    if (!strcmp(cas, "rminus1")) { uint64_t a[4] = {R_[0] - 1, R_[1], R_[2], R_[3]}; blst_scalar_from_uint64(&sc32[i], a); }
    if (!strcmp(cas, "equal") || !strcmp(cas, "negpairs")) sc32[i] = sc32[0];
    memcpy(sc + i * nbytes, sc32[i].b, nbytes);   /* flat, stride nbytes (multi_scalar.c:395) */
  }
  const uint8_t *sptr[2] = {sc, NULL};
  const uint8_t **sptrs = NULL;
  if (!strcmp(cas, "ptr")) {
    sptrs = (const uint8_t **)malloc(sizeof(uint8_t *) * n);
    for (size_t i = 0; i < n; ++i) sptrs[i] = sc32[i].b;
  }
  if (group == 1) {
    blst_p1_affine *pts = (blst_p1_affine *)calloc(n, sizeof(blst_p1_affine));
    blst_p1 cur = *blst_p1_generator();
    for (size_t i = 0; i < n; ++i) { blst_p1_double(&cur, &cur); blst_p1_to_affine(&pts[i], &cur); }
    if (!strcmp(cas, "equal")) for (size_t i = 1; i < n; ++i) pts[i] = pts[0];
    if (!strcmp(cas, "negpairs"))
      for (size_t i = 1; i < n; i += 2) { blst_p1 t; blst_p1_from_affine(&t, &pts[i - 1]); blst_p1_cneg(&t, 1); blst_p1_to_affine(&pts[i], &t); }
    const blst_p1_affine *pptr[2] = {pts, NULL};
    const blst_p1_affine **pptrs = NULL;
    if (sptrs) { pptrs = (const blst_p1_affine **)malloc(sizeof(void *) * n); for (size_t i = 0; i < n; ++i) pptrs[i] = &pts[i]; }
    limb_t *scratch = (limb_t *)malloc(blst_p1s_mult_pippenger_scratch_sizeof(n));
    blst_p1 ret;
    if (sptrs) blst_p1s_mult_pippenger(&ret, pptrs, n, sptrs, nbits, scratch);
    else blst_p1s_mult_pippenger(&ret, pptr, n, sptr, nbits, scratch);
    uint8_t out[48];
    blst_p1_compress(out, &ret);
    hex(out, 48); printf("\n");
    free(scratch); free(pts); free(pptrs);
  } else {
    blst_p2_affine *pts = (blst_p2_affine *)calloc(n, sizeof(blst_p2_affine));
    blst_p2 cur = *blst_p2_generator();
    for (size_t i = 0; i < n; ++i) { blst_p2_double(&cur, &cur); blst_p2_to_affine(&pts[i], &cur); }
    if (!strcmp(cas, "equal")) for (size_t i = 1; i < n; ++i) pts[i] = pts[0];
    if (!strcmp(cas, "negpairs"))
      for (size_t i = 1; i < n; i += 2) { blst_p2 t; blst_p2_from_affine(&t, &pts[i - 1]); blst_p2_cneg(&t, 1); blst_p2_to_affine(&pts[i], &t); }
    const blst_p2_affine *pptr[2] = {pts, NULL};
    const blst_p2_affine **pptrs = NULL;
    if (sptrs) { pptrs = (const blst_p2_affine **)malloc(sizeof(void *) * n); for (size_t i = 0; i < n; ++i) pptrs[i] = &pts[i]; }
    limb_t *scratch = (limb_t *)malloc(blst_p2s_mult_pippenger_scratch_sizeof(n));
    blst_p2 ret;
    if (sptrs) blst_p2s_mult_pippenger(&ret, pptrs, n, sptrs, nbits, scratch);
    else blst_p2s_mult_pippenger(&ret, pptr, n, sptr, nbits, scratch);
    uint8_t out[96];
    blst_p2_compress(out, &ret);
    hex(out, 96); printf("\n");
    free(scratch); free(pts); free(pptrs);
  }
  free(sc); free(sc32); free(sptrs);
  return 0;
}

static const uint64_t P_[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL, 0x6730d2a0f6b0f624ULL,
                               0x64774b84f38512bfULL, 0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
static void rand_fp(blst_fp *r, uint64_t *st) {
  for (;;) {
    for (int i = 0; i < 6; ++i) r->l[i] = sm_next(st);
    r->l[5] &= 0x1fffffffffffffffULL;
    int lt = 0;
    for (int i = 5; i >= 0; --i) { if (r->l[i] < P_[i]) { lt = 1; break; } if (r->l[i] > P_[i]) break; }
    if (lt) return;
  }
}
static int do_fpkat(int count, uint64_t seed) {
  uint64_t st = seed;
  for (int k = 0; k < count; ++k) {
    blst_fp a, b, m, ad, sb;
    rand_fp(&a, &st); rand_fp(&b, &st);
    if (k == 0) memset(&b, 0, sizeof(b));
    if (k == 1) { a.l[0] = P_[0] - 1; for (int i = 1; i < 6; ++i) a.l[i] = P_[i]; b = a; }
    blst_fp_mul(&m, &a, &b); blst_fp_add(&ad, &a, &b); blst_fp_sub(&sb, &a, &b);
    hex_limbs(a.l, 6); printf(" "); hex_limbs(b.l, 6); printf(" "); hex_limbs(m.l, 6); printf(" ");
    hex_limbs(ad.l, 6); printf(" "); hex_limbs(sb.l, 6); printf("\n");
  }
  return 0;
}

/* xyzz sequences: ops = list of (point index, sign); doubling/cancel/inf branches are forced */
static int do_xyzz(int count) {
  size_t n = 8;
  blst_p1_affine pts[8];
  blst_p1 cur = *blst_p1_generator();
  for (size_t i = 0; i < n; ++i) { blst_p1_double(&cur, &cur); blst_p1_to_affine(&pts[i], &cur); }
  uint64_t st = 99;
  for (int c = 0; c < count; ++c) {
    blst_p1xyzz acc; memset(&acc, 0, sizeof(acc));
    int len = 2 + (int)(sm_next(&st) % 6);
    printf("ops");
    for (int k = 0; k < len; ++k) {
      int idx = (int)(sm_next(&st) % 3), sg = (int)(sm_next(&st) % 2);
      if (c == 0) { idx = 0; sg = 0; }                 /* P0+P0 -> doubling branch */
      if (c == 1) { idx = 0; sg = k & 1; }             /* P0-P0 -> infinity branch */
      if (c == 2) { idx = 0; sg = 1; }                 /* -P0-P0 -> doubling of negated */
      blst_p1xyzz_dadd_affine(&acc, &acc, &pts[idx], (unsigned char)sg);
      printf(" %d:%d", idx, sg);
    }
    blst_p1xyzz acc2; memset(&acc2, 0, sizeof(acc2));
    blst_p1xyzz_dadd(&acc2, &acc2, &acc);
    blst_p1xyzz_dadd(&acc2, &acc2, &acc);   /* 2*acc via the xyzz+xyzz doubling branch */
    blst_p1 j, j2;
    blst_p1xyzz_to_Jacobian(&j, &acc);
    blst_p1xyzz_to_Jacobian(&j2, &acc2);
    uint8_t o1[48], o2[48];
    blst_p1_compress(o1, &j); blst_p1_compress(o2, &j2);
    printf(" | "); hex_limbs(acc.x.l, 6); printf(" "); hex_limbs(acc.y.l, 6); printf(" "); hex_limbs(acc.zzz.l, 6);
    printf(" "); hex_limbs(acc.zz.l, 6); printf(" | "); hex(o1, 48); printf(" "); hex(o2, 48); printf("\n");
  }
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) { fprintf(stderr, "usage\n"); return 2; }
  if (!strcmp(argv[1], "msm") && argc >= 6)
    return do_msm(atoi(argv[2]), (size_t)strtoull(argv[3], 0, 0), strtoull(argv[4], 0, 0),
                  (size_t)strtoull(argv[5], 0, 0), argc > 6 ? argv[6] : "rand");
  if (!strcmp(argv[1], "fpkat") && argc >= 4) return do_fpkat(atoi(argv[2]), strtoull(argv[3], 0, 0));
  if (!strcmp(argv[1], "xyzz") && argc >= 3) return do_xyzz(atoi(argv[2]));
  fprintf(stderr, "bad args\n");
  return 2;
}
