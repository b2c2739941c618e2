/*
 * dropin_caller.c -- a reference-side caller of the MSM entry points, linked
 * against the GPU drop-in (oracle/Makefile target `dropin`: the reference's
 * libblst with every symbol libmsm_mi355x.so exports localized, so these calls
 * bind to the GPU library).  Test infrastructure only.
 *
 * It issues exactly the call sequences of the reference's C++ binding
 * (bindings/blst.hpp) -- restated in C because blst.hpp does not compile
 * against this fork's blst.h (it uses blst_expand_message_xmd,
 * blst_pairing_as_fp12, ... whose declarations the fork's headers lack):
 *   mult_flat : P1_Affines::mult_pippenger(const P1_Affine[], ...)     blst.hpp:451-467
 *               scratch = new limb_t[scratch_sizeof/8]; {ptr, NULL}; nbits 255
 *   mult_ptrs : P1_Affines::mult_pippenger(const P1_Affine* const[], ...) blst.hpp:451-461
 *   wbits     : P1_Affines(wbits, ptrs, n) then .mult(scalars, 255)       blst.hpp:368-375, 417-424
 *               (table of n << (wbits-1) affine rows, blst_p1s_mult_wbits_precompute,
 *                blst_p1s_mult_wbits with scratch_sizeof(n) scratch)
 *   add       : P1_Affines::add(const P1_Affine[], n)                    blst.hpp:473-484
 * and, as the checker for `add`, the same sum by the reference's CPU point
 * addition (blst_p{1,2}_add_or_double_affine: not an MSM symbol, stays in libblst).
 *
 *   dropin_caller <group> <n> <seed> <wbits>   -> one JSON line
 * Points P_i = 2^(i+1) G (ref main_p1.cpp:52-66); scalars SplitMix64(seed) (SURVEY 8c').
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bindings/blst.h"

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
static void gen_scalars(byte *out, size_t n, uint64_t seed) {
  uint64_t st = seed;
  for (size_t i = 0; i < n; ++i) {
    uint64_t a[4];
    do {
      for (int k = 0; k < 4; ++k) a[k] = sm_next(&st);
      a[3] >>= 1;
    } while (!lt_r(a));
    blst_scalar s;
    blst_scalar_from_uint64(&s, a);
    memcpy(out + 32 * i, s.b, 32);
  }
}
static void phex(const char *key, const byte *b, size_t n, int last) {
  printf("\"%s\": \"", key);
  for (size_t i = 0; i < n; ++i) printf("%02x", b[i]);
  printf("\"%s", last ? "" : ", ");
}

/* one group's worth of the blst.hpp sequences; G = 1 or 2 selects the types */
#define DEFINE_RUN(g)                                                                                   \
  static void run_p##g(size_t n, uint64_t seed, size_t wbits) {                                        \
    blst_p##g##_affine *pts = malloc(n * sizeof *pts);                                                  \
    byte *sc = malloc(32 * n), out[96];                                                                 \
    blst_p##g acc = *blst_p##g##_generator(), r;                                                        \
    for (size_t i = 0; i < n; ++i) {                                                                    \
      blst_p##g##_double(&acc, &acc);                                                                   \
      blst_p##g##_to_affine(&pts[i], &acc);                                                             \
    }                                                                                                   \
    gen_scalars(sc, n, seed);                                                                           \
    const byte *sflat[2] = {sc, NULL};                                                                  \
    const blst_p##g##_affine *pflat[2] = {pts, NULL};                                                   \
    const blst_p##g##_affine **pptr = malloc(n * sizeof *pptr);                                         \
    const byte **sptr = malloc(n * sizeof *sptr);                                                       \
    for (size_t i = 0; i < n; ++i) pptr[i] = &pts[i], sptr[i] = sc + 32 * i;                            \
    printf("{\"group\": %d, \"n\": %zu, \"seed\": %llu, \"wbits\": %zu, ", g, n,                       \
           (unsigned long long)seed, wbits);                                                            \
    limb_t *scratch = malloc(blst_p##g##s_mult_pippenger_scratch_sizeof(n));                            \
    blst_p##g##s_mult_pippenger(&r, pflat, n, sflat, 255, scratch);                                     \
    blst_p##g##_compress(out, &r);                                                                      \
    phex("mult_flat", out, 48 * g, 0);                                                                  \
    blst_p##g##s_mult_pippenger(&r, pptr, n, sptr, 255, scratch);                                       \
    blst_p##g##_compress(out, &r);                                                                      \
    phex("mult_ptrs", out, 48 * g, 0);                                                                  \
    free(scratch);                                                                                      \
    blst_p##g##_affine *table = malloc(blst_p##g##s_mult_wbits_precompute_sizeof(wbits, n));            \
    blst_p##g##s_mult_wbits_precompute(table, wbits, pptr, n);                                          \
    scratch = malloc(blst_p##g##s_mult_wbits_scratch_sizeof(n));                                        \
    blst_p##g##s_mult_wbits(&r, table, wbits, n, sflat, 255, scratch);                                  \
    blst_p##g##_compress(out, &r);                                                                      \
    phex("mult_wbits", out, 48 * g, 0);                                                                 \
    free(scratch);                                                                                      \
    free(table);                                                                                        \
    blst_p##g##s_add(&r, pflat, n);                                                                     \
    blst_p##g##_compress(out, &r);                                                                      \
    phex("add", out, 48 * g, 0);                                                                        \
    memset(&acc, 0, sizeof acc);                                                                        \
    for (size_t i = 0; i < n; ++i) blst_p##g##_add_or_double_affine(&acc, &acc, &pts[i]);               \
    blst_p##g##_compress(out, &acc);                                                                    \
    phex("add_cpu", out, 48 * g, 1);                                                                    \
    printf("}\n");                                                                                      \
    free(pts), free(sc), free(pptr), free(sptr);                                                        \
  }
DEFINE_RUN(1)
DEFINE_RUN(2)

int main(int argc, char **argv) {
  const int group = argc > 1 ? atoi(argv[1]) : 1;
  const size_t n = argc > 2 ? strtoull(argv[2], NULL, 10) : 1024;
  const uint64_t seed = argc > 3 ? strtoull(argv[3], NULL, 10) : 1;
  const size_t wbits = argc > 4 ? strtoull(argv[4], NULL, 10) : 5;
  if (group == 2) run_p2(n, seed, wbits);
  else run_p1(n, seed, wbits);
  return 0;
}
