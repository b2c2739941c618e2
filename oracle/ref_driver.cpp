// ref_driver.cpp -- golden harness around the REFERENCE's own n=2^10 G1 / G2
// drivers (main_p1.cpp / main_p2.cpp compiled where they lie, main() renamed;
// their config_file.h is config_file_n_exp_10.h: q=2^13, h=20, |B|=1725).
// -DGROUP=1 (default) or -DGROUP=2 selects the driver it is linked against.
//
// Calls the reference's init_fix_point_list / init_pippenger_CHES_q_over_5 /
// init_pippenger_BGMW95 and its four timed methods on SplitMix64-seeded
// scalars, and prints one JSON object with: the bucket set, the digit hash
// table, FNV-1a hashes of the fixed points and both precomputed tables, MB and
// q/2 digits of the first scalars, and the compressed result of every method
// for seeds 1..3 plus the crafted scalar that trips the CHES last-element
// guard (SURVEY 8a defect 1).  Test infrastructure only; output is committed
// as tests/golden/ches_driver_n10.json (G1) / ches_driver_p2_n10.json (G2) by
// tests/golden/make_golden.py.
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "bindings/blst.h"
#include "src_from_aztec/numeric/uint256/uint256.hpp"

#ifndef GROUP
#define GROUP 1
#endif
#if GROUP == 1
typedef blst_p1_affine Paff;
#define PAFF_COMPRESS blst_p1_affine_compress
#else
typedef blst_p2_affine Paff;
#define PAFF_COMPRESS blst_p2_affine_compress
#endif
constexpr int H = 20, HB = 22, Q = 1 << 13, N = 1 << 10, BSZ = 1725;

extern digit_decomposition *DIGIT_CONVERSION_HASH_TABLE;
extern int *BUCKET_SET;
extern Paff *FIX_POINTS_LIST;
extern Paff *PRECOMPUTATION_POINTS_LIST_3nh;
extern Paff *PRECOMPUTATION_POINTS_LIST_BGMW95;
void init_fix_point_list();
void init_pippenger_CHES_q_over_5();
void init_pippenger_BGMW95();
Paff pippenger_variant_q_over_5_CHES(uint256_t scalars_array[]);
Paff pippenger_variant_q_over_5_CHES_integral_scalar_conversion(uint256_t scalars_array[]);
Paff pippenger_variant_BGMW95(uint256_t scalars_array[]);
Paff pippenger_blst_built_in(uint256_t scalars_array[]);
void trans_uint256_t_to_MB_radixq_expr(std::array<std::array<int, 2>, H> &ret, const uint256_t &a);
void trans_uint256_t_to_qhalf_expr(std::array<int, HB> &ret, const uint256_t &a);

static uint64_t sm_next(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static const uint64_t R_[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL,
                               0x73eda753299d7d48ULL};
static bool lt_r(const uint64_t a[4]) {
  for (int i = 3; i >= 0; --i) {
    if (a[i] < R_[i]) return true;
    if (a[i] > R_[i]) return false;
  }
  return false;
}
static void gen(uint256_t *out, size_t n, uint64_t seed) {
  uint64_t st = seed;
  for (size_t i = 0; i < n; ++i) {
    uint64_t a[4];
    do {
      for (int k = 0; k < 4; ++k) a[k] = sm_next(&st);
      a[3] >>= 1;
    } while (!lt_r(a));
    out[i] = uint256_t(a[0], a[1], a[2], a[3]);
  }
}
static uint64_t fnv(const void *p, size_t len) {
  const uint8_t *b = (const uint8_t *)p;
  uint64_t h = 1469598103934665603ULL;
  for (size_t i = 0; i < len; ++i) { h ^= b[i]; h *= 1099511628211ULL; }
  return h;
}
static void phex(const uint8_t *b, size_t n) { for (size_t i = 0; i < n; ++i) printf("%02x", b[i]); }
static void pres(const char *k, const Paff &a) {
  uint8_t o[48 * GROUP];
  PAFF_COMPRESS(o, &a);
  printf("\"%s\": \"", k); phex(o, 48 * GROUP); printf("\"");
}

int main() {
  init_fix_point_list();
  init_pippenger_CHES_q_over_5();
  init_pippenger_BGMW95();
  printf("{\"group\": %d, \"n\": %d, \"q_exp\": 13, \"h\": %d, \"b_size\": %d, \"q_exp_bgmw\": 12, \"h_bgmw\": %d,\n", GROUP, N, H, BSZ, HB);
  printf("\"bucket_set\": [");
  for (int i = 0; i < BSZ; ++i) printf("%s%d", i ? "," : "", BUCKET_SET[i]);
  printf("],\n\"digit_table\": [");
  for (int v = 0; v <= Q; ++v) {
    digit_decomposition t = DIGIT_CONVERSION_HASH_TABLE[v];
    printf("%s[%d,%d,%d]", v ? "," : "", t.m, t.b, t.alpha);
  }
  printf("],\n");
  printf("\"fnv_fixed_points\": \"%016llx\",\n", (unsigned long long)fnv(FIX_POINTS_LIST, sizeof(Paff) * N));
  printf("\"fnv_table_3nh\": \"%016llx\",\n",
         (unsigned long long)fnv(PRECOMPUTATION_POINTS_LIST_3nh, sizeof(Paff) * 3 * N * H));
  printf("\"fnv_table_bgmw\": \"%016llx\",\n",
         (unsigned long long)fnv(PRECOMPUTATION_POINTS_LIST_BGMW95, sizeof(Paff) * N * HB));
  static uint256_t sc[N];
  printf("\"runs\": [\n");
  for (int seed = 1; seed <= 4; ++seed) {
    gen(sc, N, (uint64_t)seed);
    const char *label = "rand";
    if (seed == 4) {  // crafted: last scalar's q-ary digits h-3 and h-2 zeroed (bits 221..246)
      label = "ches_last_guard";
      uint64_t *d = sc[N - 1].data;
      for (int b = 13 * (H - 3); b < 13 * (H - 1); ++b) d[b / 64] &= ~(1ULL << (b % 64));
    }
    printf("{\"seed\": %d, \"case\": \"%s\", ", seed, label);
    pres("ches_q_over_5", pippenger_variant_q_over_5_CHES(sc)); printf(", ");
    pres("ches_integral", pippenger_variant_q_over_5_CHES_integral_scalar_conversion(sc)); printf(", ");
    pres("bgmw95", pippenger_variant_BGMW95(sc)); printf(", ");
    pres("pippenger", pippenger_blst_built_in(sc)); printf(", ");
    printf("\"mb_digits\": [");
    for (int i = 0; i < 4; ++i) {
      std::array<std::array<int, 2>, H> e;
      trans_uint256_t_to_MB_radixq_expr(e, sc[i == 3 ? N - 1 : i]);
      printf("%s[", i ? "," : "");
      for (int j = 0; j < H; ++j) printf("%s[%d,%d]", j ? "," : "", e[j][0], e[j][1]);
      printf("]");
    }
    printf("], \"qhalf_digits\": [");
    for (int i = 0; i < 4; ++i) {
      std::array<int, HB> e;
      trans_uint256_t_to_qhalf_expr(e, sc[i == 3 ? N - 1 : i]);
      printf("%s[", i ? "," : "");
      for (int j = 0; j < HB; ++j) printf("%s%d", j ? "," : "", e[j]);
      printf("]");
    }
    printf("]}%s\n", seed < 4 ? "," : "");
  }
  printf("]}\n");
  return 0;
}
