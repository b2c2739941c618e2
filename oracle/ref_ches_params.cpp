// ref_ches_params.cpp -- golden harness for the CHES bucket set and MB digit
// conversion of the REFERENCE's auxiliaryfunc.h under one parameter file
// (compiled per config by oracle/Makefile with -DCFG=<config header>).
//
// Prints JSON: |B|, FNV-1a of B, first/last 16 values of B, FNV-1a of the
// digit hash table (filled as main_p1.cpp:140-152 does), and the MB digits
// (auxiliaryfunc.h:92-118) and q/2 digits (auxiliaryfunc.h:130-145) of the
// first 4 SplitMix64(seed=1) scalars.  Test infrastructure only.
#include <array>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <random>
#include <set>

#include "bindings/blst.h"
#include CFG
digit_decomposition *DIGIT_CONVERSION_HASH_TABLE;
#include "auxiliaryfunc.h"

static uint64_t sm_next(uint64_t *s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static uint64_t fnv(const void *p, size_t len) {
  const uint8_t *b = (const uint8_t *)p;
  uint64_t h = 1469598103934665603ULL;
  for (size_t i = 0; i < len; ++i) { h ^= b[i]; h *= 1099511628211ULL; }
  return h;
}

int main() {
  static int B[B_SIZE + 64];
  construct_bucket_set(B, q_RADIX, a_LEADING_TERM);
  DIGIT_CONVERSION_HASH_TABLE = new digit_decomposition[q_RADIX + 1]();
  std::set<int> MS = {1, 2, 3};
  for (int m : MS)
    for (int i = 0; i < B_SIZE; ++i) {
      int b = B[i];
      if (m * b <= q_RADIX) DIGIT_CONVERSION_HASH_TABLE[q_RADIX - m * b] = {m, b, 1};
    }
  for (int m : MS)
    for (int i = 0; i < B_SIZE; ++i) {
      int b = B[i];
      if (m * b <= q_RADIX) DIGIT_CONVERSION_HASH_TABLE[m * b] = {m, b, 0};
    }
  printf("{\"n_exp\": %d, \"q_exp\": %d, \"h\": %d, \"a_h\": %d, \"d_max\": %d, \"b_size\": %d,\n", N_EXP,
         EXPONENT_OF_q, h_LEN_SCALAR, a_LEADING_TERM, d_MAX_DIFF, B_SIZE);
  printf("\"q_exp_bgmw\": %d, \"h_bgmw\": %d,\n", EXPONENT_OF_q_BGMW95, h_BGMW95);
  printf("\"fnv_bucket_set\": \"%016llx\",\n", (unsigned long long)fnv(B, sizeof(int) * B_SIZE));
  int maxgap = 0;
  for (int i = 1; i < B_SIZE; ++i) if (B[i] - B[i - 1] > maxgap) maxgap = B[i] - B[i - 1];
  printf("\"max_gap\": %d,\n\"head\": [", maxgap);
  for (int i = 0; i < 16; ++i) printf("%s%d", i ? "," : "", B[i]);
  printf("], \"tail\": [");
  for (int i = B_SIZE - 16; i < B_SIZE; ++i) printf("%s%d", i > B_SIZE - 16 ? "," : "", B[i]);
  printf("],\n\"fnv_digit_table\": \"%016llx\",\n",
         (unsigned long long)fnv(DIGIT_CONVERSION_HASH_TABLE, sizeof(digit_decomposition) * (q_RADIX + 1)));
  uint64_t st = 1;
  printf("\"scalars\": [");
  std::array<uint256_t, 4> sc;
  for (int i = 0; i < 4; ++i) {
    uint64_t a[4];
    do {
      for (int k = 0; k < 4; ++k) a[k] = sm_next(&st);
      a[3] >>= 1;
    } while (!(uint256_t(a[0], a[1], a[2], a[3]) < r_GROUP_ORDER));
    sc[i] = uint256_t(a[0], a[1], a[2], a[3]);
    printf("%s\"%016llx%016llx%016llx%016llx\"", i ? "," : "", (unsigned long long)a[3], (unsigned long long)a[2],
           (unsigned long long)a[1], (unsigned long long)a[0]);
  }
  printf("],\n\"mb_digits\": [");
  for (int i = 0; i < 4; ++i) {
    scalar_MB_expr e;
    trans_uint256_t_to_MB_radixq_expr(e, sc[i]);
    printf("%s[", i ? "," : "");
    for (int j = 0; j < h_LEN_SCALAR; ++j) printf("%s[%d,%d]", j ? "," : "", e[j][0], e[j][1]);
    printf("]");
  }
  printf("],\n\"qhalf_digits\": [");
  for (int i = 0; i < 4; ++i) {
    std::array<int, h_BGMW95> e;
    trans_uint256_t_to_qhalf_expr(e, sc[i]);
    printf("%s[", i ? "," : "");
    for (int j = 0; j < h_BGMW95; ++j) printf("%s%d", j ? "," : "", e[j]);
    printf("]");
  }
  printf("]}\n");
  return 0;
}
