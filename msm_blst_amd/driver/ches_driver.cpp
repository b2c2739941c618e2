// ches_driver.cpp -- the reference's CHES / BGMW95 / Pippenger driver
// (ref main_p1.cpp, main_p2.cpp) rebuilt on libmsm_mi355x.so.  Compiled once
// per group (-DMSM_DRIVER_GROUP=1 -> msm_driver_p1, =2 -> msm_driver_p2), as
// the reference builds main_test_p1 / main_test_p2 (ref makefile:7-13).
//
//   ./msm_driver_p1 config=20 [beta=0] [device=0] [tests=5] [loops=N] [host_tables=0]
//                  [gpus=N | devices=d0,d1,...]
//
// gpus= / devices= shard the CHES method's points over several devices of this
// process (msm_ches_ctx_create_multi; devices may repeat): each shard uses the
// reference configuration of its size, config - ceil(log2(shards)) (2^21 points
// over 8 devices: config_file_n_exp_18.h per shard, BASELINE configs[3]); the
// other three methods stay on `device`.
//
// mirrors `./run.sh group=1 config=20` (ref run.sh:1-42): builds the fixed
// points, the CHES and BGMW95 tables (on the GPU), then test_pippengers().  The
// last stdout line is a JSON record of the mean per-method times and results.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "msm_ches_driver.hpp"

#if MSM_DRIVER_GROUP == 1
typedef blst_p1 jac_t;
#define DRV(name) msm_p1_##name
#define BLST_MULT blst_p1s_mult_pippenger
#define BLST_SCRATCH blst_p1s_mult_pippenger_scratch_sizeof
#else
typedef blst_p2 jac_t;
#define DRV(name) msm_p2_##name
#define BLST_MULT blst_p2s_mult_pippenger
#define BLST_SCRATCH blst_p2s_mult_pippenger_scratch_sizeof
#endif
static const int GROUP = MSM_DRIVER_GROUP;

int N_EXP = 0;
size_t N_POINTS = 0;
int q_RADIX_EXP = 0, h_LEN_SCALAR = 0, a_LEADING_TERM = 0, B_SIZE = 0, EXPONENT_OF_q_BGMW95 = 0, h_BGMW95 = 0;
digit_decomposition *DIGIT_CONVERSION_HASH_TABLE = nullptr;
int *BUCKET_SET = nullptr;
int *BUCKET_VALUE_TO_ITS_INDEX = nullptr;
msm_driver_affine *FIX_POINTS_LIST = nullptr;
msm_driver_affine *PRECOMPUTATION_POINTS_LIST_3nh = nullptr;
msm_driver_affine *PRECOMPUTATION_POINTS_LIST_BGMW95 = nullptr;

static int g_beta = 0, g_device = 0, g_host_tables = 0;
static std::vector<int> g_devices;  // CHES shards (empty: one shard on g_device)
static msm_ches_ctx *g_ches = nullptr;
static msm_bgmw_ctx *g_bgmw = nullptr;

static void check(int rc, const char *what) {
  if (rc != MSM_OK) {
    fprintf(stderr, "msm_driver: %s failed (%d): %s\n", what, rc, msm_last_error());
    exit(2);
  }
}

int msm_driver_configure(int n_exp, int beta, int device, int host_tables) {
  int p[9];
  int rc = msm_ches_params(n_exp, beta, p);
  if (rc != MSM_OK) return rc;
  N_EXP = n_exp;
  N_POINTS = (size_t)1 << n_exp;
  q_RADIX_EXP = p[2];
  h_LEN_SCALAR = p[3];
  a_LEADING_TERM = p[4];
  B_SIZE = p[6];
  EXPONENT_OF_q_BGMW95 = p[7];
  h_BGMW95 = p[8];
  g_beta = beta;
  g_device = device;
  g_host_tables = host_tables;
  return MSM_OK;
}

void init_fix_point_list() {
  FIX_POINTS_LIST = new msm_driver_affine[N_POINTS];
  DRV(fixed_points)(FIX_POINTS_LIST, N_POINTS);  // P_i = 2^(i+1) G
  printf("FIX_POINTS_LIST Generated\n");
}
void free_init_fix_point_list() {
  delete[] FIX_POINTS_LIST;
  FIX_POINTS_LIST = nullptr;
}

void init_pippenger_CHES_q_over_5() {
  const int q = 1 << q_RADIX_EXP;
  BUCKET_SET = new int[B_SIZE];
  if ((int)msm_ches_bucket_set(q, a_LEADING_TERM, BUCKET_SET, (size_t)B_SIZE) != B_SIZE) check(MSM_E_ARG, "bucket set");
  printf("BUCKET_SET constructed. The size of BUCKET_SET is: %d\n", B_SIZE);
  BUCKET_VALUE_TO_ITS_INDEX = new int[q / 2 + 1]();
  for (int i = 0; i < B_SIZE; ++i) BUCKET_VALUE_TO_ITS_INDEX[BUCKET_SET[i]] = i;
  DIGIT_CONVERSION_HASH_TABLE = new digit_decomposition[(size_t)q + 1];
  check(msm_ches_digit_table(q, a_LEADING_TERM, DIGIT_CONVERSION_HASH_TABLE), "digit table");
  printf("DIGIT_CONVERSION_HASH_TABLE constructed.\n");
  auto st = std::chrono::steady_clock::now();
  int h_table = h_LEN_SCALAR;
  if (g_devices.size() > 1) {
    int lg = 0;
    while ((1u << lg) < g_devices.size()) ++lg;
    int sp[9];
    check(msm_ches_params(N_EXP - lg, g_beta, sp), "per-shard CHES configuration");
    h_table = sp[3];
    check(msm_ches_ctx_create_multi(&g_ches, GROUP, g_devices.data(), (int)g_devices.size(), N_EXP - lg, g_beta),
          "msm_ches_ctx_create_multi");
    printf("CHES sharded over %zu devices, config_file_n_exp_%d per shard\n", g_devices.size(), N_EXP - lg);
  } else {
    check(msm_ches_ctx_create(&g_ches, GROUP, g_device, N_EXP, g_beta), "msm_ches_ctx_create");
  }
  check(msm_ches_ctx_build_table(g_ches, FIX_POINTS_LIST, N_POINTS, 0, nullptr), "CHES table");
  if (g_host_tables) {
    const size_t cnt = 3 * N_POINTS * (size_t)h_table;
    PRECOMPUTATION_POINTS_LIST_3nh = new msm_driver_affine[cnt];
    check(msm_ches_ctx_get_table(g_ches, PRECOMPUTATION_POINTS_LIST_3nh, 0, cnt), "CHES table read-back");
  }
  auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - st).count();
  printf("PRECOMPUTATION_POINTS_LIST_3nh SUCCESSFULLY CONSTRUCTED (GPU)\nPRECOMPUTATION Wall clock time elapse is: %lld us\n",
         (long long)us);
}
void free_init_pippenger_CHES_q_over_5() {
  delete[] BUCKET_SET;
  delete[] BUCKET_VALUE_TO_ITS_INDEX;
  delete[] DIGIT_CONVERSION_HASH_TABLE;
  delete[] PRECOMPUTATION_POINTS_LIST_3nh;
  BUCKET_SET = BUCKET_VALUE_TO_ITS_INDEX = nullptr;
  DIGIT_CONVERSION_HASH_TABLE = nullptr;
  PRECOMPUTATION_POINTS_LIST_3nh = nullptr;
  msm_ches_ctx_destroy(g_ches);
  g_ches = nullptr;
}

void init_pippenger_BGMW95() {
  auto st = std::chrono::steady_clock::now();
  check(msm_bgmw_ctx_create(&g_bgmw, GROUP, g_device, EXPONENT_OF_q_BGMW95, h_BGMW95), "msm_bgmw_ctx_create");
  check(msm_bgmw_ctx_build_table(g_bgmw, FIX_POINTS_LIST, N_POINTS, 0, nullptr), "BGMW95 table");
  if (g_host_tables) {
    const size_t cnt = N_POINTS * (size_t)h_BGMW95;
    PRECOMPUTATION_POINTS_LIST_BGMW95 = new msm_driver_affine[cnt];
    check(msm_bgmw_ctx_get_table(g_bgmw, PRECOMPUTATION_POINTS_LIST_BGMW95, 0, cnt), "BGMW95 table read-back");
  }
  auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - st).count();
  printf("PRECOMPUTATION_POINTS_LIST_BGMW95 SUCCESSFULLY CONSTRUCTED (GPU)\nPRECOMPUTATION Wall clock time elapse is: %lld us\n",
         (long long)us);
}
void free_init_pippenger_BGMW95() {
  delete[] PRECOMPUTATION_POINTS_LIST_BGMW95;
  PRECOMPUTATION_POINTS_LIST_BGMW95 = nullptr;
  msm_bgmw_ctx_destroy(g_bgmw);
  g_bgmw = nullptr;
}

static msm_driver_affine affine_of(const jac_t &j) {
  msm_driver_affine a;
  DRV(to_affine)(&a, &j);
  return a;
}

// method 1: MB digit conversion + accumulation + d-reduction, all on the device
msm_driver_affine pippenger_variant_q_over_5_CHES(uint256_t scalars_array[]) {
  jac_t ret;
  check(msm_ches_ctx_mult(g_ches, &ret, (const byte *)scalars_array, sizeof(uint256_t), 0, nullptr), "CHES mult");
  return affine_of(ret);
}

// method 2: the integral conversion (standard q-ary digits, carry into the next
// digit, hash lookup -- ref auxiliaryfunc.h:83-90 + multi_scalar.c:748-775) is
// exactly what the device digit kernel k_ches_digits does per scalar; the
// host-driven form of this method is blst_p*_construct_nh_scalars_nh_points +
// blst_p*_tile_pippenger_d_CHES (tests/test_gpu_blst_ches_abi.py)
msm_driver_affine pippenger_variant_q_over_5_CHES_integral_scalar_conversion(uint256_t scalars_array[]) {
  return pippenger_variant_q_over_5_CHES(scalars_array);
}

msm_driver_affine pippenger_variant_BGMW95(uint256_t scalars_array[]) {
  jac_t ret;
  check(msm_bgmw_ctx_mult(g_bgmw, &ret, (const byte *)scalars_array, sizeof(uint256_t), 0, nullptr), "BGMW95 mult");
  return affine_of(ret);
}

// ref main_p1.cpp:400-436: pointer arrays of points and 32-byte scalars, nbits 255
msm_driver_affine pippenger_blst_built_in(uint256_t scalars_array[]) {
  std::vector<const msm_driver_affine *> pp(N_POINTS);
  std::vector<const byte *> sp(N_POINTS);
  for (size_t i = 0; i < N_POINTS; ++i) {
    pp[i] = FIX_POINTS_LIST + i;
    sp[i] = (const byte *)&scalars_array[i];
  }
  std::vector<limb_t> scratch(BLST_SCRATCH(N_POINTS) / sizeof(limb_t) + 1);
  jac_t ret;
  BLST_MULT(&ret, pp.data(), N_POINTS, sp.data(), 255, scratch.data());
  return affine_of(ret);
}

static std::string compressed_hex(const msm_driver_affine &a) {
  // compress through a Jacobian with Z = 1 (Montgomery one): to_affine is the identity
  jac_t j;
  memset(&j, 0, sizeof j);
  memcpy(&j, &a, sizeof a);
  const bool inf = [&] {
    const uint8_t *b = (const uint8_t *)&a;
    for (size_t k = 0; k < sizeof a; ++k)
      if (b[k]) return false;
    return true;
  }();
  if (!inf) {
    static const uint64_t ONE[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL, 0x5f48985753c758baULL,
                                    0x77ce585370525745ULL, 0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
    memcpy((uint8_t *)&j + sizeof a, ONE, sizeof ONE);  // z (G2: z.c0; z.c1 stays 0)
  }
  uint8_t out[96];
  DRV(compress)(out, &j);
  std::string s;
  char buf[3];
  for (int k = 0; k < 48 * GROUP; ++k) {
    snprintf(buf, sizeof buf, "%02x", out[k]);
    s += buf;
  }
  return s;
}

static int g_tests = 5, g_loops = -1;

int test_pippengers() {
  printf("\nPIPPENGERS TEST OVER G%d for NPOINTS:  2**%d\n", GROUP, N_EXP);
  const int TEST_NUM = g_tests;
  const int LOOP_NUM = g_loops > 0 ? g_loops : (N_EXP <= 8 ? 40 : N_EXP <= 12 ? 10 : N_EXP <= 16 ? 5 : 1);
  typedef msm_driver_affine (*method_t)(uint256_t[]);
  const method_t methods[4] = {pippenger_variant_q_over_5_CHES,
                               pippenger_variant_q_over_5_CHES_integral_scalar_conversion, pippenger_variant_BGMW95,
                               pippenger_blst_built_in};
  const char *names[4] = {"ches_q_over_5", "ches_integral", "bgmw95", "pippenger_blst_built_in"};
  double acc_us[4] = {0, 0, 0, 0};
  std::string last[4];
  int agree = 1;
  std::vector<uint256_t> sc(N_POINTS);
  for (int idx = 1; idx <= TEST_NUM; ++idx) {
    msm_gen_scalars((byte *)sc.data(), N_POINTS, (uint64_t)idx);  // seeded SplitMix64
    printf("This is No.%d SCALARS_ARRAY.\n", idx);
    for (int k = 0; k < 4; ++k) {
      msm_driver_affine r;
      auto st = std::chrono::steady_clock::now();
      for (int l = 0; l < LOOP_NUM; ++l) r = methods[k](sc.data());
      acc_us[k] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - st).count();
      last[k] = compressed_hex(r);
    }
    for (int k = 1; k < 4; ++k) agree &= last[k] == last[0];
    printf("First scalar: 0x%016llx%016llx%016llx%016llx\n", (unsigned long long)sc[0].data[3],
           (unsigned long long)sc[0].data[2], (unsigned long long)sc[0].data[1], (unsigned long long)sc[0].data[0]);
  }
  const double div = (double)TEST_NUM * LOOP_NUM;
  const char *labels[4] = {"1. CHES 'nh+ q/5'", "2. CHES 'nh+ q/5' integral scalar conversion",
                           "3. pippenger_variant_BGMW95", "4. pippenger_blst_built_in"};
  for (int k = 0; k < 4; ++k)
    printf("\n%s. Wall clock time elapse is: %.1f us\n%s\n", labels[k], acc_us[k] / div, last[k].c_str());
  const double t12 = acc_us[0] < acc_us[1] ? acc_us[0] : acc_us[1];
  printf("Improvement, BGMW95 vs pipp: %.3f%%\n", 100.0 * (acc_us[3] - acc_us[2]) / acc_us[3]);
  printf("Improvement, CHES_q_over_5 vs pipp: %.3f%%\n", 100.0 * (acc_us[3] - t12) / acc_us[3]);
  printf("Improvement, CHES_q_over_5 vs BGMW95: %.3f%%\n", 100.0 * (acc_us[2] - t12) / acc_us[2]);
  printf("all four methods agree: %s\n\nTEST END\n", agree ? "yes" : "NO");
  printf("{\"group\": %d, \"n_exp\": %d, \"tests\": %d, \"loops\": %d, \"agree\": %s, \"methods\": {", GROUP, N_EXP,
         TEST_NUM, LOOP_NUM, agree ? "true" : "false");
  for (int k = 0; k < 4; ++k)
    printf("%s\"%s\": {\"us\": %.1f, \"pairs_per_s\": %.1f, \"last_compressed\": \"%s\"}", k ? ", " : "", names[k],
           acc_us[k] / div, (double)N_POINTS / (acc_us[k] / div) * 1e6, last[k].c_str());
  printf("}}\n");
  fflush(stdout);
  return agree ? 0 : 1;
}

int main(int argc, char **argv) {
  int config = 10, beta = 0, device = 0, host_tables = 0;
  for (int a = 1; a < argc; ++a) {
    const char *s = argv[a];
    if (!strncmp(s, "config=", 7)) config = atoi(s + 7);
    else if (!strncmp(s, "beta=", 5)) beta = atoi(s + 5);
    else if (!strncmp(s, "device=", 7)) device = atoi(s + 7);
    else if (!strncmp(s, "tests=", 6)) g_tests = atoi(s + 6);
    else if (!strncmp(s, "loops=", 6)) g_loops = atoi(s + 6);
    else if (!strncmp(s, "host_tables=", 12)) host_tables = atoi(s + 12);
    else if (!strncmp(s, "gpus=", 5)) {
      g_devices.clear();
      for (int d = 0; d < atoi(s + 5); ++d) g_devices.push_back(d);
    } else if (!strncmp(s, "devices=", 8)) {
      g_devices.clear();
      for (const char *c = s + 8; *c;) {
        g_devices.push_back(atoi(c));
        while (*c && *c != ',') ++c;
        if (*c == ',') ++c;
      }
    } else {
      fprintf(stderr,
              "usage: %s config=<n_exp 8..21> [beta=0|1] [device=0] [tests=5] [loops=N] [host_tables=0|1] "
              "[gpus=N | devices=d0,d1,...]\n",
              argv[0]);
      return 2;
    }
  }
  if (msm_driver_configure(config, beta, device, host_tables) != MSM_OK) {
    fprintf(stderr, "no reference configuration for config=%d beta=%d\n", config, beta);
    return 2;
  }
  if (msm_device_count() <= device) {
    fprintf(stderr, "no HIP device %d visible\n", device);
    return 2;
  }
  for (int d : g_devices)
    if (d < 0 || d >= msm_device_count()) {
      fprintf(stderr, "no HIP device %d visible\n", d);
      return 2;
    }
  init_fix_point_list();
  init_pippenger_CHES_q_over_5();
  init_pippenger_BGMW95();
  int rc = test_pippengers();
  free_init_pippenger_BGMW95();
  free_init_pippenger_CHES_q_over_5();
  free_init_fix_point_list();
  return rc;
}
