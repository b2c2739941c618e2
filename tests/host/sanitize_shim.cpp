// sanitize_shim.cpp -- the engine's host-only code under the sanitizers
// (SURVEY sec.5 aux: "ASan/UBSan on the host restatement"; the reference's only
// guard is -Werror, /root/reference/build.sh:26).  TEST INFRASTRUCTURE ONLY:
// built and run by tests/test_host_sanitize.py, twice --
//   -fsanitize=address,undefined  mode "host": everything below
//   -fsanitize=thread             mode "threads": the thread patterns only
// What runs here is the product's own header text (no HIP in any of them):
//   host_fp.hpp     the host field / curve code of the boundary (Horner
//                   combine, fold, to_affine, compress), checked against the
//                   oracle on random points
//   ptr_walk.hpp    blst's pointer-array rule (abi.cpp), against a naive walk
//   row_samples.hpp the registered-table staleness guard (table_registry.hpp)
//   workers.hpp     WorkerPool::parallel_for and ThreadTeam (multi.hpp's shard
//                   threads), incl. exceptions and concurrent callers
// plus oracle/msm_oracle.c itself (compiled with the same flags): its plain
// Pippenger and CHES MSMs against the golden keys passed on the command line.
//
// usage: sanitize_shim host <n> <g1 key hex> <g2 n> <g2 key hex> <ches n_exp> <ches key hex>
//        sanitize_shim threads
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../msm_blst_amd/csrc/host_fp.hpp"
#include "../../msm_blst_amd/csrc/ptr_walk.hpp"
#include "../../msm_blst_amd/csrc/row_samples.hpp"
#include "../../msm_blst_amd/csrc/workers.hpp"
#include "../../oracle/msm_oracle.h"

static int g_fail = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                   \
    }                                                             \
  } while (0)

static std::string hex(const uint8_t *p, size_t n) {
  static const char *d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) s += d[p[i] >> 4], s += d[p[i] & 15];
  return s;
}

// ---- oracle MSMs against the golden keys ----
static void oracle_msms(size_t n1, const char *k1, size_t n2, const char *k2, int ches_exp, const char *kc) {
  std::vector<uint8_t> sc(32 * std::max(n1, n2));
  {
    std::vector<or_p1_affine> P(n1);
    or_p1_fixed_points(P.data(), n1);
    or_gen_scalars(sc.data(), n1, 1);
    or_p1 r;
    or_p1s_mult_pippenger(&r, P.data(), n1, sc.data(), 255);
    uint8_t c[48];
    or_p1_compress(c, &r);
    CHECK(hex(c, 48) == k1);
  }
  {
    std::vector<or_p2_affine> P(n2);
    or_p2_fixed_points(P.data(), n2);
    or_gen_scalars(sc.data(), n2, 1);
    or_p2 r;
    or_p2s_mult_pippenger(&r, P.data(), n2, sc.data(), 255);
    uint8_t c[96];
    or_p2_compress(c, &r);
    CHECK(hex(c, 96) == k2);
  }
  {  // CHES "nh + q/5" on the reference configuration for 2^ches_exp points
    or_ches_params cp;
    CHECK(or_ches_params_for(ches_exp, 0, &cp) == 0);
    const size_t n = (size_t)1 << ches_exp, q = (size_t)1 << cp.q_exp;
    std::vector<or_p1_affine> P(n), T(3 * n * cp.h);
    or_p1_fixed_points(P.data(), n);
    or_p1_ches_table(T.data(), P.data(), n, cp.q_exp, cp.h);
    std::vector<int> B(or_ches_bucket_set(nullptr, (int)q, cp.a_h));
    or_ches_bucket_set(B.data(), (int)q, cp.a_h);
    std::vector<or_digit> H(q + 1);
    std::vector<int> v2i(q / 2 + 1);
    or_ches_digit_table(H.data(), v2i.data(), B.data(), B.size(), (int)q);
    std::vector<uint8_t> s(32 * n);
    or_gen_scalars(s.data(), n, 1);
    or_p1 r;
    or_p1_ches_msm(&r, T.data(), n, s.data(), H.data(), v2i.data(), B.data(), B.size(), cp.q_exp, cp.h, cp.d_max);
    uint8_t c[48];
    or_p1_compress(c, &r);
    CHECK(hex(c, 48) == kc);
  }
}

// ---- host_fp.hpp against the oracle ----
template <class J, class O>
static J as_jac(const O &o) {
  static_assert(sizeof(J) == sizeof(O), "layout");
  J j;
  memcpy(&j, &o, sizeof j);
  return j;
}
static void host_fp_vs_oracle() {
  const size_t n = 24;
  std::vector<or_p1_affine> P(n);
  or_p1_fixed_points(P.data(), n);
  std::vector<uint8_t> sc(32 * n);
  or_gen_scalars(sc.data(), n, 7);
  std::vector<or_p1> J(n);
  for (size_t i = 0; i < n; ++i) or_p1_mult(&J[i], &P[i], &sc[32 * i], 255);
  typedef hfp::Jac<hfp::Fp> HJ;
  for (size_t i = 0; i + 1 < n; ++i) {
    or_p1 s, d;
    or_p1_add(&s, &J[i], &J[i + 1]);
    or_p1_double(&d, &J[i]);
    uint8_t a[48], b[48];
    or_p1_compress(a, &s);
    hfp::compress(b, hfp::to_affine(hfp::addj(as_jac<HJ>(J[i]), as_jac<HJ>(J[i + 1]))));
    CHECK(memcmp(a, b, 48) == 0);
    or_p1_compress(a, &d);
    hfp::compress(b, hfp::to_affine(hfp::dbl(as_jac<HJ>(J[i]))));
    CHECK(memcmp(a, b, 48) == 0);
    // doubling through the general add, and P + (-P) = infinity
    hfp::compress(b, hfp::to_affine(hfp::addj(as_jac<HJ>(J[i]), as_jac<HJ>(J[i]))));
    CHECK(memcmp(a, b, 48) == 0);
    HJ neg = as_jac<HJ>(J[i]);
    neg.y = hfp::neg(neg.y);
    CHECK(hfp::is_zero(hfp::addj(as_jac<HJ>(J[i]), neg).z));
  }
  // the xyzz chain of the host helpers against the oracle's (ec_ops.h:642-785)
  or_p1xyzz ox;
  memset(&ox, 0, sizeof ox);
  hfp::Xyzz<hfp::Fp> hx;
  memset(&hx, 0, sizeof hx);
  for (size_t i = 0; i < n; ++i) {
    const int sub = (int)(i % 3 == 1);
    or_p1xyzz_dadd_affine(&ox, &ox, &P[i], sub);
    hfp::Aff<hfp::Fp> a;
    memcpy(&a, &P[i], sizeof a);
    hx = hfp::xyzz_madd(hx, a, sub != 0);
  }
  or_p1 oj;
  or_p1xyzz_to_jacobian(&oj, &ox);
  uint8_t a[48], b[48];
  or_p1_compress(a, &oj);
  hfp::compress(b, hfp::to_affine(hfp::xyzz_to_jac(hx)));
  CHECK(memcmp(a, b, 48) == 0);
  // batch to_affine with an infinity in the middle
  std::vector<HJ> in(n);
  for (size_t i = 0; i < n; ++i) in[i] = as_jac<HJ>(J[i]);
  memset(&in[n / 2], 0, sizeof(HJ));
  std::vector<hfp::Aff<hfp::Fp>> out(n);
  hfp::to_affine_batch(out.data(), in.data(), n);
  for (size_t i = 0; i < n; ++i) {
    if (i == n / 2) continue;
    hfp::compress(a, out[i]);
    or_p1_compress(b, &J[i]);
    CHECK(memcmp(a, b, 48) == 0);
  }
  // G2: add / double
  std::vector<or_p2_affine> Q(4);
  or_p2_fixed_points(Q.data(), 4);
  or_p2 q0, q1, qs;
  or_p2_mult(&q0, &Q[0], &sc[0], 255);
  or_p2_mult(&q1, &Q[3], &sc[32], 255);
  or_p2_add(&qs, &q0, &q1);
  typedef hfp::Jac<hfp::Fp2> HJ2;
  uint8_t c[96], e[96];
  or_p2_compress(c, &qs);
  hfp::compress(e, hfp::to_affine(hfp::addj(as_jac<HJ2>(q0), as_jac<HJ2>(q1))));
  CHECK(memcmp(c, e, 96) == 0);
}

// ---- ptr_walk.hpp against a naive walk of blst's rule (multi_scalar.c:390-416) ----
static void ptr_walk() {
  std::mt19937_64 rng(5);
  const size_t sz = 7, N = 300;
  std::vector<uint8_t> pool(sz * 4 * N);
  for (auto &b : pool) b = (uint8_t)rng();
  for (int t = 0; t < 400; ++t) {
    const size_t n = 1 + rng() % N;
    std::vector<const void *> ptrs(n + 1, nullptr);
    std::vector<uint8_t> want(n * sz);
    size_t cur = rng() % (2 * N);
    for (size_t i = 0; i < n; ++i) {
      const unsigned r = (unsigned)(rng() % 8);
      if (i == 0 || r < 3) {  // an explicit pointer: adjacent, or a jump
        if (i > 0 && r == 0) cur = rng() % (2 * N);
        else if (i > 0) cur += 1;
        ptrs[i] = &pool[cur * sz];
      } else if (r < 6) {  // NULL: the element right after the previous one
        cur += 1;
        ptrs[i] = nullptr;
        // blst reads NULL as "continue contiguously to the end": the rest must be NULL too
        for (size_t k = i + 1; k < n; ++k) {
          ptrs[k] = nullptr;
        }
        for (size_t k = i; k < n; ++k) memcpy(&want[k * sz], &pool[(cur + (k - i)) * sz], sz);
        break;
      } else {  // explicit pointer to the adjacent element
        cur += 1;
        ptrs[i] = &pool[cur * sz];
      }
      memcpy(&want[i * sz], &pool[cur * sz], sz);
    }
    std::vector<uint8_t> buf;
    const uint8_t *got = msm::contiguous(buf, ptrs.data(), n, sz);
    CHECK(got && memcmp(got, want.data(), n * sz) == 0);
  }
  std::vector<uint8_t> buf;
  CHECK(msm::contiguous(buf, nullptr, 0, sz) == nullptr);
}

// ---- row_samples.hpp ----
static void row_samples() {
  for (int group : {1, 2}) {
    for (size_t nrows : {(size_t)1, (size_t)2, (size_t)1000, (size_t)5000}) {
      std::vector<uint8_t> rows(nrows * 96 * group);
      for (size_t i = 0; i < rows.size(); ++i) rows[i] = (uint8_t)(i * 131 + 7);
      msm::RowSamples s;
      s.group = group;
      s.base = rows.data();
      s.nrows = nrows;
      s.take_samples();
      CHECK(s.sidx.front() == 0 && s.sidx.back() == nrows - 1);
      CHECK(s.sidx.size() == std::min(nrows, msm::RowSamples::kSamples));
      CHECK(!s.changed(0, nrows - 1));
      for (size_t row : {(size_t)0, nrows - 1, s.sidx[s.sidx.size() / 2]}) {
        uint8_t &b = rows[row * s.psz() + 5];
        b ^= 0x40;
        CHECK(s.changed(0, nrows - 1));
        CHECK(s.changed(row, row));
        if (row > 0) CHECK(!s.changed(0, row - 1));
        b ^= 0x40;
        CHECK(!s.changed(0, nrows - 1));
      }
    }
  }
}

// ---- workers.hpp ----
static void workers(int rounds) {
  msm::WorkerPool &pool = msm::WorkerPool::get();
  for (int r = 0; r < rounds; ++r) {
    const size_t n = 1 + (size_t)r * 37 % 1000;
    std::vector<uint64_t> v(n, 0);
    pool.parallel_for(n, [&](size_t i) { v[i] = i * i; });
    for (size_t i = 0; i < n; ++i) CHECK(v[i] == i * i);
  }
  bool threw = false;
  try {
    pool.parallel_for(100, [&](size_t i) {
      if (i == 57) throw std::runtime_error("57");
    });
  } catch (const std::runtime_error &e) {
    threw = std::string(e.what()) == "57";
  }
  CHECK(threw);
  {  // concurrent callers take turns
    std::atomic<uint64_t> total{0};
    std::vector<std::thread> callers;
    for (int c = 0; c < 4; ++c)
      callers.emplace_back([&] {
        for (int r = 0; r < rounds / 4 + 1; ++r) pool.parallel_for(64, [&](size_t i) { total += i; });
      });
    for (auto &t : callers) t.join();
    CHECK(total.load() == (uint64_t)4 * (rounds / 4 + 1) * (63 * 64 / 2));
  }
  {  // ThreadTeam: every member runs its task on its own thread; results visible after run()
    msm::ThreadTeam team(6);
    std::vector<uint64_t> slot(6, 0);
    std::vector<std::thread::id> who(6);
    for (int r = 0; r < rounds; ++r) {
      team.run([&](size_t g) {
        slot[g] += g + 1;
        who[g] = std::this_thread::get_id();
      });
      for (size_t g = 0; g < 6; ++g) CHECK(slot[g] == (uint64_t)(r + 1) * (g + 1));
    }
    for (size_t g = 0; g < 6; ++g) CHECK(who[g] != std::this_thread::get_id());
    threw = false;
    try {
      team.run([&](size_t g) {
        if (g == 4) throw std::runtime_error("member 4");
      });
    } catch (const std::runtime_error &e) {
      threw = std::string(e.what()) == "member 4";
    }
    CHECK(threw);
    team.run([&](size_t g) { slot[g] = 0; });  // still usable after an exception
    for (size_t g = 0; g < 6; ++g) CHECK(slot[g] == 0);
  }
}

int main(int argc, char **argv) {
  if (argc >= 2 && !strcmp(argv[1], "threads")) {
    workers(200);
  } else if (argc >= 8 && !strcmp(argv[1], "host")) {
    oracle_msms((size_t)atol(argv[2]), argv[3], (size_t)atol(argv[4]), argv[5], atoi(argv[6]), argv[7]);
    host_fp_vs_oracle();
    ptr_walk();
    row_samples();
    workers(40);
  } else {
    fprintf(stderr, "usage: %s host <n> <g1 key> <g2 n> <g2 key> <ches n_exp> <ches key> | threads\n", argv[0]);
    return 2;
  }
  printf("%s %s\n", g_fail ? "FAIL" : "OK", argv[1]);
  return g_fail ? 1 : 0;
}
