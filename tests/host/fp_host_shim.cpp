// fp_host_shim.cpp -- host (g++) build of the engine's field and xyzz headers
// (msm_blst_amd/csrc/fp.hpp, ec.hpp) with every range check enabled
// (MSM_FP_HOST_TEST: a wrapping 64-bit column, a wrapping or negative limb, or
// a negative reduced value sets msm_fp_overflow).  TEST INFRASTRUCTURE ONLY:
// loaded by tests/test_fp_bounds.py through ctypes; the same header text is
// compiled for gfx950 in the product.
#define MSM_FP_HOST_TEST 1
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <thread>

#include "../../msm_blst_amd/csrc/ec.hpp"
#include "../../msm_blst_amd/csrc/fp2l.hpp"

extern "C" {
int msm_fp_overflow = 0;

using namespace msm;

static Fp ld(const uint32_t *p) {
  Fp r;
  memcpy(r.v, p, sizeof r.v);
  return r;
}
static void st(uint32_t *p, const Fp &a) { memcpy(p, a.v, sizeof a.v); }
static Fp2 ld2(const uint32_t *p) { return Fp2{ld(p), ld(p + NL)}; }
static void st2(uint32_t *p, const Fp2 &a) {
  st(p, a.c0);
  st(p + NL, a.c1);
}

int h_overflow(int clear) {
  int v = msm_fp_overflow;
  if (clear) msm_fp_overflow = 0;
  return v;
}

// ---- Fp primitives (op codes as in tests/test_fp_bounds.py) ----
void h_fp_op(int op, uint32_t *r, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d,
             const uint32_t *e, const uint32_t *f, const uint32_t *g, const uint32_t *h) {
  Fp R;
  switch (op) {
    case 0: fp_mul(R, ld(a), ld(b)); break;
    case 1: fp_sqr(R, ld(a)); break;
    case 2: fp_mul2(R, ld(a), ld(b), ld(c), ld(d)); break;
    case 3: fp_mul4(R, ld(a), ld(b), ld(c), ld(d), ld(e), ld(f), ld(g), ld(h)); break;
    case 4: R = ld(a); fp_red(R); break;
    case 5: R = ld(a); fp_nred(R); break;
    case 6: fp_sub<4>(R, ld(a), ld(b)); break;
    case 7: fp_sub<8>(R, ld(a), ld(b)); break;
    case 8: fp_sub<32>(R, ld(a), ld(b)); break;
    case 9: f_mul_sub(R, ld(a), ld(b), ld(c), ld(d)); break;
    case 10: fp_sub_2x(R, ld(a), ld(b), ld(c)); break;
    case 11: fp_sub<16>(R, ld(a), ld(b)); break;
    default: return;
  }
  st(r, R);
}
// ---- Fp2 (components c0 | c1, 28 words) ----
void h_fp2_op(int op, uint32_t *r, const uint32_t *a, const uint32_t *b, const uint32_t *c, const uint32_t *d) {
  Fp2 R;
  switch (op) {
    case 0: f_mul(R, ld2(a), ld2(b)); break;
    case 1: f_sqr(R, ld2(a)); break;
    case 2: f_mul_bs(R, ld2(a), ld2(b)); break;
    case 3: f_mul_sub(R, ld2(a), ld2(b), ld2(c), ld2(d)); break;
    default: return;
  }
  st2(r, R);
}

}  // extern "C"

// ---- G2 lane pairs (fp2l.hpp): two threads in lockstep, lane 0 holds c0 and
// lane 1 holds c1 of every Fp2 value; pair_swap is an exchange through two
// double-buffered slots (a barrier per exchange) ----
static thread_local int t_lane = 0;
static std::mutex x_mu;
static std::condition_variable x_cv;
static uint32_t x_slot[2][2];
static int x_arrived = 0;
static uint64_t x_gen = 0;
extern "C" int msm_host_lane(void) { return t_lane; }
extern "C" uint32_t msm_host_pair_swap(uint32_t x) {
  std::unique_lock<std::mutex> lk(x_mu);
  const uint64_t my = x_gen;
  x_slot[my & 1][t_lane] = x;
  if (++x_arrived == 2) {
    x_arrived = 0;
    ++x_gen;
    x_cv.notify_all();
  } else {
    x_cv.wait(lk, [&] { return x_gen != my; });
  }
  return x_slot[my & 1][t_lane ^ 1];
}
// run f(lane) on two lockstep threads
template <class Fn>
static void pair_run(Fn f) {
  std::thread t0([&] { t_lane = 0; f(0); }), t1([&] { t_lane = 1; f(1); });
  t0.join();
  t1.join();
}
// component `lane` of the Fp2 values of an array of `count` Fp2 (c0 | c1 each)
static void ldl(Fp2L *dst, const uint32_t *src, int count, int lane) {
  for (int k = 0; k < count; ++k) memcpy(dst[k].c.v, src + (size_t)k * 2 * NL + lane * NL, NL * 4);
}
static void stl(uint32_t *dst, const Fp2L *src, int count, int lane) {
  for (int k = 0; k < count; ++k) memcpy(dst + (size_t)k * 2 * NL + lane * NL, src[k].c.v, NL * 4);
}
// op codes as h_fp2_op
extern "C" void h_fp2l_op(int op, uint32_t *r, const uint32_t *a, const uint32_t *b, const uint32_t *c,
                          const uint32_t *d) {
  pair_run([&](int lane) {
    Fp2L A, B, C, D, R;
    ldl(&A, a, 1, lane);
    if (b) ldl(&B, b, 1, lane);
    if (c) ldl(&C, c, 1, lane);
    if (d) ldl(&D, d, 1, lane);
    switch (op) {
      case 0: f_mul(R, A, B); break;
      case 1: f_sqr(R, A); break;
      case 2: f_mul_bs(R, A, B); break;
      case 3: f_mul_sub(R, A, B, C, D); break;
      default: return;
    }
    stl(r, &R, 1, lane);
  });
}
// xyzz formulas on lane pairs (ops as h_xyzz; acc: 4 Fp2, other: 2 (madd) or 4 Fp2)
extern "C" void h_xyzz_l(int op, uint32_t *acc, const uint32_t *other, int neg) {
  pair_run([&](int lane) {
    Xyzz<Fp2L> A;
    ldl(&A.x, acc, 1, lane);
    ldl(&A.y, acc + 2 * NL, 1, lane);
    ldl(&A.zzz, acc + 4 * NL, 1, lane);
    ldl(&A.zz, acc + 6 * NL, 1, lane);
    if (op == 0) {
      Aff<Fp2L> p;
      ldl(&p.x, other, 1, lane);
      ldl(&p.y, other + 2 * NL, 1, lane);
      xyzz_madd(A, p, neg != 0);
    } else if (op == 1) {
      Xyzz<Fp2L> B;
      ldl(&B.x, other, 1, lane);
      ldl(&B.y, other + 2 * NL, 1, lane);
      ldl(&B.zzz, other + 4 * NL, 1, lane);
      ldl(&B.zz, other + 6 * NL, 1, lane);
      xyzz_add(A, B);
    } else {
      Xyzz<Fp2L> t = A;
      xyzz_dbl(A, t);
    }
    stl(acc, &A.x, 1, lane);
    stl(acc + 2 * NL, &A.y, 1, lane);
    stl(acc + 4 * NL, &A.zzz, 1, lane);
    stl(acc + 6 * NL, &A.zz, 1, lane);
  });
}

// ---- xyzz formulas: op 0 madd(acc, P, neg), 1 add(acc, B), 2 dbl(acc) ----
template <class F>
static void xyzz_io(int op, uint32_t *acc, const uint32_t *other, int neg) {
  constexpr int W = sizeof(F) / 4;
  Xyzz<F> A;
  memcpy(&A, acc, sizeof A);
  if (op == 0) {
    Aff<F> p;
    memcpy(&p, other, sizeof p);
    xyzz_madd(A, p, neg != 0);
  } else if (op == 1) {
    Xyzz<F> B;
    memcpy(&B, other, sizeof B);
    xyzz_add(A, B);
  } else {
    Xyzz<F> t = A;
    xyzz_dbl(A, t);
  }
  memcpy(acc, &A, sizeof A);
  (void)W;
}
extern "C" void h_xyzz(int group, int op, uint32_t *acc, const uint32_t *other, int neg) {
  if (group == 1) xyzz_io<Fp>(op, acc, other, neg);
  else xyzz_io<Fp2>(op, acc, other, neg);
}
