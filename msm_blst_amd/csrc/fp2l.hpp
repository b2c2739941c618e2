// fp2l.hpp -- Fp2 arithmetic split over a PAIR of lanes (G2 bucket kernels).
//
// A G2 xyzz point is 4 Fp2 = 112 registers; the madd formulas keep ~12 Fp2
// values live, so one lane per G2 bucket needs 256 VGPRs + 88 AGPRs and runs at
// one wave per SIMD (measured 0.61 of the Fp-mul peak).  Here the
// two components of every Fp2 value live in two neighbouring lanes (even lane:
// c0, odd lane: c1), halving the registers per lane.  Products need the
// partner's component, fetched with one DPP quad_perm move per limb, and every
// lane runs the SAME instruction stream on lane-selected operands (v_cndmask),
// so the pair never diverges.  Round 6: the lane-dependent choice sits on the
// b side only, so the a operands enter the product in place (own a first,
// partner a' second) and one select per product is saved:
//   c0 = a0 b0 + a1 (8p - b1)        even lane: fp_mul2(a, b,  a', 8p - b')
//   c1 = a1 b0 + a0 b1               odd lane:  fp_mul2(a, b', a', b)
// (the same single-reduction sums as f_mul(Fp2) in fp.hpp, so every column and
// value bound of DESIGN 4a carries over unchanged; ' = partner component).
// ec.hpp's xyzz formulas are generic over the field type and run unchanged on
// Fp2L; ref no_asm.h:566-688 is the Fp2 tower they replace.
#pragma once
#include "fp.hpp"

namespace msm {

struct Fp2L {
  Fp c;  // this lane's component: c0 on even lanes, c1 on odd lanes
};

#ifdef MSM_FP_HOST_TEST
// host range-check build (tests/host/fp_host_shim.cpp): the pair is two host
// threads run in lockstep, and the partner's value comes through the shim
extern "C" int msm_host_lane(void);
extern "C" uint32_t msm_host_pair_swap(uint32_t x);
MSM_FN bool pair_odd() { return (msm_host_lane() & 1) != 0; }
MSM_FN uint32_t pair_swap(uint32_t x) { return msm_host_pair_swap(x); }
#else
MSM_FN bool pair_odd() { return (__lane_id() & 1) != 0; }
// the partner lane's value (DPP quad_perm [1,0,3,2]: lanes 2k <-> 2k+1)
MSM_FN uint32_t pair_swap(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true); }
#endif
MSM_FN void pair_swap(Fp &r, const Fp &a) {
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = pair_swap(a.v[i]);
}
MSM_FN void pair_sel(Fp &r, bool c, const Fp &a, const Fp &b) {  // r = c ? a : b
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = c ? a.v[i] : b.v[i];
}

// a b, a lazy (< 6p, limbs < 2^30), b lazy (normalized here) -> S
MSM_FN void f_mul(Fp2L &r, const Fp2L &a, const Fp2L &b) {
  const bool odd = pair_odd();
  Fp bn = b.c, pa, pb, nb, Y1, Y2;
  fp_norm(bn);
  pair_swap(pa, a.c);
  pair_swap(pb, bn);
  fp_neg<8>(nb, pb);
  pair_sel(Y1, odd, pb, bn);  // even b, odd b'
  pair_sel(Y2, odd, bn, nb);  // even 8p - b', odd b
  fp_mul2(r.c, a.c, Y1, pa, Y2);
}
// b already normalized (class S)
MSM_FN void f_mul_bs(Fp2L &r, const Fp2L &a, const Fp2L &b) {
  const bool odd = pair_odd();
  Fp pa, pb, nb, Y1, Y2;
  pair_swap(pa, a.c);
  pair_swap(pb, b.c);
  fp_neg<8>(nb, pb);
  pair_sel(Y1, odd, pb, b.c);  // even b, odd b'
  pair_sel(Y2, odd, b.c, nb);  // even 8p - b', odd b
  Fp t;
  fp_mul2(t, a.c, Y1, pa, Y2);
  r.c = t;
}
// (a0 + a1 i)^2: c0 = (a0 + a1)(a0 + 32p - a1), c1 = a0 (2 a1), inputs < 18p
// (P = U2 - X1 with X1 in class X; tests/fp_bounds.py sqr_fp2l)
MSM_FN void f_sqr(Fp2L &r, const Fp2L &a) {
  const bool odd = pair_odd();
  Fp own = a.c, par, s, d, X, Y;
  fp_norm(own);
  pair_swap(par, own);
  fp_add(s, own, par);       // even: a0 + a1
  fp_sub<32>(d, own, par);   // even: a0 + 32p - a1
  fp_add(Y, own, own);       // odd: 2 a1 (limbs < 2^29)
  pair_sel(X, odd, par, s);
  pair_sel(Y, odd, Y, d);
  fp_mul(r.c, X, Y);
}
MSM_FN void f_add(Fp2L &r, const Fp2L &a, const Fp2L &b) { fp_add(r.c, a.c, b.c); }
MSM_FN void f_sub4(Fp2L &r, const Fp2L &a, const Fp2L &b) { fp_sub<4>(r.c, a.c, b.c); }
MSM_FN void f_sub_2x(Fp2L &r, const Fp2L &a, const Fp2L &b, const Fp2L &c) { fp_sub_2x(r.c, a.c, b.c, c.c); }
MSM_FN void f_sub16(Fp2L &r, const Fp2L &a, const Fp2L &b) { fp_sub<16>(r.c, a.c, b.c); }
MSM_FN void f_nred(Fp2L &a) { fp_nred(a.c); }
MSM_FN void f_norm(Fp2L &a) { fp_norm(a.c); }
MSM_FN void f_neg4(Fp2L &r, const Fp2L &a) { fp_neg<4>(r.c, a.c); }
MSM_FN void f_one(Fp2L &r) {
  if (pair_odd()) fp_zero(r.c);
  else fp_one(r.c);
}
MSM_FN void f_zero(Fp2L &r) { fp_zero(r.c); }
MSM_FN bool f_is_zero_exact(const Fp2L &a) {
  const uint32_t z = fp_is_zero_exact(a.c) ? 1u : 0u;
  return (z & pair_swap(z)) != 0;
}
MSM_FN bool f_is_zero_S(const Fp2L &a) {
  const uint32_t z = fp_is_zero_lt2p(a.c) ? 1u : 0u;
  return (z & pair_swap(z)) != 0;
}
MSM_FN void f_mul3(Fp2L &r, const Fp2L &a) { f_mul3(r.c, a.c); }
// a b - c d (a lazy, b lazy normalized here, c, d in S), as f_mul_sub(Fp2):
//   r0 = a0 b0 + a1 (8p - b1) + c0 (8p - d0) + c1 d1
//   r1 = a1 b0 + a0 b1 + c1 (8p - d0) + c0 (8p - d1)
// own operands first, partner second, the lane choice on the b / d side:
//   even: a b + a' (8p - b') + c (8p - d) + c' d'
//   odd:  a b' + a' b + c (8p - d') + c' (8p - d)
MSM_FN void f_mul_sub(Fp2L &r, const Fp2L &a, const Fp2L &b, const Fp2L &c, const Fp2L &d) {
  const bool odd = pair_odd();
  Fp bn = b.c, pa, pb, pc, pd, nd, npb, Y1, Y2, Y3, Y4;
  fp_norm(bn);
  pair_swap(pa, a.c);
  pair_swap(pb, bn);
  pair_swap(pc, c.c);
  pair_swap(pd, d.c);
  fp_neg<8>(npb, pb);
  fp_neg<8>(nd, d.c);
  pair_sel(Y1, odd, pb, bn);   // even b, odd b'
  pair_sel(Y2, odd, bn, npb);  // even 8p - b', odd b
  pair_sel(Y3, odd, pd, d.c);  // even d, odd d' ...
  fp_neg<8>(Y3, Y3);           // ... negated: 8p - d / 8p - d'
  pair_sel(Y4, odd, nd, pd);   // even d', odd 8p - d
  Fp t;
  fp_mul4(t, a.c, Y1, pa, Y2, c.c, Y3, pc, Y4);
  r.c = t;
}

}  // namespace msm
