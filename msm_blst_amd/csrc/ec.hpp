// ec.hpp -- BLS12-381 point arithmetic in xyzz coordinates for gfx950,
// generic over the base field (G1: Fp, G2: Fp2).
//
// Replaces the reference's bucket formulas (src/ec_ops.h:642-785):
//   xyzz_madd  <- POINTonE1xyzz_dadd_affine (ec_ops.h:710-769), madd-2008-s
//                 with the sign twist and the mdbl-2008-s-1 doubling branch
//   xyzz_add   <- POINTonE1xyzz_dadd (ec_ops.h:642-702), add-2008-s /
//                 dbl-2008-s-1
//   xyzz_dbl   <- the doubling branch of the above, used by the reductions
// An xyzz point (X, Y, ZZZ, ZZ) stands for (X/ZZ, Y/ZZZ); infinity is ZZ == 0
// (set exactly, never produced by a product).  Every coordinate leaving these
// functions is in range class S (normalized, < 2p per component; fp.hpp)
// except x, which is left in class X (normalized, < 10p): it only enters
// products and the subtrahend of f_sub16, so its reduction is skipped.
// Branches for the rare cases (P == +-bucket, infinity) are data-dependent
// and divergent; random inputs never take them, the parity tests force them.
#pragma once
#include "fp.hpp"

namespace msm {

template <class F>
struct Aff {
  F x, y;
};
template <class F>
struct Xyzz {
  F x, y, zzz, zz;
};

template <class F>
MSM_FN bool xyzz_is_inf(const Xyzz<F> &a) {
  return f_is_zero_exact(a.zz);
}
template <class F>
MSM_FN void xyzz_set_inf(Xyzz<F> &a) {
  f_zero(a.x);
  f_zero(a.y);
  f_zero(a.zzz);
  f_zero(a.zz);
}
// bucket := +-P   (ZZ = ZZZ = 1, Y negated instead of ZZZ; same point as the
// reference's (X, Y, -1, 1) representative of ec_ops.h:720-724)
template <class F>
MSM_FN void xyzz_from_aff(Xyzz<F> &r, const Aff<F> &p, bool neg) {
  r.x = p.x;
  if (neg) {
    f_neg4(r.y, p.y);
    f_nred(r.y);
  } else {
    r.y = p.y;
  }
  f_one(r.zzz);
  f_one(r.zz);
}

// doubling of an xyzz point given in S (dbl-2008-s-1):
//   U = 2Y, V = U^2, W = U V, S = X V, M = 3 X^2 (+ a ZZ^2, a = 0)
//   X3 = M^2 - 2S, Y3 = M (S - X3) - W Y, ZZ3 = V ZZ, ZZZ3 = W ZZZ
template <class F>
MSM_FN void xyzz_dbl(Xyzz<F> &r, const Xyzz<F> &a) {
  if (xyzz_is_inf(a)) {
    r = a;
    return;
  }
  // ordered so that each input coordinate dies at its last use (ZZ3, ZZZ3
  // first; r may alias a).  Round 3 reverted this order because compiled into
  // the one-lane G2 table kernel (256 VGPR + 256 AGPR + 1.5 KB scratch) it gave
  // wrong rows on the device only: 2Q right, then Q itself corrupted across
  // the call (3Q and every later row wrong; tests/test_gpu_table_rows.py).  The
  // lane-pair table kernel has no spills and builds correct rows with it
  // (DESIGN 11).
  F U, V, W, S, M, t, X3;
  f_add(U, a.y, a.y);      // < 4p lazy
  f_sqr(V, U);             // S
  f_mul(W, V, U);          // S
  f_mul(S, a.x, V);        // S
  f_mul(r.zz, V, a.zz);    // ZZ3 = V ZZ (V, ZZ die)
  f_mul(r.zzz, W, a.zzz);  // ZZZ3 = W ZZZ
  f_sqr(M, a.x);           // S (X dies)
  f_mul3(M, M);            // < 6p lazy
  f_sqr(X3, M);            // S
  F z;
  f_zero(z);
  f_sub_2x(X3, X3, z, S);  // M^2 + 8p - 2S   < 10p
  f_norm(X3);              // X
  f_sub16(t, S, X3);       // < 18p
  f_mul_sub(r.y, t, M, W, a.y);  // Y3 = M (S - X3) - W Y   S (one reduction)
  r.x = X3;
}

// acc += (neg ? -P : P); P affine, canonical, not infinity (callers skip the
// all-zero affine point, as ec_ops.h:717 does).
template <class F>
MSM_FN void xyzz_madd(Xyzz<F> &acc, const Aff<F> &p, bool neg) {
  if (xyzz_is_inf(acc)) {
    xyzz_from_aff(acc, p, neg);
    return;
  }
  F y2, P, R, PP, PPP, t;
  if (neg) {
    f_neg4(y2, p.y);       // < 4p, limbs < 2^29
  } else {
    y2 = p.y;
  }
  f_mul_bs(P, p.x, acc.zz);   // U2 = X2 ZZ1          S
  f_mul_bs(R, y2, acc.zzz);   // S2 = Y2 ZZZ1         S
  f_sub16(P, P, acc.x);    // P = U2 - X1          < 18p lazy
  f_sub4(R, R, acc.y);     // R = S2 - Y1          < 6p lazy
  f_sqr(PP, P);            // PP                   S
  if (__builtin_expect(f_is_zero_S(PP), 0)) {
    // X1 == X2: either P == bucket (double it) or P == -bucket (infinity)
    F RR;
    f_sqr(RR, R);
    if (f_is_zero_S(RR)) {
      // +-P equals the bucket: double the bucket itself (still untouched
      // here), so the affine operand dies after U2 and S2 instead of staying
      // live through the whole madd for this branch
      Xyzz<F> b = acc;
      xyzz_dbl(acc, b);
    } else {
      xyzz_set_inf(acc);
    }
    return;
  }
  // ordered so that ZZ1, P, X1 and PP die as early as possible (register
  // pressure: 8-10 live field elements; G2 elements are 28 VGPRs each);
  // f_mul_bs: second operand normalized (every S value here)
  f_mul_bs(acc.zz, acc.zz, PP);    // ZZ3 = ZZ1 PP         S
  f_mul_bs(PPP, P, PP);         // S
  f_mul_bs(acc.x, acc.x, PP);      // Q = X1 PP  (in place of X1)   S
  f_mul_bs(acc.zzz, acc.zzz, PPP); // ZZZ3 = ZZZ1 PPP      S
  F X3;
  f_sqr(X3, R);            // R^2                  S
  f_sub_2x(X3, X3, PPP, acc.x);  // R^2 + 8p - PPP - 2Q   < 10p
  f_norm(X3);              // X3 = R^2 - PPP - 2Q  X
  f_sub16(t, acc.x, X3);   // Q - X3  < 18p
  f_mul_sub(acc.y, t, R, acc.y, PPP);  // Y3 = R (Q - X3) - Y1 PPP   S (one reduction)
  acc.x = X3;
}

// acc += b, both xyzz in S
template <class F>
MSM_FN void xyzz_add(Xyzz<F> &acc, const Xyzz<F> &b) {
  if (xyzz_is_inf(b)) return;
  if (xyzz_is_inf(acc)) {
    acc = b;
    return;
  }
  // Computed in place so that b dies early and at most ~8 field elements are
  // live (G2: 28 VGPRs each): acc is first rewritten as the representative
  // (U1, S1, ZZZ1 ZZZ2, ZZ1 ZZ2) of the same point, which is also what the
  // doubling branch doubles.
  F P, R, PP, PPP, t;
  f_mul_bs(acc.x, acc.x, b.zz);    // U1 = X1 ZZ2          S
  f_mul_bs(acc.y, acc.y, b.zzz);   // S1 = Y1 ZZZ2         S
  f_mul_bs(P, b.x, acc.zz);        // U2 = X2 ZZ1          S
  f_sub4(P, P, acc.x);          // P = U2 - U1          < 6p
  f_mul_bs(R, b.y, acc.zzz);       // S2 = Y2 ZZZ1         S
  f_sub4(R, R, acc.y);          // R = S2 - S1          < 6p
  f_mul_bs(acc.zz, acc.zz, b.zz);
  f_mul_bs(acc.zzz, acc.zzz, b.zzz);
  f_sqr(PP, P);
  if (__builtin_expect(f_is_zero_S(PP), 0)) {
    F RR;
    f_sqr(RR, R);
    if (f_is_zero_S(RR)) {
      Xyzz<F> a = acc;
      xyzz_dbl(acc, a);
    } else {
      xyzz_set_inf(acc);
    }
    return;
  }
  f_mul_bs(acc.zz, acc.zz, PP);    // ZZ3 = ZZ1 ZZ2 PP
  f_mul_bs(PPP, P, PP);
  f_mul_bs(acc.x, acc.x, PP);      // Q = U1 PP  (in place of U1)
  f_mul_bs(acc.zzz, acc.zzz, PPP); // ZZZ3 = ZZZ1 ZZZ2 PPP
  F X3;
  f_sqr(X3, R);
  f_sub_2x(X3, X3, PPP, acc.x);
  f_norm(X3);                   // X3 = R^2 - PPP - 2Q  X
  f_sub16(t, acc.x, X3);
  f_mul_sub(acc.y, t, R, acc.y, PPP);  // Y3 = R (Q - X3) - S1 PPP   S (one reduction)
  acc.x = X3;
}

}  // namespace msm
