"""Interval model of the engine's lazy-reduction arithmetic (fp.hpp / ec.hpp).

TEST INFRASTRUCTURE: proves, by exact integer interval arithmetic over the
per-limb maxima, that no 64-bit column accumulator, 32-bit limb or signed
reduction in msm_blst_amd/csrc/fp.hpp can wrap for the inputs the point
formulas of ec.hpp / coop.hpp feed it, and that every coordinate those
formulas store is in range class S (limbs 0..12 < 2^28, value < 2p).

Soundness: every quantity is an upper bound (limb maxima, value maximum) of a
non-negative integer; each transfer function below mirrors the loop structure
of the C++ routine it names (same terms per column, same carry), and all
terms are non-negative, so the modelled column maximum bounds the real one at
every mad.  fp_red is checked exhaustively over its top limb.

The constants are parsed from fp.hpp itself, so the model follows the header.
"""
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
FP_HPP = os.path.join(os.path.dirname(HERE), "msm_blst_amd", "csrc", "fp.hpp")

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
NL = 14
M = 1 << 28
R = 1 << 392
U64 = 1 << 64
U32 = 1 << 32


def _consts():
    txt = open(FP_HPP).read()
    out = {}
    for name, body in re.findall(r"MSM_CONST uint32_t (\w+)\[NL\] = \{([^}]*)\};", txt):
        out[name] = [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", body)]
    out["RED_MAG"] = int(re.search(r"RED_MAG = (0x[0-9a-fA-F]+)", txt).group(1), 16)
    return out


C = _consts()
P28 = C["P28"]
SUB = {4: C["SUB4P"], 8: C["SUB8P"], 16: C["SUB16P"], 32: C["SUB32P"]}
SUB8P3 = C["SUB8P3"]
assert sum(l << (28 * i) for i, l in enumerate(SUB8P3)) == 8 * P
RED_MAG = C["RED_MAG"]
assert sum(l << (28 * i) for i, l in enumerate(P28)) == P
for k, cs in SUB.items():
    assert sum(l << (28 * i) for i, l in enumerate(cs)) == k * P, k


class RangeError(AssertionError):
    pass


def need(cond, what):
    if not cond:
        raise RangeError(what)


class Iv:
    """upper bounds of a lazily reduced field element: limb maxima, value maximum"""
    __slots__ = ("lim", "vmax")

    def __init__(self, lim, vmax):
        self.lim = list(lim)
        self.vmax = vmax
        # a value can never exceed what its limbs can hold
        self.vmax = min(self.vmax, sum(l << (28 * i) for i, l in enumerate(self.lim)))
        # the top limb can never exceed what the value allows (low limbs >= 0)
        self.lim[NL - 1] = min(self.lim[NL - 1], self.vmax >> 364)

    def is_S(self):
        return all(l < M for l in self.lim[:NL - 1]) and self.vmax < 2 * P

    def is_X(self):
        return all(l < M for l in self.lim[:NL - 1]) and self.vmax < 10 * P

    def __repr__(self):
        return f"Iv(limbs<=2^{max(l.bit_length() for l in self.lim)}, v<{self.vmax / P:.4f}p)"


def S():
    """class S: normalized limbs, value < 2p (every stored coordinate)"""
    return Iv([M - 1] * (NL - 1) + [(2 * P - 1) >> 364], 2 * P - 1)


def Xc():
    """class X: normalized limbs, value < 10p (the stored x coordinate: X3 is
    normalized but not reduced)"""
    return Iv([M - 1] * (NL - 1) + [(10 * P - 1) >> 364], 10 * P - 1)


def canonical():
    """a canonical value < p (affine inputs, converted from blst on upload)"""
    return Iv([M - 1] * (NL - 1) + [(P - 1) >> 364], P - 1)


def union(*xs):
    return Iv([max(x.lim[i] for x in xs) for i in range(NL)], max(x.vmax for x in xs))


def _montgomery(pairs, tag):
    """fp_mul / fp_mul2 / fp_mul4: FIPS columns of sum a_i b_j + sum m_i p_j"""
    acc = 0
    m = M - 1
    out = [0] * NL
    for k in range(NL):
        for a, b in pairs:
            acc += sum(a.lim[i] * b.lim[k - i] for i in range(k + 1))
        acc += sum(m * P28[k - i] for i in range(k))
        acc += m * P28[0]
        need(acc < U64, f"{tag}: column {k} accumulator {acc.bit_length()} bits")
        acc >>= 28
    for k in range(NL, 2 * NL - 1):
        for a, b in pairs:
            acc += sum(a.lim[i] * b.lim[k - i] for i in range(k - NL + 1, NL))
        acc += sum(m * P28[k - i] for i in range(k - NL + 1, NL))
        need(acc < U64, f"{tag}: column {k} accumulator {acc.bit_length()} bits")
        out[k - NL] = min(M - 1, acc)
        acc >>= 28
    need(acc < U32, f"{tag}: top limb {acc.bit_length()} bits")
    out[NL - 1] = acc
    vmax = (sum(a.vmax * b.vmax for a, b in pairs) + (R - 1) * P) // R
    return Iv(out, vmax)


def mul(a, b):
    return _montgomery([(a, b)], "fp_mul")


def mul2(a, b, c, d):
    return _montgomery([(a, b), (c, d)], "fp_mul2")


def mul4(a, b, c, d, e, f, g, h):
    return _montgomery([(a, b), (c, d), (e, f), (g, h)], "fp_mul4")


def sqr(a):
    """fp_sqr: per column the cross products once on their own chain x, then
    acc += 2x (add_dbl: x < 2^63 and 2x + acc < 2^64)"""
    acc, m, out = 0, M - 1, [0] * NL

    def cross(k, lo):
        x = sum(a.lim[i] * a.lim[k - i] for i in range(lo, NL) if 2 * i < k and k - i < NL)
        need(x < (1 << 63), f"fp_sqr: column {k} cross sum {x.bit_length()} bits")
        return 2 * x

    for k in range(NL):
        acc += cross(k, 0)
        need(acc < U64, f"fp_sqr: column {k} after 2x")
        if k % 2 == 0:
            acc += a.lim[k // 2] ** 2
        acc += sum(m * P28[k - i] for i in range(k)) + m * P28[0]
        need(acc < U64, f"fp_sqr: column {k}")
        acc >>= 28
    for k in range(NL, 2 * NL - 1):
        acc += cross(k, k - NL + 1)
        need(acc < U64, f"fp_sqr: column {k} after 2x")
        if k % 2 == 0:
            acc += a.lim[k // 2] ** 2
        acc += sum(m * P28[k - i] for i in range(k - NL + 1, NL))
        need(acc < U64, f"fp_sqr: column {k}")
        out[k - NL] = min(M - 1, acc)
        acc >>= 28
    need(acc < U32, "fp_sqr: top limb")
    out[NL - 1] = acc
    return Iv(out, (a.vmax * a.vmax + (R - 1) * P) // R)


def add(a, b):
    lim = [x + y for x, y in zip(a.lim, b.lim)]
    need(all(l < U32 for l in lim), "fp_add: limb wraps")
    return Iv(lim, a.vmax + b.vmax)


def mul3(a):
    need(all(l <= 0x55555555 for l in a.lim), "f_mul3: limb wraps")
    return Iv([3 * l for l in a.lim], 3 * a.vmax)


def norm(a):
    lim = list(a.lim)
    for i in range(NL - 1):
        lim[i + 1] += lim[i] >> 28
        need(lim[i + 1] < U32, "fp_norm: carry wraps")
        lim[i] = min(lim[i], M - 1)
    return Iv(lim, a.vmax)


def sub(a, b, K=4):
    """fp_sub<K>: a + K p (borrow-adjusted limbs) - b, b normalized"""
    cs = SUB[K]
    need(all(b.lim[i] <= cs[i] for i in range(NL)), f"fp_sub<{K}>: subtrahend limb above K p limb (negative limb)")
    need(b.vmax <= K * P, f"fp_sub<{K}>: subtrahend above K p")
    lim = [a.lim[i] + cs[i] for i in range(NL)]
    need(all(l < U32 for l in lim), f"fp_sub<{K}>: limb wraps")
    return Iv(lim, a.vmax + K * P)


def sub2x(a, b, c):
    """fp_sub_2x: a + 8p (limbs adjusted to >= 3(2^28-1)) - b - 2c, b and c normalized"""
    need(all(b.lim[i] + 2 * c.lim[i] <= SUB8P3[i] for i in range(NL)), "fp_sub_2x: negative limb")
    need(b.vmax + 2 * c.vmax <= 8 * P, "fp_sub_2x: subtrahend above 8p")
    lim = [a.lim[i] + SUB8P3[i] for i in range(NL)]
    need(all(l < U32 for l in lim), "fp_sub_2x: limb wraps")
    return Iv(lim, a.vmax + 8 * P)


def zero():
    return Iv([0] * NL, 0)


def neg(a, K=4):
    cs = SUB[K]
    need(all(a.lim[i] <= cs[i] for i in range(NL)), f"fp_neg<{K}>: negative limb")
    return Iv(list(cs), K * P)


_red_cache = {}


def red(a):
    """fp_red: q = floor(v13 * RED_MAG / 2^32); exhaustive over the top limb v13:
    v - q p must be >= 0 for the smallest v with that top limb and < 2^392."""
    key = (tuple(a.lim), a.vmax)
    if key in _red_cache:
        return _red_cache[key]
    top = min(a.lim[NL - 1], a.vmax >> 364)
    low = sum(l << (28 * i) for i, l in enumerate(a.lim[:NL - 1]))
    out = 0
    for v13 in range(top + 1):
        q = (v13 * RED_MAG) >> 32
        lo = v13 << 364
        need(lo - q * P >= 0, f"fp_red: negative result at top limb {v13}")
        hi = min(lo + low, a.vmax)
        if hi >= lo:
            out = max(out, hi - q * P)
    need(out < R, "fp_red: result above 2^392")
    r = Iv([M - 1] * NL, out)
    _red_cache[key] = r
    return r


def nred(a):
    return red(norm(a))


# ------------------------------------------------------------- Fp2 ops ------
# an Fp2 interval is one Iv bounding both components (every op below is
# symmetric in the components, so the union is sound)
def mul2_fp2(a, b):        # f_mul(Fp2): b normalized copies, c0 = a0 b0 + a1 (8p - b1), c1 = a0 b1 + a1 b0
    bn = norm(b)
    return union(mul2(a, bn, a, neg(bn, 8)), mul2(a, bn, a, bn))


def mul_bs_fp2(a, b):      # f_mul_bs(Fp2): b normalized already
    return union(mul2(a, b, a, neg(b, 8)), mul2(a, b, a, b))


def sqr_fp2(a):            # f_sqr(Fp2): both normalized, (a0+a1)(a0+32p-a1), 2 a0 a1 (red + norm)
    an = norm(a)
    s = add(an, an)
    d = sub(an, an, 32)
    m_ = mul(an, an)
    c0 = mul(s, d)
    c1 = norm(red(add(m_, m_)))
    return union(c0, c1)


def sqr_fp2l(a):           # f_sqr(Fp2L, fp2l.hpp): own component normalized, partner swapped in;
    an = norm(a)           # even lane (a0 + a1)(a0 + 32p - a1), odd lane a0 (2 a1), one fp_mul each
    return union(mul(add(an, an), sub(an, an, 32)), mul(an, add(an, an)))


def mul_sub_fp2(a, b, c, d):   # f_mul_sub(Fp2): two fp_mul4 with 8p-adjusted negations
    b0 = norm(b)
    nb1 = neg(b0, 8)
    nd = neg(d, 8)
    return union(mul4(a, b0, a, nb1, c, nd, c, d), mul4(a, b0, a, b0, c, nd, c, nd))


class Field:
    """the f_* API of fp.hpp for one group"""

    def __init__(self, group):
        self.g = group

    def mul(self, a, b):
        return mul(a, b) if self.g == 1 else mul2_fp2(a, b)

    def mul_bs(self, a, b):
        return mul(a, b) if self.g == 1 else mul_bs_fp2(a, b)

    def sqr(self, a):  # group 3: G2 on lane pairs (fp2l.hpp) -- only the square differs
        return sqr(a) if self.g == 1 else (sqr_fp2l(a) if self.g == 3 else sqr_fp2(a))

    def mul_sub(self, a, b, c, d):
        if self.g == 1:
            return mul2(a, b, c, neg(d, 4))    # f_mul_sub(Fp): fp_mul2(a, b, c, 4p - d)
        return mul_sub_fp2(a, b, c, d)


# ------------------------------------------------------ formula traces ------
def _x3(F, R_, PPP, Q):
    return norm(sub2x(F.sqr(R_), PPP, Q))     # f_sub_2x then f_norm: class X


def trace_dbl(group, a=None):
    """xyzz_dbl (ec.hpp) of an S point"""
    F = Field(group)
    x, y, zzz, zz = a or (Xc(), S(), S(), S())
    U = add(y, y)
    V = F.sqr(U)
    W = F.mul(V, U)
    Sx = F.mul(x, V)
    Mm = mul3(F.sqr(x))
    X3 = norm(sub2x(F.sqr(Mm), zero(), Sx))
    t = sub(Sx, X3, 16)
    Y3 = F.mul_sub(t, Mm, W, y)
    return X3, Y3, F.mul(W, zzz), F.mul(V, zz)


def trace_madd(group, negate):
    """xyzz_madd (ec.hpp): S bucket += +-P, P canonical affine; both branches"""
    F = Field(group)
    x, y, zzz, zz = Xc(), S(), S(), S()
    px, py = canonical(), canonical()
    y2 = neg(py) if negate else py
    Pd = sub(F.mul_bs(px, zz), x, 16)
    Rd = sub(F.mul_bs(y2, zzz), y)
    PP = F.sqr(Pd)
    need(PP.is_S(), "madd: PP must be S for f_is_zero_S")
    zz3 = F.mul_bs(zz, PP)
    PPP = F.mul_bs(Pd, PP)
    Q = F.mul_bs(x, PP)
    zzz3 = F.mul_bs(zzz, PPP)
    X3 = _x3(F, Rd, PPP, Q)
    t = sub(Q, X3, 16)
    Y3 = F.mul_sub(t, Rd, y, PPP)
    # doubling branch (+-P equals the bucket): the untouched bucket itself is doubled
    dbl = trace_dbl(group, (x, y, zzz, zz))
    return (X3, Y3, zzz3, zz3), dbl


def trace_add(group):
    """xyzz_add (ec.hpp), in place: acc (S) += b (S)"""
    F = Field(group)
    x, y, zzz, zz = Xc(), S(), S(), S()
    bx, by, bzzz, bzz = Xc(), S(), S(), S()
    U1 = F.mul_bs(x, bzz)
    S1 = F.mul_bs(y, bzzz)
    Pd = sub(F.mul_bs(bx, zz), U1)
    Rd = sub(F.mul_bs(by, zzz), S1)
    zz12 = F.mul_bs(zz, bzz)
    zzz12 = F.mul_bs(zzz, bzzz)
    PP = F.sqr(Pd)
    need(PP.is_S(), "add: PP must be S")
    zz3 = F.mul_bs(zz12, PP)
    PPP = F.mul_bs(Pd, PP)
    Q = F.mul_bs(U1, PP)
    zzz3 = F.mul_bs(zzz12, PPP)
    X3 = _x3(F, Rd, PPP, Q)
    t = sub(Q, X3, 16)
    Y3 = F.mul_sub(t, Rd, S1, PPP)
    # doubling branch: acc rewritten as (U1, S1, ZZZ1 ZZZ2, ZZ1 ZZ2), all S, then doubled
    dbl = trace_dbl(group, (U1, S1, zzz12, zz12))
    return (X3, Y3, zzz3, zz3), dbl


def trace_coop_add(group):
    """coop_xyzz_add (coop.hpp): the same add split over 4 waves, f_mul throughout"""
    F = Field(group)
    ax, ay, azzz, azz = Xc(), S(), S(), S()
    bx, by, bzzz, bzz = Xc(), S(), S(), S()
    U1, S1, U2, S2 = F.mul(ax, bzz), F.mul(ay, bzzz), F.mul(bx, azz), F.mul(by, azzz)
    Pd, Rd = sub(U2, U1), sub(S2, S1)
    PP, RR, zz12, zzz12 = F.mul(Pd, Pd), F.mul(Rd, Rd), F.mul(azz, bzz), F.mul(azzz, bzzz)
    need(PP.is_S() and RR.is_S(), "coop: PP, RR must be S")
    PPP, Q, zz3 = F.mul(Pd, PP), F.mul(U1, PP), F.mul(zz12, PP)
    zzz3 = F.mul(zzz12, PPP)
    X3 = norm(sub2x(RR, PPP, Q))
    t = sub(Q, X3, 16)
    Y3 = F.mul_sub(t, Rd, S1, PPP)
    return X3, Y3, zzz3, zz3


def prove_all():
    """Run every trace; returns {name: [outputs]} (each output must be class S)."""
    res = {}
    for g in (1, 2):
        for negate in (False, True):
            main, dbl = trace_madd(g, negate)
            res[f"G{g} xyzz_madd{' (neg)' if negate else ''}"] = list(main)
            res[f"G{g} xyzz_madd doubling branch{' (neg)' if negate else ''}"] = list(dbl)
        main, dbl = trace_add(g)
        res[f"G{g} xyzz_add"] = list(main)
        res[f"G{g} xyzz_add doubling branch"] = list(dbl)
        res[f"G{g} xyzz_dbl"] = list(trace_dbl(g))
        res[f"G{g} coop_xyzz_add"] = list(trace_coop_add(g))
    # G2 on lane pairs (fp2l.hpp): the same formulas over f_mul / f_mul_bs / f_mul_sub
    # of the one-lane Fp2 and a square split per lane
    for negate in (False, True):
        main, dbl = trace_madd(3, negate)
        res[f"G2-pairs xyzz_madd{' (neg)' if negate else ''}"] = list(main)
        res[f"G2-pairs xyzz_madd doubling branch{' (neg)' if negate else ''}"] = list(dbl)
    main, dbl = trace_add(3)
    res["G2-pairs xyzz_add"] = list(main)
    res["G2-pairs xyzz_add doubling branch"] = list(dbl)
    res["G2-pairs xyzz_dbl"] = list(trace_dbl(3))
    for name, outs in res.items():
        for k, o in enumerate(outs):
            if k == 0:
                need(o.is_X(), f"{name}: output x not in class X: {o}")
            else:
                need(o.is_S(), f"{name}: output {'x y zzz zz'.split()[k]} not in class S: {o}")
    return res


def red_report():
    """the fp_red bound for its two kinds of callers"""
    lazy14 = sub2x(S(), S(), S())   # shape of the X3 chain input (f_sub_2x)
    rows = []
    for name, x in (("X3 chain (< 10p, normalized)", norm(lazy14)),
                    ("normalized < 32p", Iv([M - 1] * NL, 32 * P - 1)),
                    ("m + m, limbs < 2^29 (Fp2 sqr)", add(S(), S()))):
        r = red(x)
        rows.append((name, x.vmax / P, r.vmax / P))
    return rows


if __name__ == "__main__":
    for name, outs in prove_all().items():
        print(f"{name:40s} " + "  ".join(f"{c}<{o.vmax / P:.4f}p" for c, o in zip("x y zzz zz".split(), outs)))
    for name, vin, vout in red_report():
        print(f"fp_red {name:36s} in < {vin:.3f}p -> out < {vout:.6f}p")
