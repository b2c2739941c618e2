"""Range invariants of the lazy-reduction field arithmetic (fp.hpp / ec.hpp),
proven and then exercised at their bounds on the CPU (no GPU needed).

1. tests/fp_bounds.py proves by exact interval arithmetic that no 64-bit
   column, 32-bit limb or signed reduction can wrap for the operand ranges the
   point formulas produce, that fp_red (checked exhaustively over its top
   limb) leaves a value in [0, 2p), and that every stored coordinate of every
   formula (G1, G2, main and doubling branches, the 4-wave cooperative add) is
   in range class S, except x, which is in class X (normalized, < 10p).  DESIGN.md section 4a records the same table.
2. The SAME header text (msm_blst_amd/csrc/fp.hpp, ec.hpp) is compiled for the
   host with every range check enabled (tests/host/fp_host_shim.cpp,
   MSM_FP_HOST_TEST) and run on max-limb operands of every range class and on
   max-limb point coordinates, against Python big-integer arithmetic.  The
   G2 lane-pair arithmetic (fp2l.hpp) runs the same way on two host threads in
   lockstep standing in for the two lanes (pair_swap through the shim).
"""
import ctypes
import os
import random
import subprocess

import pytest

import fp_bounds as fb

HERE = os.path.dirname(os.path.abspath(__file__))
SHIM_SRC = os.path.join(HERE, "host", "fp_host_shim.cpp")
SHIM_SO = os.path.join(HERE, "host", "_build", "fp_host_shim.so")
P = fb.P
RINV = pow(fb.R, -1, P)
NL = 14
M28 = (1 << 28) - 1


@pytest.fixture(scope="module")
def shim():
    deps = [SHIM_SRC] + [os.path.join(os.path.dirname(HERE), "msm_blst_amd", "csrc", f)
                         for f in ("fp.hpp", "ec.hpp", "fp2l.hpp")]
    if not os.path.exists(SHIM_SO) or any(os.path.getmtime(d) > os.path.getmtime(SHIM_SO) for d in deps):
        os.makedirs(os.path.dirname(SHIM_SO), exist_ok=True)
        subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", "-Wno-unknown-pragmas",
                        "-o", SHIM_SO, SHIM_SRC], check=True)
    L = ctypes.CDLL(SHIM_SO)
    vp = ctypes.c_void_p
    L.h_fp_op.argtypes = [ctypes.c_int] + [vp] * 9
    L.h_fp2_op.argtypes = [ctypes.c_int] + [vp] * 5
    L.h_xyzz.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int]
    L.h_fp2l_op.argtypes = [ctypes.c_int] + [vp] * 5
    L.h_xyzz_l.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int]
    L.h_overflow.argtypes = [ctypes.c_int]
    return L


def test_interval_model_proves_every_formula():
    res = fb.prove_all()
    assert len(res) == 16 + 7  # G1, G2 (one lane), G2 on lane pairs
    for name, outs in res.items():
        assert outs[0].is_X() and all(o.is_S() for o in outs[1:]), name


def test_fp_red_exhaustive_bound():
    """fp.hpp's fp_red claim: v - q p in [0, 1.0003 p) for normalized v < 32 p, and the
    non-normalized m + m of the Fp2 square (limbs < 2^29)."""
    for name, vin, vout in fb.red_report():
        assert vout < 1.0003, (name, vout)


def test_model_rejects_an_overflowing_schedule():
    """The model is not vacuous: the previous Fp2 square schedule (lazy components
    added and subtracted without normalizing, 32p offset) overflows a column."""
    lazy = fb.sub(fb.S(), fb.S())                    # P = U2 - X1: limbs < 3 2^28, < 6p
    s = fb.add(lazy, lazy)
    d = fb.sub(lazy, fb.norm(lazy), 32)
    with pytest.raises(fb.RangeError):
        fb.mul(s, d)


# ----------------------------------------------------------- host runs ----
def _limbs(v, n=NL):
    return [(v >> (28 * i)) & M28 for i in range(n - 1)] + [v >> (28 * (n - 1))]


def _val(lim):
    return sum(int(l) << (28 * i) for i, l in enumerate(lim))


def _maxlimb(iv, rnd=None):
    """the representative with every low limb at its class maximum (or random
    below it) and the largest top limb the value bound allows"""
    low = [iv.lim[i] if rnd is None else rnd.randrange(iv.lim[i] // 2, iv.lim[i] + 1) for i in range(NL - 1)]
    lowv = _val(low + [0])
    top = min(iv.lim[NL - 1], (iv.vmax - lowv) >> 364)
    return low + [top]


def _arr(words):
    return (ctypes.c_uint32 * len(words))(*words)


def _run_fp(shim, op, *args):
    r = (ctypes.c_uint32 * NL)()
    ins = [_arr(a) for a in args] + [None] * (8 - len(args))
    shim.h_fp_op(op, r, *ins)
    return list(r)


def _mont(*pairs):
    return sum(_val(a) * _val(b) for a, b in pairs) * RINV % P


@pytest.mark.parametrize("seed", [None, 1, 2, 3])
def test_fp_primitives_at_class_bounds(shim, seed):
    rnd = random.Random(seed) if seed is not None else None
    S = _maxlimb(fb.S(), rnd)
    lazy = _maxlimb(fb.sub(fb.S(), fb.S()), rnd)         # < 6p, limbs < 3 2^28 (U2 - X1 etc.)
    lazy14 = _maxlimb(fb.norm(fb.sub(fb.norm(fb.sub(fb.norm(fb.sub(fb.S(), fb.S())), fb.S())), fb.S())), rnd)
    c = _maxlimb(fb.canonical(), rnd)
    negS = [a - b for a, b in zip(fb.SUB[4], S)]
    shim.h_overflow(1)
    cases = [
        (0, (lazy, S), _mont((lazy, S))),
        (0, (lazy, lazy), _mont((lazy, lazy))),
        (1, (lazy,), _mont((lazy, lazy))),
        (1, (_maxlimb(fb.mul3(fb.S()), rnd),), None),
        (2, (lazy, lazy, S, negS), _mont((lazy, lazy), (S, negS))),
        (9, (lazy, lazy, S, S), (_val(lazy) * _val(lazy) - _val(S) * _val(S)) * RINV % P),
        (6, (lazy, S), (_val(lazy) - _val(S)) % P),
        (5, (lazy14,), _val(lazy14) % P),
        (4, (_maxlimb(fb.Iv([M28] * NL, 32 * P - 1), rnd),), None),
        (10, (S, S, S), (_val(S) - 3 * _val(S)) % P),                     # X3 line: R^2 - PPP - 2Q
        (11, (S, _maxlimb(fb.Xc(), rnd)), None),                          # P = U2 - X1, X1 in class X
    ]
    for op, args, want in cases:
        r = _run_fp(shim, op, *args)
        assert shim.h_overflow(1) == 0, (op, args)
        if op == 6:
            assert _val(r) < 10 * P   # lazy (< 6p) + 4p - S
        elif op in (10, 11):
            assert all(x < (1 << 31) for x in r) and _val(r) < 18 * P, op   # lazy, limbs < 2^31
        else:  # products and reductions land in class S
            assert all(x <= M28 for x in r[:NL - 1]) and _val(r) < 2 * P, op
        if want is None:
            want = {1: lambda: _mont((args[0], args[0])), 4: lambda: _val(args[0]) % P,
                    11: lambda: (_val(args[0]) - _val(args[1])) % P}[op]()
        assert _val(r) % P == want, op
    # c (canonical affine) enters as the first operand of the madd products
    r = _run_fp(shim, 0, c, S)
    assert shim.h_overflow(1) == 0 and _val(r) % P == _mont((c, S))


def _fp2_mont(a, b):
    a0, a1, b0, b1 = _val(a[:NL]), _val(a[NL:]), _val(b[:NL]), _val(b[NL:])
    return (a0 * b0 - a1 * b1) * RINV % P, (a0 * b1 + a1 * b0) * RINV % P


@pytest.mark.parametrize("seed", [None, 5, 6])
def test_fp2_primitives_at_class_bounds(shim, seed):
    rnd = random.Random(seed) if seed is not None else None
    S2 = _maxlimb(fb.S(), rnd) + _maxlimb(fb.S(), rnd)
    lazy2 = _maxlimb(fb.sub(fb.S(), fb.S()), rnd) + _maxlimb(fb.sub(fb.S(), fb.S()), rnd)
    # P = U2 - X1 with X1 in class X: < 18p, the widest square input
    lazy18 = _maxlimb(fb.sub(fb.S(), fb.Xc(), 16), rnd) + _maxlimb(fb.sub(fb.S(), fb.Xc(), 16), rnd)
    shim.h_overflow(1)
    for op, a, b in ((0, lazy2, lazy2), (1, lazy2, lazy2), (2, lazy2, S2), (1, lazy18, lazy18), (2, lazy18, S2)):
        r = (ctypes.c_uint32 * (2 * NL))()
        shim.h_fp2_op(op, r, _arr(a), _arr(b), None, None)
        assert shim.h_overflow(1) == 0, op
        r = list(r)
        assert all(x <= M28 for x in r[:NL - 1] + r[NL:2 * NL - 1]), op
        assert _val(r[:NL]) < 2 * P and _val(r[NL:]) < 2 * P, op
        want = _fp2_mont(a, a if op == 1 else b)
        assert (_val(r[:NL]) % P, _val(r[NL:]) % P) == want, op
    # f_mul_sub: a b - c d
    r = (ctypes.c_uint32 * (2 * NL))()
    shim.h_fp2_op(3, r, _arr(lazy2), _arr(lazy2), _arr(S2), _arr(S2))
    assert shim.h_overflow(1) == 0
    ab, cd = _fp2_mont(lazy2, lazy2), _fp2_mont(S2, S2)
    assert (_val(list(r)[:NL]) % P, _val(list(r)[NL:]) % P) == ((ab[0] - cd[0]) % P, (ab[1] - cd[1]) % P)


@pytest.mark.parametrize("seed", [None, 7, 8])
def test_fp2l_lane_pair_primitives_at_class_bounds(shim, seed):
    """fp2l.hpp's f_mul / f_sqr / f_mul_bs / f_mul_sub: each lane computes one
    component from operands selected through pair_swap (its own products, e.g.
    the odd lane's c1 = a0 (2 a1) in f_sqr), checked like the Fp2 versions."""
    rnd = random.Random(seed) if seed is not None else None
    S2 = _maxlimb(fb.S(), rnd) + _maxlimb(fb.S(), rnd)
    lazy2 = _maxlimb(fb.sub(fb.S(), fb.S()), rnd) + _maxlimb(fb.sub(fb.S(), fb.S()), rnd)
    lazy18 = _maxlimb(fb.sub(fb.S(), fb.Xc(), 16), rnd) + _maxlimb(fb.sub(fb.S(), fb.Xc(), 16), rnd)
    shim.h_overflow(1)
    for op, a, b in ((0, lazy2, lazy2), (1, lazy2, lazy2), (2, lazy2, S2), (1, lazy18, lazy18), (2, lazy18, S2)):
        r = (ctypes.c_uint32 * (2 * NL))()
        shim.h_fp2l_op(op, r, _arr(a), _arr(b), None, None)
        assert shim.h_overflow(1) == 0, op
        r = list(r)
        assert all(x <= M28 for x in r[:NL - 1] + r[NL:2 * NL - 1]), op
        assert _val(r[:NL]) < 2 * P and _val(r[NL:]) < 2 * P, op
        assert (_val(r[:NL]) % P, _val(r[NL:]) % P) == _fp2_mont(a, a if op == 1 else b), op
    r = (ctypes.c_uint32 * (2 * NL))()
    shim.h_fp2l_op(3, r, _arr(lazy2), _arr(lazy2), _arr(S2), _arr(S2))
    assert shim.h_overflow(1) == 0
    ab, cd = _fp2_mont(lazy2, lazy2), _fp2_mont(S2, S2)
    assert (_val(list(r)[:NL]) % P, _val(list(r)[NL:]) % P) == ((ab[0] - cd[0]) % P, (ab[1] - cd[1]) % P)


# ---- the xyzz formulas on max-limb coordinates vs the same algebra mod p ----
class _F:
    """Montgomery-domain field algebra mod p (R = 2^392) for G1 (ints) / G2 (pairs)"""

    def __init__(self, g):
        self.g = g

    def mul(self, a, b):
        if self.g == 1:
            return a * b * RINV % P
        return ((a[0] * b[0] - a[1] * b[1]) * RINV % P, (a[0] * b[1] + a[1] * b[0]) * RINV % P)

    def add(self, a, b):
        return (a + b) % P if self.g == 1 else ((a[0] + b[0]) % P, (a[1] + b[1]) % P)

    def sub(self, a, b):
        return (a - b) % P if self.g == 1 else ((a[0] - b[0]) % P, (a[1] - b[1]) % P)

    def neg(self, a):
        return self.sub(self.zero(), a)

    def zero(self):
        return 0 if self.g == 1 else (0, 0)


def _ref_madd(F, acc, p, neg):
    X1, Y1, ZZZ1, ZZ1 = acc
    x2, y2 = p
    if neg:
        y2 = F.neg(y2)
    Pd = F.sub(F.mul(x2, ZZ1), X1)
    Rd = F.sub(F.mul(y2, ZZZ1), Y1)
    PP = F.mul(Pd, Pd)
    PPP = F.mul(Pd, PP)
    Q = F.mul(X1, PP)
    X3 = F.sub(F.sub(F.mul(Rd, Rd), PPP), F.add(Q, Q))
    Y3 = F.sub(F.mul(Rd, F.sub(Q, X3)), F.mul(Y1, PPP))
    return X3, Y3, F.mul(ZZZ1, PPP), F.mul(ZZ1, PP)


def _ref_add(F, a, b):
    X1, Y1, ZZZ1, ZZ1 = a
    X2, Y2, ZZZ2, ZZ2 = b
    U1, S1 = F.mul(X1, ZZ2), F.mul(Y1, ZZZ2)
    Pd, Rd = F.sub(F.mul(X2, ZZ1), U1), F.sub(F.mul(Y2, ZZZ1), S1)
    PP = F.mul(Pd, Pd)
    PPP = F.mul(Pd, PP)
    Q = F.mul(U1, PP)
    X3 = F.sub(F.sub(F.mul(Rd, Rd), PPP), F.add(Q, Q))
    Y3 = F.sub(F.mul(Rd, F.sub(Q, X3)), F.mul(S1, PPP))
    return X3, Y3, F.mul(F.mul(ZZZ1, ZZZ2), PPP), F.mul(F.mul(ZZ1, ZZ2), PP)


def _ref_dbl(F, a):
    X, Y, ZZZ, ZZ = a
    U = F.add(Y, Y)
    V = F.mul(U, U)
    W = F.mul(U, V)
    Sx = F.mul(X, V)
    XX = F.mul(X, X)
    Mm = F.add(F.add(XX, XX), XX)
    X3 = F.sub(F.mul(Mm, Mm), F.add(Sx, Sx))
    Y3 = F.sub(F.mul(Mm, F.sub(Sx, X3)), F.mul(W, Y))
    return X3, Y3, F.mul(W, ZZZ), F.mul(V, ZZ)


def _elem(g, rnd, iv):
    if g == 1:
        return _maxlimb(iv, rnd)
    return _maxlimb(iv, rnd) + _maxlimb(iv, rnd)


def _dec(g, words):
    if g == 1:
        return _val(words) % P
    return (_val(words[:NL]) % P, _val(words[NL:]) % P)


def _check_S(g, words, bound=2):
    for k in range(g):
        w = words[k * NL:(k + 1) * NL]
        assert all(x <= M28 for x in w[:NL - 1]) and _val(w) < bound * P


@pytest.mark.parametrize("group", [1, 2])
@pytest.mark.parametrize("seed", [None, 11, 12, 13])
def test_xyzz_formulas_at_class_bounds(shim, group, seed):
    rnd = random.Random(seed) if seed is not None else None
    F = _F(group)
    W = NL * group
    # seed None: x at the exact class maximum, the other coordinates near it (equal
    # coordinates everywhere would make P = 0, the doubling/infinity branch)
    r2 = rnd or random.Random(98)
    # x in class X (normalized, < 10p: the stored x is not reduced), the rest in S
    acc = [_elem(group, rnd, fb.Xc())] + [_elem(group, r2, fb.S()) for _ in range(3)]
    # (the second operand of the add must differ from acc, else the doubling branch runs)
    r3 = rnd or random.Random(99)
    oth = [_elem(group, r3, fb.Xc())] + [_elem(group, r3, fb.S()) for _ in range(3)]
    pt = [_elem(group, rnd, fb.canonical()) for _ in range(2)]
    dec = lambda ws: tuple(_dec(group, w) for w in ws)  # noqa: E731
    shim.h_overflow(1)
    for op, neg in ((0, 0), (0, 1), (1, 0), (2, 0)):
        a = _arr(sum(acc, []))
        other = _arr(sum(pt if op == 0 else oth, []))
        shim.h_xyzz(group, op, a, other, neg)
        assert shim.h_overflow(1) == 0, (op, neg)
        out = list(a)
        coords = [out[k * W:(k + 1) * W] for k in range(4)]
        _check_S(group, coords[0], 10)
        for c in coords[1:]:
            _check_S(group, c)
        if op == 0:
            want = _ref_madd(F, dec(acc), dec(pt), neg)
        elif op == 1:
            want = _ref_add(F, dec(acc), dec(oth))
        else:
            want = _ref_dbl(F, dec(acc))
        assert dec(coords) == want, (op, neg)


@pytest.mark.parametrize("seed", [None, 21, 22])
def test_xyzz_lane_pair_formulas_at_class_bounds(shim, seed):
    """ec.hpp's madd / add / dbl on Fp2L (the G2 accumulation and reduction
    kernels' arithmetic), two lockstep host threads as the lane pair."""
    group = 2
    rnd = random.Random(seed) if seed is not None else None
    F = _F(group)
    W = NL * group
    r2 = rnd or random.Random(96)
    acc = [_elem(group, rnd, fb.Xc())] + [_elem(group, r2, fb.S()) for _ in range(3)]
    r3 = rnd or random.Random(97)
    oth = [_elem(group, r3, fb.Xc())] + [_elem(group, r3, fb.S()) for _ in range(3)]
    pt = [_elem(group, rnd, fb.canonical()) for _ in range(2)]
    dec = lambda ws: tuple(_dec(group, w) for w in ws)  # noqa: E731
    shim.h_overflow(1)
    for op, neg in ((0, 0), (0, 1), (1, 0), (2, 0)):
        a = _arr(sum(acc, []))
        other = _arr(sum(pt if op == 0 else oth, []))
        shim.h_xyzz_l(op, a, other, neg)
        assert shim.h_overflow(1) == 0, (op, neg)
        out = list(a)
        coords = [out[k * W:(k + 1) * W] for k in range(4)]
        _check_S(group, coords[0], 10)
        for c in coords[1:]:
            _check_S(group, c)
        want = (_ref_madd(F, dec(acc), dec(pt), neg) if op == 0 else
                _ref_add(F, dec(acc), dec(oth)) if op == 1 else _ref_dbl(F, dec(acc)))
        assert dec(coords) == want, (op, neg)
