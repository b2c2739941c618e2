"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and the pinned CPU oracle.  Marked gpu; run on an MI355X."""
import ctypes
import struct

import pytest

import oracle_ffi as of
from test_oracle_golden import _limbs, _msm_cases, _prepare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m.lib()


def _u64s(hexes):
    vals = []
    for h in hexes:
        vals += _limbs(h)
    return (ctypes.c_uint64 * len(vals))(*vals)


def test_field_kat_g1(L, golden):
    vec = golden("fp_kat.json")["vectors"]
    n = len(vec)
    a = _u64s([v["a"] for v in vec])
    b = _u64s([v["b"] for v in vec])
    out = (ctypes.c_uint64 * (6 * n))()
    for op, key in ((0, "mul"), (1, "add"), (2, "sub")):
        assert L.msm_test_field(1, op, a, b, out, n) == 0
        for i, v in enumerate(vec):
            assert list(out[6 * i:6 * i + 6]) == _limbs(v[key]), (key, i)
    assert L.msm_test_field(1, 3, a, b, out, n) == 0
    for i, v in enumerate(vec):
        if v["a"] == v["b"]:
            assert list(out[6 * i:6 * i + 6]) == _limbs(v["mul"])


def test_field_fp2_vs_oracle(L):
    n = 257
    import random
    rnd = random.Random(5)
    P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
    vals = [rnd.randrange(P) for _ in range(4 * n)]
    vals[0] = 0
    vals[1] = P - 1
    def arr(xs):
        limbs = []
        for x in xs:
            limbs += [(x >> (64 * k)) & (2**64 - 1) for k in range(6)]
        return (ctypes.c_uint64 * len(limbs))(*limbs)
    a = arr(vals[:2 * n])
    b = arr(vals[2 * n:])
    out = (ctypes.c_uint64 * (12 * n))()
    for op in (0, 3):
        assert L.msm_test_field(2, op, a, b, out, n) == 0
        for i in range(n):
            r = (ctypes.c_uint64 * 12)()
            aa = (ctypes.c_uint64 * 12)(*a[12 * i:12 * i + 12])
            bb = (ctypes.c_uint64 * 12)(*(b[12 * i:12 * i + 12] if op == 0 else a[12 * i:12 * i + 12]))
            of.lib().or_fp2_mul(r, aa, bb)
            assert list(out[12 * i:12 * i + 12]) == list(r), (op, i)


def test_xyzz_kat_g1(L, golden):
    seqs = golden("xyzz_kat.json")["sequences"]
    pts = of.fixed_points(1, 8)
    ln = max(len(s["ops"]) for s in seqs)
    ops = []
    for s in seqs:
        o = [idx | (sg << 31) for idx, sg in s["ops"]]
        ops += o + [0xffffffff] * (ln - len(o))
    opsa = (ctypes.c_uint32 * len(ops))(*ops)
    out = (ctypes.c_uint8 * (2 * 144 * len(seqs)))()
    assert L.msm_test_xyzz(1, pts, 8, opsa, ln, len(seqs), out) == 0
    raw = bytes(out)
    for i, s in enumerate(seqs):
        j1 = raw[288 * i:288 * i + 144]
        j2 = raw[288 * i + 144:288 * i + 288]
        assert of.compress(1, (ctypes.c_uint8 * 144).from_buffer_copy(j1)) == s["compressed"], i
        assert of.compress(1, (ctypes.c_uint8 * 144).from_buffer_copy(j2)) == s["compressed_double"], i


def test_xyzz_edge_branches_g2(L):
    """P+P (doubling), P-P (infinity), -P-P through the G2 madd/add paths vs the oracle."""
    pts = of.fixed_points(2, 4)
    seqs = [[0, 0, 0], [0, 0 | 1 << 31, 0], [0 | 1 << 31, 0 | 1 << 31], [1, 2, 3, 1 << 31 | 2], [3, 3, 3, 3]]
    ln = max(len(s) for s in seqs)
    ops = []
    for s in seqs:
        ops += s + [0xffffffff] * (ln - len(s))
    opsa = (ctypes.c_uint32 * len(ops))(*ops)
    out = (ctypes.c_uint8 * (2 * 288 * len(seqs)))()
    assert L.msm_test_xyzz(2, pts, 4, opsa, ln, len(seqs), out) == 0
    raw = bytes(out)
    for i, s in enumerate(seqs):
        acc = of.buf(384)
        for o in s:
            of.lib().or_p2xyzz_dadd_affine(acc, acc, ctypes.byref(pts, 192 * (o & 0x7fffffff)), o >> 31)
        j = of.buf(288)
        of.lib().or_p2xyzz_to_jacobian(j, acc)
        want = of.compress(2, j)
        got = of.compress(2, (ctypes.c_uint8 * 288).from_buffer_copy(raw[576 * i:576 * i + 288]))
        assert got == want, i


@pytest.mark.parametrize("group,nmax", [(1, 4096), (2, 1024)])
def test_msm_blst_abi_matches_reference(L, golden, group, nmax):
    import msm_blst_amd as m
    mult = m.p1s_mult_pippenger if group == 1 else m.p2s_mult_pippenger
    seen = 0
    for c in _msm_cases(golden, group, nmax):
        pts, sc = _prepare(group, c)
        r = mult(pts, sc, c["n"], c["nbits"])
        assert m.compress(group, r).hex() == c["compressed"], c
        seen += 1
    assert seen > 10


def test_msm_ctx_window_sweep(L, golden):
    import msm_blst_amd as m
    c = [x for x in _msm_cases(golden, 1, 1000) if x["n"] == 1000 and x["case"] == "rand" and x["nbits"] == 255][0]
    pts, sc = _prepare(1, c)
    for w in (8, 10, 12, 13, 14, 15, 16, 17, 18):
        ctx = m.MSMContext(1, 0, w)
        ctx.set_points(pts, c["n"])
        r = ctx.mult(sc, c["nbits"], stride=32)
        assert m.compress(1, r).hex() == c["compressed"], w
        ctx.close()


@pytest.mark.parametrize("group,n", [(1, 1 << 16), (1, 1 << 20), (2, 1 << 16), (2, 1 << 20)])
def test_msm_large_vs_reference(L, golden, points, group, n):
    """configs[1] (G1 2^16) and configs[4] (G2 2^20, the Fp2 path) by plain Pippenger"""
    import msm_blst_amd as m
    want = [c for c in golden(f"msm_g{group}.json")["cases"] if c["n"] == n and c["seed"] == 1][0]["compressed"]
    pts = points(group, n)
    sc = m.gen_scalars(n, 1)
    ctx = m.MSMContext(group, 0, 16 if n >= (1 << 18) else 13)
    ctx.set_points(pts, n)
    r = ctx.mult(sc, 255)
    assert m.compress(group, r).hex() == want
    # second call on the same context (buffers reused) gives the same answer
    assert ctx.mult(sc, 255) == r or m.compress(group, ctx.mult(sc, 255)).hex() == want


R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def _times_p0(m, k):
    """k * P_0 (P_0 = fixed_points(1, 1)) by the CPU oracle, compressed."""
    p0 = of.fixed_points(1, 1)
    s = (ctypes.c_uint8 * 32).from_buffer_copy((k % R_ORDER).to_bytes(32, "little"))
    return of.compress(1, of.msm(1, p0, s, 1, 255, "naive"))


@pytest.mark.parametrize("n,kind", [(1 << 16, "pippenger"), (1 << 18, "pippenger"), (1 << 16, "ches")])
def test_sort_heavy_bucket_equal_scalars(L, n, kind):
    """Every scalar equal: each window's entries all land in ONE bucket, so one
    coarse bin holds n entries -- the fine sort's LDS-window overflow path
    (n = 2^16) and its unstaged fallback (n = 2^18, > BS_FINE_MAXW windows).
    Expected value by linearity: s * sum P_i = s (2^n - 1) P_0 (P_i = 2^i P_0)."""
    import msm_blst_amd as m
    s0 = int.from_bytes(bytes(m.gen_scalars(1, 77)), "little")
    sc = s0.to_bytes(32, "little") * n
    pts = m.fixed_points(1, n)
    if kind == "pippenger":
        ctx = m.MSMContext(1, 0, 16)
        ctx.set_points(pts, n)
        r = ctx.mult(sc, 255)
    else:
        ctx = m.CHESContext(1, 0, n_exp=16)
        ctx.build_table(pts, n)
        r = ctx.mult(sc)
    assert m.compress(1, r).hex() == _times_p0(m, s0 * ((1 << n) - 1))
    ctx.close()


def test_sort_heavy_bucket_mixed(L):
    """Half the scalars equal (one heavy bucket per window beside ~13-entry
    buckets): staged windows with entries past the LDS capacity."""
    import msm_blst_amd as m
    n = 1 << 17
    rnd = bytes(m.gen_scalars(n, 5))
    s0 = rnd[:32]
    sc = bytearray(rnd)
    for i in range(0, n, 2):
        sc[32 * i:32 * i + 32] = s0
    pts = m.fixed_points(1, n)
    ctx = m.MSMContext(1, 0, 16)
    ctx.set_points(pts, n)
    got = m.compress(1, ctx.mult(bytes(sc), 255)).hex()
    ctx.close()
    P = of.fixed_points(1, n)
    S = (ctypes.c_uint8 * len(sc)).from_buffer_copy(bytes(sc))
    assert got == of.compress(1, of.msm(1, P, S, n, 255, "pippenger"))
