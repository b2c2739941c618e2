"""GPU parity of blst's fixed-window MSM (ref src/multi_scalar.c:63-261,
blst.h:228-236 / :367-375) against the reference's own outputs
(tests/golden/wbits.json, written by make_wbits_golden.py from the reference
libblst): the precomputed table byte for byte (FNV of the rows) and the MSM
result, through the blst-named entry points and the resident-table context."""
import ctypes

import pytest

from test_oracle_golden import _fnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _inputs(m, c):
    g, n, nbits = c["group"], c["n"], c["nbits"]
    pts = bytearray(bytes(m.fixed_points(g, n)))
    raw = bytes(m.gen_scalars(n, c["seed"]))
    vals = [int.from_bytes(raw[32 * i:32 * i + 32], "little") & ((1 << nbits) - 1) for i in range(n)]
    if c["case"] == "inf":
        pts[3 * 96 * g:4 * 96 * g] = bytes(96 * g)
        vals[5] = 0
    nb = (nbits + 7) // 8
    return bytes(pts), b"".join(v.to_bytes(32, "little")[:nb] for v in vals), vals


def _cases(golden):
    return golden("wbits.json")["cases"]


def test_wbits_blst_entry_points_match_reference(m, golden):
    from msm_blst_amd import wbits as W
    for c in _cases(golden):
        g = c["group"]
        pts, sc, _ = _inputs(m, c)
        table = W.precompute(g, pts, c["n"], c["wbits"])
        assert _fnv(bytes(table)) == c["table_fnv"], c
        got = m.compress(g, W.mult(g, table, c["wbits"], c["n"], sc, c["nbits"]))
        assert got.hex() == c["compressed"], c


def test_wbits_context_resident_table(m, golden):
    for c in _cases(golden):
        if c["n"] > 1024:
            continue
        g = c["group"]
        pts, sc, vals = _inputs(m, c)
        ctx = m.WbitsContext(g, 0, c["wbits"])
        ctx.precompute(pts, c["n"])
        assert _fnv(bytes(ctx.get_table())) == c["table_fnv"]
        assert m.compress(g, ctx.mult(sc, c["nbits"])).hex() == c["compressed"]
        # 32-byte stride (wider than (nbits+7)/8) selects the same low nbits bits
        sc32 = b"".join(v.to_bytes(32, "little") for v in vals)
        assert m.compress(g, ctx.mult(sc32, c["nbits"], stride=32)).hex() == c["compressed"]
        # a table uploaded in the reference layout gives the same result
        ctx2 = m.WbitsContext(g, 0, c["wbits"])
        ctx2.set_table(bytes(ctx.get_table()), c["n"])
        assert m.compress(g, ctx2.mult(sc, c["nbits"])).hex() == c["compressed"]
        ctx.close()
        ctx2.close()


def test_wbits_in_place_precompute_and_pointer_rules(m, golden):
    """blst.hpp:383-393 calls precompute with the points stored at the end of the
    output table; scalars[] may be pointers with a NULL after k entries
    (ref multi_scalar.c:191: NULL continues after the previous scalar)."""
    L = m.lib()
    c = [c for c in _cases(golden) if c["group"] == 1 and c["n"] == 1024][0]
    n, wbits, nbits = c["n"], c["wbits"], c["nbits"]
    pts, sc, _ = _inputs(m, c)
    size = L.blst_p1s_mult_wbits_precompute_sizeof(wbits, n)
    table = (ctypes.c_uint8 * size)()
    ctypes.memmove(ctypes.byref(table, size - 96 * n), pts, 96 * n)
    pp = (ctypes.c_void_p * 2)(ctypes.addressof(table) + size - 96 * n, None)
    L.blst_p1s_mult_wbits_precompute(table, wbits, pp, n)
    assert _fnv(bytes(table)) == c["table_fnv"]
    nb = (nbits + 7) // 8
    S = (ctypes.c_uint8 * len(sc)).from_buffer_copy(sc)
    base = ctypes.addressof(S)
    ptrs = (ctypes.c_void_p * (n + 1))(*([base + i * nb for i in range(5)] + [None] * (n - 4)))
    ret = (ctypes.c_uint8 * 144)()
    L.blst_p1s_mult_wbits(ret, table, wbits, n, ptrs, nbits, None)
    assert m.compress(1, bytes(ret)).hex() == c["compressed"]
    assert L.blst_p1s_mult_wbits_scratch_sizeof(100) == 144 * 100
    assert L.blst_p1s_mult_wbits_scratch_sizeof(1 << 20) == 144 * 8192
    assert L.blst_p2s_mult_wbits_scratch_sizeof(1 << 20) == 288 * 4096


def test_error_mode_returns_infinity_instead_of_abort(m):
    """With msm_set_abort_on_error(0) a failing void entry point (wbits = 15 is
    outside blst's [2, 14]) returns the all-zero point and raises
    msm_error_pending() instead of aborting the process."""
    L = m.lib()
    prev = L.msm_set_abort_on_error(0)
    try:
        n = 4
        pts = bytes(m.fixed_points(1, n))
        table = (ctypes.c_uint8 * (96 * n * 2))()
        sc = bytes(m.gen_scalars(n, 1))
        ret = (ctypes.c_uint8 * 144)(*([0xAB] * 144))
        S = (ctypes.c_uint8 * len(sc)).from_buffer_copy(sc)
        sp = (ctypes.c_void_p * 2)(ctypes.cast(S, ctypes.c_void_p), None)
        L.blst_p1s_mult_wbits(ret, table, 15, n, sp, 255, None)
        assert bytes(ret) == bytes(144)
        assert L.msm_error_pending() == 1
        assert L.msm_error_pending() == 0
        assert b"wbits" in L.msm_last_error()
        # a failing precompute zeroes the caller's whole table (never half written)
        wb = 15
        tsz = L.blst_p1s_mult_wbits_precompute_sizeof(wb, n)
        big = (ctypes.c_uint8 * tsz)(*([0xCD] * tsz))
        P = (ctypes.c_uint8 * len(pts)).from_buffer_copy(pts)
        pp = (ctypes.c_void_p * 2)(ctypes.cast(P, ctypes.c_void_p), None)
        L.blst_p1s_mult_wbits_precompute(big, wb, pp, n)
        assert L.msm_error_pending() == 1
        assert bytes(big) == bytes(tsz)
    finally:
        L.msm_set_abort_on_error(prev)
