"""GPU parity of the blst pointer-array inputs whose elements are NOT one
contiguous range -- the gather path of abi.cpp `contiguous()` (the reference's
iteration rule, multi_scalar.c:390-416 / :136 / :191: the first pointer is
taken, a non-NULL entry names the next element, a NULL continues right after
the previous one).  Real callers build such arrays: Go's []*P1Affine pointing
at separately allocated points (blst.go:2019-2049), permuted arrays, or a few
explicit pointers into one buffer followed by NULL and a second buffer.

Cases: every element through its own pointer into a shuffled copy of the
inputs; and two buffers -- explicit adjacent pointers into buffer A, one
explicit pointer into buffer B, then NULL (the rest continues in B).  Entry
points: blst_p{1,2}s_mult_pippenger (against the golden), blst_p1s_tile_pippenger,
blst_p1s_add and blst_p1s_mult_wbits[_precompute] (against the same call with
flat {ptr, NULL} arrays)."""
import ctypes
import random

import pytest

from test_oracle_golden import _prepare

pytestmark = pytest.mark.gpu

vp = ctypes.c_void_p


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _case(golden, group, n):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == 1 and c["nbits"] == 255 and c["case"] == "rand"][0]


def _shuffled(raw, sz, n, seed):
    """(keep-alive buffer, pointer array): element i lives at slot perm[i] of a
    permuted copy, so consecutive pointers are never adjacent."""
    perm = list(range(n))
    random.Random(seed).shuffle(perm)
    buf = (ctypes.c_uint8 * (sz * n))()
    for i in range(n):
        ctypes.memmove(ctypes.addressof(buf) + sz * perm[i], raw[sz * i:sz * (i + 1)], sz)
    return buf, (vp * n)(*[ctypes.addressof(buf) + sz * perm[i] for i in range(n)])


def _two_buffers(raw, sz, n, k):
    """elements 0..k-1 in buffer A (explicit adjacent pointers), elements k..n-1
    in buffer B: one explicit pointer to B[0], then NULL (continue after it)."""
    A = (ctypes.c_uint8 * (sz * k)).from_buffer_copy(raw[:sz * k])
    B = (ctypes.c_uint8 * (sz * (n - k))).from_buffer_copy(raw[sz * k:sz * n])
    ptrs = [ctypes.addressof(A) + sz * i for i in range(k)] + [ctypes.addressof(B), None]
    return (A, B), (vp * len(ptrs))(*ptrs)


def _flat(raw):
    buf = (ctypes.c_uint8 * len(raw)).from_buffer_copy(raw)
    return buf, (vp * 2)(ctypes.addressof(buf), None)


@pytest.mark.parametrize("group,n", [(1, 1024), (2, 256)])
@pytest.mark.parametrize("layout", ["shuffled", "two_buffers"])
def test_mult_pippenger_gathered_pointers(m, golden, group, n, layout):
    c = _case(golden, group, n)
    pts, sc = _prepare(group, c)
    P, S = bytes(pts), bytes(sc)
    if layout == "shuffled":
        kp, pp = _shuffled(P, 96 * group, n, 1)
        ks, sp = _shuffled(S, 32, n, 2)
    else:
        kp, pp = _two_buffers(P, 96 * group, n, 37)
        ks, sp = _two_buffers(S, 32, n, 5)
    ret = (ctypes.c_uint8 * (144 * group))()
    getattr(m.lib(), f"blst_p{group}s_mult_pippenger")(ret, pp, n, sp, 255, None)
    assert m.compress(group, bytes(ret)).hex() == c["compressed"]
    del kp, ks


def test_tile_and_points_add_gathered_pointers(m, golden):
    n = 1024
    c = _case(golden, 1, n)
    pts, sc = _prepare(1, c)
    P, S = bytes(pts), bytes(sc)
    L = m.lib()
    fp, fpp = _flat(P)
    fs, fsp = _flat(S)
    for layout in ("shuffled", "two_buffers"):
        if layout == "shuffled":
            kp, pp = _shuffled(P, 96, n, 3)
            ks, sp = _shuffled(S, 32, n, 4)
        else:
            kp, pp = _two_buffers(P, 96, n, 100)
            ks, sp = _two_buffers(S, 32, n, 1)
        for bit0, w in ((0, 9), (120, 13), (250, 8)):
            a, b = (ctypes.c_uint8 * 144)(), (ctypes.c_uint8 * 144)()
            L.blst_p1s_tile_pippenger(a, pp, n, sp, 255, None, bit0, w)
            L.blst_p1s_tile_pippenger(b, fpp, n, fsp, 255, None, bit0, w)
            assert m.compress(1, bytes(a)) == m.compress(1, bytes(b)), (layout, bit0, w)
        a, b = (ctypes.c_uint8 * 144)(), (ctypes.c_uint8 * 144)()
        L.blst_p1s_add(a, pp, n)
        L.blst_p1s_add(b, fpp, n)
        assert m.compress(1, bytes(a)) == m.compress(1, bytes(b)), layout
        del kp, ks


def test_wbits_gathered_pointers(m, golden):
    c = [c for c in golden("wbits.json")["cases"] if c["group"] == 1 and c["n"] == 1024 and c["case"] != "inf"][0]
    n, wbits, nbits = c["n"], c["wbits"], c["nbits"]
    L = m.lib()
    P = bytes(m.fixed_points(1, n))
    raw = bytes(m.gen_scalars(n, c["seed"]))
    nb = (nbits + 7) // 8
    S = b"".join((int.from_bytes(raw[32 * i:32 * i + 32], "little") & ((1 << nbits) - 1)).to_bytes(32, "little")[:nb]
                 for i in range(n))
    size = L.blst_p1s_mult_wbits_precompute_sizeof(wbits, n)
    fp, fpp = _flat(P)
    ref_table = (ctypes.c_uint8 * size)()
    L.blst_p1s_mult_wbits_precompute(ref_table, wbits, fpp, n)
    for layout in ("shuffled", "two_buffers"):
        if layout == "shuffled":
            kp, pp = _shuffled(P, 96, n, 5)
            ks, sp = _shuffled(S, nb, n, 6)
        else:
            kp, pp = _two_buffers(P, 96, n, 64)
            ks, sp = _two_buffers(S, nb, n, 3)
        table = (ctypes.c_uint8 * size)()
        L.blst_p1s_mult_wbits_precompute(table, wbits, pp, n)
        assert bytes(table) == bytes(ref_table), layout
        ret = (ctypes.c_uint8 * 144)()
        L.blst_p1s_mult_wbits(ret, table, wbits, n, sp, nbits, None)
        assert m.compress(1, bytes(ret)).hex() == c["compressed"], layout
        del kp, ks
