"""Registered host points behind the plain blst drop-in (ref multi_scalar.c:549-607
blst_p{1,2}s_mult_pippenger, :383-419 _tile_pippenger).

A caller that multiplies the same point array again and again (an SRS)
registers it once with msm_register_host_table (include/msm_mi355x.h); a flat
{ptr, NULL} call whose points lie inside a registered table then reads the
device copy instead of uploading 96 G bytes per point (abi.cpp
registered_rows).  Results must equal the unregistered calls and the goldens,
for the whole array, a sub-range at an offset, and a range running past the
registered rows (which falls back to the upload)."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


def _golden(golden, group, n, seed=1):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["case"] == "rand" and c["nbits"] == 255][0]["compressed"]


def _mult(m, group, base, n, sc):
    L = m.lib()
    pp = (ctypes.c_void_p * 2)(base, None)
    spp = (ctypes.c_void_p * 2)(ctypes.cast(sc, ctypes.c_void_p), None)
    r = (ctypes.c_uint8 * (144 * group))()
    getattr(L, f"blst_p{group}s_mult_pippenger")(r, pp, n, spp, 255, None)  # aborts on an error (blst has no code)
    return m.compress(group, bytes(r)).hex()


def _tile(m, group, base, n, sc, bit0, window):
    L = m.lib()
    pp = (ctypes.c_void_p * 2)(base, None)
    spp = (ctypes.c_void_p * 2)(ctypes.cast(sc, ctypes.c_void_p), None)
    r = (ctypes.c_uint8 * (144 * group))()
    getattr(L, f"blst_p{group}s_tile_pippenger")(r, pp, n, spp, 255, None, bit0, window)
    return m.compress(group, bytes(r)).hex()


@pytest.mark.parametrize("group,n", [(1, 4096), (2, 1024)])
def test_registered_points_dropin(golden, points, group, n):
    import msm_blst_amd as m
    L = m.lib()
    big = points(group, 2 * n)  # 2n points; the golden is over the first n
    P = (ctypes.c_uint8 * len(big)).from_buffer_copy(big)
    base = ctypes.addressof(P)
    psz = 96 * group
    sc = (ctypes.c_uint8 * (32 * n)).from_buffer_copy(m.gen_scalars(n, 1))
    off = n // 4
    want_full = _golden(golden, group, n)
    want_off = _mult(m, group, base + off * psz, n, sc)  # unregistered: uploads the points
    want_tail = _mult(m, group, base + (n + off) * psz, n - off, sc)
    want_tile = _tile(m, group, base, n, sc, 16, 8)
    assert _mult(m, group, base, n, sc) == want_full
    assert L.msm_register_host_table(group, P, 2 * n) == 0, L.msm_last_error()
    try:
        for _ in range(2):
            assert _mult(m, group, base, n, sc) == want_full
            assert _mult(m, group, base + off * psz, n, sc) == want_off
            assert _mult(m, group, base + (n + off) * psz, n - off, sc) == want_tail  # ends at the last row
            assert _tile(m, group, base, n, sc, 16, 8) == want_tile
        # a range past the registered rows falls back to the upload
        assert L.msm_unregister_host_table(P) == 0
        assert L.msm_register_host_table(group, P, n) == 0
        assert _mult(m, group, base + off * psz, n, sc) == want_off
    finally:
        L.msm_unregister_host_table(P)
    assert _mult(m, group, base, n, sc) == want_full


@pytest.mark.parametrize("group,n", [(1, 4096), (2, 1024)])
def test_registered_rows_edited_between_calls(golden, points, group, n):
    """The staleness guard (row_samples.hpp, ADVICE/VERDICT r05): the reference
    reads the caller's points on every call (ref multi_scalar.c:549-607), so a
    registered array whose rows change between calls must give the MSM of the
    NEW rows.  Edits of a sampled row (the first and the last row are always
    sampled) and a wholesale rewrite of the buffer (a reused allocation) are
    each followed by a call that must equal the oracle's MSM of the edited
    points; restoring the rows gives the golden again."""
    import oracle_ffi as of

    import msm_blst_amd as m
    L = m.lib()
    psz = 96 * group
    orig = bytes(points(group, n + 1))
    P = (ctypes.c_uint8 * (psz * n)).from_buffer_copy(orig[:psz * n])
    base = ctypes.addressof(P)
    sc = (ctypes.c_uint8 * (32 * n)).from_buffer_copy(m.gen_scalars(n, 1))
    want = _golden(golden, group, n)

    def oracle_of(buf):
        return of.compress(group, of.msm(group, buf, sc, n))

    assert L.msm_register_host_table(group, P, n) == 0, L.msm_last_error()
    try:
        assert _mult(m, group, base, n, sc) == want
        for row in (0, n - 1):  # one row edited in place: the point of row (row + 1) % n
            src = ((row + 1) % n) * psz
            ctypes.memmove(base + row * psz, orig[src:src + psz], psz)
            assert _mult(m, group, base, n, sc) == oracle_of(P)
            ctypes.memmove(base + row * psz, orig[row * psz:(row + 1) * psz], psz)
            assert _mult(m, group, base, n, sc) == want
        # the whole buffer reused for another point set: P_1 .. P_n
        ctypes.memmove(base, orig[psz:psz * (n + 1)], psz * n)
        assert _mult(m, group, base, n, sc) == oracle_of(P)
        assert _tile(m, group, base, n, sc, 16, 8) == _tile_unregistered(m, group, P, n, sc, 16, 8)
    finally:
        L.msm_unregister_host_table(P)


def _tile_unregistered(m, group, P, n, sc, bit0, window):
    """the same tile over a private copy of the rows (never registered)"""
    Q = (ctypes.c_uint8 * len(P)).from_buffer_copy(bytes(P))
    return _tile(m, group, ctypes.addressof(Q), n, sc, bit0, window)
