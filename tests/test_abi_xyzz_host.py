"""CPU tests of the per-point blst_p*xyzz_* helpers the C ABI exports (host
code; ref src/ec_ops.h:642-785, multi_scalar.c:609-641), pinned by the
reference's own xyzz sequences (tests/golden/xyzz_kat.json: the same formula
sequence must give the identical xyzz representative, incl. the doubling and
P == -bucket branches)."""
import ctypes
import struct

import pytest

from test_oracle_golden import _limbs


@pytest.fixture(scope="module")
def L():
    import msm_blst_amd as m
    L = m.lib()
    vp = ctypes.c_void_p
    for g in (1, 2):
        getattr(L, f"blst_p{g}xyzz_dadd_affine").argtypes = [vp, vp, vp, ctypes.c_ubyte]
        getattr(L, f"blst_p{g}xyzz_dadd").argtypes = [vp, vp, vp]
        getattr(L, f"blst_p{g}xyzz_to_Jacobian").argtypes = [vp, vp]
        getattr(L, f"blst_p{g}_to_xyzz").argtypes = [vp, vp]
        getattr(L, f"blst_p{g}_bucket_CHES").argtypes = [vp, ctypes.c_int, vp, ctypes.c_ubyte]
        getattr(L, f"blst_p{g}s_mult_pippenger_scratch_sizeof_CHES").argtypes = [ctypes.c_size_t]
        getattr(L, f"blst_p{g}s_mult_pippenger_scratch_sizeof_CHES").restype = ctypes.c_size_t
    return L


def _compress(L, group, jac):
    out = (ctypes.c_uint8 * (48 * group))()
    getattr(L, f"msm_p{group}_compress")(out, jac)
    return bytes(out).hex()


def test_xyzz_sequences_match_reference_raw_limbs(L, golden):
    import msm_blst_amd as m
    pts = m.fixed_points(1, 8)
    for seq in golden("xyzz_kat.json")["sequences"]:
        acc = (ctypes.c_uint8 * 192)()
        for idx, sg in seq["ops"]:
            L.blst_p1xyzz_dadd_affine(acc, acc, ctypes.byref(pts, 96 * idx), sg)
        raw = struct.unpack("<24Q", bytes(acc))
        assert list(raw[0:6]) == _limbs(seq["x"])
        assert list(raw[6:12]) == _limbs(seq["y"])
        assert list(raw[12:18]) == _limbs(seq["zzz"])
        assert list(raw[18:24]) == _limbs(seq["zz"])
        j = (ctypes.c_uint8 * 144)()
        L.blst_p1xyzz_to_Jacobian(j, acc)
        assert _compress(L, 1, j) == seq["compressed"]
        acc2 = (ctypes.c_uint8 * 192)()
        L.blst_p1xyzz_dadd(acc2, acc2, acc)
        L.blst_p1xyzz_dadd(acc2, acc2, acc)
        L.blst_p1xyzz_to_Jacobian(j, acc2)
        assert _compress(L, 1, j) == seq["compressed_double"]
        # Jacobian -> xyzz -> Jacobian keeps the point
        x = (ctypes.c_uint8 * 192)()
        L.blst_p1_to_xyzz(x, j)
        j2 = (ctypes.c_uint8 * 144)()
        L.blst_p1xyzz_to_Jacobian(j2, x)
        assert _compress(L, 1, j2) == seq["compressed_double"]


def test_bucket_ches_and_g2_helpers_vs_msm(L):
    """bucket[k] += +-P through blst_p2_bucket_CHES equals the G2 MSM of +-1 scalars."""
    import msm_blst_amd as m
    import oracle_ffi as of
    n = 16
    pts = m.fixed_points(2, n)
    buckets = (ctypes.c_uint8 * (384 * 3))()
    signs = [(i * 7) % 3 == 0 for i in range(n)]
    for i in range(n):
        L.blst_p2_bucket_CHES(buckets, 1 + (i % 2), ctypes.byref(pts, 192 * i), int(signs[i]))
    tot = (ctypes.c_uint8 * 384)()
    L.blst_p2xyzz_dadd(tot, ctypes.byref(buckets, 384), ctypes.byref(buckets, 768))
    j = (ctypes.c_uint8 * 288)()
    L.blst_p2xyzz_to_Jacobian(j, tot)
    R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    sc = b"".join(((R - 1) if s else 1).to_bytes(32, "little") for s in signs)
    S = (ctypes.c_uint8 * len(sc)).from_buffer_copy(sc)
    assert _compress(L, 2, j) == of.compress(2, of.msm(2, pts, S, n, 255, "naive"))


def test_scratch_sizeof_ches(L):
    assert L.blst_p1s_mult_pippenger_scratch_sizeof_CHES(1 << 13) == 192 * (1 << 12)
    assert L.blst_p2s_mult_pippenger_scratch_sizeof_CHES(1 << 13) == 384 * (1 << 12)
