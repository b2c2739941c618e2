"""GPU parity of the blst-level CHES / BGMW95 entry points (ref
bindings/blst.h:249-357) driven the way the reference's driver drives them
(ref main_p1.cpp:192-291, :294-398) at the n = 2^10 configuration
(q = 2^13, h = 20; BGMW95 q = 2^12, h = 22), against the reference's own
driver results (tests/golden/ches_driver_n10.json)."""
import ctypes

import pytest

import oracle_ffi as of

pytestmark = pytest.mark.gpu

vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


@pytest.fixture(scope="module")
def env(golden):
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    L = m.lib()
    L.blst_p1_construct_nh_scalars_nh_points.argtypes = [vp, vp, vp, sz, vp, vp]
    L.blst_p1_tile_pippenger_d_CHES.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp, sz, i32]
    L.blst_p1_tile_pippenger_d_CHES_noindexhash.argtypes = [vp, vp, sz, vp, vp, vp, vp, sz, i32]
    L.blst_p1_tile_pippenger_CHES_prefetch_2step_ahead_input_std_scalar.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp,
                                                                                   sz, i32]
    L.blst_p1_integrate_buckets_accumulation_d_CHES.argtypes = [vp, vp, vp, sz, i32]
    L.blst_p1_tile_pippenger_BGMW95.argtypes = [vp, vp, sz, vp, vp, vp, sz]
    g = golden("ches_driver_n10.json")
    n, h, qe = g["n"], g["h"], g["q_exp"]
    ctx = m.CHESContext(1, 0, n_exp=10)
    ctx.build_table(m.fixed_points(1, n), n)
    T = ctx.get_table()                      # 3 n h blst affine, main_p1.cpp:155-172 order
    ctx.close()
    bctx = m.BGMWContext(1, 0, n_exp=10)
    bctx.build_table(m.fixed_points(1, n), n)
    TB = bctx.get_table()                    # n h_bgmw, main_p1.cpp:109-119 order
    bctx.close()
    B = of.bucket_set(1 << qe, 231)
    H, v2i = of.digit_table(B, 1 << qe)
    return m, L, g, T, TB, B, H, v2i


def _std_digits(sc, n, qe, h):
    """trans_uint256_t_to_standard_q_ary_expr (ref auxiliaryfunc.h:83-90) of every scalar, flat + 2 pad."""
    out = (ctypes.c_int * (n * h + 2))()
    raw = bytes(sc)
    for i in range(n):
        v = int.from_bytes(raw[32 * i:32 * i + 32], "little")
        for j in range(h):
            out[i * h + j] = (v >> (qe * j)) & ((1 << qe) - 1)
    return out


def _runs(g):
    return [r for r in g["runs"] if r["case"] == "rand"]


def test_integral_conversion_then_tile_d_ches(env):
    """method 2 (main_p1.cpp:249-291): construct_nh_scalars_nh_points + tile_pippenger_d_CHES,
    then integrate_buckets_accumulation_d_CHES over the buckets it leaves filled."""
    m, L, g, T, TB, B, H, v2i = env
    n, h, qe = g["n"], g["h"], g["q_exp"]
    for run in _runs(g):
        sc = m.gen_scalars(n, run["seed"])
        nh = _std_digits(sc, n, qe, h)
        signs = (ctypes.c_ubyte * (n * h))()
        ptrs = (ctypes.c_void_p * (n * h))()
        L.blst_p1_construct_nh_scalars_nh_points(nh, signs, ptrs, n * h, T, H)
        buckets = (ctypes.c_uint8 * (192 * len(B)))()
        ret = (ctypes.c_uint8 * 144)()
        L.blst_p1_tile_pippenger_d_CHES(ret, ptrs, n * h, nh, signs, buckets, B, v2i, len(B), 6)
        assert m.compress(1, bytes(ret)).hex() == run["ches_integral"] == run["pippenger"]
        ret2 = (ctypes.c_uint8 * 144)()
        L.blst_p1_integrate_buckets_accumulation_d_CHES(ret2, buckets, B, len(B), 6)
        assert m.compress(1, bytes(ret2)).hex() == run["pippenger"]
        # noindexhash: buckets indexed by value, same entries
        bk = (ctypes.c_uint8 * (192 * (B[len(B) - 1] + 1)))()
        L.blst_p1_tile_pippenger_d_CHES_noindexhash(ret, ptrs, n * h, nh, signs, bk, B, len(B), 6)
        assert m.compress(1, bytes(ret)).hex() == run["pippenger"]


def test_tile_prefetch_2step_std_scalar(env):
    m, L, g, T, TB, B, H, v2i = env
    n, h, qe = g["n"], g["h"], g["q_exp"]
    for run in _runs(g):
        nh = _std_digits(m.gen_scalars(n, run["seed"]), n, qe, h)
        buckets = (ctypes.c_uint8 * (192 * len(B)))()
        ret = (ctypes.c_uint8 * 144)()
        L.blst_p1_tile_pippenger_CHES_prefetch_2step_ahead_input_std_scalar(ret, T, n * h, nh, H, buckets, B, v2i,
                                                                             len(B), 6)
        assert m.compress(1, bytes(ret)).hex() == run["pippenger"]


def test_tile_bgmw95(env):
    m, L, g, T, TB, B, H, v2i = env
    n, qb, hb = g["n"], g["q_exp_bgmw"], g["h_bgmw"]
    for run in _runs(g):
        sc = m.gen_scalars(n, run["seed"])
        vals = (ctypes.c_int * (n * hb))()
        signs = (ctypes.c_ubyte * (n * hb))()
        ptrs = (ctypes.c_void_p * (n * hb))()
        base = ctypes.addressof(TB)
        d = (ctypes.c_int * hb)()
        for i in range(n):
            of.lib().or_bgmw_digits(d, ctypes.byref(sc, 32 * i), qb, hb)  # signed q/2 digits, r - s rule
            for j in range(hb):
                vals[i * hb + j] = abs(d[j])
                signs[i * hb + j] = 1 if d[j] < 0 else 0
                ptrs[i * hb + j] = base + 96 * (i * hb + j)
        buckets = (ctypes.c_uint8 * (192 * ((1 << (qb - 1)) + 1)))()
        ret = (ctypes.c_uint8 * 144)()
        L.blst_p1_tile_pippenger_BGMW95(ret, ptrs, n * hb, vals, signs, buckets, qb)
        assert m.compress(1, bytes(ret)).hex() == run["bgmw95"] == run["pippenger"]
