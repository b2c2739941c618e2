"""GPU parity of the blst-level CHES / BGMW95 entry points (ref
bindings/blst.h:249-357) driven the way the reference's drivers drive them
(ref main_p1.cpp / main_p2.cpp :192-291, :294-398) at the n = 2^10
configuration (q = 2^13, h = 20; BGMW95 q = 2^12, h = 22), for G1 and the p2
twins, against the reference's own driver results
(tests/golden/ches_driver_n10.json, ches_driver_p2_n10.json)."""
import ctypes

import pytest

import oracle_ffi as of
from test_oracle_golden import _fnv

pytestmark = pytest.mark.gpu

vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int


class _Env:
    """The blst-level entry points of one group under their blst names."""

    def __init__(self, m, L, group, g, T, TB, B, H, v2i):
        self.m, self.L, self.G, self.g, self.T, self.TB, self.B, self.H, self.v2i = m, L, group, g, T, TB, B, H, v2i

    def fn(self, name):
        return getattr(self.L, name.format(g=self.G))


@pytest.fixture(scope="module", params=[1, 2], ids=["g1", "g2"])
def env(golden, request):
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    G = request.param
    L = m.lib()
    getattr(L, f"blst_p{G}_construct_nh_scalars_nh_points").argtypes = [vp, vp, vp, sz, vp, vp]
    getattr(L, f"blst_p{G}_tile_pippenger_d_CHES").argtypes = [vp, vp, sz, vp, vp, vp, vp, vp, sz, i32]
    getattr(L, f"blst_p{G}_tile_pippenger_d_CHES_noindexhash").argtypes = [vp, vp, sz, vp, vp, vp, vp, sz, i32]
    getattr(L, f"blst_p{G}_tile_pippenger_CHES_prefetch_2step_ahead_input_std_scalar").argtypes = [
        vp, vp, sz, vp, vp, vp, vp, vp, sz, i32]
    getattr(L, f"blst_p{G}_integrate_buckets_accumulation_d_CHES").argtypes = [vp, vp, vp, sz, i32]
    getattr(L, f"blst_p{G}_tile_pippenger_BGMW95").argtypes = [vp, vp, sz, vp, vp, vp, sz]
    g = golden("ches_driver_n10.json" if G == 1 else "ches_driver_p2_n10.json")
    n, h, qe = g["n"], g["h"], g["q_exp"]
    ctx = m.CHESContext(G, 0, n_exp=10)
    ctx.build_table(m.fixed_points(G, n), n)
    T = ctx.get_table()                      # 3 n h blst affine, main_p{1,2}.cpp:155-172 order
    ctx.close()
    bctx = m.BGMWContext(G, 0, n_exp=10)
    bctx.build_table(m.fixed_points(G, n), n)
    TB = bctx.get_table()                    # n h_bgmw, main_p{1,2}.cpp:109-119 order
    bctx.close()
    B = of.bucket_set(1 << qe, 231)
    H, v2i = of.digit_table(B, 1 << qe)
    return _Env(m, L, G, g, T, TB, B, H, v2i)


def test_tables_match_reference(env):
    """the GPU-built CHES and BGMW95 tables equal the reference driver's (FNV-1a of the
    blst affine bytes), incl. the G2 tables of main_p2.cpp"""
    assert _fnv(bytes(env.T)) == env.g["fnv_table_3nh"]
    assert _fnv(bytes(env.TB)) == env.g["fnv_table_bgmw"]


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
    m, G, g, T, B, H, v2i = env.m, env.G, env.g, env.T, env.B, env.H, env.v2i
    n, h, qe = g["n"], g["h"], g["q_exp"]
    for run in _runs(g):
        sc = m.gen_scalars(n, run["seed"])
        nh = _std_digits(sc, n, qe, h)
        signs = (ctypes.c_ubyte * (n * h))()
        ptrs = (ctypes.c_void_p * (n * h))()
        env.fn("blst_p{g}_construct_nh_scalars_nh_points")(nh, signs, ptrs, n * h, T, H)
        buckets = (ctypes.c_uint8 * (192 * G * len(B)))()
        ret = (ctypes.c_uint8 * (144 * G))()
        env.fn("blst_p{g}_tile_pippenger_d_CHES")(ret, ptrs, n * h, nh, signs, buckets, B, v2i, len(B), 6)
        assert m.compress(G, bytes(ret)).hex() == run["ches_integral"] == run["pippenger"]
        ret2 = (ctypes.c_uint8 * (144 * G))()
        env.fn("blst_p{g}_integrate_buckets_accumulation_d_CHES")(ret2, buckets, B, len(B), 6)
        assert m.compress(G, bytes(ret2)).hex() == run["pippenger"]
        # noindexhash: buckets indexed by value, same entries
        bk = (ctypes.c_uint8 * (192 * G * (B[len(B) - 1] + 1)))()
        env.fn("blst_p{g}_tile_pippenger_d_CHES_noindexhash")(ret, ptrs, n * h, nh, signs, bk, B, len(B), 6)
        assert m.compress(G, bytes(ret)).hex() == run["pippenger"]


def test_tile_prefetch_2step_std_scalar(env):
    m, G, g, T, B, H, v2i = env.m, env.G, env.g, env.T, env.B, env.H, env.v2i
    n, h, qe = g["n"], g["h"], g["q_exp"]
    for run in _runs(g):
        nh = _std_digits(m.gen_scalars(n, run["seed"]), n, qe, h)
        buckets = (ctypes.c_uint8 * (192 * G * len(B)))()
        ret = (ctypes.c_uint8 * (144 * G))()
        env.fn("blst_p{g}_tile_pippenger_CHES_prefetch_2step_ahead_input_std_scalar")(
            ret, T, n * h, nh, H, buckets, B, v2i, len(B), 6)
        assert m.compress(G, bytes(ret)).hex() == run["pippenger"]


def test_tile_bgmw95(env):
    m, G, g, TB = env.m, env.G, env.g, env.TB
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
                ptrs[i * hb + j] = base + 96 * G * (i * hb + j)
        buckets = (ctypes.c_uint8 * (192 * G * ((1 << (qb - 1)) + 1)))()
        ret = (ctypes.c_uint8 * (144 * G))()
        env.fn("blst_p{g}_tile_pippenger_BGMW95")(ret, ptrs, n * hb, vals, signs, buckets, qb)
        assert m.compress(G, bytes(ret)).hex() == run["bgmw95"] == run["pippenger"]


def test_registered_table_tiles(env):
    """msm_register_host_table: the driver's host table registered once, then the
    method-2 tile (main_p1.cpp:249-291) ships row indices instead of gathering
    rows -- same result, same buckets left filled (integrate over them), the
    same for noindexhash and the BGMW95 tile over its registered table; a
    pointer outside the registered rows falls back to the gather; after
    unregistering, the gather path again."""
    m, G, g, T, TB, B, H, v2i = env.m, env.G, env.g, env.T, env.TB, env.B, env.H, env.v2i
    L = m.lib()
    n, h, qe = g["n"], g["h"], g["q_exp"]
    run = _runs(g)[0]
    sc = m.gen_scalars(n, run["seed"])
    nh = _std_digits(sc, n, qe, h)
    signs = (ctypes.c_ubyte * (n * h))()
    ptrs = (ctypes.c_void_p * (n * h))()
    env.fn("blst_p{g}_construct_nh_scalars_nh_points")(nh, signs, ptrs, n * h, T, H)
    ref_buckets = (ctypes.c_uint8 * (192 * G * len(B)))()
    ret = (ctypes.c_uint8 * (144 * G))()
    env.fn("blst_p{g}_tile_pippenger_d_CHES")(ret, ptrs, n * h, nh, signs, ref_buckets, B, v2i, len(B), 6)
    assert L.msm_register_host_table(G, T, 3 * n * h) == 0, L.msm_last_error()
    try:
        for _ in range(2):
            buckets = (ctypes.c_uint8 * (192 * G * len(B)))()
            ret = (ctypes.c_uint8 * (144 * G))()
            env.fn("blst_p{g}_tile_pippenger_d_CHES")(ret, ptrs, n * h, nh, signs, buckets, B, v2i, len(B), 6)
            assert m.compress(G, bytes(ret)).hex() == run["pippenger"]
            ret2 = (ctypes.c_uint8 * (144 * G))()
            env.fn("blst_p{g}_integrate_buckets_accumulation_d_CHES")(ret2, buckets, B, len(B), 6)
            assert m.compress(G, bytes(ret2)).hex() == run["pippenger"]
        bk = (ctypes.c_uint8 * (192 * G * (B[len(B) - 1] + 1)))()
        env.fn("blst_p{g}_tile_pippenger_d_CHES_noindexhash")(ret, ptrs, n * h, nh, signs, bk, B, len(B), 6)
        assert m.compress(G, bytes(ret)).hex() == run["pippenger"]
        # one entry pointing at a copy of its row outside the table: the gather path
        moved = (ctypes.c_uint8 * (96 * G)).from_buffer_copy(ctypes.string_at(ptrs[7], 96 * G))
        saved = ptrs[7]
        ptrs[7] = ctypes.addressof(moved)
        env.fn("blst_p{g}_tile_pippenger_d_CHES")(ret, ptrs, n * h, nh, signs, ref_buckets, B, v2i, len(B), 6)
        assert m.compress(G, bytes(ret)).hex() == run["pippenger"]
        ptrs[7] = saved
        # BGMW95 over its own registered table
        assert L.msm_register_host_table(G, TB, n * g["h_bgmw"]) == 0
        qb, hb = g["q_exp_bgmw"], g["h_bgmw"]
        vals = (ctypes.c_int * (n * hb))()
        bsig = (ctypes.c_ubyte * (n * hb))()
        bptr = (ctypes.c_void_p * (n * hb))()
        d = (ctypes.c_int * hb)()
        for i in range(n):
            of.lib().or_bgmw_digits(d, ctypes.byref(sc, 32 * i), qb, hb)
            for j in range(hb):
                vals[i * hb + j] = abs(d[j])
                bsig[i * hb + j] = 1 if d[j] < 0 else 0
                bptr[i * hb + j] = ctypes.addressof(TB) + 96 * G * (i * hb + j)
        bb = (ctypes.c_uint8 * (192 * G * ((1 << (qb - 1)) + 1)))()
        env.fn("blst_p{g}_tile_pippenger_BGMW95")(ret, bptr, n * hb, vals, bsig, bb, qb)
        assert m.compress(G, bytes(ret)).hex() == run["pippenger"]
    finally:
        assert L.msm_unregister_host_table(T) == 0
        L.msm_unregister_host_table(TB)
    assert L.msm_unregister_host_table(T) != 0  # not registered any more
    env.fn("blst_p{g}_tile_pippenger_d_CHES")(ret, ptrs, n * h, nh, signs, ref_buckets, B, v2i, len(B), 6)
    assert m.compress(G, bytes(ret)).hex() == run["pippenger"]


def test_registered_table_row_edited(env):
    """The staleness guard of a registered table (row_samples.hpp): one row of
    the registered host table edited between tile calls -- a row some entry
    points at and that the guard samples (rows i (R - 1) / (k - 1), k = min(R,
    1024)) -- must give what the gather path gives over the edited table (the
    reference reads the host rows on every call, main_p1.cpp:279-282); the
    restored row gives the golden again."""
    m, G, g, T, B, H, v2i = env.m, env.G, env.g, env.T, env.B, env.H, env.v2i
    L = m.lib()
    n, h, qe = g["n"], g["h"], g["q_exp"]
    run = _runs(g)[0]
    nh = _std_digits(m.gen_scalars(n, run["seed"]), n, qe, h)
    signs = (ctypes.c_ubyte * (n * h))()
    ptrs = (ctypes.c_void_p * (n * h))()
    env.fn("blst_p{g}_construct_nh_scalars_nh_points")(nh, signs, ptrs, n * h, T, H)
    psz, R = 96 * G, 3 * n * h
    k = min(R, 1024)
    sampled = {i * (R - 1) // (k - 1) for i in range(k)}
    base = ctypes.addressof(T)
    row = next(r for r in ((p - base) // psz for p in ptrs) if r in sampled)
    other = (row + 1) % R
    saved = ctypes.string_at(base + row * psz, psz)

    def tile():
        bk = (ctypes.c_uint8 * (192 * G * len(B)))()
        ret = (ctypes.c_uint8 * (144 * G))()
        env.fn("blst_p{g}_tile_pippenger_d_CHES")(ret, ptrs, n * h, nh, signs, bk, B, v2i, len(B), 6)
        return m.compress(G, bytes(ret)).hex()

    assert L.msm_register_host_table(G, T, R) == 0, L.msm_last_error()
    try:
        assert tile() == run["pippenger"]
        ctypes.memmove(base + row * psz, ctypes.string_at(base + other * psz, psz), psz)
        edited = tile()
        assert edited != run["pippenger"]
        assert L.msm_unregister_host_table(T) == 0
        assert tile() == edited  # the gather path over the edited host table
        assert L.msm_register_host_table(G, T, R) == 0
        ctypes.memmove(base + row * psz, saved, psz)
        assert tile() == run["pippenger"]
    finally:
        ctypes.memmove(base + row * psz, saved, psz)
        L.msm_unregister_host_table(T)
