"""GPU parity of the one-window reductions at tiny sizes (CHES and BGMW95,
G1 and G2): with a handful of points the final segment partials are few and
sparse, which is where the synchronous bit-sum tail (WeightedReducer plan:
2 s bit sums + host Horner, ches.hip) has its smallest buffers and emptiest
bit segments.  Checked against the oracle's naive MSM (oracle/msm_oracle.c),
the reference's result on the same inputs (ref main_p1.cpp:470-580 compares
every method with Pippenger)."""
import ctypes

import pytest

import oracle_ffi as of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _oracle(group, pts, sc, n):
    P = (ctypes.c_uint8 * len(pts)).from_buffer_copy(pts)
    S = (ctypes.c_uint8 * len(sc)).from_buffer_copy(sc)
    return of.compress(group, of.msm(group, P, S, n, 255, "naive"))


@pytest.mark.parametrize("group", [1, 2])
@pytest.mark.parametrize("method", ["ches", "bgmw"])
@pytest.mark.parametrize("n", [1, 2, 5, 64])
def test_tiny_msm_vs_oracle(m, group, method, n):
    pts = bytes(m.fixed_points(group, n))
    ctor = m.CHESContext if method == "ches" else m.BGMWContext
    ctx = ctor(group, 0, n_exp=8)
    try:
        ctx.build_table(pts, n)
        for seed in (5, 6):
            sc = bytes(m.gen_scalars(n, seed))
            assert m.compress(group, ctx.mult(sc)).hex() == _oracle(group, pts, sc, n), (method, group, n, seed)
        # one nonzero scalar of 1: a single bucket, a single bit sum
        one = (1).to_bytes(32, "little") + bytes(32 * (n - 1))
        assert m.compress(group, ctx.mult(one)).hex() == _oracle(group, pts, one, n)
    finally:
        ctx.close()
