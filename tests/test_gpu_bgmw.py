"""GPU parity of the BGMW95 fixed-base path (table q^j P_i built on the GPU,
signed radix-q digits, accumulation and reduction in HIP) against the
reference: the n = 2^10 driver runs of ref main_p1.cpp (`bgmw95` result and
the BGMW95 table hash, tests/golden/ches_driver_n10.json) and the golden
Pippenger values (BGMW95 equals Pippenger on the same scalars, ref driver
test_pippengers main_p1.cpp:470-580)."""
import pytest

from test_oracle_golden import _fnv

pytestmark = pytest.mark.gpu

R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _golden(golden, group, n, seed=1, case="rand"):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["case"] == case and c["nbits"] == 255][0]["compressed"]


@pytest.fixture(scope="module")
def ctx10(m):
    ctx = m.BGMWContext(1, 0, n_exp=10)
    ctx.build_table(m.fixed_points(1, 1024), 1024)
    yield ctx
    ctx.close()


def test_table_n10_matches_reference(ctx10, golden):
    g = golden("ches_driver_n10.json")
    assert (ctx10.q_exp, ctx10.h) == (g["q_exp_bgmw"], g["h_bgmw"])
    assert _fnv(bytes(ctx10.get_table())) == g["fnv_table_bgmw"]


def test_driver_runs_n10(m, ctx10, golden):
    g = golden("ches_driver_n10.json")
    for run in g["runs"]:
        if run["case"] != "rand":
            continue
        r = ctx10.mult(bytes(m.gen_scalars(g["n"], run["seed"])))
        assert m.compress(1, r).hex() == run["bgmw95"] == run["pippenger"]


def test_edge_scalars_n10(m, ctx10, golden):
    n = 1024
    assert m.compress(1, ctx10.mult(bytes(32 * n))).hex() == "c0" + "00" * 47
    # r - 1 everywhere: top digit > q/2 -> the r - s branch for every scalar
    gold = [c for c in golden("msm_g1.json")["cases"] if c["case"] == "rminus1"][0]
    ctx = m.BGMWContext(1, 0, n_exp=10)
    ctx.build_table(m.fixed_points(1, gold["n"]), gold["n"])
    assert m.compress(1, ctx.mult((R - 1).to_bytes(32, "little") * gold["n"])).hex() == gold["compressed"]
    ctx.close()
    # s and s + r, and a mix of large (r - small) and small scalars, against CHES on the same points
    base = bytes(m.gen_scalars(n, 4))
    mixed = bytearray()
    for i in range(n):
        v = int.from_bytes(base[32 * i:32 * i + 32], "little")
        if i % 3 == 0:
            v = R - 1 - (v >> 200)
        elif i % 3 == 1:
            v = v + R if v + R < (1 << 256) else v
        mixed += v.to_bytes(32, "little")
    ches = m.CHESContext(1, 0, n_exp=10)
    ches.build_table(m.fixed_points(1, n), n)
    want = m.compress(1, ches.mult(bytes(mixed)))
    ches.close()
    assert m.compress(1, ctx10.mult(bytes(mixed))) == want


@pytest.mark.parametrize("n_exp", [16, 20])
def test_bgmw_g1_large_vs_reference(m, golden, points, n_exp):
    n = 1 << n_exp
    ctx = m.BGMWContext(1, 0, n_exp=n_exp)
    ctx.build_table(points(1, n), n)
    assert m.compress(1, ctx.mult(bytes(m.gen_scalars(n, 1)))).hex() == _golden(golden, 1, n)
    ctx.close()


@pytest.mark.parametrize("n_exp", [10, 16, 20])
def test_bgmw_g2_vs_reference(m, golden, points, n_exp):
    n = 1 << n_exp
    ctx = m.BGMWContext(2, 0, n_exp=n_exp)
    ctx.build_table(points(2, n), n)
    assert m.compress(2, ctx.mult(bytes(m.gen_scalars(n, 1)))).hex() == _golden(golden, 2, n)
    ctx.close()


def test_set_table_roundtrip_and_other_q(m, golden):
    n = 1000
    ctx = m.BGMWContext(1, 0, q_exp=16, h=16)
    ctx.build_table(m.fixed_points(1, n), n)
    T = ctx.get_table()
    ctx2 = m.BGMWContext(1, 0, q_exp=16, h=16)
    ctx2.set_table(T, n)
    sc = bytes(m.gen_scalars(n, 1))
    want = _golden(golden, 1, n)
    assert m.compress(1, ctx.mult(sc)).hex() == want
    assert m.compress(1, ctx2.mult(sc)).hex() == want
    ctx.close()
    ctx2.close()
