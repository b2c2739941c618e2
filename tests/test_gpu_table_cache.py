"""GPU tests: the table file cache (save / load of the CHES and BGMW95 tables in
blst affine layout; the reference rebuilds them on every run, ref
main_p1.cpp:94-178) and the sum of affine points blst_p{1,2}s_add (ref
src/bulk_addition.c:145-164), against the reference's golden values and the
CPU oracle."""
import ctypes

import pytest

import oracle_ffi as of
from test_oracle_golden import _fnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _golden(golden, group, n, seed=1):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["case"] == "rand" and c["nbits"] == 255][0]["compressed"]


@pytest.mark.parametrize("kind", ["ches", "bgmw"])
def test_table_file_roundtrip(m, golden, tmp_path, kind):
    n = 1024
    Ctx = m.CHESContext if kind == "ches" else m.BGMWContext
    a = Ctx(1, 0, n_exp=10)
    a.build_table(m.fixed_points(1, n), n)
    path = tmp_path / f"{kind}.tbl"
    a.save_table(path)
    rows = a.get_table()
    b = Ctx(1, 0, n_exp=10)
    b.load_table(path)
    assert b.n == n
    assert _fnv(bytes(b.get_table())) == _fnv(bytes(rows))
    assert path.stat().st_size == 64 + len(bytes(rows))
    if kind == "ches":
        assert _fnv(bytes(rows)) == golden("ches_driver_n10.json")["fnv_table_3nh"]
    else:
        assert _fnv(bytes(rows)) == golden("ches_driver_n10.json")["fnv_table_bgmw"]
    assert m.compress(1, b.mult(bytes(m.gen_scalars(n, 1)))).hex() == _golden(golden, 1, n)
    a.close()
    b.close()


def test_table_file_rejects_other_parameters(m, tmp_path):
    n = 256
    a = m.BGMWContext(1, 0, n_exp=10)
    a.build_table(m.fixed_points(1, n), n)
    path = tmp_path / "bgmw.tbl"
    a.save_table(path)
    c = m.CHESContext(1, 0, n_exp=10)
    with pytest.raises(m.MsmError):
        c.load_table(path)
    g2 = m.BGMWContext(2, 0, n_exp=10)
    with pytest.raises(m.MsmError):
        g2.load_table(path)
    for x in (a, c, g2):
        x.close()


def _naive_sum(group, pts, n):
    one = (1).to_bytes(32, "little") * n
    S = (ctypes.c_uint8 * len(one)).from_buffer_copy(one)
    return of.compress(group, of.msm(group, pts, S, n, 255, "naive"))


@pytest.mark.parametrize("group,n", [(1, 1), (1, 1000), (1, 5000), (2, 300)])
def test_points_add_matches_oracle(m, group, n):
    pts = m.fixed_points(group, n)
    assert m.compress(group, m.ps_add(group, pts, n)).hex() == _naive_sum(group, pts, n)


def test_points_add_pointer_rule_and_infinity(m):
    """bulk_addition.c:155: a NULL entry continues after the previous point; all-zero = infinity."""
    n = 64
    raw = bytearray(bytes(m.fixed_points(1, n)))
    raw[96 * 5:96 * 6] = bytes(96)                  # point 5 at infinity
    P = (ctypes.c_uint8 * len(raw)).from_buffer_copy(bytes(raw))
    base = ctypes.addressof(P)
    ptrs = (ctypes.c_void_p * n)()
    for i in range(n):                              # explicit pointers for even i, NULL for odd i
        ptrs[i] = base + 96 * i if i % 2 == 0 else None
    ret = (ctypes.c_uint8 * 144)()
    m.lib().blst_p1s_add(ret, ptrs, n)
    assert m.compress(1, bytes(ret)).hex() == _naive_sum(1, P, n)
    # all infinity -> infinity
    Z = (ctypes.c_uint8 * (96 * 8))()
    assert m.compress(1, m.ps_add(1, Z, 8)).hex() == "c0" + "00" * 47


@pytest.mark.parametrize("kind", ["ches", "bgmw"])
def test_table_file_truncated_or_padded_is_rejected(m, golden, tmp_path, kind):
    """A file whose size disagrees with its header is refused before the context is
    touched; a context whose load failed has no table and its mult raises
    (MSM_E_STATE) instead of returning a point."""
    n = 256
    Ctx = m.CHESContext if kind == "ches" else m.BGMWContext
    a = Ctx(1, 0, n_exp=10)
    a.build_table(m.fixed_points(1, n), n)
    good = tmp_path / "good.tbl"
    a.save_table(good)
    raw = good.read_bytes()
    sc = bytes(m.gen_scalars(n, 1))
    want = m.compress(1, a.mult(sc))
    for name, data in (("short", raw[:-96]), ("long", raw + bytes(96)), ("header_only", raw[:64])):
        bad = tmp_path / f"{name}.tbl"
        bad.write_bytes(data)
        b = Ctx(1, 0, n_exp=10)
        with pytest.raises(m.MsmError):
            b.load_table(bad)
        with pytest.raises(m.MsmError):
            b.mult(sc)
        # a context with a valid table keeps it usable after a rejected load? No:
        # a failed load leaves no table (never a half-loaded one) -> mult raises
        b.load_table(good)
        assert m.compress(1, b.mult(sc)) == want
        with pytest.raises(m.MsmError):
            b.load_table(bad)
        with pytest.raises(m.MsmError):
            b.mult(sc)
        b.close()
    # header with a row count that disagrees with its point count
    hdr = bytearray(raw[:64])
    hdr[32:40] = (int.from_bytes(hdr[32:40], "little") + 1).to_bytes(8, "little")
    bad = tmp_path / "rows.tbl"
    bad.write_bytes(bytes(hdr) + raw[64:])
    b = Ctx(1, 0, n_exp=10)
    with pytest.raises(m.MsmError):
        b.load_table(bad)
    b.close()
    a.close()


@pytest.mark.parametrize("kind", ["ches", "bgmw"])
def test_mult_without_table_raises(m, kind):
    Ctx = m.CHESContext if kind == "ches" else m.BGMWContext
    c = Ctx(1, 0, n_exp=10)
    with pytest.raises(m.MsmError):
        c.mult(bytes(32 * 4))
    c.close()
