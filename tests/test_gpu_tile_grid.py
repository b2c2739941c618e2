"""GPU parity of blst_p{1,2}s_tile_pippenger driven the way its real callers
drive it: the Go binding's multi-threaded grid (ref bindings/go/blst.go
:2064-2197, breakdown :3181-3211) splits (points x windows) into tiles, calls
the tile entry point per tile and recombines rows top-down with `wnd`
doublings between rows.  The recombined sum must equal the reference's golden
MSM value.  The grids used here include bit0 = 0 (lookback bit taken as 0),
the partial top window (bit0 + window > nbits: cbits = wbits + 1, ref
multi_scalar.c:596-599), negative Booth digits (every full window), pointer
arrays (`&val[x]`, the Go []*P1Affine case) and flat {ptr, NULL} inputs.
Also: the reference's pointer-iteration rule (multi_scalar.c:390-416) on
blst_p{1,2}s_mult_pippenger with a NULL after k explicit pointers."""
import ctypes

import pytest

from test_oracle_golden import _prepare

pytestmark = pytest.mark.gpu

vp, sz = ctypes.c_void_p, ctypes.c_size_t


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _case(golden, group, n, seed, nbits):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["nbits"] == nbits and c["case"] == "rand"][0]


def _go_grid(nbits, window, nx):
    """blst.go:3207-3208 (final lines of breakdown) for a chosen window and nx, then the
    grid of :2073-2096: nx point ranges, ny rows, top row first."""
    ny = nbits // window + 1
    wnd = nbits // ny + 1
    return nx, ny, wnd


def _grid_msm(m, group, pts, sc, n, nbits, window, nx, ptr_points=False, ptr_scalars=False):
    L = m.lib()
    tile = getattr(L, f"blst_p{group}s_tile_pippenger")
    add = getattr(L, f"msm_p{group}_add")
    nx, ny, wnd = _go_grid(nbits, window, nx)
    psz, nb, jb = 96 * group, (nbits + 7) // 8, 144 * group
    base_p, base_s = ctypes.addressof(pts), ctypes.addressof(sc)
    dx = n // nx
    xs = [(i * dx, dx if i < nx - 1 else n - i * dx) for i in range(nx)]
    ret = (ctypes.c_uint8 * jb)()                    # infinity (all zero)
    y = wnd * (ny - 1)
    while True:
        for x, cnt in xs:
            if ptr_points:                           # []*P1Affine: &val[x], one pointer per point
                pp = (vp * cnt)(*[base_p + psz * (x + i) for i in range(cnt)])
            else:                                    # []P1Affine: {&val[x], NULL}
                pp = (vp * 2)(base_p + psz * x, None)
            if ptr_scalars:
                sp = (vp * cnt)(*[base_s + nb * (x + i) for i in range(cnt)])
            else:
                sp = (vp * 2)(base_s + nb * x, None)
            t = (ctypes.c_uint8 * jb)()
            tile(t, pp, cnt, sp, nbits, None, y, wnd)
            add(ret, ret, t)
        if y == 0:
            break
        for _ in range(wnd):
            add(ret, ret, ret)                       # doubling-aware add = blst_p1_double
        y -= wnd
    return bytes(ret), (nx, ny, wnd)


@pytest.mark.parametrize("group,n,seed,nbits,window,nx,ptrs", [
    (1, 1000, 1, 255, 10, 3, (False, False)),   # 26 rows of 10 bits, top row bits 250..254 (partial)
    (1, 1000, 2, 64, 10, 2, (True, False)),     # nbits = 64: 7 rows, top row 4 bits; pointer arrays
    (1, 1024, 1, 255, 13, 1, (False, True)),    # window 13 (partial top), scalar pointers
    (1, 64, 1, 256, 8, 2, (True, True)),        # 256-bit scalars: top row at bit0 = nbits (carry tile)
    (2, 256, 1, 255, 12, 2, (False, False)),    # G2: 22 rows of 12 bits, top row 3 bits
    (2, 64, 1, 64, 9, 1, (True, True)),
])
def test_tile_grid_reassembles_msm(m, golden, group, n, seed, nbits, window, nx, ptrs):
    c = _case(golden, group, n, seed, nbits)
    pts, sc = _prepare(group, c)
    got, (gx, gy, wnd) = _grid_msm(m, group, pts, sc, n, nbits, window, nx, *ptrs)
    # the top window is partial; for nbits = 256, window 8 it starts AT nbits (wbits = 0,
    # cbits = 1: the tile is the Booth carry of bit 255 alone, ref multi_scalar.c:596-599)
    assert (gy - 1) * wnd <= nbits < gy * wnd
    assert m.compress(group, got).hex() == c["compressed"], (gx, gy, wnd)


def test_tile_single_windows_vs_oracle(m):
    """Individual tiles (not only their sum): tile(bit0, w) == sum_i d_i P_i with d_i the
    Booth digit of scalar i, computed here from the scalar bits, for bit0 = 0, a middle
    window with negative digits, and the partial top window."""
    import oracle_ffi as of
    n, nbits = 200, 255
    R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    pts = of.fixed_points(1, n)
    sc = of.scalars(n, 11)
    raw = bytes(sc)
    L = m.lib()
    for bit0, w in ((0, 9), (100, 11), (250, 8), (247, 8)):
        wbits, cbits = (nbits - bit0, nbits - bit0 + 1) if bit0 + w > nbits else (w, w)
        digits = []
        for i in range(n):
            v = int.from_bytes(raw[32 * i:32 * i + 32], "little")
            wv = ((v << 1) >> bit0) & ((1 << (wbits + 1)) - 1)      # bits [bit0-1, bit0+wbits)
            d = (wv + 1) >> 1
            if (wv >> cbits) & 1:
                d -= 1 << cbits
            digits.append(d)
        if bit0 + w <= nbits:
            assert any(d < 0 for d in digits)
        dsc = b"".join((d % R).to_bytes(32, "little") for d in digits)
        want = of.compress(1, of.msm(1, pts, (ctypes.c_uint8 * len(dsc)).from_buffer_copy(dsc), n, 255, "naive"))
        t = (ctypes.c_uint8 * 144)()
        L.blst_p1s_tile_pippenger(t, (vp * 2)(ctypes.addressof(pts), None), n,
                                  (vp * 2)(ctypes.addressof(sc), None), nbits, None, bit0, w)
        assert m.compress(1, bytes(t)).hex() == want, (bit0, w)


@pytest.mark.parametrize("group", [1, 2])
def test_pointer_rule_null_after_k_pointers(m, golden, group):
    """points = {&P[0], &P[1], &P[2], NULL, ...}: after the NULL the points continue
    right after P[2] (multi_scalar.c:413 `*points ? *points++ : point+1`); same for
    scalars, which advance by nbytes."""
    n = 64
    c = _case(golden, group, n, 1, 255)
    pts, sc = _prepare(group, c)
    psz, nb = 96 * group, 32
    bp, bs = ctypes.addressof(pts), ctypes.addressof(sc)
    for k in (1, 2, 3, 17):
        pp = (vp * (k + 1))(*([bp + psz * i for i in range(k)] + [None]))
        sp = (vp * (k + 1))(*([bs + nb * i for i in range(k)] + [None]))
        ret = (ctypes.c_uint8 * (144 * group))()
        getattr(m.lib(), f"blst_p{group}s_mult_pippenger")(ret, pp, n, sp, 255, None)
        assert m.compress(group, bytes(ret)).hex() == c["compressed"], k
