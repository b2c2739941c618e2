"""GPU parity of the pipelined plain-Pippenger batch (msm_ctx_mult_batch,
Pippenger<G>::run_batch): K MSMs over one point set with K distinct scalar
sets must equal K synchronous msm_ctx_mult calls, and set 0 (the seed-1
stream) the reference's golden value (tests/golden, written from the
reference's own blst_p1s_mult_pippenger).  Covers device and host scalar
sets, G1 and G2, window sizes with a partial top window (bucket copies),
64-bit scalars (short window plan) and batch lengths that are not a multiple
of the plain-Pippenger reduction group (Pippenger::kGroup = 10,
engine.hpp; the CHES batch groups 20)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _golden(golden, group, n, nbits=255):
    return [c["compressed"] for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == nbits][0]


def _sets(m, n, k):
    return b"".join(m.gen_scalars(n, 1 if i == 0 else 100 + i) for i in range(k))


@pytest.mark.parametrize("group,lg,c,count,on_device", [
    (1, 16, 14, 10, True),   # configs[1]: 2^16, the drop-in's window
    (1, 16, 13, 17, False),  # blst's window for 2^16; host sets; 2 groups (9/8)
    (1, 12, 12, 23, True),   # 3 reduction groups (8/8/7), two front-group ramps
    (1, 10, 10, 3, True),
    (2, 10, 10, 9, True),
])
def test_batch_equals_sync_and_golden(m, golden, points, group, lg, c, count, on_device):
    import torch
    n = 1 << lg
    raw = _sets(m, n, count)
    ctx = m.MSMContext(group, 0, c)
    ctx.set_points(points(group, n), n)
    if on_device:
        d = torch.tensor(np.frombuffer(raw, dtype=np.uint8), device="cuda:0")
        got = ctx.mult_batch(d.data_ptr(), count, 255, on_device=True)
    else:
        got = ctx.mult_batch(raw, count, 255)
    sync = [ctx.mult(raw[k * 32 * n:(k + 1) * 32 * n], 255) for k in range(count)]
    ctx.close()
    keys = [m.compress(group, j) for j in got]
    assert keys == [m.compress(group, j) for j in sync]
    assert keys[0].hex() == _golden(golden, group, n)


def test_batch_short_scalars(m, golden):
    """nbits = 64 (the reference's 64-bit scalar case, golden n = 1000 seed 2):
    fewer windows, the top window partial; packed 8-byte scalars."""
    from test_oracle_golden import _prepare
    c = [c for c in golden("msm_g1.json")["cases"]
         if c["n"] == 1000 and c["seed"] == 2 and c["nbits"] == 64 and c["case"] == "rand"][0]
    n, count = 1000, 5
    pts, sc = _prepare(1, c)
    other = _sets(m, n, count - 1)
    raw = bytes(sc) + b"".join(other[32 * i:32 * i + 8] for i in range(n * (count - 1)))
    ctx = m.MSMContext(1, 0, 10)
    ctx.set_points(bytes(pts), n)
    got = ctx.mult_batch(raw, count, 64, stride=8)
    sync = [ctx.mult(raw[k * 8 * n:(k + 1) * 8 * n], 64, stride=8) for k in range(count)]
    ctx.close()
    assert [m.compress(1, j) for j in got] == [m.compress(1, j) for j in sync]
    assert m.compress(1, got[0]).hex() == c["compressed"]
