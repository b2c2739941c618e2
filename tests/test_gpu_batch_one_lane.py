"""GPU parity of the ONE-lane CHES batch schedule -- the exact code path the
headline bench times (Ches::run_jobs with batch_lanes() == 1, ches.hip: front
groups on the greatest-priority front stream, accumulation k waiting for level
0 of MSM k - 1, reduction groups of up to kGroup = 20 MSMs alternating between
two reducer sets / tail streams, one device scalar slot per host set).

The reference computations these stages restate: the CHES accumulation
ref src/multi_scalar.c:421-463 and its d-trick reduction :301-321 (driven by
main_p1.cpp:192-246).  Every batch result must equal the synchronous MSM of
its set, and set 0 (the seed-1 stream) the reference's golden key
(tests/golden/msm_g*.json, written by the reference's blst_p1s_mult_pippenger).

- G1 n = 2^20 (config_file_n_exp_20.h) with K = 22 host sets in page-locked
  memory: two reduction groups of 11, so the reducer-set alternation runs.
- G2 n = 2^20 with K = 21 (two groups, 11 + 10).
- G1 n = 2^16 forced onto the one-lane branch (MSM_BATCH_LANES=1, read once
  per process, so in a child process) with K = 40 host sets > the 32 device
  slot groups: the slot-reuse wait (copy of group g after front g - 32) and
  two reduction groups; and with MSM_H2D_SLOTS=4 so the reuse wait runs every
  few MSMs.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _golden(golden, group, n):
    return [c["compressed"] for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == 255][0]


def _pinned_sets(m, n, K, seed0):
    import torch
    host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
    for k in range(K):
        host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(
            m.gen_scalars(n, 1 if k == 0 else seed0 + k), dtype=np.uint8)
    return host


@pytest.mark.parametrize("group,K", [(1, 22), (2, 21)])
def test_one_lane_batch_2p20(m, golden, points, group, K):
    n = 1 << 20
    ctx = m.CHESContext(group, 0, n_exp=20)
    ctx.build_table(points(group, n), n)
    assert ctx.batch_lanes() == 1, "n = 2^20 must take the headline's one-lane schedule"
    host = _pinned_sets(m, n, K, 500)
    got = [m.compress(group, r) for r in ctx.mult_batch(host.data_ptr(), K, set_stride=n * 32, on_device=False)]
    assert got[0].hex() == _golden(golden, group, n)
    view = host.numpy()
    for k in range(K):
        want = m.compress(group, ctx.mult(bytes(view[k * n * 32:(k + 1) * n * 32])))
        assert got[k] == want, f"set {k} of {K}"
    ctx.close()


_ONE_LANE_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
import msm_blst_amd as m
n, K = 1 << 16, int(sys.argv[2])
ctx = m.CHESContext(1, 0, n_exp=16)
ctx.build_table(m.fixed_points(1, n), n)
print("LANES", ctx.batch_lanes())
host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
for k in range(K):
    host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 1 if k == 0 else 700 + k), dtype=np.uint8)
got = [m.compress(1, r).hex() for r in ctx.mult_batch(host.data_ptr(), K, set_stride=n * 32, on_device=False)]
# a second batch on the same context: every ring (slots, fronts, reducer sets) reused
again = [m.compress(1, r).hex() for r in ctx.mult_batch(host.data_ptr(), K, set_stride=n * 32, on_device=False)]
want = [m.compress(1, ctx.mult(bytes(host.numpy()[k * n * 32:(k + 1) * n * 32]))).hex() for k in range(K)]
print("SET0", got[0])
print("OK" if got == want and again == want else "MISMATCH " + str([k for k in range(K) if got[k] != want[k]]))
"""


@pytest.mark.parametrize("slots", [None, 4])
def test_one_lane_batch_slot_reuse_2p16(golden, slots):
    env = dict(os.environ, MSM_BATCH_LANES="1")
    if slots:
        env["MSM_H2D_SLOTS"] = str(slots)
    K = 40
    r = subprocess.run([sys.executable, "-c", _ONE_LANE_SCRIPT, REPO, str(K)], capture_output=True, text=True,
                       env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = dict(ln.split(" ", 1) for ln in r.stdout.splitlines() if " " in ln)
    assert out.get("LANES") == "1", r.stdout[-2000:]
    assert out.get("SET0") == _golden(golden, 1, 1 << 16)
    assert r.stdout.strip().endswith("OK"), r.stdout[-2000:]
