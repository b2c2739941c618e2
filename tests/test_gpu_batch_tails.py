"""GPU parity of round 6's batch tails (ches.hip / engine.hip).

The batch's LAST reduction group of a one-window CHES plan ends in 2 s bit sums
per MSM and a host Horner (WeightedReducer::launch_tail_group_bits) instead of
the dense stage; earlier groups keep the dense stage, whose levels now run over
4 waves per add only when they have <= 16 384 adds (MSM_DENSE_COOP_MAX).  The
reduction they restate is ref src/multi_scalar.c:301-321 (sum_b b S_b over the
bucket set), driven by main_p1.cpp:192-246.

In child processes (the knobs are read once per process): G1 2^16 and G2 2^10
CHES batches of K sets spanning several reduction groups and lanes, with the
bit tail on / off and the dense stage all-coop / all-one-lane, must all give
the same K results, equal to the synchronous MSMs, with set 0 the golden key;
and configs[1]'s plain batch (19 windows: no bit tail) under both dense-stage
settings."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
torch.cuda.init()  # torch's HIP runtime first (tests/conftest.py _torch_hip_first)
import msm_blst_amd as m
out = {}
for group, n_exp, K in ((1, 16, 25), (2, 10, 23)):
    n = 1 << n_exp
    ctx = m.CHESContext(group, 0, n_exp=n_exp)
    ctx.build_table(m.fixed_points(group, n), n)
    sets = b"".join(bytes(m.gen_scalars(n, 1 if k == 0 else 300 + k)) for k in range(K))
    got = [m.compress(group, r).hex() for r in ctx.mult_batch(sets, K)]
    sync = [m.compress(group, ctx.mult(sets[32 * n * k:32 * n * (k + 1)])).hex() for k in (0, K - 1)]
    out[f"ches{group}"] = {"got": got, "sync_ok": sync == [got[0], got[K - 1]], "lanes": ctx.batch_lanes()}
    ctx.close()
n, K = 1 << 12, 21
pc = m.MSMContext(1, 0, 12)
pc.set_points(m.fixed_points(1, n), n)
raw = b"".join(bytes(m.gen_scalars(n, 1 if k == 0 else 400 + k)) for k in range(K))
d = torch.tensor(np.frombuffer(raw, dtype=np.uint8), device="cuda:0")
got = [m.compress(1, r).hex() for r in pc.mult_batch(d.data_ptr(), K, 255, on_device=True)]
sync = [m.compress(1, pc.mult(d.data_ptr() + 32 * n * k, 255, on_device=True)).hex() for k in (0, K - 1)]
out["pip"] = {"got": got, "sync_ok": sync == [got[0], got[K - 1]]}
print("RESULT", json.dumps(out))
"""


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(line[0][7:])


def test_bit_tail_and_dense_coop_choices_agree(golden):
    want = {g: [c["compressed"] for c in golden(f"msm_g{g}.json")["cases"]
                if c["n"] == n and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == 255][0]
            for g, n in ((1, 1 << 16), (2, 1 << 10))}
    want_pip = [c["compressed"] for c in golden("msm_g1.json")["cases"]
                if c["n"] == 1 << 12 and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == 255][0]
    g8 = {"MSM_RED_GROUP": "8", "MSM_PIP_GROUP": "8"}  # several reduction groups per batch
    runs = [_run(g8),                                         # defaults
            _run(dict(g8, MSM_BIT_TAIL="0")),                 # dense stage for every group
            _run(dict(g8, MSM_DENSE_COOP_MAX="1000000")),     # every dense level coop
            _run(dict(g8, MSM_DENSE_COOP_MAX="0"))]           # no dense level coop
    for key, w in (("ches1", want[1]), ("ches2", want[2]), ("pip", want_pip)):
        for r in runs:
            assert r[key]["sync_ok"], key
            assert r[key]["got"][0] == w, key
            assert r[key]["got"] == runs[0][key]["got"], key


@pytest.mark.parametrize("group,n_exp", [(1, 12), (2, 10)])
def test_short_batches_equal_sync(group, n_exp):
    """Batches of 1, 2 and 3 sets: a single reduction group that is also the
    last (bit tail over one to three MSMs), the first front groups of the ramp
    (1, 1, 2, ...) and, for K = 1, no second lane -- each result equal to the
    synchronous MSM of its set."""
    import msm_blst_amd as m
    n = 1 << n_exp
    ctx = m.CHESContext(group, 0, n_exp=n_exp)
    ctx.build_table(m.fixed_points(group, n), n)
    try:
        for K in (1, 2, 3, 1):
            sets = [bytes(m.gen_scalars(n, 500 + 10 * K + k)) for k in range(K)]
            got = [m.compress(group, r) for r in ctx.mult_batch(b"".join(sets), K)]
            want = [m.compress(group, ctx.mult(s)) for s in sets]
            assert got == want, K
    finally:
        ctx.close()


def test_short_plain_batches_equal_sync():
    """configs[1]'s plain-Pippenger batch with 1, 2 and 3 sets (one reduction
    group, dense tail) against the synchronous MSMs."""
    import msm_blst_amd as m
    n = 1 << 12
    ctx = m.MSMContext(1, 0, 12)
    ctx.set_points(m.fixed_points(1, n), n)
    try:
        for K in (1, 2, 3):
            raw = b"".join(bytes(m.gen_scalars(n, 600 + 10 * K + k)) for k in range(K))
            got = [m.compress(1, r) for r in ctx.mult_batch(raw, K, 255)]
            want = [m.compress(1, ctx.mult(raw[32 * n * k:32 * n * (k + 1)], 255)) for k in range(K)]
            assert got == want, K
    finally:
        ctx.close()
