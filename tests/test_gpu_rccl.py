"""The RCCL leg of the multi-GPU path on a real MI355X: torch.distributed with
backend "nccl" (RCCL on ROCm) in a child process with world size 1 -- the code
path `bench.py --gpus N` runs per rank (ProcessGroup with device_id, the batch's
all_gather of 144-B partials through msm_blst_amd.dist.gather_partials_batch,
host fold, Bracket's MAX all_reduce) -- on device 0.  World size > 1 needs
several GPUs (the driver's 8-GPU run); the CPU suite covers N = 2 / 3 with gloo
(tests/test_dist.py).  Parity: the folded set-0 result of a 2^16 CHES batch
against the reference's golden key."""
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
import numpy as np, torch, torch.distributed as dist
import msm_blst_amd as m
from msm_blst_amd import dist as mdist
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl"
n, K = 1 << 16, 3
ctx = m.CHESContext(1, 0, n_exp=16)
ctx.build_table(m.fixed_points(1, n), n)
host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
for k in range(K):
    host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 1 if k == 0 else 40 + k), dtype=np.uint8)
parts = ctx.mult_batch(host.data_ptr(), K, 32, set_stride=n * 32, on_device=False)
gathered = mdist.gather_partials_batch(parts, 1, dev)
res = [mdist.fold(ps, mdist.engine_add(1)) for ps in gathered]
t = torch.tensor([1.5], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
dist.barrier()
print("RESULT", json.dumps({"set0": m.compress(1, res[0]).hex(), "same": [m.compress(1, a) == m.compress(1, b) for a, b in zip(res, parts)], "max": float(t.item()), "world": dist.get_world_size()}))
dist.destroy_process_group()
"""


def test_rccl_world1_gather_and_fold(golden):
    want = [c["compressed"] for c in golden("msm_g1.json")["cases"]
            if c["n"] == 1 << 16 and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == 255][0]
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29631")
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads(line[0][7:])
    assert d["world"] == 1 and d["max"] == 1.5
    assert d["set0"] == want
    assert all(d["same"])


CHILD_MULTI = r"""
import sys
sys.path.insert(0, sys.argv[1])
import msm_blst_amd as m
out = []
for group, n_exp, K in ((1, 16, 4), (2, 10, 3)):
    n = 1 << n_exp
    ctx = m.CHESContext(group, n_exp=n_exp, devices=[0])
    ctx.build_table(m.fixed_points(group, n), n)
    sets = b"".join(bytes(m.gen_scalars(n, 1 if k == 0 else 60 + k)) for k in range(K))
    got = [m.compress(group, r).hex() for r in ctx.mult_batch(sets, K)]
    want = [m.compress(group, ctx.mult(sets[32 * n * k:32 * n * (k + 1)])).hex() for k in range(K)]
    out.append((group, got[0], got == want, m.lib().msm_ches_ctx_rccl_exchange(ctx._ctx)))
    ctx.close()
print("RESULT", out)
"""


def test_c_abi_multi_device_rccl_gather(golden):
    """The C-ABI multi-device batch exchanging over RCCL (csrc/multi.hpp
    run_batch_rccl: every shard's window sums into a device exchange buffer, ONE
    ncclGather onto the first shard's device, one read-back, host combine +
    fold), forced with MSM_MULTI_RCCL=1 on a one-device context (a communicator
    of one rank: the gather is a device copy).  Set 0 against the golden keys,
    every set against the synchronous MSM."""
    want = {g: [c["compressed"] for c in golden(f"msm_g{g}.json")["cases"]
                if c["n"] == n and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == 255][0]
            for g, n in ((1, 1 << 16), (2, 1 << 10))}
    env = dict(os.environ, MSM_MULTI_RCCL="1")
    r = subprocess.run([sys.executable, "-c", CHILD_MULTI, REPO], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    res = eval(line[0][7:])  # noqa: S307 -- our own child's repr of tuples of str/bool/int
    for group, set0, same, rccl in res:
        assert rccl == 1, "the RCCL exchange was not selected"
        assert set0 == want[group]
        assert same


CHILD_ORDER = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
torch.cuda.init()
import msm_blst_amd as m
n, K = 1 << 16, 4
ctx = m.CHESContext(1, n_exp=16, devices=[0])
ctx.build_table(m.fixed_points(1, n), n)
raw = b"".join(bytes(m.gen_scalars(n, 1 if k == 0 else 70 + k)) for k in range(K))
host = torch.tensor(np.frombuffer(raw, dtype=np.uint8)).pin_memory()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    d = torch.empty_like(host, device="cuda:0")
    x = torch.randn(4096, 4096, device="cuda:0")
    for _ in range(30):                   # keep the caller's stream busy ...
        x = (x @ x).clamp_(-1, 1)
    d.copy_(host, non_blocking=True)      # ... so the sets land late on it
    got = [m.compress(1, r).hex() for r in ctx.mult_batch(d.data_ptr(), K, on_device=True, stream=s.cuda_stream)]
torch.cuda.synchronize()
want = [m.compress(1, ctx.mult(raw[32 * n * k:32 * n * (k + 1)])).hex() for k in range(K)]
print("RESULT", [got[0], got == want, m.lib().msm_ches_ctx_rccl_exchange(ctx._ctx)])
"""


def test_rccl_batch_waits_for_the_callers_stream(golden):
    """the RCCL exchange path (forced, one device) reads device
    scalar sets that the caller's stream is still writing; it must order after
    that stream (multi.hpp run_batch_rccl syncs it first).  The copy is queued
    behind 30 GEMMs on the caller's stream; every result must equal the
    synchronous MSM and set 0 the golden."""
    want = [c["compressed"] for c in golden("msm_g1.json")["cases"]
            if c["n"] == 1 << 16 and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == 255][0]
    env = dict(os.environ, MSM_MULTI_RCCL="1")
    r = subprocess.run([sys.executable, "-c", CHILD_ORDER, REPO], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    set0, same, rccl = eval(line[0][7:])  # noqa: S307 -- our own child's repr of a list of str/bool/int
    assert rccl == 1 and set0 == want and same
