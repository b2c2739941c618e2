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
