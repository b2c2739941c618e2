#!/usr/bin/env python3
"""Why the bench's 2^17-shard leg (bench.py shard_legs: 8 shard contexts, each
one warm-up batch then ONE timed H2D batch of K sets sliced out of the 2^20
sets) reads slower than tools/shard_study.py (best of 3): times 3 consecutive
H2D batches per shard, for shards 0..S-1 of the 2^20 problem.
usage: python tools/shard_leg_probe.py [--shards 8] [--use 3] [--steps 20]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import msm_blst_amd as m  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shards", type=int, default=8)
ap.add_argument("--use", type=int, default=3, help="shards timed (0 .. use-1)")
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
sp = torch.cuda.current_stream(dev).cuda_stream
K, N, n20 = a.steps, a.shards, 1 << 20
host = bench.make_scalar_sets(m, n20, K, 0, 1)
n = n20 // N
ne, cb = bench.ches_config(n.bit_length() - 1)
for r in range(a.use):
    ctx = m.CHESContext(1, 0, n_exp=ne, beta=cb)
    ctx.build_table(m.fixed_points(1, n, r * n), n, stream=sp)
    base = host.data_ptr() + r * n * 32
    ctx.mult_batch(base, K, 32, set_stride=32 << 20, on_device=False, stream=sp)
    torch.cuda.synchronize(dev)
    ts = []
    for rep in range(3):
        t = time.perf_counter()
        ctx.mult_batch(base, K, 32, set_stride=32 << 20, on_device=False, stream=sp)
        torch.cuda.synchronize(dev)
        ts.append(round((time.perf_counter() - t) / K * 1e3, 4))
    print({"shard": r, "cfg": f"q{ctx.params['q_exp']}h{ctx.params['h']}", "ms_per_msm": ts,
           "env": {k: v for k, v in os.environ.items() if k.startswith("MSM_")}}, flush=True)
    ctx.close()
