#!/usr/bin/env python3
"""configs[1] window sweep: the 2^16 plain-Pippenger pipelined batch (K = 20
resident sets, msm_ctx_mult_batch) at window widths c = argv (default 12..16),
each after one untimed batch; prints ms per MSM for three timed batches and
whether every c gives the same 20 results.
usage: python3 tools/cfg1_window_sweep.py [c ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import msm_blst_amd as m  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
sp = torch.cuda.current_stream(dev).cuda_stream
n, K = 1 << 16, 20
raw = b"".join(m.gen_scalars(n, 1 + k) for k in range(K))
d = torch.tensor(np.frombuffer(raw, dtype=np.uint8), device=dev)
pts = m.fixed_points(1, n)
ref = None
for c in [int(x) for x in sys.argv[1:]] or [12, 13, 14, 15, 16]:
    ctx = m.MSMContext(1, 0, c)
    ctx.set_points(pts, n, stream=sp)
    res = ctx.mult_batch(d.data_ptr(), K, 255, on_device=True, stream=sp)
    torch.cuda.synchronize(dev)
    keys = [m.compress(1, r) for r in res]
    ref = ref or keys
    ms = []
    for rep in range(3):
        t = time.perf_counter()
        ctx.mult_batch(d.data_ptr(), K, 255, on_device=True, stream=sp)
        torch.cuda.synchronize(dev)
        ms.append(round((time.perf_counter() - t) / K * 1e3, 4))
    print(f"c={c} ms per MSM {ms} same={keys == ref}", flush=True)
    ctx.close()
