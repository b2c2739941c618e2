#!/usr/bin/env python3
"""Batch-rate probe used for the schedule studies of DESIGN 5
(profiles/archive_r01_r04.txt (r02_batch_sched2.txt)): G1 CHES 2^20, K distinct scalar sets, resident
and pinned-host batches, best of R runs, results checked equal across runs.
usage: exp_batch.py [K] [R]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import msm_blst_amd as m  # noqa: E402

if os.environ.get("MSM_LIB"):  # A/B of two builds on one box (e.g. tools/ablib/libmsm_prev.so)
    m._ffi.LIB_PATH = os.environ["MSM_LIB"]

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = 1 << 20
pts = m.fixed_points(1, n, 0)
host = bench.make_scalar_sets(m, n, K, 0, 1)
dev = torch.device("cuda", 0)
d_all = host.to(dev)
sp = torch.cuda.current_stream(dev).cuda_stream
ctx = m.CHESContext(1, 0, n_exp=20)
ctx.build_table(pts, n, stream=sp)
torch.cuda.synchronize()
ctx.set_profiling(True)
ref = None
for name, ptr, ondev in (("resident", d_all.data_ptr(), True), ("h2d", host.data_ptr(), False)):
    best, runs = 1e9, []
    for r in range(R):
        torch.cuda.synchronize()
        t = time.perf_counter()
        parts = ctx.mult_batch(ptr, K, 32, set_stride=n * 32, on_device=ondev, stream=sp)
        torch.cuda.synchronize()
        runs.append(n * K / (time.perf_counter() - t) / 1e6)
        best = min(best, time.perf_counter() - t)
        keys = [m.compress(1, j) for j in parts]
        ok = ref is None or keys == ref
        ref = ref or keys
    print(f"EXP {name}: {n * K / best / 1e6:.1f} M pairs/s "
          f"({best / K * 1e3:.3f} ms/MSM, acc {ctx.phase_times()['accumulate']:.3f} ms) same={ok} runs={[round(x) for x in runs]}",
          flush=True)

if os.environ.get("EXP_SYNC"):
    best = 1e9
    for r in range(R):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(K):
            ctx.mult(d_all.data_ptr() + k * n * 32, 32, on_device=True, stream=sp)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    ph = ctx.phase_times()
    print(f"EXP sync: {n * K / best / 1e6:.1f} M pairs/s ({best / K * 1e3:.3f} ms/MSM) "
          f"phases {{{', '.join(f'{k}: {v:.3f}' for k, v in ph.items())}}}", flush=True)
