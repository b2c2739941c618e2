#!/usr/bin/env python3
"""Kernel-trace workload for the small-MSM batches (round 6): configs[1]'s
plain-Pippenger batch (2^16, c = 14, K = 20 resident sets) and the 2^17 CHES
shard batch of `bench.py --gpus 8` (bench.ches_config(17): config_file_n_exp_17_beta.h
since round 6, K = 20 pinned host sets), each after one untimed batch, separated by 50-ms host sleeps so
tools/batch_profile.py can split the trace into segments.
usage: rocprofv3 --kernel-trace --output-format csv -d D -o run -- python3 tools/r06_small_trace.py
"""
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
K = 20
cases = sys.argv[1:] or ["pip16", "ches17"]
for case in cases:
    if case == "pip16":
        n = 1 << 16
        raw = b"".join(m.gen_scalars(n, 1 + k) for k in range(K))
        d = torch.tensor(np.frombuffer(raw, dtype=np.uint8), device=dev)
        ctx = m.MSMContext(1, 0, 14)
        ctx.set_points(m.fixed_points(1, n), n, stream=sp)
        run = lambda: ctx.mult_batch(d.data_ptr(), K, 255, on_device=True, stream=sp)  # noqa: E731
    else:
        n = 1 << 17
        host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
        for k in range(K):
            host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 1 + k), dtype=np.uint8)
        import bench  # noqa: E402
        ne, beta = bench.ches_config(17)
        ctx = m.CHESContext(1, 0, n_exp=ne, beta=beta)
        ctx.build_table(m.fixed_points(1, n), n, stream=sp)
        run = lambda: ctx.mult_batch(host.data_ptr(), K, 32, set_stride=n * 32, on_device=False, stream=sp)  # noqa: E731
    run()
    torch.cuda.synchronize(dev)
    time.sleep(0.05)
    for rep in range(2):
        t = time.perf_counter()
        run()
        torch.cuda.synchronize(dev)
        print(case, rep, round((time.perf_counter() - t) / K * 1e3, 4), "ms per MSM", flush=True)
        time.sleep(0.05)
    ctx.close()
