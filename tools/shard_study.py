#!/usr/bin/env python3
"""Strong-scaling shard study (one GPU): the per-MSM time of a CHES batch on
one shard of the 2^20 problem (2^20 / N points, N = 2, 4, 8) for each of the
reference's (q, h) configurations (ches_config_files: every n_exp's q, h, a_h
is usable for any point count; the table is 3 n h rows).  Prints one JSON line
per (shard, config): resident and H2D batch ms per MSM, the 2^20 per-point
efficiency (T_2^20 / N / T_shard), and whether every configuration gives the
same set-0 result.
usage: python tools/shard_study.py [--steps K] [--logs 17,18,19] [--cfgs 22,20,19,18,16]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# (n_exp, beta) of a reference configuration file with the given q exponent
CFG_BY_Q = {22: (20, 0), 20: (18, 0), 19: (17, 1), 18: (16, 1), 16: (14, 0), 14: (12, 0), 13: (10, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--logs", default="17,18,19")
    ap.add_argument("--cfgs", default="22,20,19,18,16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--warm", type=int, default=3, help="sets in the untimed warm-up batch")
    ap.add_argument("--heat", type=int, default=0, help="bf16 GEMMs (8192^3) on the GPU right before the timed batches")
    ap.add_argument("--all", action="store_true", help="also print every repetition's ms per MSM")
    a = ap.parse_args()
    import numpy as np
    import torch
    import msm_blst_amd as m
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    K = a.steps
    base = None
    for lg in [int(x) for x in a.logs.split(",")]:
        n = 1 << lg
        pts = m.fixed_points(1, n)
        host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
        for k in range(K):
            host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 1 + k), dtype=np.uint8)
        d = host.to(dev)
        keys = {}
        for qe in [int(x) for x in a.cfgs.split(",")]:
            ne, beta = CFG_BY_Q[qe]
            t = time.time()
            ctx = m.CHESContext(1, 0, n_exp=ne, beta=beta)
            ctx.build_table(pts, n, stream=sp)
            torch.cuda.synchronize(dev)
            setup = time.time() - t
            ctx.mult_batch(host.data_ptr(), min(a.warm, K), 32, set_stride=n * 32, on_device=False, stream=sp)
            if a.heat:  # GPU busy without touching the MSM's data: clocks / power state, not caches
                x = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
                for _ in range(a.heat):
                    x = (x @ x).clamp_(-1, 1)
                torch.cuda.synchronize(dev)
                del x
            res, every = {}, {}
            for mode, ptr, on_dev in (("resident", d.data_ptr(), True), ("h2d", host.data_ptr(), False)):
                best = None
                every[mode] = []
                for _ in range(a.reps):
                    torch.cuda.synchronize(dev)
                    t = time.perf_counter()
                    out = ctx.mult_batch(ptr, K, 32, set_stride=n * 32, on_device=on_dev, stream=sp)
                    torch.cuda.synchronize(dev)
                    el = (time.perf_counter() - t) / K * 1e3
                    best = el if best is None else min(best, el)
                    every[mode].append(round(el, 4))
                res[mode] = round(best, 4)
            keys[qe] = m.compress(1, out[0]).hex()
            p = ctx.params
            line = {"log_n": lg, "q_exp": qe, "h": p["h"], "b_size": p["b_size"], "lanes": ctx.batch_lanes(),
                    "buckets": ctx.bucket_count(), "ms_resident": res["resident"], "ms_h2d": res["h2d"],
                    "setup_s": round(setup, 2)}
            if a.all:
                line["every"] = every
            ctx.close()
            print(json.dumps(line), flush=True)
        print(json.dumps({"log_n": lg, "all_configs_agree": len(set(keys.values())) == 1}), flush=True)
        del d, host


if __name__ == "__main__":
    main()
