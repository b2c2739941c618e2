#!/usr/bin/env python3
"""Accumulation rate alone vs sets per launch (msm_ches_ctx_time_accumulation):
for each shard size and R sets in one grid, ms per launch, ms per set, and the
madd rate against the 7.32 G madd/s register-resident rate."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import msm_blst_amd as m  # noqa: E402

for lg in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "17,18,20").split(",")]:
    n = 1 << lg
    ctx = m.CHESContext(1, 0, n_exp=lg)
    ctx.build_table(m.fixed_points(1, n), n)
    R = 16 if lg < 20 else 4
    raw = b"".join(m.gen_scalars(n, 1 + k) for k in range(R))
    d = torch.tensor(np.frombuffer(raw, dtype=np.uint8), device="cuda:0")
    h = ctx.params["h"]
    for r in (1, 2, 4, 8, 16):
        if r > R:
            break
        ms = ctx.time_accumulation(d.data_ptr(), r, reps=5)
        print(json.dumps({"log_n": lg, "sets": r, "ms_launch": round(ms, 4), "ms_per_set": round(ms / r, 4),
                          "madd_rate_frac": round(n * h * r / (ms / 1e3) / 7.32e9, 3),
                          "buckets": ctx.bucket_count()}), flush=True)
    ctx.close()
