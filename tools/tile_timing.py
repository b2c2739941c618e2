#!/usr/bin/env python3
"""Host-side phase times of the blst-level CHES tile (bench.py tile_d_ches_legs:
main_p1.cpp:249-291 call sequence at 2^16 and 2^20, plain and registered table)
with MSM_TILE_TIMING=1 (compat.hip TileClock lines on stderr)."""
import json
import os
import sys

os.environ.setdefault("MSM_TILE_TIMING", "1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import msm_blst_amd as m  # noqa: E402

n = 1 << 20
pts = m.fixed_points(1, n)
host = torch.empty(2 * n * 32, dtype=torch.uint8, pin_memory=True)
host.numpy()[:n * 32] = np.frombuffer(m.gen_scalars(n, 1), dtype=np.uint8)
legs = bench.tile_d_ches_legs(m, pts, host)
print(json.dumps({k: {kk: v[kk] for kk in ("ms_per_step", "ctx_sync_ms", "ratio_vs_ctx_sync", "parity_vs_reference")}
                  for k, v in legs.items()}, indent=1))
