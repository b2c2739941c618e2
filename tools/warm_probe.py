"""Is the slow first H2D batch a property of the host-scalar path or of a cold
GPU?  The same 20-set batch timed in the order: resident (cold), H2D, resident,
H2D, each after a 3-MSM warm-up batch of its own kind.  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import msm_blst_amd as m  # noqa: E402


def main():
    n, K, W = 1 << 20, 20, int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    pts = m.fixed_points(1, n)
    ctx = m.CHESContext(1, 0, n_exp=20)
    ctx.build_table(pts, n)
    host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
    for k in range(K):
        host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 50 + k), dtype=np.uint8)
    d = host.to(dev)
    torch.cuda.synchronize()
    ctx.set_profiling(True)
    out = []
    for tag in ("resident", "h2d", "resident", "h2d", "resident"):
        on_dev = tag == "resident"
        ptr = d.data_ptr() if on_dev else host.data_ptr()
        ctx.mult_batch(ptr, W, 32, set_stride=n * 32, on_device=on_dev)
        torch.cuda.synchronize()
        t = time.perf_counter()
        ctx.mult_batch(ptr, K, 32, set_stride=n * 32, on_device=on_dev)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        r = {"leg": tag, "ms_per_msm": round(el / K * 1e3, 4), "acc_ms": round(ctx.phase_times()["accumulate"], 4)}
        print(r, file=sys.stderr, flush=True)
        out.append(r)
    print(json.dumps({"warmup": W, "legs": out}))


if __name__ == "__main__":
    main()
