"""Does an independent H2D copy stream slow the CHES accumulations?  Resident
batch of K MSMs (scalar sets already in HBM) timed alone, then beside 80
32-MiB pinned->HBM copies (SDMA, the whole batch long) queued on an unrelated
stream, then beside 80 32-MiB HBM->HBM copies (mean and best of 3).  No dependency links the copies to the batch.  One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import msm_blst_amd as m  # noqa: E402


def main():
    n, K = 1 << 20, 20
    dev = torch.device("cuda", 0)
    pts = m.fixed_points(1, n)
    ctx = m.CHESContext(1, 0, n_exp=20)
    ctx.build_table(pts, n)
    host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
    for k in range(K):
        host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 50 + k), dtype=np.uint8)
    d = host.to(dev)
    ctx.set_profiling(True)
    side = torch.cuda.Stream(dev)
    src_h = torch.empty(32 << 20, dtype=torch.uint8, pin_memory=True)
    src_d = torch.empty(32 << 20, dtype=torch.uint8, device=dev)
    dst = torch.empty(32 << 20, dtype=torch.uint8, device=dev)
    out = {}

    def run(tag, copies=None, ncopy=0):
        ctx.mult_batch(d.data_ptr(), 3, 32, set_stride=n * 32, on_device=True)
        torch.cuda.synchronize()
        best, tot, acc = 1e9, 0.0, 0.0
        for _ in range(3):
            if copies is not None:
                with torch.cuda.stream(side):
                    for _ in range(ncopy):
                        dst.copy_(copies, non_blocking=True)
            t = time.perf_counter()
            ctx.mult_batch(d.data_ptr(), K, 32, set_stride=n * 32, on_device=True)
            el = time.perf_counter() - t
            torch.cuda.synchronize()
            best = min(best, el)
            tot += el
            acc += ctx.phase_times()["accumulate"]
        out[tag] = {"ms_per_msm_best": round(best / K * 1e3, 4), "ms_per_msm_mean": round(tot / 3 / K * 1e3, 4),
                    "acc_ms_mean": round(acc / 3, 4)}
        print(tag, out[tag], file=sys.stderr, flush=True)

    # 80 x 32 MiB back to back (~45 ms of H2D at ~57 GB/s): copies beside the whole batch
    run("alone")
    run("h2d_copies", src_h, 80)
    run("d2d_copies", src_d, 80)
    run("alone_again")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
