"""Per-MSM fixed cost study (round 4): timings of the small plain-Pippenger and
CHES shard MSMs, run under rocprofv3 --kernel-trace to get launch counts and
per-level times.  Each case is bracketed by a marker kernel-free gap (a
host sleep) so the trace can be split by case.

usage: python tools/r04_small_trace.py [cases...]   (default: all)
"""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

import msm_blst_amd as m  # noqa: E402

dev = torch.device("cuda", 0)
K = 20


def dev_sets(n, k, seed0=1):
    import numpy as np
    raw = b"".join(m.gen_scalars(n, seed0 + i) for i in range(k))
    return torch.tensor(np.frombuffer(raw, dtype=np.uint8), device=dev)


def timed(fn, k):
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for i in range(k):
        fn(i)
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t) / k


def plain(lg, c):
    n = 1 << lg
    pts = m.fixed_points(1, n)
    d = dev_sets(n, K)
    ctx = m.MSMContext(1, 0, c)
    ctx.set_points(pts, n)
    for _ in range(3):
        ctx.mult(d.data_ptr(), 255, stride=32, on_device=True)
    time.sleep(0.05)
    ms = timed(lambda i: ctx.mult(d.data_ptr() + i * 32 * n, 255, stride=32, on_device=True), K) * 1e3
    ctx.set_profiling(True)
    ctx.mult(d.data_ptr(), 255, stride=32, on_device=True)
    ph = ctx.phase_times()
    print(f"plain 2^{lg} c={c}: {ms:.3f} ms/MSM sync = {n / ms / 1e3:.1f} M pairs/s | "
          + " ".join(f"{k}={v:.3f}" for k, v in ph.items()), flush=True)
    ctx.close()
    time.sleep(0.05)


def plain_batch(lg, c):
    n = 1 << lg
    pts = m.fixed_points(1, n)
    d = dev_sets(n, K)
    ctx = m.MSMContext(1, 0, c)
    ctx.set_points(pts, n)
    ctx.mult_batch(d.data_ptr(), K, 255, on_device=True)
    ref = [m.compress(1, ctx.mult(d.data_ptr() + i * 32 * n, 255, on_device=True)) for i in range(3)]
    time.sleep(0.05)
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        got = ctx.mult_batch(d.data_ptr(), K, 255, on_device=True)
        torch.cuda.synchronize(dev)
        best = min(best, (time.perf_counter() - t) / K * 1e3)
    ok = [m.compress(1, j) for j in got[:3]] == ref
    print(f"plain batch 2^{lg} c={c}: {best:.3f} ms/MSM = {n / best / 1e3:.1f} M pairs/s (K={K}, equals sync: {ok})",
          flush=True)
    ctx.close()
    time.sleep(0.05)


def ches(lg, beta=0):
    n = 1 << lg
    pts = m.fixed_points(1, n)
    d = dev_sets(n, K)
    ctx = m.CHESContext(1, 0, n_exp=lg, beta=beta)
    ctx.build_table(pts, n)
    p = ctx.params
    for _ in range(3):
        ctx.mult(d.data_ptr(), on_device=True)
    time.sleep(0.05)
    ms = timed(lambda i: ctx.mult(d.data_ptr() + i * 32 * n, on_device=True), K) * 1e3
    ctx.set_profiling(True)
    ctx.mult(d.data_ptr(), on_device=True)
    ph = ctx.phase_times()
    time.sleep(0.05)
    ctx.mult_batch(d.data_ptr(), K, 32, set_stride=32 * n, on_device=True)
    torch.cuda.synchronize(dev)
    time.sleep(0.05)
    t = time.perf_counter()
    ctx.mult_batch(d.data_ptr(), K, 32, set_stride=32 * n, on_device=True)
    torch.cuda.synchronize(dev)
    bms = (time.perf_counter() - t) / K * 1e3
    acc = ctx.phase_times()["accumulate"]
    print(f"ches 2^{lg} beta={beta} (q=2^{p['q_exp']} h={p['h']} |B|={p['b_size']}): sync {ms:.3f} ms "
          f"({n / ms / 1e3:.1f} M/s), batch {bms:.3f} ms/MSM ({n / bms / 1e3:.1f} M/s, acc {acc:.3f}) | sync phases "
          + " ".join(f"{k}={v:.3f}" for k, v in ph.items()), flush=True)
    ctx.close()
    time.sleep(0.05)


CASES = {
    "p10": lambda: plain(10, 10),
    "p16": lambda: plain(16, 14),
    "p16c13": lambda: plain(16, 13),
    "pb16": lambda: plain_batch(16, 14),
    "pb16c13": lambda: plain_batch(16, 13),
    "pb16c12": lambda: plain_batch(16, 12),
    "c17": lambda: ches(17),
    "c17b": lambda: ches(17, 1),
    "c18": lambda: ches(18),
    "c19": lambda: ches(19),
    "c20": lambda: ches(20),
    "c20b": lambda: ches(20, 1),
}

if __name__ == "__main__":
    for name in (sys.argv[1:] or list(CASES)):
        CASES[name]()
