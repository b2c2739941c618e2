"""Repeated H2D / resident headline batches in ONE process (the bench's
ches_batch_h2d leg: K = 20 distinct 2^20 scalar sets in pinned host memory,
CHES config_file_n_exp_20), for A/B studies of the batch schedule whose single
bench run is too noisy (round 4: the bimodal H2D headline).

usage: python tools/h2d_ab.py [--reps R] [--warmup W] [--steps K] [--log-n L]
Prints one line per repetition and the median / min / max of each series.
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--label", default=os.environ.get("AB_LABEL", ""))
    ap.add_argument("--profiling", type=int, default=0, help="ctx.set_profiling (bench.py turns it on)")
    ap.add_argument("--pre", type=int, default=0, help="an untimed batch of this many sets after the warm-up")
    ap.add_argument("--pre-h2d", type=int, default=0, help="the --pre batch from host memory (else resident)")
    a = ap.parse_args()
    import torch
    import msm_blst_amd as m
    from bench import make_scalar_sets
    m.lib()
    n, K, W = 1 << a.log_n, a.steps, a.warmup
    pts = m.fixed_points(1, n, 0)
    host = make_scalar_sets(m, n, K, 0, 1)
    dev = torch.device("cuda", 0)
    d_all = host.to(dev)
    sp = torch.cuda.current_stream(dev).cuda_stream
    ctx = m.CHESContext(1, 0, n_exp=a.log_n, beta=0)
    ctx.build_table(pts, n, stream=sp)
    torch.cuda.synchronize()
    ctx.set_profiling(bool(a.profiling))
    SS = n * 32

    def timed(ptr, on_device):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = ctx.mult_batch(ptr, K, 32, set_stride=SS, on_device=on_device, stream=sp)
        torch.cuda.synchronize()
        return n * K / (time.perf_counter() - t), r

    ctx.mult_batch(host.data_ptr(), min(W, K), 32, set_stride=SS, on_device=False, stream=sp)
    if a.pre:
        ctx.mult_batch(host.data_ptr() if a.pre_h2d else d_all.data_ptr(), min(a.pre, K), 32, set_stride=SS,
                       on_device=not a.pre_h2d, stream=sp)
    h2d, res, ref = [], [], None
    for i in range(a.reps):
        v, r = timed(host.data_ptr(), False)
        h2d.append(v / 1e6)
        keys = [m.compress(1, j) for j in r]
        ref = ref or keys
        v2, r2 = timed(d_all.data_ptr(), True)
        res.append(v2 / 1e6)
        same = keys == ref and [m.compress(1, j) for j in r2] == ref
        print(f"{a.label} rep {i}: h2d {h2d[-1]:.1f} M  resident {res[-1]:.1f} M  equal {same}", flush=True)
    for name, xs in (("h2d", h2d), ("resident", res)):
        print(f"{a.label} {name}: first {xs[0]:.1f} median {statistics.median(xs):.1f} min {min(xs):.1f} "
              f"max {max(xs):.1f}", flush=True)


if __name__ == "__main__":
    main()
