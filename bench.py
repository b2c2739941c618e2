#!/usr/bin/env python3
"""bench.py -- G1 MSM point-scalar pairs/s at n=2^20 per MI355X (BASELINE.json metric).

One step = one complete G1 MSM over this rank's 2^20 fixed points with the
scalars already resident in HBM, by the reference's CHES "nh + q/5" method
(BASELINE.json configs[2]: q = 2^22, h = 12, |B| = 874 437, precomputed table
T = m q^j P_i resident in HBM): MB digit conversion -> bucket sort -> bucket
accumulation -> weighted bucket reduction, plus, for N > 1, the single exchange
of the partial sums (all_gather of 144-B Jacobians over RCCL) and their fold.
The plain Pippenger path (configs[1] method) is timed beside it (`methods`).
Weak scaling: every GPU owns its own 2^20-point shard of the sequence
P_i = 2^(i+1) G, so the job computes an MSM of N * 2^20 pairs per step.

Usage:
  python bench.py [--gpus N --steps K --warmup W]                 (N = 1)
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Prints ONE JSON line on rank 0 with value = total pairs / (max-over-ranks
time of K steps), a `roofline` object for the dominant kernel (bucket
accumulation, timed with HIP events on the stream it runs on), and a
`cpu_baseline` object (the reference's own blst_p1s_mult_pippenger built from
/root/reference into oracle/_ref, 1 thread, on the same points and scalars;
rank 0, N = 1 only; the oracle port if that build is absent).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "G1 MSM point-scalar pairs/sec at n=2^20, 1/2/4/8 MI355X; bit-exact vs CPU"
METRIC_G2 = "G2 MSM point-scalar pairs/sec at n=2^20 (BASELINE configs[4]); bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_LANE_OPS = 78.6e12   # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (one VALU op / lane / clk)
MADS_PER_FPMUL = 392           # 14x14 product + 14x14 reduction, one v_mad_u64_u32 each (fp.hpp)
FPMUL_PEAK = 76.8e9            # measured register-resident Fp-mul/s, tools/microbench/fp_rate.hip (profiles/)
AFFINE_BYTES = 96              # one G1 affine point (blst layout), SURVEY 8d
FPMUL_PER_MADD = 10            # 8M + 2S (ec_ops.h:727-748)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def timed_steps(step, ctx, steps, warmup, world, dev):
    """W untimed + K timed steps bracketed by barrier + synchronize; max over ranks."""
    import torch
    for _ in range(warmup):
        res = step()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    acc_ms, tot_ms = [], []
    t_start = time.perf_counter()
    for _ in range(steps):
        res = step()
        ph = ctx.phase_times()
        acc_ms.append(ph["accumulate"])
        tot_ms.append(ph["total"])
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return res, elapsed, acc_ms, tot_ms, ctx.phase_times()


def timed_batch(ctx, steps, warmup, world, dev, add):
    """CHES batch mode: the K steps are K MSMs issued as one pipelined batch
    (msm_ches_ctx_mult_batch: MSM k's bucket-reduction tail overlaps MSM k+1);
    for N > 1 each step's partial is then exchanged and folded.  Same bracketing
    (barrier + synchronize, max over ranks) as timed_steps."""
    import torch
    from msm_blst_amd import dist as mdist
    if warmup:
        ctx._bench_batch(warmup)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)
    ctx.set_profiling(True)
    t_start = time.perf_counter()
    parts = ctx._bench_batch(steps)
    if world > 1:
        res = [mdist.fold(mdist.gather_partials(p, ctx.group, dev), add) for p in parts][-1]
    else:
        res = parts[-1]
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t_start
    acc_ms = [ctx.phase_times()["accumulate"]]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return res, elapsed, acc_ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=20, help="points per GPU = 2^log_n")
    ap.add_argument("--method", choices=("ches", "pippenger", "bgmw"), default="ches")
    ap.add_argument("--group", type=int, choices=(1, 2), default=1,
                    help="1: G1 (the BASELINE metric); 2: G2 (configs[4], Fp2 tower), reported under its own metric")
    ap.add_argument("--window", type=int, default=16, help="plain Pippenger window bits")
    ap.add_argument("--no-compare", action="store_true", help="skip timing the other method (N = 1)")
    ap.add_argument("--no-batch", action="store_true",
                    help="CHES: time K independent synchronous MSMs instead of one pipelined batch of K")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-log-n", type=int, default=20)
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    import torch
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from msm_blst_amd import _ffi
    if not os.path.exists(_ffi.LIB_PATH):
        from msm_blst_amd import build
        build.build()
    import msm_blst_amd as m
    from msm_blst_amd import dist as mdist

    n = 1 << args.log_n
    t0 = time.time()
    start, _ = mdist.shard_range(n * world, world, rank)
    G = args.group
    pts = m.fixed_points(G, n, start)
    sc = m.gen_scalars(n, 1 + rank)
    log(f"[rank {rank}] inputs generated in {time.time() - t0:.1f}s (points {start}..{start + n})")
    stream = torch.cuda.current_stream(dev)
    d_sc = torch.frombuffer(bytearray(bytes(sc)), dtype=torch.uint8).to(dev)
    add = mdist.engine_add(G)

    def make(method):
        t = time.time()
        if method == "ches":
            ctx = m.CHESContext(G, local, n_exp=args.log_n)
            ctx.build_table(pts, n, stream=stream.cuda_stream)

            def mult():
                return ctx.mult(d_sc.data_ptr(), 32, on_device=True, stream=stream.cuda_stream)

            def mult_batch(k):  # k MSMs on the same resident scalars, pipelined (set_stride 0)
                return ctx.mult_batch(d_sc.data_ptr(), k, 32, set_stride=0, on_device=True,
                                      stream=stream.cuda_stream)
            ctx._bench_batch = mult_batch
        elif method == "bgmw":
            ctx = m.BGMWContext(G, local, n_exp=args.log_n)
            ctx.build_table(pts, n, stream=stream.cuda_stream)

            def mult():
                return ctx.mult(d_sc.data_ptr(), 32, on_device=True, stream=stream.cuda_stream)
        else:
            ctx = m.MSMContext(G, local, args.window)
            ctx.set_points(pts, n, stream=stream.cuda_stream)

            def mult():
                return ctx.mult(d_sc.data_ptr(), 255, stride=32, on_device=True, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        log(f"[rank {rank}] {method} setup {time.time() - t:.3f}s")
        ctx.set_profiling(True)

        def step():
            part = mult()
            if world > 1:
                return mdist.fold(mdist.gather_partials(part, G, dev), add)
            return part
        return ctx, step

    ctx, step = make(args.method)
    batched = args.method == "ches" and not args.no_batch
    if batched:
        res, elapsed, acc_ms = timed_batch(ctx, args.steps, args.warmup, world, dev, add)
        ctx.mult(d_sc.data_ptr(), 32, on_device=True, stream=stream.cuda_stream)  # one profiled single MSM
        phases = ctx.phase_times()
    else:
        res, elapsed, acc_ms, tot_ms, phases = timed_steps(step, ctx, args.steps, args.warmup, world, dev)

    gold = json.load(open(os.path.join(REPO, "tests", "golden", f"msm_g{G}.json")))
    want = [c["compressed"] for c in gold["cases"] if c["n"] == n and c["seed"] == 1 and c["case"] == "rand"]
    parity = (m.compress(G, res).hex() == want[0]) if (world == 1 and want) else None

    sync = None
    if batched and world == 1 and not args.no_compare:  # the same MSMs issued one by one (no overlap)
        sres, sel, _, _, sph = timed_steps(step, ctx, args.steps, 1, world, dev)
        sync = {"value": round(n * args.steps / sel, 1), "unit": "pairs/s",
                "ms_per_step": round(sel / args.steps * 1e3, 4),
                "parity_vs_reference": (m.compress(G, sres).hex() == want[0]) if want else None,
                "note": "K synchronous msm_ches_ctx_mult calls (per-MSM latency)"}
    others = {}
    if world == 1 and not args.no_compare:  # the reference's other methods, same points and scalars
        for ometh in ("ches", "pippenger", "bgmw"):
            if ometh == args.method:
                continue
            octx, ostep = make(ometh)
            k = max(5, args.steps // 2)
            ores, oel, oacc, _, oph = timed_steps(ostep, octx, k, 2, world, dev)
            others[ometh] = {"value": round(n * k / oel, 1), "unit": "pairs/s",
                             "ms_per_step": round(oel / k * 1e3, 4),
                             "phases_ms": {kk: round(v, 4) for kk, v in oph.items()},
                             "parity_vs_reference": (m.compress(G, ores).hex() == want[0]) if want else None}
            octx.close()

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    value = n * world * args.steps / elapsed
    acc_s = sum(acc_ms) / len(acc_ms) / 1e3
    if args.method == "ches":
        h = ctx.params["h"]
        madds = n * h                                 # one table point per (i, j) digit
        alg_bytes = n * h * AFFINE_BYTES * G              # h affine gathers per pair (1184 B/pair incl. scalar)
        workload = (f"G{G} MSM n=2^{args.log_n} per GPU, CHES nh+q/5 (q=2^{ctx.params['q_exp']}, h={h}, "
                    f"|B|={ctx.params['b_size']}), table T=m*q^j*P_i resident in HBM, scalars resident in HBM")
        cfg_extra = {"method": "ches_q_over_5", "q_exp": ctx.params["q_exp"], "h": h,
                     "bucket_set": ctx.params["b_size"], "buckets_incl_top_digit_copies": ctx.bucket_count()}
    elif args.method == "bgmw":
        h = ctx.h
        madds = n * h
        alg_bytes = n * h * AFFINE_BYTES * G
        workload = (f"G{G} MSM n=2^{args.log_n} per GPU, BGMW95 (q=2^{ctx.q_exp}, h={h}), table q^j*P_i resident in HBM, "
                    f"scalars resident in HBM")
        cfg_extra = {"method": "bgmw95", "q_exp": ctx.q_exp, "h": h}
    else:
        W = (255 + 1 + args.window - 1) // args.window
        madds = n * W
        alg_bytes = n * (AFFINE_BYTES * G + 32)
        workload = (f"G{G} MSM n=2^{args.log_n} per GPU, plain Pippenger c={args.window} ({W} windows), "
                    f"points+scalars resident in HBM")
        cfg_extra = {"method": "pippenger", "window_bits": args.window}
    achieved_gbs = alg_bytes / acc_s / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("method") == args.method and tj.get("log_n") == args.log_n and tj.get("group", 1) == G:
                traffic = tj.get("accumulate_bytes_per_launch")
        except Exception:
            traffic = None
    fpm_per_madd = FPMUL_PER_MADD if G == 1 else 28   # Fp2: 8M + 2S = 8*3 + 2*2 Fp-mul
    fpmul_rate = madds * fpm_per_madd / acc_s

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(m, pts, sc, args.cpu_sample_log_n if G == 1 else min(args.cpu_sample_log_n, 18), G)

    line = {
        "metric": METRIC if G == 1 else METRIC_G2,
        "value": round(value, 1),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (exact Fp381 integer arithmetic, 14x28-bit limbs)" + ("" if G == 1 else ", Fp2 = Fp[i]/(i^2+1)"),
        "data": "synthetic: P_i = 2^(i+1) G1 (main_p1.cpp:52-66), SplitMix64 scalars < r (BASELINE.md sec.3)",
        "config": dict({"workload": workload, "n_per_gpu": n, "n_total": n * world,
                        "parallelism": f"points sharded x{world}, RCCL all_gather of {144 * G}-B partials"}, **cfg_extra),
        "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved_gbs / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "kernel": "k_accumulate (bucket accumulation)", "kernel_ms": round(acc_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "note": "integer-VALU bound (v_mad_u64_u32 issue), see valu_roofline"},
        "valu_roofline": {"bound": "valu-int", "achieved": round(fpmul_rate / 1e9, 2),
                          "peak": round(FPMUL_PEAK / 1e9, 2), "unit": "G Fp-mul/s",
                          "frac": round(fpmul_rate / FPMUL_PEAK, 4),
                          "work": f"{madds} xyzz madds x {fpm_per_madd} Fp-mul",
                          "peak_basis": "measured register-resident Fp-mul kernel (tools/microbench/fp_rate.hip)"},
        "phases_ms": {k: round(v, 4) for k, v in phases.items()},
        "phases_note": "one synchronous MSM (profiled) after the timed region" if batched else "last timed step",
        "pipelined_batch": batched,
        "parity_vs_reference": parity,
        "methods": {args.method + ("_batch" if batched else ""): {"value": round(value, 1),
                                                                   "ms_per_step": round(elapsed / args.steps * 1e3, 4)},
                    **({"ches_sync": sync} if sync else {}),
                    **others},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def cpu_baseline(m, pts, sc, log_n, G=1):
    """The reference's own blst_p{1,2}s_mult_pippenger (libblst built from /root/reference
    sources into oracle/_ref/libblst_ref.so, x86-64 mulx asm), 1 thread -- the
    reference has no threading -- timed on this host's cores on the same points and
    scalars; falls back to the oracle port (oracle/msm_oracle.c) if the reference
    build is absent.  The result is cross-checked against the GPU result."""
    import ctypes
    k = 1 << log_n
    P = (ctypes.c_uint8 * (96 * G * k)).from_buffer_copy(bytes(pts)[:96 * G * k])
    S = (ctypes.c_uint8 * (32 * k)).from_buffer_copy(bytes(sc)[:32 * k])
    ref_so = os.path.join(REPO, "oracle", "_ref", "libblst_ref.so")
    if os.path.exists(ref_so):
        R = ctypes.CDLL(ref_so)
        sizeof = getattr(R, f"blst_p{G}s_mult_pippenger_scratch_sizeof")
        sizeof.restype = ctypes.c_size_t
        sizeof.argtypes = [ctypes.c_size_t]
        mult = getattr(R, f"blst_p{G}s_mult_pippenger")
        mult.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                         ctypes.c_void_p]
        scratch = (ctypes.c_uint8 * sizeof(k))()
        pp = (ctypes.c_void_p * 2)(ctypes.cast(P, ctypes.c_void_p), None)
        sp = (ctypes.c_void_p * 2)(ctypes.cast(S, ctypes.c_void_p), None)
        r = (ctypes.c_uint8 * (144 * G))()
        t = time.perf_counter()
        mult(r, pp, k, sp, 255, scratch)
        dt = time.perf_counter() - t
        out = (ctypes.c_uint8 * (48 * G))()
        getattr(R, f"blst_p{G}_compress")(out, r)
        cpu_res, kind = bytes(out).hex(), "reference"
        what = f"reference libblst blst_p{G}s_mult_pippenger (oracle/_ref)"
    else:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_ffi as of
        t = time.perf_counter()
        r = of.msm(G, P, S, k, 255, "pippenger")
        dt = time.perf_counter() - t
        cpu_res, kind, what = of.compress(G, r), "port", "oracle port of blst Pippenger (oracle/msm_oracle.c)"
    ctx = m.CHESContext(G, 0, n_exp=log_n)
    ctx.build_table(P, k)
    gpu_res = m.compress(G, ctx.mult(S)).hex()
    ctx.close()
    return {"value": round(k / dt, 1), "unit": "pairs/s", "cores": 1, "kind": kind,
            "sample": f"{what}, 1 thread, first 2^{log_n} points/scalars of the rank-0 workload, {dt:.1f}s",
            "matches_gpu": cpu_res == gpu_res}


if __name__ == "__main__":
    main()
