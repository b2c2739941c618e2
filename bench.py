#!/usr/bin/env python3
"""bench.py -- G1 MSM point-scalar pairs/s at n=2^20 on 1/2/4/8 MI355X (BASELINE.json metric).

One step = one complete G1 MSM of n = 2^20 point-scalar pairs by the
reference's CHES "nh + q/5" method, split over the N ranks (strong scaling,
the metric as stated: "pairs/sec at n=2^20, 1/2/4/8 MI355X"): rank r owns the
contiguous points [r 2^20/N, (r+1) 2^20/N) and the CHES table of its shard,
built with the reference's configuration for that shard size
(ches_config_files/config_file_n_exp_{20 - log2 N}.h; at N = 1 configs[2]:
q = 2^22, h = 12, |B| = 874 437, table T = m q^j P_i resident in HBM), and gets
only its shard's scalars.  Per MSM: MB digit conversion -> bucket sort ->
bucket accumulation -> weighted bucket reduction on every rank, then the single
exchange of the partial sums (all_gather of 144-B Jacobians over RCCL) and
their fold.

Headline `value` ("scalars H2D included"): the K steps are K MSMs
over K DISTINCT scalar sets that start in page-locked host memory; each set's
H2D copy is inside the timed region, issued by the pipelined batch
(msm_ches_ctx_mult_batch) on its copy stream so it overlaps earlier MSMs'
accumulations; one all_gather per batch.  value = 2^20 K / max-over-ranks time.
Reported beside it: the same batch with the scalar sets already resident in
HBM (`methods.ches_batch_resident`), K synchronous MSMs (`methods.ches_sync`),
the reference's other methods on the same points (plain Pippenger = configs[1]
method, BGMW95), and for N > 1 the weak-scaling leg (2^20 points per rank,
`methods.ches_weak_2^20_per_rank`) and configs[3] (2^21 over the ranks).

Parity (bit-exact): set 0 is the seed-1 scalar stream of BASELINE.md sec.3
(rank r takes its slice of the 2^20-scalar stream), so the folded set-0 result
must equal the golden n = 2^20 MSM of tests/golden; every batch result must
equal the synchronous MSM of the same set; the last set is recomputed by the
reference's own multi-threaded CPU grid (cpu_baseline, N = 1).

--log-n L instead fixes 2^L points per rank (weak scaling, the round-3 mode).

Usage:
  python bench.py [--gpus N --steps K --warmup W]                 (N = 1)
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "G1 MSM point-scalar pairs/sec at n=2^20, 1/2/4/8 MI355X; bit-exact vs CPU"
METRIC_G2 = "G2 MSM point-scalar pairs/sec at n=2^20 (BASELINE configs[4]); bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
MADS_PER_FPMUL = 392           # 14x14 product + 14x14 reduction, one v_mad_u64_u32 each (fp.hpp)
FPMUL_PEAK = 76.8e9            # round-2 register-resident Fp-mul/s (profiles/archive_r01_r04.txt (r02_fp_rate.txt)): fallback only, the
                               # line prices against msm_valu_probe's rates measured in the same run
MADD_RATE_R02 = 7.32e9         # round-2 register-resident G1 xyzz madd/s: fallback only
AFFINE_BYTES = 96              # one G1 affine point (blst layout), SURVEY 8d
FPMUL_PER_MADD = 10            # 8M + 2S (ec_ops.h:727-748)
MAD_RATE = 30.36e12            # round-2 chip v_mad_u64_u32 rate (profiles/archive_r01_r04.txt (r02_instr_rate.txt)): fallback only
CPU_THREADS = 16               # the GPU box's CPU share per GPU (16 threads)
CPU_SETS = 3                   # scalar sets in the 1-thread CPU sample (~12 s at 2^20)
# (group, log_n) -> the ches_config_files variant used by default: G1 2^20 keeps config_file_n_exp_20.h
# (_beta measured slower); G2 2^20 takes config_file_n_exp_20_beta.h (q = 2^20, h = 13), faster in
# 3 of 3 alternating runs, 164-167 vs 159-165 M pairs/s (profiles/r05_g2_beta_ab.txt)
DEFAULT_BETA = {(2, 20): 1}
# CHES configuration per point count (n_exp, beta of a ches_config_files header; its q, h and a_h are valid
# for any point count): the strong-scaling shards of `--gpus N` (2^20 / N points per rank) take the
# configuration MEASURED fastest for that shard size on MI355X (tools/shard_study.py,
# profiles/r05_shard_pip_study.txt), not necessarily the reference's config_file_n_exp_<log2 shard>.h
# round 6 (profiles/r06_tail_ab.txt, one box, two rounds): the 2^17 shard runs 0.410 ms per MSM with q = 2^19
# (config_file_n_exp_17_beta.h: h = 14, |B| = 109 244) vs 0.425 with q = 2^20; 2^18 keeps q = 2^20 (0.668 vs 0.721)
SHARD_CONFIG = {17: (17, 1)}


def ches_config(log_n, beta=None, group=1):
    """(n_exp, beta) of the CHES configuration for 2^log_n points per GPU."""
    if beta is not None:
        return log_n, beta
    if group == 1 and log_n in SHARD_CONFIG:
        return SHARD_CONFIG[log_n]
    return log_n, DEFAULT_BETA.get((group, log_n), 0)


def isa_mads_per_madd(G=1, path=os.path.join(REPO, "profiles", "r06_isa_counts.txt")):
    """v_mad_u64_u32 per xyzz madd on its main path, from the gfx950 ISA of the
    shipped field code (tools/isa_report.sh): the madd is 6 products (U2, S2,
    PPP, Q, ZZ3, ZZZ3), 2 squares (PP, R^2) and one fused two-product sum
    (Y3 = R (Q - X3) - S1 PPP), ec.hpp xyzz_madd.  G1: Fp ops on one lane; G2:
    the lane-pair Fp2 ops (fp2l.hpp), counted per lane, times the two lanes."""
    import re
    keys = (("k_op_fp_mulP", "k_op_fp_sqr", "k_op_fp_mul2") if G == 1 else
            ("k_op_g2l_mul_bs", "k_op_g2l_sqr", "k_op_g2l_mul_sub"))
    try:
        txt = open(path).read()
        cnt = [int(re.search(k + r"\w*\n\s+vgpr \d+ scratch \d+ total \d+ v_mad_u64_u32 (\d+)", txt).group(1))
               for k in keys]
        return (6 * cnt[0] + 2 * cnt[1] + cnt[2]) * (1 if G == 1 else 2), os.path.basename(path)
    except Exception:
        return (3567, "profiles/archive_r01_r04.txt (r03_isa_counts.txt) (constant)") if G == 1 else (None, "no lane-pair counts")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def leg(value, ms, ok=None, **kw):
    """One leg of the JSON line in its compact form (round 6: the whole line
    must fit the driver's record): M = M pairs/s, ms = ms per MSM, ok = parity
    (bit-exact vs the reference's golden result); the leg names and extra keys
    are documented in DESIGN.md sec.13."""
    d = {"M": None if value is None else round(value / 1e6, 2), "ms": None if ms is None else round(ms, 4)}
    if ok is not None:
        d["ok"] = ok
    d.update(kw)
    return d


def valu_probe(m, device):
    """The device's VALU ceilings measured now (msm_valu_probe, csrc/probe.hip):
    v_mad_u64_u32 lane-ops/s, Fp-mul/s and register-resident G1 madd/s; None
    when the library lacks the probe."""
    out = (ctypes.c_double * 4)()
    try:
        rc = m.lib().msm_valu_probe(device, out)
    except AttributeError:
        return None
    return {"mad": out[0], "fpmul": out[1], "madd": out[2], "ms": out[3]} if rc == 0 else None


class Bracket:
    """W untimed warmup already done by the caller; barrier + synchronize on both
    sides of the timed region, max over ranks."""

    def __init__(self, world, dev, xdev=None):
        self.world, self.dev, self.xdev = world, dev, xdev

    def __enter__(self):
        import torch
        if self.world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(self.dev)
        self.t = time.perf_counter()
        return self

    def __exit__(self, *exc):
        import torch
        torch.cuda.synchronize(self.dev)
        if self.world > 1:
            torch.distributed.barrier()
        el = time.perf_counter() - self.t
        if self.world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=self.xdev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        self.elapsed = el
        return False


def all_true(flag, world, dev):
    """Logical AND of a per-rank boolean (None counts as unknown -> None)."""
    if world == 1:
        return flag
    import torch
    v = torch.tensor([-1 if flag is None else int(bool(flag))], dtype=torch.int32, device=dev)
    torch.distributed.all_reduce(v, op=torch.distributed.ReduceOp.MIN)
    x = int(v.item())
    return None if x < 0 else bool(x)


def make_scalar_sets(m, n, K, rank, world):
    """K scalar sets of n 32-byte scalars in one page-locked host tensor.
    Set 0: slice `rank` of the seed-1 stream of world*n scalars (golden key);
    set k >= 1: its own seed per (k, rank)."""
    import numpy as np
    import torch
    host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
    hv = host.numpy()
    s0 = m.gen_scalars(world * n, 1)
    hv[:n * 32] = np.frombuffer(s0, dtype=np.uint8)[rank * n * 32:(rank + 1) * n * 32]
    for k in range(1, K):
        hv[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 1000 * k + rank + 1), dtype=np.uint8)
    return host


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=20,
                    help="untimed warm-up MSMs (default: one batch as long as the timed one)")
    ap.add_argument("--log-n", type=int, default=None,
                    help="weak scaling: 2^log_n points per GPU (default: strong scaling, 2^log_n_total / N per GPU)")
    ap.add_argument("--log-n-total", type=int, default=20, help="strong scaling: total points 2^log_n_total")
    ap.add_argument("--no-weak-leg", action="store_true", help="N > 1: skip the 2^20-points-per-rank leg")
    ap.add_argument("--method", choices=("ches", "pippenger", "bgmw"), default="ches")
    ap.add_argument("--group", type=int, choices=(1, 2), default=1,
                    help="1: G1 (the BASELINE metric); 2: G2 (configs[4], Fp2 tower), reported under its own metric")
    ap.add_argument("--window", type=int, default=16, help="plain Pippenger window bits")
    ap.add_argument("--beta", type=int, choices=(0, 1), default=None,
                    help="CHES/BGMW95 configuration: ches_config_files/config_file_n_exp_<log_n>[_beta].h "
                         "(default: the faster one measured on MI355X where the reference ships both)")
    ap.add_argument("--no-compare", action="store_true", help="skip the resident/sync/other-method legs")
    ap.add_argument("--no-batch", action="store_true",
                    help="CHES: time K independent synchronous MSMs instead of one pipelined batch of K")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--setup-batch", type=int, choices=(0, 1), default=0,
                    help="study knob: the context's setup ends with one untimed pipelined batch over the K resident "
                         "sets, before the W warm-up steps (measured no effect on the first timed batch, "
                         "profiles/archive_r01_r04.txt (r04_setup_batch_ab.txt))")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other BASELINE configs' legs (configs[0], [1], [4], the blst drop-in at 2^20)")
    ap.add_argument("--no-shards", action="store_true",
                    help="N = 1: skip the one-GPU projection of the N = 2/4/8 strong-scaling shards")
    ap.add_argument("--cpu-sample-log-n", type=int, default=20)
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl = RCCL over xGMI (the multi-GPU bench); gloo only for --one-device rehearsals")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses device 0 (with --dist-backend gloo)")
    ap.add_argument("--multi-context", type=int, default=0, metavar="D",
                    help="N = 1: also time configs[3] (2^21 points) through ONE process driving D shards "
                         "(msm_ches_ctx_create_multi; devices 0..D-1, or D shards on device 0 with --one-device)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")

    if args.log_n is None:  # strong scaling: one 2^log_n_total MSM split over the ranks
        if world & (world - 1) or world > (1 << args.log_n_total):
            raise SystemExit(f"strong scaling needs a power-of-two world size <= 2^{args.log_n_total}, got {world}")
        args.log_n = args.log_n_total - (world.bit_length() - 1)
        scaling = "strong"
    else:
        scaling = "weak"
    import torch
    if args.one_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    xdev = dev if args.dist_backend == "nccl" else None  # where exchanged tensors live

    import msm_blst_amd as m
    from msm_blst_amd import dist as mdist
    m.lib()  # fails loudly when the HIP library is missing (build() first)

    n, G, K, W = 1 << args.log_n, args.group, args.steps, args.warmup
    t0 = time.time()
    start, _ = mdist.shard_range(n * world, world, rank)
    pts = m.fixed_points(G, n, start)
    host = make_scalar_sets(m, n, K, rank, world)
    log(f"[rank {rank}] inputs generated in {time.time() - t0:.1f}s (points {start}..{start + n}, {K} scalar sets)")
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    d_all = host.to(dev)  # the same K sets resident in HBM (resident / sync legs)
    hptr, dptr, SS = host.data_ptr(), d_all.data_ptr(), n * 32
    add = mdist.engine_add(G)

    def keys(jacs):  # canonical comparison key: the compressed affine point (Jacobians differ in representative)
        return [m.compress(G, j) for j in jacs]

    def fold_all(parts):
        if world == 1:
            return parts
        return [mdist.fold(ps, add) for ps in mdist.gather_partials_batch(parts, G, xdev)]

    cfg_n, beta = ches_config(args.log_n, args.beta, G)  # the config file this point count uses (SHARD_CONFIG)

    def has_config(b):
        try:
            m.ches.params(cfg_n, b)
            return True
        except Exception:
            return False

    if not has_config(beta):
        log(f"no reference configuration n_exp={cfg_n} beta={beta}; using n_exp={args.log_n} beta=0")
        cfg_n, beta = args.log_n, 0

    def make(method, b=None):
        t = time.time()
        b = beta if b is None else b
        if method == "ches":
            ctx = m.CHESContext(G, local, n_exp=cfg_n, beta=b)
            ctx.build_table(pts, n, stream=sp)
        elif method == "bgmw":
            ctx = m.BGMWContext(G, local, n_exp=args.log_n, beta=b)
            ctx.build_table(pts, n, stream=sp)
        else:
            ctx = m.MSMContext(G, local, args.window)
            ctx.set_points(pts, n, stream=sp)
        torch.cuda.synchronize(dev)
        log(f"[rank {rank}] {method} setup {time.time() - t:.3f}s")
        ctx.set_profiling(True)

        def mult(k, on_device=True):
            base = (dptr if on_device else hptr) + k * SS
            if method == "pippenger":
                return ctx.mult(base, 255, stride=32, on_device=on_device, stream=sp)
            return ctx.mult(base, 32, on_device=on_device, stream=sp)
        return ctx, mult

    def sync_steps(mult, k_steps, on_device):
        """k_steps synchronous MSMs over sets 0..k_steps-1 (exchange + fold per step)."""
        out = []
        with Bracket(world, dev, xdev) as b:
            for k in range(k_steps):
                part = mult(k, on_device)
                out.append(part if world == 1 else mdist.fold(mdist.gather_partials(part, G, xdev), add))
        return out, b.elapsed

    ctx, mult = make(args.method)
    batched = args.method == "ches" and not args.no_batch
    legs = {}
    if batched:
        if args.setup_batch:  # part of the context's setup, before the W warm-up steps (see --setup-batch)
            ctx.mult_batch(dptr, K, 32, set_stride=SS, on_device=True, stream=sp)
            torch.cuda.synchronize(dev)
        if W:
            ctx.mult_batch(hptr, min(W, K), 32, set_stride=SS, on_device=False, stream=sp)
        with Bracket(world, dev, xdev) as b:  # headline: host scalars, H2D inside the pipeline
            parts = ctx.mult_batch(hptr, K, 32, set_stride=SS, on_device=False, stream=sp)
            res = fold_all(parts)
        elapsed, acc_ms = b.elapsed, ctx.phase_times()["accumulate"]
        legs["ches_h2d"] = leg(n * world * K / elapsed, elapsed / K * 1e3, kernel_ms=round(acc_ms, 4))
        if not args.no_compare:
            with Bracket(world, dev, xdev) as b:
                rparts = fold_all(ctx.mult_batch(dptr, K, 32, set_stride=SS, on_device=True, stream=sp))
            legs["ches_res"] = leg(n * world * K / b.elapsed, b.elapsed / K * 1e3, keys(rparts) == keys(res),
                                   kernel_ms=round(ctx.phase_times()["accumulate"], 4))
            if world == 1 and has_config(1 - beta):  # the reference's other configuration for this n
                octx, _ = make("ches", 1 - beta)
                octx.mult_batch(dptr, min(max(W, 1), K), 32, set_stride=SS, on_device=True, stream=sp)
                with Bracket(world, dev, xdev) as b:
                    oparts = octx.mult_batch(dptr, K, 32, set_stride=SS, on_device=True, stream=sp)
                op = octx.params
                legs[f"ches_res_beta{1 - beta}"] = leg(n * K / b.elapsed, b.elapsed / K * 1e3, keys(oparts) == keys(res),
                                                       kernel_ms=round(octx.phase_times()["accumulate"], 4),
                                                       cfg=f"q{op['q_exp']}h{op['h']}")
                octx.close()
            sres, sel = sync_steps(mult, K, True)
            batch_eq_sync = keys(sres) == keys(res)
            legs["ches_sync"] = leg(n * world * K / sel, sel / K * 1e3, batch_eq_sync)
        else:
            batch_eq_sync = None
        mult(0)  # one profiled synchronous MSM for the phase split
        phases = ctx.phase_times()
    else:
        for k in range(W):
            mult(k % K, False)
        res, elapsed = sync_steps(mult, K, False)
        phases = ctx.phase_times()
        acc_ms = phases["accumulate"]
        batch_eq_sync = None
        legs[args.method + "_sync_h2d"] = leg(n * world * K / elapsed, elapsed / K * 1e3)

    # ---- parity ----
    gold = json.load(open(os.path.join(REPO, "tests", "golden", f"msm_g{G}.json")))
    want = [c["compressed"] for c in gold["cases"]
            if c["n"] == n * world and c["seed"] == 1 and c["case"] == "rand"]
    golden_ok = (m.compress(G, res[0]).hex() == want[0]) if want else None
    cross = None
    if world > 1 and not want:  # no golden for this total size: plain Pippenger on the same shard and set 0
        pctx = m.MSMContext(G, local, args.window)
        pctx.set_points(pts, n, stream=sp)
        pp = pctx.mult(dptr, 255, stride=32, on_device=True, stream=sp)
        mine = ctx.mult(dptr, 32, on_device=True, stream=sp) if args.method != "pippenger" else pp
        cross = all_true(m.compress(G, pp) == m.compress(G, mine), world, xdev)
        pctx.close()

    # the device's VALU ceilings, measured now (after the timed region, GPU warm):
    # twice, keeping the higher rate (the first call also warms the probe kernels)
    probe = None
    for _ in range(2):
        p = valu_probe(m, local)
        if p is not None:
            probe = p if probe is None else {k: max(probe[k], p[k]) for k in p}
    others = {}
    if world == 1 and not args.no_compare:  # the reference's other methods, same points, resident sets
        for ometh in ("ches", "pippenger", "bgmw"):
            if ometh == args.method:
                continue
            octx, omult = make(ometh)
            k = max(5, K // 2)
            for _ in range(2):
                omult(0)
            ores, oel = sync_steps(omult, k, True)
            others[ometh[:4] + "_sync"] = leg(n * k / oel, oel / k * 1e3,
                                             ((m.compress(G, ores[0]).hex() == want[0]) if want else True)
                                             and keys(ores) == keys(res[:k]))
            octx.close()

    if world == 1 and not args.no_compare and not args.no_shards and G == 1 and args.log_n == 20 and batched:
        others.update(shard_legs(m, mdist, torch, dev, local, sp, host, K, W, n * K / elapsed))
    if world == 1 and not args.no_compare and not args.no_configs and G == 1 and args.log_n == 20:
        others.update(config_legs(m, torch, dev, local, sp, pts, host, K, W, probe))
    # configs[3]: G1 n = 2^21 sharded over the ranks (RCCL path) or over the
    # shards of one process (--multi-context), against the golden 2^21 result
    if G == 1 and not args.no_compare and world > 1 and (1 << 21) % world == 0:
        others.update(cfg3_ranks(m, mdist, torch, dev, local, sp, world, rank, K, W, xdev, add))
    if G == 1 and not args.no_compare and world > 1 and scaling == "strong" and not args.no_weak_leg:
        others.update(weak_leg(m, mdist, torch, dev, local, sp, world, rank, K, W, xdev, add))
    if G == 1 and world == 1 and args.multi_context > 1:
        others.update(cfg3_multi_context(m, torch, args.multi_context, args.one_device, K, W))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(m, pts, host, n, K, res, G, args.cpu_sample_log_n if G == 1 else min(args.cpu_sample_log_n, 18))

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    value = n * world * K / elapsed
    acc_s = acc_ms / 1e3
    if args.method == "ches":
        h = ctx.params["h"]
        madds = n * h                                 # one table point per (i, j) digit
        alg_bytes = n * h * AFFINE_BYTES * G              # h affine gathers per pair (1184 B/pair incl. scalar)
        workload = (f"G{G} MSM n=2^{args.log_n} per GPU, CHES nh+q/5, table in HBM, K distinct scalar sets H2D "
                    f"from pinned host memory in the timed region")
        cfg_extra = {"method": "ches_q_over_5",
                     "config_file": f"config_file_n_exp_{cfg_n}{'_beta' if beta else ''}.h",
                     "q_exp": ctx.params["q_exp"], "h": h,
                     "bucket_set": ctx.params["b_size"], "buckets_incl_top_digit_copies": ctx.bucket_count()}
    elif args.method == "bgmw":
        h = ctx.h
        madds = n * h
        alg_bytes = n * h * AFFINE_BYTES * G
        workload = (f"G{G} MSM n=2^{args.log_n} per GPU, BGMW95 (q=2^{ctx.q_exp}, h={h}), table q^j*P_i resident in HBM, "
                    f"scalars H2D per MSM")
        cfg_extra = {"method": "bgmw95", "q_exp": ctx.q_exp, "h": h}
    else:
        Wn = (255 + 1 + args.window - 1) // args.window
        madds = n * Wn
        alg_bytes = n * (AFFINE_BYTES * G + 32)
        workload = (f"G{G} MSM n=2^{args.log_n} per GPU, plain Pippenger c={args.window} ({Wn} windows), "
                    f"points resident in HBM, scalars H2D per MSM")
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
    mads, mads_src = isa_mads_per_madd(G)
    acc_alone = phases.get("accumulate") and phases["accumulate"] / 1e3
    # VALU roofline, priced against ceilings measured in THIS run on this device
    # (msm_valu_probe, csrc/probe.hip): the register-resident G1 madd loop (the
    # accumulation's body without its row loads) and the chip's v_mad_u64_u32
    # rate.  G2 has no madd probe: its valu fraction is the mad fraction.
    pk = probe or {"mad": MAD_RATE, "madd": MADD_RATE_R02, "fpmul": FPMUL_PEAK}
    mad_frac = round(madds * mads / acc_s / pk["mad"], 4) if mads else None
    mad_frac_alone = round(madds * mads / acc_alone / pk["mad"], 4) if mads and acc_alone else None
    valu = {"valu_bound": "valu-int (v_mad_u64_u32 issue)",
            "valu_unit": "G madd/s" if G == 1 else "T mad/s",
            "valu_achieved": round(madds / acc_s / 1e9, 3) if G == 1 else round(madds * mads / acc_s / 1e12, 3),
            "valu_peak": round(pk["madd"] / 1e9, 3) if G == 1 else round(pk["mad"] / 1e12, 3),
            "valu_frac": round(madds / acc_s / pk["madd"], 4) if G == 1 else mad_frac,
            "valu_frac_alone": (round(madds / acc_alone / pk["madd"], 4) if acc_alone else None) if G == 1
            else mad_frac_alone,
            "mad_frac": mad_frac, "mad_frac_alone": mad_frac_alone, "mads_per_madd": mads,
            "mad_peak_T": round(pk["mad"] / 1e12, 3), "fpmul_peak_G": round(pk["fpmul"] / 1e9, 2),
            "peak_basis": "this run (msm_valu_probe)" if probe else "round-2 constants (probe unavailable)"}

    parity = golden_ok if golden_ok is not None else cross
    if batch_eq_sync is False:
        parity = False
    line = {
        "legs": dict(legs, **others),
        "legs_key": "M = M pairs/s, ms = ms per MSM, ok = bit-exact vs the reference; DESIGN.md sec.13",
        "phases_ms": [round(v, 4) for v in phases.values()],
        "parity_detail": {"set0_golden": golden_ok, "batch_eq_sync": batch_eq_sync, "pip_cross_ranks": cross},
        "metric": METRIC if G == 1 else METRIC_G2,
        "value": round(value, 1),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32 (exact Fp381 integer arithmetic, 14x28-bit limbs)" + ("" if G == 1 else ", Fp2 = Fp[i]/(i^2+1)"),
        "data": ("synthetic: P_i = 2^(i+1) G%d (main_p1.cpp:52-66), SplitMix64 scalars < r (BASELINE.md sec.3), "
                 "K distinct scalar sets" % G),
        "config": dict({"workload": workload, "n_per_gpu": n, "n_total": n * world,
                        "parallelism": (f"one n=2^{args.log_n + world.bit_length() - 1} MSM: points sharded x{world}, "
                                        f"RCCL all_gather of {144 * G}-B partials" if world > 1 else "1 GPU")},
                       **cfg_extra),
        "roofline": dict({"bound": "hbm", "achieved": round(achieved_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(achieved_gbs / HBM_PEAK_GBS, 5), "traffic": traffic,
                          "kernel": "k_accumulate", "kernel_ms": round(acc_s * 1e3, 4),
                          "kernel_ms_alone": round(acc_alone * 1e3, 4) if acc_alone else None,
                          "algorithmic_bytes_per_launch": alg_bytes}, **valu),
        "cpu_baseline": cpu,
        "parity_vs_reference": parity,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def _golden(m, G, n):
    gold = json.load(open(os.path.join(REPO, "tests", "golden", f"msm_g{G}.json")))
    want = [c["compressed"] for c in gold["cases"] if c["n"] == n and c["seed"] == 1 and c["case"] == "rand"
            and c["nbits"] == 255]
    return want[0] if want else None


def config_legs(m, torch, dev, local, sp, pts, host, K, W, probe):
    """The other single-GPU BASELINE configs and the blst drop-in boundary, each
    timed and parity-checked against the reference's golden (set 0 = the seed-1
    stream, whose first 2^k scalars are the seed-1 set of 2^k points):
      configs[1]  G1 n=2^16 plain Pippenger: device-resident context (scalar sets
                  resident) and the blst drop-in blst_p1s_mult_pippenger (points
                  and scalars in the caller's pageable host memory, per call)
      boundary    blst_p1s_mult_pippenger at n=2^20 (the north star's
                  pippenger_blst_built_in, main_p1.cpp:400-436), per call
      configs[4]  G2 n=2^20 CHES batch (table resident), scalars H2D / resident
      configs[0]  G1 n=2^10 on the CPU: the reference's blst_p1s_mult_pippenger
                  (oracle/_ref), beside the GPU drop-in at the same size"""
    import numpy as np
    legs = {}
    hv = host.numpy()
    nsets = host.numel() // (32 << 20)

    def set_bytes(k, n):  # first n scalars of set k, in fresh pageable host memory
        off = (k % nsets) * (32 << 20)
        return (ctypes.c_uint8 * (32 * n)).from_buffer_copy(hv[off:off + 32 * n].tobytes())

    def dropin(G, P, S, n):
        pp = (ctypes.c_void_p * 2)(ctypes.cast(P, ctypes.c_void_p), None)
        spp = (ctypes.c_void_p * 2)(ctypes.cast(S, ctypes.c_void_p), None)
        r = (ctypes.c_uint8 * (144 * G))()
        getattr(m.lib(), f"blst_p{G}s_mult_pippenger")(r, pp, n, spp, 255, None)
        return bytes(r)

    def timed(fn, k):
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        out = [fn(i) for i in range(k)]
        torch.cuda.synchronize(dev)
        return out, time.perf_counter() - t

    # ---- configs[1]: G1 2^16 plain Pippenger ----
    n16 = 1 << 16
    P16 = (ctypes.c_uint8 * (96 * n16)).from_buffer_copy(bytes(pts)[:96 * n16])
    want16 = _golden(m, 1, n16)
    sets16 = [set_bytes(k, n16) for k in range(K)]
    d16 = torch.tensor(np.frombuffer(b"".join(bytes(x) for x in sets16), dtype=np.uint8), device=dev)
    for c in (13, 14):  # blst's rule for 2^16 (multi_scalar.c:268-275) / the drop-in's measured best
        pc = m.MSMContext(1, local, c)
        pc.set_points(P16, n16, stream=sp)
        pc.mult(d16.data_ptr(), 255, stride=32, on_device=True, stream=sp)
        r, el = timed(lambda k: pc.mult(d16.data_ptr() + k * 32 * n16, 255, stride=32, on_device=True, stream=sp), K)
        pc.set_profiling(True)
        pc.mult(d16.data_ptr(), 255, stride=32, on_device=True, stream=sp)
        legs[f"cfg1_ctx_c{c}"] = leg(n16 * K / el, el / K * 1e3, m.compress(1, r[0]).hex() == want16,
                                     phases=[round(v, 4) for v in pc.phase_times().values()])
        # the same K sets through the pipelined batch (msm_ctx_mult_batch): throughput
        pc.mult_batch(d16.data_ptr(), K, 255, on_device=True, stream=sp)  # untimed: sizes the batch buffers
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        rb = pc.mult_batch(d16.data_ptr(), K, 255, on_device=True, stream=sp)
        torch.cuda.synchronize(dev)
        elb = time.perf_counter() - t
        # ms_steady: two more batches right after the timed one (the timed batch is the first after one
        # untimed batch; later ones run ~3-5 % faster as the board's clocks settle)
        more = []
        for _ in range(2):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            pc.mult_batch(d16.data_ptr(), K, 255, on_device=True, stream=sp)
            torch.cuda.synchronize(dev)
            more.append((time.perf_counter() - t) / K * 1e3)
        legs[f"cfg1_batch_c{c}"] = leg(n16 * K / elb, elb / K * 1e3, m.compress(1, rb[0]).hex() == want16
                                       and [m.compress(1, x) for x in rb] == [m.compress(1, x) for x in r],
                                       ms_steady=round(min(more), 4))
        pc.close()
    for _ in range(max(W, 1)):
        dropin(1, P16, sets16[0], n16)
    r, el = timed(lambda k: dropin(1, P16, sets16[k], n16), K)
    legs["cfg1_dropin"] = leg(n16 * K / el, el / K * 1e3, m.compress(1, r[0]).hex() == want16)
    del d16

    # ---- the blst drop-in at 2^20 ----
    n20 = 1 << 20
    P20 = (ctypes.c_uint8 * (96 * n20)).from_buffer_copy(bytes(pts)[:96 * n20])
    k20 = min(K, 10)
    sets20 = [set_bytes(k, n20) for k in range(k20)]
    for _ in range(max(W, 1)):
        dropin(1, P20, sets20[0], n20)
    r, el = timed(lambda k: dropin(1, P20, sets20[k], n20), k20)
    legs["dropin20"] = leg(n20 * k20 / el, el / k20 * 1e3, m.compress(1, r[0]).hex() == _golden(m, 1, n20))
    # the same calls with the point array registered once (msm_register_host_table): no point upload
    L = m.lib()
    if L.msm_register_host_table(1, P20, n20) == 0:
        for _ in range(2):
            dropin(1, P20, sets20[0], n20)
        r, el = timed(lambda k: dropin(1, P20, sets20[k], n20), k20)
        L.msm_unregister_host_table(P20)
        legs["dropin20_reg"] = leg(n20 * k20 / el, el / k20 * 1e3, m.compress(1, r[0]).hex() == _golden(m, 1, n20))
    del sets20, P20

    # ---- configs[0]: CPU reference at 2^10, and the drop-in at the same size ----
    n10 = 1 << 10
    P10 = (ctypes.c_uint8 * (96 * n10)).from_buffer_copy(bytes(pts)[:96 * n10])
    S10 = set_bytes(0, n10)
    want10 = _golden(m, 1, n10)
    R = _ref_lib("libblst_ref.so")
    if R is not None:
        mult = R.blst_p1s_mult_pippenger
        mult.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        R.blst_p1s_mult_pippenger_scratch_sizeof.restype = ctypes.c_size_t
        R.blst_p1s_mult_pippenger_scratch_sizeof.argtypes = [ctypes.c_size_t]
        scratch = (ctypes.c_uint8 * R.blst_p1s_mult_pippenger_scratch_sizeof(n10))()
        pp = (ctypes.c_void_p * 2)(ctypes.cast(P10, ctypes.c_void_p), None)
        spp = (ctypes.c_void_p * 2)(ctypes.cast(S10, ctypes.c_void_p), None)
        rr = (ctypes.c_uint8 * 144)()
        reps, t = 0, time.perf_counter()
        while reps < 5 or time.perf_counter() - t < 0.5:
            mult(rr, pp, n10, spp, 255, scratch)
            reps += 1
        el = time.perf_counter() - t
        legs["cfg0_cpu_ref"] = leg(n10 * reps / el, el / reps * 1e3, m.compress(1, bytes(rr)).hex() == want10)
    for _ in range(3):
        dropin(1, P10, S10, n10)
    r, el = timed(lambda k: dropin(1, P10, S10, n10), 20)
    legs["cfg0_gpu_dropin"] = leg(n10 * 20 / el, el / 20 * 1e3, m.compress(1, r[0]).hex() == want10)

    # ---- the blst-level CHES tile (main_p1.cpp:249-291 call sequence) at 2^16 and 2^20 ----
    legs.update(tile_d_ches_legs(m, pts, host))

    # ---- configs[4]: G2 2^20 CHES batch ----
    t = time.time()
    pts2_host = m.fixed_points(2, n20)
    c2 = m.CHESContext(2, local, n_exp=20, beta=ches_config(20, group=2)[1])
    c2.build_table(pts2_host, n20, stream=sp)
    c2.set_profiling(True)
    torch.cuda.synchronize(dev)
    setup = time.time() - t
    k2 = K  # the headline's batch length
    hptr, SS = host.data_ptr(), 32 * n20
    d2 = host[:k2 * SS].to(dev)
    c2.mult_batch(hptr, min(max(W, 1), k2), 32, set_stride=SS, on_device=False, stream=sp)
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    bh = c2.mult_batch(hptr, k2, 32, set_stride=SS, on_device=False, stream=sp)
    torch.cuda.synchronize(dev)
    elh = time.perf_counter() - t
    acc_h = c2.phase_times()["accumulate"]
    t = time.perf_counter()
    br = c2.mult_batch(d2.data_ptr(), k2, 32, set_stride=SS, on_device=True, stream=sp)
    torch.cuda.synchronize(dev)
    elr = time.perf_counter() - t
    sync = [c2.mult(d2.data_ptr() + k * SS, 32, on_device=True, stream=sp) for k in range(2)]
    c2.set_profiling(True)
    c2.mult(d2.data_ptr(), 32, on_device=True, stream=sp)
    ph = c2.phase_times()
    eq = [m.compress(2, x) for x in bh[:2]] == [m.compress(2, x) for x in sync] and \
        [m.compress(2, x) for x in br] == [m.compress(2, x) for x in bh]
    par = c2.params
    mads2, _ = isa_mads_per_madd(2)
    legs["cfg4_g2_h2d"] = leg(n20 * k2 / elh, elh / k2 * 1e3, m.compress(2, bh[0]).hex() == _golden(m, 2, n20) and eq,
                              kernel_ms=round(acc_h, 4), cfg=f"q{par['q_exp']}h{par['h']}",
                              mad_frac_alone=(round(n20 * par["h"] * mads2 / (ph["accumulate"] / 1e3) / probe["mad"], 4)
                                              if probe and mads2 else None),
                              phases=[round(v, 4) for v in ph.values()])
    # the G2 blst drop-in at 2^20 (main_p2.cpp:424 pippenger_blst_built_in): points + scalars per call
    P2 = (ctypes.c_uint8 * (192 * n20)).from_buffer_copy(bytes(pts2_host))
    S2 = set_bytes(0, n20)
    dropin(2, P2, S2, n20)
    r2, el2 = timed(lambda k: dropin(2, P2, S2, n20), 3)
    legs["g2_dropin20"] = leg(n20 * 3 / el2, el2 / 3 * 1e3, m.compress(2, r2[0]).hex() == _golden(m, 2, n20))
    del P2, pts2_host
    legs["cfg4_g2_res"] = leg(n20 * k2 / elr, elr / k2 * 1e3, m.compress(2, br[0]).hex() == _golden(m, 2, n20))
    c2.close()
    del d2
    return legs


def _std_digits(raw, n, q_exp, h):
    """trans_uint256_t_to_standard_q_ary_expr (ref auxiliaryfunc.h:83-90) of n
    32-byte scalars: n h ints, digit j of scalar i at i h + j, plus 2 pad slots
    (main_p1.cpp:254)."""
    import numpy as np
    w = np.frombuffer(raw, dtype=np.uint64, count=4 * n).reshape(n, 4)
    out = np.zeros(n * h + 2, dtype=np.int32)
    mask = np.uint64((1 << q_exp) - 1)
    for j in range(h):
        o = q_exp * j
        wi, sh = o // 64, o % 64
        v = w[:, wi] >> np.uint64(sh)
        if sh and wi + 1 < 4:
            v = v | (w[:, wi + 1] << np.uint64(64 - sh))
        out[j:n * h:h] = (v & mask).astype(np.int32)
    return out


def tile_d_ches_legs(m, pts, host):
    """The blst-level CHES tile through the reference driver's method-2 call
    sequence (main_p1.cpp:249-291): standard q-ary digits of every scalar,
    blst_p1_construct_nh_scalars_nh_points (MB digits + one pointer per entry
    into the host table T[3 n h], main_p1.cpp:155-172), then
    blst_p1_tile_pippenger_d_CHES over the n h pointers -- the boundary hands the
    table over by pointer, so every call gathers and uploads n h rows (1.2 GB
    at 2^20) before the same GPU accumulation and reduction as the context.
    Timed: the tile call; parity: set 0 against the golden MSM."""
    import numpy as np
    vp, sz, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L = m.lib()
    L.blst_p1_construct_nh_scalars_nh_points.argtypes = [vp, vp, vp, sz, vp, vp]
    L.blst_p1_tile_pippenger_d_CHES.argtypes = [vp, vp, sz, vp, vp, vp, vp, vp, sz, i32]
    L.msm_register_host_table.argtypes = [i32, vp, sz]
    L.msm_unregister_host_table.argtypes = [vp]
    legs = {}
    hv = host.numpy()
    for lg in (16, 20):
        n = 1 << lg
        ctx = m.CHESContext(1, 0, n_exp=lg)
        ctx.build_table(bytes(pts)[:96 * n], n)
        p = ctx.params
        T = ctx.get_table()
        ctx.mult(hv[:32 * n].tobytes())
        t = time.perf_counter()
        for _ in range(3):
            ctx.mult(hv[:32 * n].tobytes())
        sync_ms = (time.perf_counter() - t) / 3 * 1e3
        ctx.close()
        q, h = 1 << p["q_exp"], p["h"]
        B = m.ches.bucket_set(q, p["a_h"])
        H = m.ches.digit_table(q, p["a_h"])
        Bn = np.frombuffer(B, dtype=np.int32)
        v2i_np = np.zeros(int(Bn[-1]) + 1, dtype=np.int32)
        v2i_np[Bn] = np.arange(len(Bn), dtype=np.int32)
        v2i = (ctypes.c_int * len(v2i_np)).from_buffer_copy(v2i_np.tobytes())
        ne = n * h
        t0 = time.perf_counter()
        nh_np = _std_digits(hv[:32 * n].tobytes(), n, p["q_exp"], h)
        nh = (ctypes.c_int * len(nh_np)).from_buffer_copy(nh_np.tobytes())
        signs = (ctypes.c_ubyte * ne)()
        ptrs = (ctypes.c_void_p * ne)()
        L.blst_p1_construct_nh_scalars_nh_points(nh, signs, ptrs, ne, T, H)
        prep = time.perf_counter() - t0
        buckets = (ctypes.c_uint8 * (192 * len(B)))()
        ret = (ctypes.c_uint8 * 144)()
        L.blst_p1_tile_pippenger_d_CHES(ret, ptrs, ne, nh, signs, buckets, B, v2i, len(B), p["d_max"])
        reps = 3
        t = time.perf_counter()
        for _ in range(reps):
            L.blst_p1_tile_pippenger_d_CHES(ret, ptrs, ne, nh, signs, buckets, B, v2i, len(B), p["d_max"])
        el = (time.perf_counter() - t) / reps
        legs[f"tile{lg}"] = leg(n / el, el * 1e3, m.compress(1, bytes(ret)).hex() == _golden(m, 1, n),
                                ratio=round(el * 1e3 / sync_ms, 2))
        # the same calls after registering the host table once (msm_register_host_table): row indices
        # instead of gathered rows
        t = time.perf_counter()
        rc = L.msm_register_host_table(1, T, 3 * n * h)
        reg_s = time.perf_counter() - t
        if rc == 0:
            L.blst_p1_tile_pippenger_d_CHES(ret, ptrs, ne, nh, signs, buckets, B, v2i, len(B), p["d_max"])
            t = time.perf_counter()
            for _ in range(reps):
                L.blst_p1_tile_pippenger_d_CHES(ret, ptrs, ne, nh, signs, buckets, B, v2i, len(B), p["d_max"])
            el = (time.perf_counter() - t) / reps
            L.msm_unregister_host_table(T)
            legs[f"tile{lg}_reg"] = leg(n / el, el * 1e3, m.compress(1, bytes(ret)).hex() == _golden(m, 1, n),
                                        ratio=round(el * 1e3 / sync_ms, 2))
        del T, ptrs, nh, signs, buckets
    return legs


def shard_legs(m, mdist, torch, dev, local, sp, host, K, W, headline_value):
    """The metric's N-GPU strong-scaling shards, measured on ONE GPU (a
    projection, not a scaling number): the 2^20 problem of the headline split
    into N = 2, 4, 8 contiguous shards exactly as `bench.py --gpus N` splits it
    (rank r: points [r 2^20/N, (r+1) 2^20/N), the CHES configuration
    ches_config(20 - log2 N), the r-th slice of each of the K pinned host sets).
    Every shard runs the same pipelined H2D batch of K sets the rank would run,
    one shard after another on device 0; per_shard_ms = the slowest shard's ms
    per MSM, projected_value = 2^20 K / (K per_shard_ms) -- the N-GPU rate if
    the ranks ran at this speed side by side with a free exchange -- and
    efficiency = projected_value / (N x the headline value).  Parity: set 0's
    shard partials folded (exact host add) against the 2^20 golden; each shard's
    batch against its synchronous MSM on sets 0 and K-1."""
    n20, SS = 1 << 20, 32 << 20
    add = mdist.engine_add(1)
    want = _golden(m, 1, n20)
    hptr = host.data_ptr()
    out = {}
    for N in (2, 4, 8):
        n = n20 // N
        lg = n.bit_length() - 1
        n_exp, cbeta = ches_config(lg)
        times, parts0, eqs, setup, params = [], [], [], 0.0, None
        for r in range(N):
            t = time.time()
            ctx = m.CHESContext(1, local, n_exp=n_exp, beta=cbeta)
            ctx.build_table(m.fixed_points(1, n, r * n), n, stream=sp)
            torch.cuda.synchronize(dev)
            setup += time.time() - t
            params = ctx.params
            base = hptr + r * n * 32
            ctx.mult_batch(base, min(max(W, 1), K), 32, set_stride=SS, on_device=False, stream=sp)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            res = ctx.mult_batch(base, K, 32, set_stride=SS, on_device=False, stream=sp)
            torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t)
            parts0.append(res[0])
            sync = [ctx.mult(base + k * SS, 32, on_device=False, stream=sp) for k in (0, K - 1)]
            eqs.append([m.compress(1, x) for x in sync] == [m.compress(1, res[0]), m.compress(1, res[K - 1])])
            lanes = ctx.batch_lanes()
            ctx.close()
        worst = max(times)
        proj = n20 * K / worst
        folded = mdist.fold(parts0, add)
        out[f"shard{N}"] = leg(proj, worst / K * 1e3, (m.compress(1, folded).hex() == want if want else None)
                               and all(eqs), eff=round(proj / (N * headline_value), 4),
                               cfg=f"q{params['q_exp']}h{params['h']}",
                               ms_all=[round(x / K * 1e3, 3) for x in times])
    return out


def _cfg3_sets(m, K, lo, hi):
    """K scalar sets of the 2^21-point configs[3] problem, points [lo, hi) only:
    set 0 = the seed-1 stream (golden), set k = seed 5000 + k; pinned host memory."""
    import numpy as np
    import torch
    N = 1 << 21
    n = hi - lo
    host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
    for k in range(K):
        full = np.frombuffer(m.gen_scalars(N, 1 if k == 0 else 5000 + k), dtype=np.uint8)
        host.numpy()[k * n * 32:(k + 1) * n * 32] = full[lo * 32:hi * 32]
    return host


def weak_leg(m, mdist, torch, dev, local, sp, world, rank, K, W, xdev, add):
    """The round-3 weak-scaling mode as a leg: every rank owns its own 2^20
    points (configs[2] per rank, n_total = N 2^20), K distinct host scalar sets
    per rank (set 0 = slice `rank` of the seed-1 stream of N 2^20 scalars),
    pipelined batch with H2D, one all_gather of the batch's partials.  Parity:
    the folded set 0 against the golden N 2^20 MSM where tests/golden holds it
    (N = 2: 2^21), and on every rank the batch against the synchronous MSM."""
    n = 1 << 20
    start, _ = mdist.shard_range(n * world, world, rank)
    t = time.time()
    ctx = m.CHESContext(1, local, n_exp=20)
    ctx.build_table(m.fixed_points(1, n, start), n, stream=sp)
    host = make_scalar_sets(m, n, K, rank, world)
    torch.cuda.synchronize(dev)
    setup = time.time() - t
    ctx.mult_batch(host.data_ptr(), min(max(W, 1), K), 32, set_stride=n * 32, on_device=False, stream=sp)
    with Bracket(world, dev, xdev) as b:
        parts = ctx.mult_batch(host.data_ptr(), K, 32, set_stride=n * 32, on_device=False, stream=sp)
        res = [mdist.fold(ps, add) for ps in mdist.gather_partials_batch(parts, 1, xdev)]
    sync0 = ctx.mult(host.data_ptr(), 32, on_device=False, stream=sp)
    eq = all_true(m.compress(1, sync0) == m.compress(1, parts[0]), world, xdev)
    want = _golden(m, 1, n * world)
    ok = all_true(m.compress(1, res[0]).hex() == want, world, xdev) if want else None
    ctx.close()
    return {"weak_2p20_per_rank": leg(n * world * K / b.elapsed, b.elapsed / K * 1e3, (ok is not False) and eq,
                                      golden=ok is not None, setup_s=round(setup, 2))}


def cfg3_ranks(m, mdist, torch, dev, local, sp, world, rank, K, W, xdev, add):
    """configs[3] on the ranks: each rank builds the CHES table of its 2^21/world
    points (ches_config_files for that shard size), multiplies its slices of K
    distinct 2^21-scalar sets in one pipelined batch, then ONE all_gather (RCCL)
    of the batch's partials and a host fold.  Strong scaling of a fixed 2^21."""
    N = 1 << 21
    lo, hi = mdist.shard_range(N, world, rank)
    n = hi - lo
    n_exp, cbeta = ches_config(n.bit_length() - 1)
    t = time.time()
    ctx = m.CHESContext(1, local, n_exp=n_exp, beta=cbeta)
    ctx.build_table(m.fixed_points(1, n, lo), n, stream=sp)
    host = _cfg3_sets(m, K, lo, hi)
    torch.cuda.synchronize(dev)
    setup = time.time() - t
    ctx.mult_batch(host.data_ptr(), min(max(W, 1), K), 32, set_stride=n * 32, on_device=False, stream=sp)
    with Bracket(world, dev, xdev) as b:
        parts = ctx.mult_batch(host.data_ptr(), K, 32, set_stride=n * 32, on_device=False, stream=sp)
        res = [mdist.fold(ps, add) for ps in mdist.gather_partials_batch(parts, 1, xdev)]
    want = _golden(m, 1, N)
    ok = all_true(m.compress(1, res[0]).hex() == want, world, xdev)
    ctx.close()
    return {"cfg3_ranks": leg(N * K / b.elapsed, b.elapsed / K * 1e3, ok, setup_s=round(setup, 2))}


def cfg3_multi_context(m, torch, D, one_device, K, W):
    """configs[3] through ONE process driving D shards (msm_ches_ctx_create_multi:
    persistent shard workers, host fold)."""
    N = 1 << 21
    n = N // D
    n_exp = n.bit_length() - 1
    devs = [0] * D if one_device else list(range(D))
    t = time.time()
    ctx = m.CHESContext(1, n_exp=n_exp, devices=devs)
    ctx.build_table(m.fixed_points(1, N), N)
    host = _cfg3_sets(m, K, 0, N)
    setup = time.time() - t
    ctx.mult(host.data_ptr())
    ctx.mult_batch(host.data_ptr(), min(max(W, 1), K), 32, set_stride=N * 32)
    for d in set(devs):
        torch.cuda.synchronize(d)
    t = time.perf_counter()
    res = ctx.mult_batch(host.data_ptr(), K, 32, set_stride=N * 32)
    el = time.perf_counter() - t
    t = time.perf_counter()
    sres = [ctx.mult(host.data_ptr() + k * N * 32) for k in range(min(K, 5))]
    sel = (time.perf_counter() - t) / min(K, 5)
    want = _golden(m, 1, N)
    eq = [m.compress(1, x) for x in sres] == [m.compress(1, x) for x in res[:len(sres)]]
    ctx.close()
    return {"cfg3_multi_ctx": leg(N * K / el, el / K * 1e3, m.compress(1, res[0]).hex() == want and eq,
                                  sync_ms=round(sel * 1e3, 4), devices=len(set(devs)))}


def _ref_lib(name):
    p = os.path.join(REPO, "oracle", "_ref", name)
    return ctypes.CDLL(p) if os.path.exists(p) else None


def cpu_baseline(m, pts, host, n, K, gpu_res, G, log_n):
    """The reference's own blst_p{G}s_mult_pippenger (libblst built from the
    /root/reference sources into oracle/_ref, x86-64 mulx asm) on the host cores:
    1 thread (the reference driver is single-threaded) on set 0, and all of this
    GPU's CPU share (CPU_THREADS) through the Go binding's tile grid
    (oracle/ref_grid.c over the reference's blst_p{G}s_tile_pippenger) on the last
    set; both cross-checked against the GPU.  Falls back to the oracle port when
    the reference build is absent."""
    k = min(1 << log_n, n)
    sc = host.numpy()
    P = (ctypes.c_uint8 * (96 * G * k)).from_buffer_copy(bytes(pts)[:96 * G * k])
    S0 = (ctypes.c_uint8 * (32 * k)).from_buffer_copy(sc[:32 * k].tobytes())
    last = (K - 1) * n * 32
    SL = (ctypes.c_uint8 * (32 * k)).from_buffer_copy(sc[last:last + 32 * k].tobytes())
    full = k == n
    R = _ref_lib("libblst_ref.so")
    out = {}
    if R is not None:
        sizeof = getattr(R, f"blst_p{G}s_mult_pippenger_scratch_sizeof")
        sizeof.restype = ctypes.c_size_t
        sizeof.argtypes = [ctypes.c_size_t]
        mult = getattr(R, f"blst_p{G}s_mult_pippenger")
        mult.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        scratch = (ctypes.c_uint8 * sizeof(k))()
        pp = (ctypes.c_void_p * 2)(ctypes.cast(P, ctypes.c_void_p), None)
        # a bounded sample of ~10-15 s: the first CPU_SETS scalar sets, each checked against the GPU
        nsets = min(CPU_SETS, K)
        dt1, match = 0.0, True
        for j in range(nsets):
            Sj = S0 if j == 0 else (ctypes.c_uint8 * (32 * k)).from_buffer_copy(sc[j * n * 32:j * n * 32 + 32 * k].tobytes())
            sp = (ctypes.c_void_p * 2)(ctypes.cast(Sj, ctypes.c_void_p), None)
            r = (ctypes.c_uint8 * (144 * G))()
            t = time.perf_counter()
            mult(r, pp, k, sp, 255, scratch)
            dt1 += time.perf_counter() - t
            match = match and m.compress(G, bytes(r)) == m.compress(G, gpu_res[j])
        one = {"value": round(nsets * k / dt1, 1), "cores": 1, "seconds": round(dt1, 2), "sets": nsets,
               "matches_gpu": match if full else None}
        kind = "reference"
        Gd = _ref_lib("libref_grid.so")
        if Gd is not None:
            Gd.ref_grid_msm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
            r2 = (ctypes.c_uint8 * (144 * G))()
            t = time.perf_counter()
            Gd.ref_grid_msm(G, r2, P, k, SL, 255, CPU_THREADS)
            dtn = time.perf_counter() - t
            multi = {"value": round(k / dtn, 1), "cores": CPU_THREADS, "seconds": round(dtn, 2),
                     "matches_gpu": (m.compress(G, bytes(r2)) == m.compress(G, gpu_res[-1])) if full else None,
                     "what": f"Go-binding tile grid (bindings/go/blst.go:2064-2197) over the reference's "
                             f"blst_p{G}s_tile_pippenger, {CPU_THREADS} threads, last scalar set"}
        else:
            multi = None
        out = {"value": one["value"], "unit": "pairs/s", "cores": 1, "kind": kind,
               "sample": f"reference libblst blst_p{G}s_mult_pippenger (oracle/_ref), 1 thread, "
                         f"first 2^{log_n} points, scalar sets 0-{one['sets'] - 1}, {dt1:.1f}s",
               "matches_gpu": one["matches_gpu"],
               # the Go binding's tile grid (bindings/go/blst.go:2064-2197) on CPU_THREADS threads, last set
               "all_cores_value": multi and multi["value"], "all_cores_cores": multi and multi["cores"],
               "all_cores_matches_gpu": multi and multi["matches_gpu"]}
    else:
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_ffi as of
        t = time.perf_counter()
        r = of.msm(G, P, S0, k, 255, "pippenger")
        dt1 = time.perf_counter() - t
        out = {"value": round(k / dt1, 1), "unit": "pairs/s", "cores": 1, "kind": "port",
               "sample": f"oracle port of blst Pippenger (oracle/msm_oracle.c), 1 thread, 2^{log_n} pairs, {dt1:.1f}s",
               "matches_gpu": (of.compress(G, r) == m.compress(G, gpu_res[0]).hex()) if full else None}
    return out


if __name__ == "__main__":
    main()
