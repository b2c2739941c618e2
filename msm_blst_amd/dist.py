"""Multi-GPU MSM: one process per GPU, points sharded, one exchange.

MSM is linear: Q = sum_g Q_g with Q_g = sum_{i in shard g} s_i P_i.  Each rank
owns a contiguous point range (and its CHES tables) in its own HBM and gets only
its shard's scalars; the single exchange is an all_gather of the per-rank
partial Jacobian points (144 B for G1, 288 B for G2) over torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X, "gloo" in the CPU tests), folded
with an exact EC addition.  RCCL's reduction ops (sum/prod/min/max) cannot
express EC addition, hence gather + fold instead of a literal reduce
(SURVEY.md section 8e).  The reference has no multi-device path; its Go/Rust
bindings split (points x windows) over threads (ref bindings/go/blst.go:1959-2198),
which would replicate points on every GPU, so points are sharded instead.
"""
import torch
import torch.distributed as dist

JAC_BYTES = {1: 144, 2: 288}


def shard_range(n_total, world, rank):
    """Contiguous [start, stop) of a balanced split of n_total points."""
    base, rem = divmod(n_total, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_partials(partial: bytes, group: int, device=None):
    """all_gather the raw Jacobian bytes of every rank's partial sum."""
    nb = JAC_BYTES[group]
    assert len(partial) == nb
    world = dist.get_world_size()
    t = torch.frombuffer(bytearray(partial), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return [bytes(o.cpu().numpy().tobytes()) for o in outs]


def gather_partials_batch(partials, group: int, device=None):
    """One all_gather for a whole batch: partials[k] is this rank's Jacobian of
    MSM k; returns, per MSM k, the list of every rank's partial (rank order)."""
    nb = JAC_BYTES[group]
    assert all(len(p) == nb for p in partials)
    world = dist.get_world_size()
    t = torch.frombuffer(bytearray(b"".join(partials)), dtype=torch.uint8)
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    raw = [bytes(o.cpu().numpy().tobytes()) for o in outs]
    return [[r[k * nb:(k + 1) * nb] for r in raw] for k in range(len(partials))]


def fold(partials, add_fn):
    """Sum a list of Jacobian byte strings with an exact EC add (host, rank order)."""
    acc = partials[0]
    for p in partials[1:]:
        acc = add_fn(acc, p)
    return acc


def engine_add(group):
    """EC addition of two blst Jacobians via the engine library (host helper)."""
    import ctypes

    from . import lib

    def add(a, b):
        out = (ctypes.c_uint8 * JAC_BYTES[group])()
        A = (ctypes.c_uint8 * len(a)).from_buffer_copy(a)
        B = (ctypes.c_uint8 * len(b)).from_buffer_copy(b)
        getattr(lib(), f"msm_p{group}_add")(out, A, B)
        return bytes(out)

    return add


def sharded_msm(local_mult, group, device=None, add_fn=None):
    """Run this rank's partial MSM, exchange, fold.  Returns the full result."""
    part = local_mult()
    parts = gather_partials(part, group, device)
    return fold(parts, add_fn or engine_add(group))
