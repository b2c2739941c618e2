"""Multi-process (N > 1) path of the sharded MSM (msm_blst_amd/dist.py).

CPU tests: world_size 2 and 3 over gloo on 127.0.0.1, partial sums from the CPU
oracle, exchanged with all_gather and folded with the engine's host EC add;
the folded result must equal the reference's golden MSM over all points.
GPU tests: the same exchange with partials computed by the HIP engines (ranks
share cuda:0), and the 8-way shard of the n = 2^21 configuration (BASELINE
configs[3]) computed shard by shard on one GPU and folded.
"""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _golden(golden, group, n, seed=1):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["case"] == "rand" and c["nbits"] == 255][0]["compressed"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(world, group, n, seed, compute, timeout=240):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), MSM_DIST_COMPUTE=compute, OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_worker.py"), str(group), str(n),
                                       str(seed)], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            outs.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
    res = [ln.split()[1] for ln in outs[0][1].splitlines() if ln.startswith("RESULT")]
    assert len(res) == 1
    return res[0]


def test_shard_range_partitions():
    from msm_blst_amd.dist import shard_range
    for n in (1, 7, 1000, 1 << 21):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[k][1] == rs[k + 1][0] for k in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


@pytest.mark.parametrize("world,group,n", [(2, 1, 1024), (3, 1, 1000), (2, 2, 256)])
def test_gloo_sharded_fold_matches_reference(golden, world, group, n):
    assert _run_ranks(world, group, n, 1, "oracle") == _golden(golden, group, n)


@pytest.mark.gpu
@pytest.mark.parametrize("compute", ["ches", "pip"])
def test_gloo_sharded_gpu_partials(golden, compute):
    assert _run_ranks(2, 1, 4096, 1, compute) == _golden(golden, 1, 4096)


@pytest.mark.gpu
def test_eight_shards_of_2e21_on_one_gpu(golden):
    """configs[3]: n = 2^21 split 8 ways (2^18 points per rank, CHES n_exp = 18
    configuration per shard), each shard's partial computed on the GPU, folded."""
    import msm_blst_amd as m
    from msm_blst_amd import dist as mdist
    n_total, world = 1 << 21, 8
    sc = bytes(m.gen_scalars(n_total, 1))
    add = mdist.engine_add(1)
    parts = []
    for r in range(world):
        a, b = mdist.shard_range(n_total, world, r)
        ctx = m.CHESContext(1, 0, n_exp=18)
        ctx.build_table(m.fixed_points(1, b - a, a), b - a)
        parts.append(ctx.mult(sc[32 * a:32 * b]))
        ctx.close()
    assert m.compress(1, mdist.fold(parts, add)).hex() == _golden(golden, 1, n_total)
