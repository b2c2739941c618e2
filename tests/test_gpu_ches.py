"""GPU parity of the CHES bucket-set path (table built on the GPU, digits,
accumulation and reduction in HIP) against the reference's golden values.
The CHES result equals the reference's Pippenger result on the same scalars
(ref driver test_pippengers, main_p1.cpp:470-580), so msm_g*.json pins it."""
import ctypes

import pytest

import oracle_ffi as of
from test_oracle_golden import _fnv

pytestmark = pytest.mark.gpu

R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _golden(golden, group, n, seed=1, case="rand"):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["case"] == case and c["nbits"] == 255][0]["compressed"]


@pytest.fixture(scope="module")
def ctx10(m):
    ctx = m.CHESContext(1, 0, n_exp=10)
    ctx.build_table(m.fixed_points(1, 1024), 1024)
    yield ctx
    ctx.close()


def test_table_n10_matches_reference(ctx10, golden):
    g = golden("ches_driver_n10.json")
    T = ctx10.get_table()
    assert len(bytes(T)) == 96 * 3 * 1024 * g["h"]
    assert _fnv(bytes(T)) == g["fnv_table_3nh"]


def test_driver_runs_n10(m, ctx10, golden):
    g = golden("ches_driver_n10.json")
    n, h = g["n"], g["h"]
    for run in g["runs"]:
        sc = bytearray(bytes(m.gen_scalars(n, run["seed"])))
        if run["case"] == "ches_last_guard":  # crafted: digits h-3, h-2 of the last scalar zeroed
            v = int.from_bytes(sc[32 * (n - 1):], "little")
            for bit in range(13 * (h - 3), 13 * (h - 1)):
                v &= ~(1 << bit)
            sc[32 * (n - 1):] = v.to_bytes(32, "little")
        r = ctx10.mult(bytes(sc))
        assert m.compress(1, r).hex() == run["pippenger"], run["case"]


def test_edge_scalars_n10(m, ctx10, golden):
    n = 1024
    # all zero -> infinity (compressed 0xc0 00..)
    r = ctx10.mult(bytes(32 * n))
    assert m.compress(1, r).hex() == "c0" + "00" * 47
    # s and s + r give the same point (scalars >= r reduced mod r)
    base = bytes(m.gen_scalars(n, 3))
    want = m.compress(1, ctx10.mult(base))
    shifted = bytearray()
    for i in range(n):
        v = int.from_bytes(base[32 * i:32 * i + 32], "little") + (R if i % 3 == 0 else 0)
        shifted += v.to_bytes(32, "little")
    assert m.compress(1, ctx10.mult(bytes(shifted))) == want
    # r - 1 everywhere == golden 'rminus1' (-sum P_i)
    rm1 = (R - 1).to_bytes(32, "little") * n
    gold = [c for c in golden("msm_g1.json")["cases"] if c["case"] == "rminus1"][0]
    if gold["n"] == n:
        assert m.compress(1, ctx10.mult(rm1)).hex() == gold["compressed"]
    else:
        sc = bytearray(rm1)
        pts = of.fixed_points(1, n)
        ref = of.msm(1, pts, (ctypes.c_uint8 * len(sc)).from_buffer_copy(bytes(sc)), n, 255, "pippenger")
        assert m.compress(1, ctx10.mult(rm1)).hex() == of.compress(1, ref)


def test_equal_points_doubling_branch(m):
    """Equal points with equal scalars: every bucket add hits P == bucket (doubling branch)."""
    n = 64
    ctx = m.CHESContext(1, 0, n_exp=8)
    p0 = bytes(m.fixed_points(1, 1))
    ctx.build_table(p0 * n, n)
    s0 = bytes(m.gen_scalars(1, 9))
    got = m.compress(1, ctx.mult(s0 * n))
    pts = (ctypes.c_uint8 * (96 * n)).from_buffer_copy(p0 * n)
    sc = (ctypes.c_uint8 * (32 * n)).from_buffer_copy(s0 * n)
    assert got.hex() == of.compress(1, of.msm(1, pts, sc, n, 255, "naive"))
    ctx.close()


@pytest.mark.parametrize("method", ["ches", "bgmw"])
def test_equal_points_doubling_branch_g2(m, method):
    """G2 (lane-pair kernels): equal points with equal scalars -- every bucket add
    takes the doubling branch of xyzz_madd, and equal bucket sums meet in the
    reduction's pairwise adds (xyzz_add / the cooperative tail's doubling branch,
    coop.hpp) -- vs the CPU oracle's naive sum."""
    n = 64
    ctx = m.CHESContext(2, 0, n_exp=8) if method == "ches" else m.BGMWContext(2, 0, n_exp=8)
    p0 = bytes(m.fixed_points(2, 1))
    ctx.build_table(p0 * n, n)
    s0 = bytes(m.gen_scalars(1, 9))
    got = m.compress(2, ctx.mult(s0 * n))
    pts = (ctypes.c_uint8 * (192 * n)).from_buffer_copy(p0 * n)
    sc = (ctypes.c_uint8 * (32 * n)).from_buffer_copy(s0 * n)
    assert got.hex() == of.compress(2, of.msm(2, pts, sc, n, 255, "naive"))
    ctx.close()


@pytest.mark.parametrize("group,n_exp", [(1, 16), (2, 12)])
def test_skewed_buckets_mixed_payload_layout(m, group, n_exp):
    """A quarter of the scalars equal: their digits pile into h buckets of n/4
    entries each, whose wave groups keep the bucket-ordered payload (padding
    would exceed 2x), beside interleaved groups of ordinary buckets
    (bucket_sort.hpp k_wave_len / k_interleave) -- vs the CPU oracle."""
    n = 1 << n_exp
    pts = bytes(m.fixed_points(group, n))
    sc = bytearray(bytes(m.gen_scalars(n, 11)))
    same = bytes(m.gen_scalars(1, 12))
    for i in range(0, n, 4):
        sc[32 * i:32 * i + 32] = same
    ctx = m.CHESContext(group, 0, n_exp=n_exp)
    ctx.build_table(pts, n)
    got = m.compress(group, ctx.mult(bytes(sc)))
    ctx.close()
    cp = (ctypes.c_uint8 * len(pts)).from_buffer_copy(pts)
    cs = (ctypes.c_uint8 * len(sc)).from_buffer_copy(bytes(sc))
    assert got.hex() == of.compress(group, of.msm(group, cp, cs, n, 255, "pippenger"))


@pytest.mark.parametrize("n_exp", [16, 20])
def test_ches_g1_large_vs_reference(m, golden, points, n_exp):
    n = 1 << n_exp
    ctx = m.CHESContext(1, 0, n_exp=n_exp)
    ctx.build_table(points(1, n), n)
    r = ctx.mult(m.gen_scalars(n, 1))
    assert m.compress(1, r).hex() == _golden(golden, 1, n)
    # buffers reused; the atomics-ordered accumulation may pick another Jacobian
    # representative of the same point, so compare the canonical encoding
    assert m.compress(1, ctx.mult(m.gen_scalars(n, 1))) == m.compress(1, r)
    ctx.close()


@pytest.mark.parametrize("n_exp", [10, 16, 20])
def test_ches_g2_vs_reference(m, golden, points, n_exp):
    """G2 CHES incl. configs[4] (n = 2^20: q = 2^22, h = 12, table 9.7 GB in HBM)"""
    n = 1 << n_exp
    ctx = m.CHESContext(2, 0, n_exp=n_exp)
    ctx.build_table(points(2, n), n)
    r = ctx.mult(m.gen_scalars(n, 1))
    assert m.compress(2, r).hex() == _golden(golden, 2, n)
    ctx.close()


def test_set_table_roundtrip(m, ctx10):
    """A table uploaded in blst layout (e.g. one the reference built) gives the same result."""
    T = bytes(ctx10.get_table())
    ctx = m.CHESContext(1, 0, n_exp=10)
    ctx.set_table(T, 1024)
    sc = m.gen_scalars(1024, 4)
    assert m.compress(1, ctx.mult(sc)) == m.compress(1, ctx10.mult(sc))
    ctx.close()


def test_mult_batch_matches_single(m, golden):
    """The pipelined batch (tail of MSM k beside MSM k+1) equals independent mults."""
    n = 1 << 16
    ctx = m.CHESContext(1, 0, n_exp=16)
    ctx.build_table(m.fixed_points(1, n), n)
    sets = [bytes(m.gen_scalars(n, seed)) for seed in (1, 2, 3, 4, 5)]
    got = ctx.mult_batch(b"".join(sets), 5)
    for k, sc in enumerate(sets):
        assert m.compress(1, got[k]) == m.compress(1, ctx.mult(sc)), k
    assert m.compress(1, got[0]).hex() == _golden(golden, 1, n)
    rep = ctx.mult_batch(sets[0], 3, set_stride=0)  # one set repeated
    assert all(m.compress(1, r).hex() == _golden(golden, 1, n) for r in rep)
    ctx.close()


@pytest.mark.parametrize("group,log_n,K", [(1, 16, 7), (2, 10, 7), (1, 12, 9), (1, 12, 17), (2, 10, 9),
                                           (2, 10, 17)])
def test_mult_batch_sets_resident_and_pinned(m, group, log_n, K):
    """K distinct sets from device memory and from page-locked host memory
    (copied set by set inside the pipeline) equal the synchronous MSMs.  These
    sizes take the small-MSM LANE schedule of Ches::run_jobs (batch_lanes() = 3
    for G1, 2 for G2: MSMs accumulate side by side on rotating streams and
    bucket sets, kFrontsMax = 5 front sets, front groups of 1, 1, 2, 4, 4, ...,
    four reducer sets).  One reduction group holds up to kGroup = 20 MSMs, so
    these K form one group; the headline's one-lane schedule and batches of
    more than 20 are test_gpu_batch_one_lane.py."""
    import numpy as np
    import torch
    n = 1 << log_n
    ctx = m.CHESContext(group, 0, n_exp=log_n)
    ctx.build_table(m.fixed_points(group, n), n)
    host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
    for k in range(K):
        host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 100 + k), dtype=np.uint8)
    dev = host.to("cuda:0")
    torch.cuda.synchronize()
    want = [m.compress(group, ctx.mult(dev.data_ptr() + k * n * 32, on_device=True)) for k in range(K)]
    got_d = ctx.mult_batch(dev.data_ptr(), K, set_stride=n * 32, on_device=True)
    got_h = ctx.mult_batch(host.data_ptr(), K, set_stride=n * 32, on_device=False)
    assert [m.compress(group, r) for r in got_d] == want
    assert [m.compress(group, r) for r in got_h] == want
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("group,log_n,K", [(1, 12, 6), (2, 10, 4)])
def test_mult_batch_waits_for_host_sets_written_on_its_stream(m, group, log_n, K):
    """The batch's copy stream does not wait on the caller's stream (a copy
    enqueued behind a cross-stream wait could block the host, ches.hip
    run_jobs); the batch waits for the caller's prior work on the host instead.
    Here the pinned host sets are produced by a D2H copy queued on the batch's
    own stream behind ~20 ms of GPU spinning, and the batch is called without a
    synchronise: it must see the new sets, not the zeros before them."""
    import numpy as np
    import torch
    n = 1 << log_n
    ctx = m.CHESContext(group, 0, n_exp=log_n)
    ctx.build_table(m.fixed_points(group, n), n)
    raw = np.concatenate([np.frombuffer(m.gen_scalars(n, 700 + k), dtype=np.uint8) for k in range(K)])
    src = torch.tensor(raw, device="cuda:0")
    want = [m.compress(group, ctx.mult(src.data_ptr() + k * n * 32, on_device=True)) for k in range(K)]
    host = torch.zeros(K * n * 32, dtype=torch.uint8, pin_memory=True)
    st = torch.cuda.Stream()
    # a first host-set batch sizes the batch buffers (their first sizing
    # synchronises the stream, which would hide a missing wait)
    ctx.mult_batch(host.data_ptr(), K, set_stride=n * 32, on_device=False, stream=st.cuda_stream)
    torch.cuda.synchronize()
    with torch.cuda.stream(st):
        torch.cuda._sleep(50_000_000)
        host.copy_(src, non_blocking=True)
    got = ctx.mult_batch(host.data_ptr(), K, set_stride=n * 32, on_device=False, stream=st.cuda_stream)
    torch.cuda.synchronize()
    assert [m.compress(group, r) for r in got] == want
    ctx.close()


_FRONT_GROUP_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
import msm_blst_amd as m
ok = True
for group, log_n, K in ((1, 12, 17), (2, 10, 9)):
    n = 1 << log_n
    ctx = m.CHESContext(group, 0, n_exp=log_n)
    ctx.build_table(m.fixed_points(group, n), n)
    host = torch.empty(K * n * 32, dtype=torch.uint8, pin_memory=True)
    for k in range(K):
        host.numpy()[k * n * 32:(k + 1) * n * 32] = np.frombuffer(m.gen_scalars(n, 300 + k), dtype=np.uint8)
    dev = host.to("cuda:0")
    torch.cuda.synchronize()
    want = [m.compress(group, ctx.mult(dev.data_ptr() + k * n * 32, on_device=True)) for k in range(K)]
    got_d = ctx.mult_batch(dev.data_ptr(), K, set_stride=n * 32, on_device=True)
    got_h = ctx.mult_batch(host.data_ptr(), K, set_stride=n * 32, on_device=False)
    ok &= [m.compress(group, r) for r in got_d] == want and [m.compress(group, r) for r in got_h] == want
    ctx.close()
print("FRONT_GROUPS_OK" if ok else "FRONT_GROUPS_MISMATCH")
"""


@pytest.mark.parametrize("knobs", [{"MSM_FRONT_GROUP": "8"}, {"MSM_ACC_GROUP": "0"},
                                   {"MSM_ACC_GROUP": "0", "MSM_BATCH_LANES": "2"}])
def test_batch_front_groups_of_eight(knobs):
    """Non-default small-MSM batch schedules, selected by knobs the library reads
    once per process: MSM_FRONT_GROUP=8 (digits + sort of up to 8 MSMs in one
    pass per stage, and accumulation groups of up to 8 sets in one launch:
    front groups 1, 1, 2, 4, 8, 1); MSM_ACC_GROUP=0 (the per-MSM accumulation
    lanes of round 4, three lanes / two lanes).  A child process runs batches
    of 17 (G1) and 9 (G2) distinct sets from device and pinned host memory
    against the synchronous MSMs."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, **knobs)
    r = subprocess.run([sys.executable, "-c", _FRONT_GROUP_SCRIPT, repo], capture_output=True, text=True, env=env,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "FRONT_GROUPS_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


_UNFUSED_SCRIPT = r"""
import sys
sys.path.insert(0, sys.argv[1])
import msm_blst_amd as m
out = []
for group, log_n in ((1, 12), (2, 10)):
    n = 1 << log_n
    ctx = m.CHESContext(group, 0, n_exp=log_n)
    ctx.build_table(m.fixed_points(group, n), n)
    out.append(m.compress(group, ctx.mult(m.gen_scalars(n, 77))).hex())
    ctx.close()
print("RESULTS", " ".join(out))
"""


def test_unfused_front_equals_fused(m):
    """The fused CHES front (ches_kernels.hpp k_ches_front_hist / _coarse: digits
    counted per coarse bin, then recomputed and binned from registers; the default
    for every h the reference configurations use except 15 and 22) and the unfused
    one (k_ches_digits writing keys / vals, then BucketSort::run), selected with
    MSM_FRONT_FUSED=0 in a child process (read once per process), give the same
    MSMs for G1 2^12 (h = 19) and G2 2^10 (h = 20)."""
    import os
    import subprocess
    import sys
    want = []
    for group, log_n in ((1, 12), (2, 10)):
        n = 1 << log_n
        ctx = m.CHESContext(group, 0, n_exp=log_n)
        ctx.build_table(m.fixed_points(group, n), n)
        want.append(m.compress(group, ctx.mult(m.gen_scalars(n, 77))).hex())
        ctx.close()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _UNFUSED_SCRIPT, repo], capture_output=True, text=True,
                       env=dict(os.environ, MSM_FRONT_FUSED="0"), timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULTS")]
    assert line and line[0].split()[1:] == want, r.stdout[-2000:]
