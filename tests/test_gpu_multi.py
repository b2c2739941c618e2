"""The C/C++ multi-device CHES path (msm_ches_ctx_create_multi, csrc/multi.hpp):
points sharded contiguously over several devices of ONE process, per-shard
tables, concurrent per-shard MSMs and the exact host fold of the partials
(SURVEY 8e).  On the 1-GPU box the shards share device 0 (devices = [0]*k).
Shards sharing a device are merged into one engine by default (multi.hpp);
`shard_mode` also runs the unmerged paths the 8-GPU node takes -- one engine
per shard as one pipeline over (set, shard) jobs ("pipeline") or concurrently
("engines") -- so the split / route / fold code is exercised on one GPU."""
import pytest

MODES = {"merged": {}, "pipeline": {"MSM_MULTI_MERGE": "0"},
         "engines": {"MSM_MULTI_MERGE": "0", "MSM_MULTI_PIPELINE": "0"}}


def _mode(monkeypatch, mode):
    """set the shard mode for contexts created after this call (read at creation)"""
    for k in ("MSM_MULTI_MERGE", "MSM_MULTI_PIPELINE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def m():
    import msm_blst_amd as m
    if m.device_count() < 1:
        pytest.fail("no HIP device visible")
    return m


def _golden(golden, group, n, seed=1):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["case"] == "rand" and c["nbits"] == 255][0]["compressed"]


@pytest.mark.parametrize("mode", ["merged", "pipeline"])
def test_configs3_2e21_over_8_shards(m, golden, monkeypatch, mode):
    """BASELINE configs[3]: n = 2^21 over 8 shards, config_file_n_exp_18 per shard,
    against the reference's golden MSM of 2^21 points."""
    _mode(monkeypatch, mode)
    n = 1 << 21
    ctx = m.CHESContext(1, n_exp=18, devices=[0] * 8)
    assert ctx.shards() == 8
    ctx.build_table(m.fixed_points(1, n), n)
    sc = m.gen_scalars(n, 1)
    assert m.compress(1, ctx.mult(sc)).hex() == _golden(golden, 1, n)
    # the batch: all 8 shards share device 0, so it runs as one 2^21 MSM per set
    # (merged) or as ONE pipeline over (set, shard) jobs (Ches::run_jobs), each
    # job reading its shard's table
    sets = bytes(sc) + bytes(m.gen_scalars(n, 7))
    got = ctx.mult_batch(sets, 2)
    assert m.compress(1, got[0]).hex() == _golden(golden, 1, n)
    assert m.compress(1, got[1]) == m.compress(1, ctx.mult(sets[32 * n:]))
    ctx.close()


@pytest.mark.parametrize("mode", ["merged", "pipeline", "engines"])
@pytest.mark.parametrize("group,shards,count", [(1, 4, 6), (2, 2, 3)])
def test_one_device_shard_pipeline(m, golden, monkeypatch, group, shards, count, mode):
    """Equal shards on one device: the batch of `count` sets runs as one
    pipeline of count x shards jobs (several reduction groups, front groups of
    one job); every folded result equals the single-device context's batch, and
    set 0 the golden MSM."""
    _mode(monkeypatch, mode)
    n = 1 << 12 if group == 1 else 1 << 10
    pts = m.fixed_points(group, n)
    one = m.CHESContext(group, 0, n_exp=10)
    one.build_table(pts, n)
    multi = m.CHESContext(group, n_exp=10, devices=[0] * shards)
    multi.build_table(pts, n)
    sets = b"".join(bytes(m.gen_scalars(n, 1 if k == 0 else 40 + k)) for k in range(count))
    got = [m.compress(group, r) for r in multi.mult_batch(sets, count)]
    want = [m.compress(group, r) for r in one.mult_batch(sets, count)]
    assert got == want
    assert got[0].hex() == _golden(golden, group, n)
    one.close()
    multi.close()


@pytest.mark.parametrize("mode", ["merged", "engines"])
@pytest.mark.parametrize("group,shards", [(1, 3), (2, 2)])
def test_uneven_shards_table_layout_and_batch(m, golden, monkeypatch, group, shards, mode):
    """n = 2^10 over an uneven split (341/341/342): the sharded table reads back
    byte-identical to the single-device table in the reference layout; mult and
    a 4-set batch equal the golden / single-device results."""
    _mode(monkeypatch, mode)
    n = 1 << 10
    pts = m.fixed_points(group, n)
    one = m.CHESContext(group, 0, n_exp=10)
    one.build_table(pts, n)
    multi = m.CHESContext(group, n_exp=10, devices=[0] * shards)
    multi.build_table(pts, n)
    assert bytes(multi.get_table()) == bytes(one.get_table())
    rows = 3 * n * one.params["h"]
    mid = rows // shards - 5  # a range straddling a shard boundary
    assert bytes(multi.get_table(mid, 11)) == bytes(one.get_table(mid, 11))
    assert m.compress(group, multi.mult(m.gen_scalars(n, 1))).hex() == _golden(golden, group, n)
    sets = b"".join(bytes(m.gen_scalars(n, s)) for s in (2, 3, 4, 5))
    got = [m.compress(group, r) for r in multi.mult_batch(sets, 4)]
    want = [m.compress(group, r) for r in one.mult_batch(sets, 4)]
    assert got == want
    one.close()
    multi.close()


@pytest.mark.parametrize("mode", ["merged", "engines"])
def test_sharded_table_file_roundtrip(m, golden, tmp_path, monkeypatch, mode):
    """save_table / load_table on a sharded context keep the reference layout:
    a file written by a 2-shard context loads into a single-device one."""
    _mode(monkeypatch, mode)
    n = 1 << 10
    multi = m.CHESContext(1, n_exp=10, devices=[0, 0])
    multi.build_table(m.fixed_points(1, n), n)
    path = tmp_path / "t.bin"
    multi.save_table(path)
    one = m.CHESContext(1, 0, n_exp=10)
    one.load_table(path)
    back = m.CHESContext(1, n_exp=10, devices=[0, 0, 0])
    back.load_table(path)
    sc = m.gen_scalars(n, 1)
    want = _golden(golden, 1, n)
    assert m.compress(1, one.mult(sc)).hex() == want
    assert m.compress(1, back.mult(sc)).hex() == want
    for c in (multi, one, back):
        c.close()


def test_driver_sharded_ches(golden):
    """msm_driver_p1 devices=0,0,0,0: the CHES method on 4 shards agrees with the
    other three methods and the golden value (config 16: config 14 per shard)."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "msm_blst_amd", "bin",
                       "msm_driver_p1")
    r = subprocess.run([exe, "config=16", "tests=1", "loops=1", "devices=0,0,0,0"], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "config_file_n_exp_14 per shard" in r.stdout
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["agree"] is True
    assert rec["methods"]["ches_q_over_5"]["last_compressed"] == _golden(golden, 1, 1 << 16)
