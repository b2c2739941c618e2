"""CPU tests of bench.py's host-side accounting: the per-madd v_mad_u64_u32
count behind `valu_roofline.mad_frac` is parsed from the committed gfx950 ISA
counts (tools/isa_report.sh -> profiles/r06_isa_counts.txt) for G1 (Fp ops on
one lane) and G2 (lane-pair Fp2 ops, both lanes)."""
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

ISA = os.path.join(REPO, "profiles", "r06_isa_counts.txt")


def _mads(txt, key):
    return int(re.search(key + r"\w*\n\s+vgpr \d+ scratch \d+ total \d+ v_mad_u64_u32 (\d+)", txt).group(1))


def test_mads_per_madd_from_isa_counts():
    txt = open(ISA).read()
    mul, sqr, mul2 = (_mads(txt, k) for k in ("k_op_fp_mulP", "k_op_fp_sqr", "k_op_fp_mul2"))
    g1, src = bench.isa_mads_per_madd(1, ISA)
    # ec.hpp xyzz_madd: 6 products, 2 squares, 1 fused two-product sum
    assert g1 == 6 * mul + 2 * sqr + mul2 and src == os.path.basename(ISA)
    bs, sq2, ms = (_mads(txt, k) for k in ("k_op_g2l_mul_bs", "k_op_g2l_sqr", "k_op_g2l_mul_sub"))
    g2, _ = bench.isa_mads_per_madd(2, ISA)
    assert g2 == 2 * (6 * bs + 2 * sq2 + ms)  # per lane, times the lane pair
    assert 3000 < g1 < 4000 and 2 * g1 < g2 < 4 * g1


def test_mads_per_madd_without_counts(tmp_path):
    missing = str(tmp_path / "none.txt")
    assert bench.isa_mads_per_madd(1, missing)[0] == 3567  # the round-3 constant
    assert bench.isa_mads_per_madd(2, missing)[0] is None  # no G2 figure without lane-pair counts


def test_ches_config_per_group_and_shard_size():
    """The configuration each bench line uses: G1 2^20 the reference's
    config_file_n_exp_20.h, G2 2^20 its _beta variant (measured faster for G2,
    profiles/r05_g2_beta_ab.txt), the strong-scaling shards the reference's
    file measured fastest for their point count, and an explicit --beta wins."""
    assert bench.ches_config(20) == (20, 0)
    assert bench.ches_config(20, group=2) == (20, 1)
    assert bench.ches_config(17) == (17, 1)  # q = 2^19, measured faster for the 2^17 shard (r06_tail_ab.txt)
    for lg in (18, 19):
        assert bench.ches_config(lg) == (lg, 0)
    assert bench.ches_config(20, 0, 2) == (20, 0)
    assert bench.ches_config(20, 1, 1) == (20, 1)


def test_default_warmup_is_one_batch():
    """bench.py's default warm-up is one untimed batch as long as the timed one
    (the first short-warm-up batch runs below steady-state clocks,
    profiles/r05_warmup_ab.txt)."""
    src = open(os.path.join(REPO, "bench.py")).read()
    steps = int(re.search(r'"--steps", type=int, default=(\d+)', src).group(1))
    warm = int(re.search(r'"--warmup", type=int, default=(\d+)', src).group(1))
    assert warm == steps == 20
