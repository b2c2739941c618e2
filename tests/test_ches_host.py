"""CPU tests of the engine's own CHES host setup (msm_blst_amd, not the oracle):
configuration table, bucket set and digit hash against the reference's values
(tests/golden, generated from /root/reference by tests/golden/make_golden.py).
No GPU is touched: these entry points are pure host code of libmsm_mi355x.so."""
import pytest

from test_oracle_golden import _fnv


@pytest.fixture(scope="module")
def ches():
    import os
    from msm_blst_amd import _ffi
    if not os.path.exists(_ffi.LIB_PATH):
        from msm_blst_amd import build
        build.build()
    from msm_blst_amd import ches
    return ches


def test_params_match_every_reference_config(ches, golden):
    for cfg in golden("ches_configs.json")["configs"]:
        p = ches.params(cfg["n_exp"], cfg["beta"])
        for k in ches.PARAM_KEYS:
            if k in cfg:
                assert p[k] == cfg[k], (cfg, k)


def test_bucket_set_sizes_all_configs(ches, golden):
    for cfg in golden("ches_configs.json")["configs"]:
        if cfg["q_exp"] > 20:
            continue
        B = list(ches.bucket_set(1 << cfg["q_exp"], cfg["a_h"]))
        assert len(B) == cfg["b_size"]
        assert B[0] == 0 and B == sorted(set(B))
        assert max(b - a for a, b in zip(B, B[1:])) <= cfg["d_max"]


@pytest.mark.parametrize("cfg", [10, 16, 20])
def test_bucket_set_and_digit_hash_vs_reference(ches, golden, cfg):
    g = golden(f"ches_params_n{cfg}.json")
    q = 1 << g["q_exp"]
    B = ches.bucket_set(q, g["a_h"])
    assert len(B) == g["b_size"]
    assert list(B[:16]) == g["head"] and list(B[len(B) - 16:]) == g["tail"]
    assert max(b - a for a, b in zip(B, B[1:])) == g["max_gap"]
    if len(bytes(B)) < 4_000_000:
        assert _fnv(bytes(B)) == g["fnv_bucket_set"]
    H = ches.digit_table(q, g["a_h"])
    if q <= (1 << 19):
        assert _fnv(bytes(H)) == g["fnv_digit_table"]
    Bs = set(B)
    for v in range(0, q + 1, 1 if q <= (1 << 16) else 101):
        t = H[v]
        assert t.b in Bs and 1 <= t.m <= 3
        assert (t.m * t.b == v) if t.alpha == 0 else (q - t.m * t.b == v)


def test_driver_tables_n10(ches, golden):
    g = golden("ches_driver_n10.json")
    q = 1 << g["q_exp"]
    assert list(ches.bucket_set(q, 231)) == g["bucket_set"]
    H = ches.digit_table(q, 231)
    assert [[H[v].m, H[v].b, H[v].alpha] for v in range(q + 1)] == g["digit_table"]


@pytest.mark.parametrize("cfg", [20, 16])
def test_device_digit_code_matches_oracle_table(ches, golden, cfg):
    """The device's compact digit code + rank tables, decoded with the device
    arithmetic (msm_ches_digit_table), equal the oracle's digit hash entry for
    entry (ref main_p1.cpp:140-152) over the whole digit range."""
    import numpy as np
    import oracle_ffi as of
    g = golden(f"ches_params_n{cfg}.json")
    q = 1 << g["q_exp"]
    got = np.frombuffer(bytes(ches.digit_table(q, g["a_h"])), dtype=np.int32)
    H, _ = of.digit_table(of.bucket_set(q, g["a_h"]), q)
    want = np.frombuffer(bytes(H), dtype=np.int32)
    assert got.shape == want.shape and np.array_equal(got, want)
