"""The drop-in on the GPU: the reference's own callers, linked against the
reference's libblst with the GPU library's symbols localized (oracle/Makefile
`dropin`, binding proved by tests/test_dropin_link.py), reproduce the
reference's results.

* dropin_driver_p{1,2}: the reference's unmodified main_p1.cpp / main_p2.cpp
  (n = 2^10 configuration) through oracle/ref_driver.cpp -- CPU setup by the
  reference, every tile / Pippenger call on the GPU -- against
  ches_driver_n10.json / ches_driver_p2_n10.json (the same harness linked
  against the plain reference).  The crafted last-guard scalar set (SURVEY 8a
  defect 1) returns the correct sum (the reference's Pippenger value) where the
  reference's CHES tile drops the last digit.
* dropin_caller: blst.hpp's P{1,2}_Affines call sequences (mult_pippenger flat
  and pointer arrays, wbits precompute + mult, add) against msm_g{1,2}.json.
* libref_grid_gpu.so: the Go binding's multi-threaded tile grid, concurrent
  blst_p{1,2}s_tile_pippenger calls from 4 threads, against the goldens.
"""
import ctypes
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_OUT = os.path.join(REPO, "oracle", "_ref")


def _bin(name):
    p = os.path.join(REF_OUT, name)
    if not os.path.exists(p):
        pytest.fail(f"{p} missing: build it with `make -C oracle dropin` (needs /root/reference)")
    return p


def _golden_msm(golden, group, n, seed, case="rand"):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["case"] == case and c["nbits"] == 255][0]["compressed"]


@pytest.mark.parametrize("group,fixture", [(1, "ches_driver_n10.json"), (2, "ches_driver_p2_n10.json")])
def test_reference_driver_on_the_gpu(golden, group, fixture):
    r = subprocess.run([_bin(f"dropin_driver_p{group}")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout[r.stdout.index('{"group"'):])  # after the reference's own progress lines
    want = golden(fixture)
    for k in ("bucket_set", "digit_table", "fnv_fixed_points", "fnv_table_3nh", "fnv_table_bgmw"):
        assert got[k] == want[k], k
    assert len(got["runs"]) == len(want["runs"]) == 4
    for g, w in zip(got["runs"], want["runs"]):
        assert (g["seed"], g["case"]) == (w["seed"], w["case"])
        assert g["mb_digits"] == w["mb_digits"] and g["qhalf_digits"] == w["qhalf_digits"]
        truth = w["pippenger"]
        for meth in ("ches_q_over_5", "ches_integral", "bgmw95", "pippenger"):
            assert g[meth] == truth, (g["case"], meth)
        if w["case"] == "rand":
            assert all(w[m] == truth for m in ("ches_q_over_5", "ches_integral", "bgmw95"))
        else:  # the reference's CHES tile loses the last digit here; the GPU does not
            assert w["ches_q_over_5"] != truth


@pytest.mark.parametrize("group,n,seed,wbits", [(1, 1024, 1, 5), (1, 1024, 2, 8), (1, 1000, 3, 4), (1, 4096, 1, 6),
                                                (2, 1024, 1, 4), (2, 256, 2, 6)])
def test_blst_hpp_call_sequences_on_the_gpu(golden, group, n, seed, wbits):
    r = subprocess.run([_bin("dropin_caller"), str(group), str(n), str(seed), str(wbits)], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    got = json.loads(r.stdout)
    want = _golden_msm(golden, group, n, seed)
    assert got["mult_flat"] == want
    assert got["mult_ptrs"] == want
    assert got["mult_wbits"] == want
    assert got["add"] == got["add_cpu"]


@pytest.mark.parametrize("group,n", [(1, 4096), (2, 1024)])
def test_go_grid_on_the_gpu(golden, points, group, n):
    import msm_blst_amd as m
    L = ctypes.CDLL(_bin("libref_grid_gpu.so"))
    L.ref_grid_msm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_int]
    L.ref_grid_msm.restype = ctypes.c_int
    pts = points(group, n)
    sc = m.gen_scalars(n, 1)
    ret = ctypes.create_string_buffer(144 * group)
    assert L.ref_grid_msm(group, ret, pts, n, sc, 255, 4) == 0
    assert m.compress(group, ret.raw).hex() == _golden_msm(golden, group, n, 1)
