"""CPU-side checks of the C-ABI library: it loads, and exports every function
include/msm_mi355x.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "msm_mi355x.h")
LIB = os.path.join(REPO, "msm_blst_amd", "libmsm_mi355x.so")


def declared_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set()
    for m in re.finditer(r"\b([a-z_][a-z0-9_]*)\s*\(", txt):
        name = m.group(1)
        if name.startswith(("blst_", "msm_")):
            names.add(name)
    return sorted(names)


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        from msm_blst_amd import build
        build.build()
    return LIB


def test_header_declares_drop_in_entry_points():
    names = declared_functions()
    for must in ("blst_p1s_mult_pippenger", "blst_p2s_mult_pippenger", "blst_p1s_tile_pippenger",
                 "blst_p1s_mult_pippenger_scratch_sizeof", "msm_ctx_create", "msm_ctx_mult"):
        assert must in names


def test_library_exports_every_declared_symbol(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing


def test_library_loads_and_scratch_sizeof_matches_blst(built):
    L = ctypes.CDLL(built)
    L.blst_p1s_mult_pippenger_scratch_sizeof.argtypes = [ctypes.c_size_t]
    L.blst_p1s_mult_pippenger_scratch_sizeof.restype = ctypes.c_size_t
    # sizeof(blst_p1xyzz) << (window(n)-1), window rule of multi_scalar.c:268-275
    for n, w in ((1024, 8), (65536, 13), (1 << 20, 17), (1 << 21, 18), (16, 2), (2, 2), (1, 1)):
        assert L.blst_p1s_mult_pippenger_scratch_sizeof(n) == 192 << (w - 1)


def test_error_mode_switch(built):
    """msm_set_abort_on_error toggles the void entry points' failure mode and
    returns the previous one (default: abort); nothing is pending initially."""
    L = ctypes.CDLL(built)
    L.msm_set_abort_on_error.argtypes = [ctypes.c_int]
    assert L.msm_set_abort_on_error(0) == 1
    assert L.msm_set_abort_on_error(1) == 0
    assert L.msm_error_pending() == 0
