"""The drop-in binds (CPU side, no GPU needed).

The reference's libblst is one unity object (ref src/server.c:7-24 includes
multi_scalar.c and bulk_addition.c), so a caller that links it gets its strong
MSM definitions whatever the link order -- the recipe of round 2's
INTEGRATION.md silently ran the CPU code.  `make -C oracle dropin` localizes
every symbol libmsm_mi355x.so exports in the reference's server.o; these tests
prove with `nm` that the reference's own callers (main_p1.cpp / main_p2.cpp
through oracle/ref_driver.cpp, the blst.hpp call sequences in
oracle/dropin_caller.c, the Go-style grid oracle/ref_grid.c) then leave every
MSM symbol undefined, i.e. bound to the GPU library, and that the naive link
does not (so the check has teeth).  The GPU run is tests/test_gpu_dropin.py.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_OUT = os.path.join(REPO, "oracle", "_ref")
LIB = os.path.join(REPO, "msm_blst_amd", "libmsm_mi355x.so")
BINS = ["dropin_driver_p1", "dropin_driver_p2", "dropin_caller", "libref_grid_gpu.so"]
# what each caller must reach on the GPU (its MSM calls in the reference source)
MUST = {
    "dropin_driver_p1": ["blst_p1s_mult_pippenger", "blst_p1_tile_pippenger_d_CHES", "blst_p1_tile_pippenger_BGMW95"],
    "dropin_driver_p2": ["blst_p2s_mult_pippenger", "blst_p2_tile_pippenger_d_CHES", "blst_p2_tile_pippenger_BGMW95"],
    "dropin_caller": ["blst_p1s_mult_pippenger", "blst_p1s_mult_wbits_precompute", "blst_p1s_mult_wbits",
                      "blst_p1s_add", "blst_p2s_mult_pippenger", "blst_p2s_mult_wbits", "blst_p2s_add"],
    "libref_grid_gpu.so": ["blst_p1s_tile_pippenger", "blst_p2s_tile_pippenger"],
}


def _nm(path, dynamic):
    args = ["nm", "-D"] if dynamic else ["nm"]
    out = subprocess.run(args + [path], capture_output=True, text=True, check=True).stdout
    syms = {}
    for line in out.splitlines():
        parts = line.split()
        if len(parts) >= 2:
            syms.setdefault(parts[-1], set()).add(parts[-2])
    return syms


@pytest.fixture(scope="module")
def dropin():
    if not os.path.isdir("/root/reference") and not all(os.path.exists(os.path.join(REF_OUT, b)) for b in BINS):
        pytest.skip("reference sources absent and drop-in binaries not prebuilt")
    if not os.path.exists(LIB):
        from msm_blst_amd import build
        build.build()
    if os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "dropin"], check=True)
    with open(os.path.join(REF_OUT, "dropin.syms")) as f:
        syms = [s.strip() for s in f if s.strip()]
    return syms


def test_localized_set_is_the_gpu_export_set(dropin):
    """dropin.syms = every blst_* symbol the GPU library defines; all of them were
    global (T) in the reference's server.o and none is global after objcopy."""
    exported = {s for s, t in _nm(LIB, True).items() if t & {"T", "W"} and s.startswith("blst_")}
    assert set(dropin) == exported
    before = _nm(os.path.join(REF_OUT, "server.o"), False)
    after = _nm(os.path.join(REF_OUT, "server_gpu.o"), False)
    for s in dropin:
        assert "T" in before.get(s, set()), s
        assert not (after.get(s, set()) & {"T", "W"}), s
    # what the reference's other callers need from libblst stays global
    for s in ("blst_p1s_to_affine", "blst_p2s_to_affine", "blst_p1_double", "blst_p1_to_affine",
              "blst_p1_add_or_double_affine", "blst_scalar_from_uint64"):
        assert "T" in after.get(s, set()), s


@pytest.mark.parametrize("binary", BINS)
def test_reference_callers_bind_msm_symbols_to_the_gpu_library(dropin, binary):
    path = os.path.join(REF_OUT, binary)
    dyn = _nm(path, True)
    full = _nm(path, False)
    for s in dropin:
        # no global definition of an exported MSM symbol anywhere in the binary
        assert not (full.get(s, set()) & {"T", "W"}), f"{binary} defines {s} itself"
        if s in dyn:
            assert dyn[s] == {"U"}, f"{binary}: {s} {dyn[s]}"
    for s in MUST[binary]:
        assert dyn.get(s) == {"U"}, f"{binary} does not import {s} from libmsm_mi355x.so"
    needed = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    assert "libmsm_mi355x.so" in needed


def test_naive_link_order_binds_the_cpu_code(dropin, tmp_path):
    """The round-2 recipe (GPU library first, then the unmodified libblst.a)
    puts the reference's CPU Pippenger into the executable -- the reason the
    drop-in localizes the symbols."""
    exe = tmp_path / "naive"
    subprocess.run(["gcc", "-std=gnu11", "-O1", f"-I{'/root/reference'}", "-o", str(exe),
                    os.path.join(REPO, "oracle", "dropin_caller.c"), f"-L{os.path.dirname(LIB)}",
                    "-l:libmsm_mi355x.so", os.path.join(REF_OUT, "libblst_ref.a")], check=True)
    assert "T" in _nm(str(exe), False)["blst_p1s_mult_pippenger"]


def test_call_lands_in_the_gpu_library_without_a_device(dropin):
    """With no HIP device (this container), the first MSM call of the drop-in
    caller fails inside libmsm_mi355x.so with its own error message: the call
    reached the GPU library, not libblst's CPU code (which would just return)."""
    import msm_blst_amd as m
    if m.device_count() > 0:
        pytest.skip("a HIP device is present: the GPU run is tests/test_gpu_dropin.py")
    r = subprocess.run([os.path.join(REF_OUT, "dropin_caller"), "1", "16", "1", "4"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0
    assert "msm_mi355x: blst_p1s_mult_pippenger failed" in r.stderr
