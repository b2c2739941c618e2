"""Scratch / spill gate for every gfx950 kernel in the product library (CPU).

The G2 CHES table bug of round 4 (device-only wrong rows from (i=0, j=0, m=3)
on) appeared in a kernel that spilled 1.5 KB per lane to
scratch and disappeared when the spill was removed; its mechanism was never
proven.  So no product kernel may use scratch memory: this test reads the
AMDHSA metadata of every kernel in libmsm_mi355x.so (tools/kernel_scratch.py:
the .hip_fatbin bundles unbundled with clang-offload-bundler, llvm-readelf
--notes) and fails on any private segment (scratch) and on any VGPR spill,
except the two G2 cooperative tail kernels below whose few spilled VGPRs land
in AGPRs (v_accvgpr moves, no memory; private segment 0) -- capped at today's
counts so any growth fails too.
"""
import os
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "msm_blst_amd", "libmsm_mi355x.so")
sys.path.insert(0, os.path.join(REPO, "tools"))

# (kernel name substring, max VGPRs spilled into AGPRs): one G2 xyzz add over 4
# waves (coop.hpp) keeps both operands, their four-way selects and the
# pair-swap temporaries live at the 256 architectural VGPRs (k_suffix_step_c2p:
# 12 since round 6's lane-pair operand forms, fp2l.hpp, which cut 182 selects
# from the G2 accumulation; the tail kernel's AGPR moves cost nothing measurable)
AGPR_SPILL_CEILING = {"k_segsum_c2p": 2, "k_suffix_step_c2p": 12}


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.fail("libmsm_mi355x.so not built (python -c 'import __graft_entry__ as g; g.build()')")
    if not shutil.which("objcopy") or not os.path.exists("/opt/rocm/lib/llvm/bin/clang-offload-bundler"):
        pytest.fail("objcopy / clang-offload-bundler missing")
    import kernel_scratch
    ks = kernel_scratch.kernels(LIB)
    assert len(ks) > 150, f"only {len(ks)} kernels found in the code objects"
    return ks


def test_every_kernel_found(kernels):
    names = " ".join(kernels)
    for k in ("k_accumulate", "k_accumulate2p", "k_segsum", "k_segsum2p", "k_ches_table", "k_ches_table2p",
              "k_ches_front_hist", "k_finalize", "k_wbits_table2p", "k_wbits_sums2p", "k_test_xyzz2p"):
        assert k in names, k


def test_no_scratch(kernels):
    bad = {n: d["private_segment_fixed_size"] for n, d in kernels.items() if d.get("private_segment_fixed_size", 0)}
    assert not bad, f"kernels with scratch (private segment bytes): {bad}"


def test_no_vgpr_spill(kernels):
    bad = {}
    for n, d in kernels.items():
        sp = d.get("vgpr_spill_count", 0) + d.get("sgpr_spill_count", 0)
        if not sp:
            continue
        ceiling = [c for k, c in AGPR_SPILL_CEILING.items() if k in n]
        if ceiling and d.get("sgpr_spill_count", 0) == 0 and d.get("vgpr_spill_count", 0) <= ceiling[0] \
                and d.get("agpr_count", 0) > 0 and d.get("private_segment_fixed_size", 0) == 0:
            continue  # the documented spills into AGPRs
        bad[n] = (d.get("vgpr_spill_count", 0), d.get("sgpr_spill_count", 0))
    assert not bad, f"kernels with spills (vgpr, sgpr): {bad}"
