"""msm_valu_probe (csrc/probe.hip): the VALU ceilings bench.py prices its
roofline with, measured on the device in the caller's process.  The rates must
be positive and physically plausible for an MI355X (256 CUs x 4 SIMDs, ~2-2.4
GHz): a mad rate of tens of T lane-ops/s, Fp-mul and madd rates whose ratio to
the mad rate matches the instruction counts of one product / one madd (392 /
~3 600 v_mad_u64_u32, profiles/r06_isa_counts.txt), and a bad device id is
refused."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


def test_valu_probe_rates():
    import msm_blst_amd as m
    L = m.lib()
    out = (ctypes.c_double * 4)()
    assert L.msm_valu_probe(0, out) == 0, L.msm_last_error()
    mad, fpmul, madd, ms = list(out)
    assert 15e12 < mad < 60e12
    # a product is 392 mads plus ~25 % other VALU work: between 0.5x and 1x of mad / 392
    assert 0.5 * mad / 392 < fpmul < 1.0 * mad / 392
    # a madd is ~3 570 mads plus other work, and reads its rows from cache
    assert 0.5 * mad / 3573 < madd < 1.0 * mad / 3573
    assert 0 < ms < 2000
    assert L.msm_valu_probe(-1, out) != 0
    assert L.msm_valu_probe(m.device_count(), out) != 0
