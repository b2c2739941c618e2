"""The bench line's shape, on the line bench.py printed in the final-tree
session (profiles/r06_bench.json, N = 1) and a gloo rehearsal (N = 2 / 8,
profiles/r06_strong_rehearsal.txt): the contract keys, the roofline and
cpu_baseline objects, every leg compact, and the whole line small enough for
the driver's record (under ~7 KB, so the stdout tail the
driver keeps holds all of it)."""
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONTRACT = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")
ROOF = ("bound", "achieved", "peak", "unit", "frac", "traffic", "valu_achieved", "valu_peak", "valu_frac",
        "mad_frac", "peak_basis")


def _last_line(path):
    return [ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1]


def test_n1_line_shape_and_size():
    raw = _last_line(os.path.join(REPO, "profiles", "r06_bench.json"))
    assert len(raw) < 7000
    d = json.loads(raw)
    for k in CONTRACT:
        assert k in d, k
    assert d["metric"] == json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["unit"] == "pairs/s"
    assert d["config"]["workload"]
    r = d["roofline"]
    for k in ROOF:
        assert k in r, k
    assert 0 < r["frac"] < 1 and 0 < r["valu_frac"] <= 1 and r["peak_basis"].startswith("this run")
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    c = d["cpu_baseline"]
    assert c["kind"] in ("reference", "port") and c["cores"] >= 1 and c["value"] > 0 and c["sample"]
    assert d["parity_vs_reference"] is True
    for name, leg in d["legs"].items():
        assert set(leg) >= {"M", "ms"}, name
        assert leg.get("ok", True) is True, name
    # the headline equals its leg
    assert abs(d["legs"]["ches_h2d"]["M"] * 1e6 - d["value"]) / d["value"] < 1e-3


def test_rehearsal_lines_are_strong_scaling_with_parity():
    for ln in open(os.path.join(REPO, "profiles", "r06_strong_rehearsal.txt")):
        if not ln.startswith("N="):
            continue
        n, raw = ln.split(" ", 1)
        d = json.loads(raw)
        assert d["n_gpus"] == int(n[2:]) and d["scaling"] == "strong"
        assert d["config"]["n_total"] == 1 << 20
        assert d["parity_vs_reference"] is True
        assert len(raw) < 7000


def test_g2_line_shape():
    """configs[4]'s line (bench.py --group 2): its own metric name, the G2
    roofline priced on the probe's mad rate, parity, under 7 KB."""
    raw = _last_line(os.path.join(REPO, "profiles", "r06_bench_g2.json"))
    assert len(raw) < 7000
    d = json.loads(raw)
    for k in CONTRACT:
        assert k in d, k
    assert "G2" in d["metric"] and d["parity_vs_reference"] is True
    r = d["roofline"]
    assert r["valu_unit"] == "T mad/s" and 0 < r["valu_frac"] <= 1 and r["peak_basis"].startswith("this run")
    for name, leg in d["legs"].items():
        assert leg.get("ok", True) is True, name


def test_profiles_agree_with_the_line():
    """The committed evidence behind the N = 1 line's roofline (final
    session): the rocprofv3 kernel stats list the dominant kernel, the HIP-event
    kernel time agrees with rocprof's average over the same timed launches
    (roofline_check.json), and the line's `traffic` is the PMC pass's bytes per
    launch (pmc_traffic.json, which bench.py reads)."""
    prof = os.path.join(REPO, "profiles")
    d = json.loads(_last_line(os.path.join(prof, "r06_bench.json")))
    stats = open(os.path.join(prof, "r06_kernel_stats.csv")).read()
    assert "k_accumulate<1" in stats
    chk = json.load(open(os.path.join(prof, "r06_roofline_check.json")))
    assert 0.95 < chk["rocprof_vs_bench"] < 1.05 and chk["timed_launches"] == d["steps"]
    assert chk["scratch"] == "0"
    pmc = json.load(open(os.path.join(prof, "r06_pmc_traffic.json")))
    assert pmc == json.load(open(os.path.join(prof, "pmc_traffic.json")))
    assert abs(pmc["accumulate_bytes_per_launch"] - d["roofline"]["traffic"]) / pmc["accumulate_bytes_per_launch"] < 1e-3
    assert d["roofline"]["traffic"] > d["roofline"]["algorithmic_bytes_per_launch"]  # 128-B lines of 112-B rows
