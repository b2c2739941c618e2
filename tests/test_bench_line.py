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
