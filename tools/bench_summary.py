#!/usr/bin/env python3
"""Print the headline and every leg of a bench.py JSON line (M pairs/s, ms, parity)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("headline", d["value"], d["ms_per_step"], "parity", d["parity_vs_reference"], "frac", r["frac"],
      "valu_frac", r.get("valu_frac"), "alone", r.get("valu_frac_alone"), "mad_frac", r.get("mad_frac"),
      "basis", r.get("peak_basis"), "bytes", len(open(sys.argv[1]).read().strip().splitlines()[-1]))
for k, v in d["legs"].items():
    print(" ", k, v)
if d.get("cpu_baseline"):
    print("  cpu", d["cpu_baseline"]["value"], d["cpu_baseline"].get("all_cores_value"))
