#!/usr/bin/env python3
"""Print the headline and every leg of a bench.py JSON line (value, ms, parity)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"], "parity", d["parity_vs_reference"], "frac", d["roofline"]["frac"],
      "mad_frac", d["valu_roofline"].get("mad_frac"))
for k, v in d["methods"].items():
    extra = {kk: v[kk] for kk in ("kernel_ms", "ratio_vs_ctx_sync", "efficiency", "projected_value") if kk in v}
    print(" ", k, v.get("value"), v.get("ms_per_step"), v.get("parity_vs_reference"), extra or "")
if d.get("cpu_baseline"):
    print("  cpu", d["cpu_baseline"]["value"], (d["cpu_baseline"].get("all_cores") or {}).get("value"))
