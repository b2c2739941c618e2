#!/usr/bin/env python3
"""Summarise a VALU PMC pass (tools/r06_final.sh: rocprofv3 --pmc
SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES)
per dispatch of a kernel: held clock, VALU-busy fraction per SIMD and resident
waves.  usage: valu_pmc_summary.py run_counter_collection.csv [kernel-substring]
  clk            = GRBM_GUI_ACTIVE / 8 XCDs / duration
  valu/SIMD      = SQ_ACTIVE_INST_VALU (quad-cycles) x 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8)
  waves-resident = SQ_WAVE_CYCLES x 4 / (GRBM_GUI_ACTIVE / 8)"""
import csv
import json
import sys

path = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "k_accumulate"
rows = {}
for r in csv.DictReader(open(path)):
    if key not in r["Kernel_Name"]:
        continue
    d = rows.setdefault(int(r["Dispatch_Id"]), {"grid": int(r["Grid_Size"]),
                                                 "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
                                                 "raw": {}})
    d["raw"][r["Counter_Name"]] = float(r["Counter_Value"])
for disp, d in sorted(rows.items()):
    raw = d["raw"]
    per_xcd = raw["GRBM_GUI_ACTIVE"] / 8
    print(f"dispatch {disp} grid {d['grid']} dur {d['dur']:.3f} ms  clk {per_xcd / d['dur'] / 1e6:.3f} GHz  "
          f"valu/SIMD {raw['SQ_ACTIVE_INST_VALU'] * 4 / 1024 / per_xcd:.3f}  "
          f"waves-resident {raw['SQ_WAVE_CYCLES'] * 4 / per_xcd:.0f}  raw {json.dumps(dict(sorted(raw.items())))}")
