#!/usr/bin/env python3
"""The exposed tail of the last batch of each case in a kernel trace of
tools/r06_small_trace.py: every kernel that ends after the start of the last
accumulation launch of a segment, with its start / end (us from that
accumulation's start), duration, queue and grid.  Segments are split at host
gaps > --gap ms (the script sleeps 50 ms between batches).
usage: python3 tools/tail_listing.py run_kernel_trace.csv [--gap 20] [--segments 3,6]"""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--gap", type=float, default=20.0)
ap.add_argument("--segments", default="", help="comma-separated segment numbers to list (default: every one)")
a = ap.parse_args()
rows = []
for r in csv.DictReader(open(a.csv)):
    name = re.sub(r"\(.*", "", r["Kernel_Name"])
    name = re.sub(r"msm::|void |<.*", "", name)
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "?"),
                 r.get("Grid_Size", r.get("Grid_Size_X", "?")), r.get("Workgroup_Size", "")))
rows.sort()
segs, cur, last_end = [], [], None
for row in rows:
    if last_end is not None and row[0] - last_end > a.gap * 1e6:
        segs.append(cur)
        cur = []
    cur.append(row)
    last_end = max(last_end or 0, row[1])
segs.append(cur)
want = {int(x) for x in a.segments.split(",") if x}
for i, seg in enumerate(segs, 1):
    accs = [r for r in seg if r[2].startswith("k_accumulate")]
    if not accs or (want and i not in want):
        continue
    t0 = accs[-1][0]
    tail = [r for r in seg if r[1] > t0]
    span = (max(r[1] for r in seg) - t0) / 1e3
    print(f"== segment {i}: {len(seg)} kernels; from the last accumulation's start to the end {span:.1f} us")
    for s, e, nm, q, g, wg in tail:
        print(f"  {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{q} {nm} grid {g} wg {wg}")
