"""Convert rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into the bench's
`roofline.traffic` figure: HBM bytes per k_accumulate launch.

FETCH_SIZE/WRITE_SIZE are in KiB.  Calibration (tools/microbench/gather_cal.hip,
profiles/r02_gather_cal.json): for a coalesced 16-B/lane stream FETCH_SIZE is half
the bytes (MI355X_MICROARCH.md, HBM section); for the accumulation's pattern --
each lane gathering one random 128-B table row with seven 16-B loads -- FETCH_SIZE
is 64 B per row, i.e. x2 gives the full 128-B lines.  So FETCH x2 counts whole
128-B lines; WRITE_SIZE is exact for 16-B/lane stores.
usage: python tools/pmc_traffic.py <fetch.csv> <write.csv> <method> <log_n> [out.json] [calibration.json]
"""
import csv
import json
import sys


def per_kernel(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        vals.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
acc = [k for k in fetch if "k_accumulate" in k][0]
f_kib, w_kib = fetch[acc], write.get(acc, 0.0)
out = {"method": sys.argv[3], "log_n": int(sys.argv[4]), "group": 1, "kernel": "k_accumulate",
       "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
       "accumulate_bytes_per_launch": int(f_kib * 1024 * 2 + w_kib * 1024),
       "correction": "FETCH_SIZE x2 (whole 128-B lines, calibrated by tools/microbench/gather_cal.hip), WRITE_SIZE x1"}
if sys.argv[4] == "20" and sys.argv[3] == "ches":
    n, h, nb = 1 << 20, 12, 961017
    out["decomposition_bytes"] = {
        "table_rows_128B_lines": n * h * 128,          # 112-B internal rows padded to one 128-B line
        "table_rows_blst_96B_algorithmic": n * h * 96,
        "payload_4B": n * h * 4,                       # interleaved rows: one coalesced 256-B read per wave step
        "schedule_order_counts_offsets_wave_rows": nb * 12 + (nb // 64) * 8,
        "bucket_xyzz_writes_224B": nb * 224,
        "note": "round 3: counts/offsets are read by schedule position (coalesced) and the payload from "
                "per-wave interleaved rows (bucket_sort.hpp k_interleave); before, counts[id]/offsets[id] "
                "were random 4-B reads and each lane's payload run was re-fetched per step (2.63 GB/launch)"}
if len(sys.argv) > 6:
    out["calibration"] = json.load(open(sys.argv[6]))
js = json.dumps(out, indent=1)
print(js)
if len(sys.argv) > 5:
    open(sys.argv[5], "w").write(js + "\n")
