"""Convert a rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE collection into the bench's
`roofline.traffic` figure: HBM bytes per k_accumulate launch.

FETCH_SIZE/WRITE_SIZE are in KiB.  MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) reads -> x2; WRITE_SIZE
is exact for 16 B/lane stores.  Our gathers are 16 B/lane loads of 112-B rows.
usage: python tools/pmc_traffic.py <counter_collection.csv[,second_pass.csv]> <method> <log_n> [out.json]
"""
import csv
import json
import sys

rows = [r for f in sys.argv[1].split(",") for r in csv.DictReader(open(f))]
vals = {}
for r in rows:
    if "k_accumulate" not in r["Kernel_Name"]:
        continue
    vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
fetch = sum(vals.get("FETCH_SIZE", [0])) / max(1, len(vals.get("FETCH_SIZE", [])))
write = sum(vals.get("WRITE_SIZE", [0])) / max(1, len(vals.get("WRITE_SIZE", [])))
out = {"method": sys.argv[2], "log_n": int(sys.argv[3]), "kernel": "k_accumulate",
       "fetch_size_kib_raw": fetch, "write_size_kib_raw": write, "launches": len(vals.get("FETCH_SIZE", [])),
       "accumulate_bytes_per_launch": int(fetch * 1024 * 2 + write * 1024),
       "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section), WRITE_SIZE x1"}
js = json.dumps(out, indent=1)
print(js)
if len(sys.argv) > 4:
    open(sys.argv[4], "w").write(js + "\n")
