"""Recompute the bench line's roofline from a committed rocprofv3 kernel trace.

usage: python tools/roofline_check.py <bench.json> <run_kernel_trace.csv> [out.json]

The bench command run under `rocprofv3 --kernel-trace --stats` launches, in
order: W warmup accumulations (one batch), the K accumulations of the timed
host-scalar batch, then the resident batch, the synchronous MSMs and the other
methods.  The CHES accumulations are the k_accumulate launches whose grid is
the CHES bucket count; launches [W, W+K) of them are the timed region.  Their
average rocprof duration gives achieved = algorithmic bytes / duration, to be
compared with the bench line's HIP-event `kernel_ms` (events on the
accumulation stream fire when the stream reaches them, so under the batch's
concurrent kernels they include dispatch waits the rocprof span does not)."""
import csv
import json
import sys

line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
rows = [r for r in csv.DictReader(open(sys.argv[2])) if "k_accumulate" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nb = line["config"].get("buckets_incl_top_digit_copies")
grid = -(-nb // 256) * 256
ches = [r for r in rows if int(r["Grid_Size_X"]) == grid]
W, K = line["warmup"], line["steps"]
timed = ches[W:W + K]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
avg = sum(dur) / len(dur)
alg = line["roofline"]["algorithmic_bytes_per_launch"]
all_avg = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows) / len(rows)
out = {
    "timed_launches": len(dur), "rocprof_avg_ms_timed": round(avg, 4), "rocprof_avg_ms_all_k_accumulate": round(all_avg, 4),
    "bench_kernel_ms": line["roofline"]["kernel_ms"],
    "rocprof_vs_bench": round(avg / line["roofline"]["kernel_ms"], 4),
    "achieved_gbs_rocprof": round(alg / avg / 1e6, 2), "frac_rocprof": round(alg / avg / 1e6 / line["roofline"]["peak"], 5),
    "valu_frac_rocprof": round(line["roofline"]["valu_frac"] * line["roofline"]["kernel_ms"] / avg, 4),
    "vgpr": timed[0]["VGPR_Count"], "scratch": timed[0]["Scratch_Size"],
}
js = json.dumps(out, indent=1)
print(js)
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(js + "\n")
