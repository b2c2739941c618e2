"""Per-MSM timeline of bench.py's timed H2D batch from a rocprofv3 kernel +
memory-copy trace: for each accumulation k of the timed batch, its start,
duration, the gap since accumulation k-1 ended, the end of level 0 of k-1,
the end of front k (k_interleave of its sort) and the H2D copy bytes/time
overlapping it.  A fast/slow run comparison aid (round 4, the bimodal H2D
headline).

usage: python tools/h2d_trace.py <trace_dir_prefix> <warmup> <steps>
  (<prefix>_kernel_trace.csv and <prefix>_memory_copy_trace.csv)
"""
import csv
import sys


def main(prefix, W, K):
    W, K = int(W), int(K)
    ks = list(csv.DictReader(open(prefix + "_kernel_trace.csv")))
    try:
        cs = list(csv.DictReader(open(prefix + "_memory_copy_trace.csv")))
    except FileNotFoundError:
        cs = []
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    acc = [r for r in ks if "k_accumulate<1" in r["Kernel_Name"] and int(r["Grid_Size_X"]) > 500000]
    seg = [r for r in ks if "k_segsum<1>" in r["Kernel_Name"] and int(r["Grid_Size_Y"]) == 1
           and int(r["Grid_Size_X"]) > 100000]
    inter = [r for r in ks if "k_interleave" in r["Kernel_Name"]]
    h2d = [r for r in cs if "HOST_TO_DEVICE" in r.get("Direction", r.get("Kind", "")) or
           r.get("Src_Agent_Type", "") == "CPU"]
    timed = acc[W:W + K]
    if len(timed) < K:
        print("not enough accumulations", len(acc))
        return
    t0 = int(timed[0]["Start_Timestamp"])
    S = lambda r: int(r["Start_Timestamp"])
    E = lambda r: int(r["End_Timestamp"])
    prev_end = None
    tot_gap = 0
    print(" k   start_ms  dur_ms  gap_ms  l0prev_end  front_end  copy_overlap_ms")
    for k, a in enumerate(timed):
        s, e = S(a), E(a)
        gap = (s - prev_end) / 1e6 if prev_end else 0.0
        tot_gap += gap
        l0 = [r for r in seg if S(r) < s and (prev_end is None or E(r) >= prev_end - 1)]
        l0e = max((E(r) for r in l0), default=None)
        fr = [r for r in inter if E(r) <= s + 1000]
        fre = max((E(r) for r in fr), default=None)
        ov = sum(max(0, min(e, E(c)) - max(s, S(c))) for c in h2d) / 1e6
        f = lambda x: f"{(x - t0) / 1e6:9.3f}" if x is not None else "        -"
        print(f"{k:2d} {f(s)} {(e - s) / 1e6:7.3f} {gap:7.3f} {f(l0e)} {f(fre)} {ov:8.3f}")
        prev_end = e
    span = (E(timed[-1]) - S(timed[0])) / 1e6
    dur = sum((E(a) - S(a)) for a in timed) / 1e6
    print(f"span {span:.3f} ms  sum(acc) {dur:.3f}  sum(gaps) {tot_gap:.3f}  per MSM {span / K:.3f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
