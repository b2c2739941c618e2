"""Print the kernel sequence of a rocprofv3 kernel trace between two
timestamps (or the k-th run of a kernel-name pattern): name, duration, gap to
the previous kernel's end.  Development aid for the per-MSM fixed-cost study.

usage: python tools/trace_seq.py run_kernel_trace.csv START_PATTERN K [COUNT]
  prints COUNT (default 80) kernels starting at the K-th dispatch whose name
  contains START_PATTERN.
"""
import csv
import re
import sys


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"msm::|void |rocprim::ROCPRIM_\w+::detail::", "", n)
    return n[:60]


def main(path, pat, k, count=80):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    hits = [i for i, r in enumerate(rows) if pat in r["Kernel_Name"]]
    i0 = hits[k]
    prev_end = int(rows[i0]["Start_Timestamp"])
    t0 = prev_end
    tot = {}
    for r in rows[i0:i0 + count]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        nm = short(r["Kernel_Name"])
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {(s - prev_end) / 1e3:7.1f}  q{r['Queue_Id']} "
              f"grid {r['Grid_Size_X']}x{r['Grid_Size_Y']} v{r['VGPR_Count']}  {nm}")
        prev_end = max(prev_end, e)
        tot[nm] = tot.get(nm, 0) + (e - s)
    print("span", (prev_end - t0) / 1e3, "us")
    for nm, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {v / 1e3:9.1f} us  {nm}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else 80)
