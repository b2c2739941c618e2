"""Print the kernel timeline of the last CHES batch in a rocprofv3 kernel trace.
usage: python tools/timeline.py gpurun_out/<tag>/prof/run_kernel_trace.csv [nlines]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))


def short(n):
    m = re.search(r"(k_[a-z_0-9]+|rocprim|copyBuffer|fillBuffer)", n)
    return m.group(1) if m else n[:30]


ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows)
acc = [e for e in ev if e[2] == "k_accumulate"]
t0 = acc[-9][0] - 100000
sel = [e for e in ev if e[0] >= t0]
base = sel[0][0]
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 120
for s, e, n, q in sel[:nl]:
    print(f"{(s - base) / 1000:9.1f} {(e - base) / 1000:9.1f} {(e - s) / 1000:8.1f} q{q} {n}")
a = [e for e in sel if e[2] == "k_accumulate"]
print("accumulate starts delta (us):", [round((a[i + 1][0] - a[i][0]) / 1000, 1) for i in range(len(a) - 1)])
