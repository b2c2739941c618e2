#!/usr/bin/env python3
"""Where does a pipelined batch spend its time?  Splits a rocprofv3 kernel
trace into segments at host gaps (> --gap ms with no kernel running) and, for
each segment with accumulation kernels, prints: span; the time with >= 1
accumulation running; the exposed time before the first / after the last
accumulation; per kernel family the summed duration and the busy union; the
mean accumulation duration and how many ran concurrently.
usage: python tools/batch_profile.py run_kernel_trace.csv [--gap 20] [--min-acc 10]
"""
import argparse
import csv
import re


def fam(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"msm::|void |rocprim::ROCPRIM_\w+::detail::", "", n)
    n = re.sub(r"<.*", "", n)
    return n[:40]


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=float, default=20.0)
    ap.add_argument("--min-acc", type=int, default=10)
    a = ap.parse_args()
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"]))
                   for r in csv.DictReader(open(a.trace))))
    segs, cur, end = [], [], None
    for r in rows:
        if end is not None and r[0] - end > a.gap * 1e6:
            segs.append(cur)
            cur = []
        cur.append(r)
        end = r[1] if end is None else max(end, r[1])
    segs.append(cur)
    for si, sg in enumerate(segs):
        acc = [r for r in sg if r[2].startswith("k_accumulate")]
        if len(acc) < a.min_acc:
            continue
        t0, t1 = sg[0][0], max(r[1] for r in sg)
        a0, a1 = min(r[0] for r in acc), max(r[1] for r in acc)
        span = (t1 - t0) / 1e3
        print(f"segment {si}: {len(sg)} kernels, span {span:.1f} us, {len(acc)} accumulations "
              f"({span / len(acc):.1f} us per accumulation)")
        print(f"  before first accumulation {(a0 - t0) / 1e3:.1f} us, after last {(t1 - a1) / 1e3:.1f} us, "
              f"accumulation busy union {union([(r[0], r[1]) for r in acc]) / 1e3:.1f} us")
        durs = [(r[1] - r[0]) / 1e3 for r in acc]
        conc = sum(durs) / (union([(r[0], r[1]) for r in acc]) / 1e3)
        print(f"  accumulation mean {sum(durs) / len(durs):.1f} us (min {min(durs):.1f}, max {max(durs):.1f}), "
              f"mean concurrency {conc:.2f}")
        fams = {}
        for r in sg:
            fams.setdefault(r[2], []).append((r[0], r[1]))
        for f, iv in sorted(fams.items(), key=lambda x: -sum(e - s for s, e in x[1])):
            tot = sum(e - s for s, e in iv) / 1e3
            print(f"  {f:40s} n {len(iv):5d} sum {tot:9.1f} us  union {union(iv) / 1e3:9.1f} us")
        # what runs after the last accumulation (the exposed tail)
        tail = [r for r in sg if r[0] >= a1 - 1000]
        if tail:
            tf = {}
            for r in tail:
                tf.setdefault(r[2], [0, 0])
                tf[r[2]][0] += 1
                tf[r[2]][1] += r[1] - r[0]
            print("  after the last accumulation: " + ", ".join(f"{k} x{v[0]} {v[1] / 1e3:.0f} us" for k, v in tf.items()))


if __name__ == "__main__":
    main()
