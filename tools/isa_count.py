"""Instruction histogram of one kernel in a gfx950 .s file (hipcc -S
--cuda-device-only): total, v_mad_u64_u32 and the main-loop body, VGPRs.
usage: python tools/isa_count.py file.s kernel_substring"""
import collections
import re
import sys


def main(path, pat):
    s = open(path).read()
    names = [n for n in re.findall(r"^(_Z\w+):", s, re.M) if pat in n]
    for name in names:
        i = s.index(name + ":")
        j = s.index("s_endpgm", i)
        ins = [l.split()[0] for l in s[i:j].split("\n")
               if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
        c = collections.Counter(ins)
        vg = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", s)
        sc = re.search(re.escape(name) + r"\.private_seg_size, (\d+)", s)
        print(f"{name[:100]}\n  vgpr {vg.group(1) if vg else '?'} scratch {sc.group(1) if sc else '?'} "
              f"total {sum(c.values())} v_mad_u64_u32 {c['v_mad_u64_u32']}")
        print("  " + ", ".join(f"{k} {v}" for k, v in c.most_common(14)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
