"""Per-kernel register / scratch / occupancy summary of a gfx950 .s file
(hipcc -S --cuda-device-only): the compiler's "; Kernel info:" blocks.
usage: python tools/kernel_resources.py file.s [name_substring]"""
import re
import sys


def main(path, pat=""):
    name, info, cur = None, {}, None
    for line in open(path):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            name = m.group(1)
        if line.startswith("; Kernel info:") or line.startswith("; Function info:"):
            cur = {"kind": "kernel" if "Kernel" in line else "function"}
            continue
        if cur is not None:
            m = re.match(r"^; (NumVgprs|NumAgprs|ScratchSize|Occupancy): (\d+)", line)
            if m:
                cur[m.group(1)] = int(m.group(2))
            if line.startswith("; Occupancy") or (cur["kind"] == "function" and line.startswith("; MemoryBound")):
                info[name] = cur
                cur = None
    for n, d in info.items():
        if pat in n:
            print(f"{d['kind']:8s} vgpr {d.get('NumVgprs', '?'):>3} agpr {d.get('NumAgprs', '?'):>3} "
                  f"scratch {d.get('ScratchSize', '?'):>5} occ {d.get('Occupancy', '-')}  {n[:110]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
