#!/usr/bin/env python3
"""Hygiene: fold the round-1..4 profile files into one
text archive, profiles/archive_r01_r04.txt (one '=== <name> ===' section per
file, in name order), delete the originals, and point every citation of
`profiles/<name>` in the docs and sources at the archive section.  Files a
tool reads at run time stay (KEEP)."""
import glob
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(REPO, "profiles")
KEEP = {"r02_gather_cal.json"}  # tools/pmc_traffic.py's FETCH calibration input
ARCH = os.path.join(P, "archive_r01_r04.txt")

names = sorted(os.path.basename(f) for f in glob.glob(os.path.join(P, "r0[1-4]*")) if os.path.basename(f) not in KEEP)
with open(ARCH, "w") as out:
    out.write("# profiles of rounds 1-4, one section per former file (tools/archive_profiles.py);\n"
              "# DESIGN.md cites them as profiles/archive_r01_r04.txt (<name>)\n")
    for n in names:
        with open(os.path.join(P, n), errors="replace") as f:
            out.write(f"\n=== {n} ===\n" + f.read().rstrip("\n") + "\n")
for n in names:
    os.remove(os.path.join(P, n))
pat = re.compile(r"profiles/(" + "|".join(re.escape(n) for n in names) + r")\b")
files = [os.path.join(REPO, f) for f in ("DESIGN.md", "README.md", "INTEGRATION.md", "bench.py")]
files += glob.glob(os.path.join(REPO, "msm_blst_amd", "**", "*.*"), recursive=True)
files += glob.glob(os.path.join(REPO, "tools", "**", "*.*"), recursive=True)
files += glob.glob(os.path.join(REPO, "tests", "*.py"))
for f in files:
    if not f.endswith((".md", ".py", ".hpp", ".hip", ".cpp", ".sh", ".h")) or f.endswith("archive_profiles.py"):
        continue
    s = open(f).read()
    t = pat.sub(lambda m: f"profiles/archive_r01_r04.txt ({m.group(1)})", s)
    if t != s:
        open(f, "w").write(t)
        print("rewrote", os.path.relpath(f, REPO))
print(len(names), "files archived")
