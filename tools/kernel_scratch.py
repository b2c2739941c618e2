#!/usr/bin/env python3
"""Per-kernel register, spill and scratch use of every gfx950 kernel inside a
built HIP library (the code objects' AMDHSA metadata: .vgpr_count,
.agpr_count, .vgpr_spill_count, .sgpr_spill_count,
.private_segment_fixed_size).

The library's .hip_fatbin section holds one offload bundle per compiled
source; each is unbundled with clang-offload-bundler and read with
llvm-readelf --notes (both from /opt/rocm/lib/llvm/bin).  No GPU needed.
usage: python tools/kernel_scratch.py [lib.so]   (default: the product library)
"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
KEYS = ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size")


def kernels(lib=os.path.join(REPO, "msm_blst_amd", "libmsm_mi355x.so"), arch="gfx950"):
    """{mangled kernel name: {key: int}} over every bundle of `lib`."""
    out = {}
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for k, s in enumerate(starts):
            e = starts[k + 1] if k + 1 < len(starts) else len(data)
            part, co = os.path.join(td, f"b{k}.bin"), os.path.join(td, f"b{k}.co")
            open(part, "wb").write(data[s:e])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            f"--targets=hipv4-amdgcn-amd-amdhsa--{arch}", f"--output={co}"], check=True)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            cur = None
            for line in notes.splitlines():
                m = re.match(r"^\s+-?\s*\.(\w+):\s+(\S+)", line)
                if not m:
                    continue
                key, val = m.group(1), m.group(2)
                if line.lstrip().startswith("- .agpr_count"):
                    cur = {}
                if cur is None:
                    continue
                if key == "name":
                    out[val] = cur
                elif key in KEYS:
                    cur[key] = int(val)
    return out


def main():
    ks = kernels(*sys.argv[1:2])
    for name, d in sorted(ks.items()):
        print(f"vgpr {d.get('vgpr_count', 0):>3} agpr {d.get('agpr_count', 0):>3} "
              f"spill v{d.get('vgpr_spill_count', 0)} s{d.get('sgpr_spill_count', 0)} "
              f"scratch {d.get('private_segment_fixed_size', 0):>5}  {name[:120]}")
    print(f"{len(ks)} kernels", file=sys.stderr)


if __name__ == "__main__":
    main()
