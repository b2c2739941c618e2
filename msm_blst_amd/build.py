"""Build libmsm_mi355x.so (HIP, gfx950) in-tree.

`python -m msm_blst_amd.build` or `msm_blst_amd.build.build()`.  Sources in
msm_blst_amd/csrc are compiled with hipcc --offload-arch=gfx950 into objects
under msm_blst_amd/_build/ and linked into msm_blst_amd/libmsm_mi355x.so.
Rebuilds only what changed (mtime of sources and headers).
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# MSM_BUILD_VARIANT=<tag>: objects in _build_<tag>, library tools/ablib/libmsm_<tag>.so
# (A/B variants built with MSM_EXTRA_FLAGS; the product build leaves both unset)
_VAR = os.environ.get("MSM_BUILD_VARIANT")
OBJ = os.path.join(HERE, "_build" + (f"_{_VAR}" if _VAR else ""))
LIB = (os.path.join(os.path.dirname(HERE), "tools", "ablib", f"libmsm_{_VAR}.so") if _VAR
       else os.path.join(HERE, "libmsm_mi355x.so"))
BIN = os.path.join(HERE, "bin")
REPO = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MSM_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-value",
         "-Wno-unused-function", f"-I{os.path.join(REPO, 'include')}"] + os.environ.get("MSM_EXTRA_FLAGS", "").split()
# (source, MSM_GROUP or None): the group-templated engines compile once per
# group in parallel (the G2 instantiations dominate the build time)
SOURCES = [("engine.hip", 1), ("engine.hip", 2), ("ches.hip", 1), ("ches.hip", 2), ("bgmw.hip", 1), ("bgmw.hip", 2),
           ("compat.hip", 1), ("compat.hip", 2), ("wbits.hip", 1), ("wbits.hip", 2),
           ("probe.hip", None), ("abi.cpp", None)]


def _deps():
    return glob.glob(os.path.join(CSRC, "*.hpp")) + [os.path.join(REPO, "include", "msm_mi355x.h")]


def _stale(target, inputs):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(i) > t for i in inputs if os.path.exists(i))


def build(verbose=False, jobs=5):
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    hdrs = _deps()
    jobs_list = []
    objs = []
    for src, grp in SOURCES:
        sp = os.path.join(CSRC, src)
        if not os.path.exists(sp):
            continue
        stem = os.path.splitext(src)[0] + (f"_g{grp}" if grp else "")
        op = os.path.join(OBJ, stem + ".o")
        objs.append(op)
        if _stale(op, [sp] + hdrs):
            defs = [f"-DMSM_GROUP={grp}"] if grp else []
            jobs_list.append([HIPCC] + FLAGS + defs + ["-c", sp, "-o", op])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(run, jobs_list))
    if jobs_list or _stale(LIB, objs):
        # RCCL: the multi-device CHES batches gather their partials with ncclGather (csrc/multi.hpp)
        run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs + ["-L/opt/rocm/lib", "-lrccl"])
    if _VAR:
        return LIB
    # the reference-driver executables (ref main_p1.cpp / main_p2.cpp), host C++ on the C ABI
    drv = os.path.join(HERE, "driver", "ches_driver.cpp")
    hdr = os.path.join(REPO, "include", "msm_ches_driver.hpp")
    for g in (1, 2):
        exe = os.path.join(BIN, f"msm_driver_p{g}")
        if _stale(exe, [drv, hdr, LIB]):
            os.makedirs(BIN, exist_ok=True)
            run(["g++", "-O2", "-std=c++17", "-Wall", f"-DMSM_DRIVER_GROUP={g}", f"-I{os.path.join(REPO, 'include')}",
                 drv, "-o", exe, f"-L{HERE}", "-l:libmsm_mi355x.so", "-Wl,-rpath,$ORIGIN/.."])
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
