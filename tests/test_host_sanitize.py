"""The engine's host-only code under the sanitizers (SURVEY sec.5 aux; the
reference's only guard is -Werror, /root/reference/build.sh:26).

tests/host/sanitize_shim.cpp compiles the product's HIP-free host headers --
host_fp.hpp (boundary field/curve code), ptr_walk.hpp (blst's pointer-array
rule), row_samples.hpp (the registered-table staleness guard), workers.hpp
(WorkerPool, ThreadTeam: the batch's host Horner and the multi-device shard
threads) -- together with oracle/msm_oracle.c:
  * -fsanitize=address,undefined: the oracle's plain Pippenger (G1 2^10, G2
    2^6) and CHES (2^10) MSMs against the golden keys, host_fp against the
    oracle, the pointer walker against a naive walk, the guard, the workers;
  * -fsanitize=thread: the worker patterns alone (concurrent callers,
    exceptions, 200 rounds).
Any sanitizer report aborts the binary (-fno-sanitize-recover=all,
halt_on_error)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "host", "sanitize_shim.cpp")
ORACLE = os.path.join(REPO, "oracle", "msm_oracle.c")
OUT = os.path.join(HERE, "host", "_build")
COMMON = ["-O1", "-g", "-fno-omit-frame-pointer", "-Wall", "-Werror", "-Wno-unused-function"]


def _build(kind, flags):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, f"sanitize_{kind}")
    deps = [SRC, ORACLE] + [os.path.join(REPO, "msm_blst_amd", "csrc", h)
                            for h in ("host_fp.hpp", "ptr_walk.hpp", "row_samples.hpp", "workers.hpp")]
    if os.path.exists(exe) and all(os.path.getmtime(d) <= os.path.getmtime(exe) for d in deps):
        return exe
    obj = os.path.join(OUT, f"msm_oracle_{kind}.o")
    subprocess.run(["gcc", "-std=c11", "-c", ORACLE, "-o", obj] + COMMON + flags, check=True,
                   capture_output=True, text=True)
    r = subprocess.run(["g++", "-std=c++17", SRC, obj, "-o", exe, "-pthread"] + COMMON + flags,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def _key(golden, group, n):
    return [c["compressed"] for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == 1 and c["case"] == "rand" and c["nbits"] == 255][0]


def _env(extra):
    env = dict(os.environ, **extra)
    env.pop("LD_PRELOAD", None)  # the sanitizer runtimes are linked statically; nothing else is needed
    return env


def test_host_code_under_asan_ubsan(golden):
    exe = _build("asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-static-libasan",
                          "-static-libubsan"])
    args = [exe, "host", "1024", _key(golden, 1, 1024), "64", _key(golden, 2, 64), "10", _key(golden, 1, 1024)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600,
                       env=_env({"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1:abort_on_error=0",
                                 "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}))
    assert r.returncode == 0 and "OK host" in r.stdout, (r.stdout + r.stderr)[-4000:]


def test_worker_threads_under_tsan():
    try:
        exe = _build("tsan", ["-fsanitize=thread", "-static-libtsan"])
    except subprocess.CalledProcessError as e:  # pragma: no cover - toolchain without TSan
        pytest.skip(f"no TSan toolchain: {e.stderr[-300:]}")
    r = subprocess.run([exe, "threads"], capture_output=True, text=True, timeout=600,
                       env=_env({"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}))
    if "FATAL: ThreadSanitizer" in r.stderr and "memory mapping" in r.stderr:  # pragma: no cover
        pytest.skip("TSan cannot map its shadow memory in this environment: " + r.stderr[-300:])
    assert r.returncode == 0 and "OK threads" in r.stdout, (r.stdout + r.stderr)[-4000:]
