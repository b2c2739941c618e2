"""blst_p1s_mult_pippenger (the drop-in) at n = 2^k: per-call time with the
same caller buffers reused vs fresh pageable buffers every call, and the
context MSM on resident data for comparison.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import msm_blst_amd as m  # noqa: E402


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = 1 << lg
    pts = m.fixed_points(1, n)
    sc = bytes(m.gen_scalars(n, 1))
    L = m.lib()

    def call(P, S):
        pp = (ctypes.c_void_p * 2)(ctypes.cast(P, ctypes.c_void_p), None)
        sp = (ctypes.c_void_p * 2)(ctypes.cast(S, ctypes.c_void_p), None)
        r = (ctypes.c_uint8 * 144)()
        L.blst_p1s_mult_pippenger(r, pp, n, sp, 255, None)
        return bytes(r)

    S = (ctypes.c_uint8 * len(sc)).from_buffer_copy(sc)
    ref = call(pts, S)
    out = {}
    t = time.perf_counter()
    for _ in range(5):
        call(pts, S)
    out["reused_ms"] = round((time.perf_counter() - t) / 5 * 1e3, 3)
    fresh = []
    for _ in range(5):
        P2 = (ctypes.c_uint8 * len(pts)).from_buffer_copy(bytes(pts))
        S2 = (ctypes.c_uint8 * len(sc)).from_buffer_copy(sc)
        t = time.perf_counter()
        r = call(P2, S2)
        fresh.append(time.perf_counter() - t)
        assert m.compress(1, r) == m.compress(1, ref)
    out["fresh_ms"] = [round(x * 1e3, 3) for x in fresh]
    ctx = m.MSMContext(1, 0, 16 if lg >= 17 else 14)
    ctx.set_points(pts, n)
    d = torch.tensor(bytearray(sc), dtype=torch.uint8, device="cuda:0")
    ctx.mult(d.data_ptr(), 255, on_device=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        ctx.mult(d.data_ptr(), 255, on_device=True)
    out["ctx_resident_ms"] = round((time.perf_counter() - t) / 5 * 1e3, 3)
    ctx.set_profiling(True)
    ctx.mult(d.data_ptr(), 255, on_device=True)
    out["ctx_phases"] = {k: round(v, 3) for k, v in ctx.phase_times().items()}
    out["n"] = n
    print(json.dumps(out))


if __name__ == "__main__":
    main()
