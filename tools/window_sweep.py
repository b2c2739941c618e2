"""Plain Pippenger window sweep on one GPU: ms per MSM (resident points and
scalars, msm_ctx_mult) for n = 2^k and window c, plus the blst drop-in at the
auto window.  Used to pick abi.cpp auto_window().  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import msm_blst_amd as m  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for lg in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "10,12,14,16,18,20").split(",")]:
        n = 1 << lg
        pts = m.fixed_points(1, n)
        sc = m.gen_scalars(n, 1)
        d = torch.tensor(bytearray(bytes(sc)), dtype=torch.uint8, device=dev)
        row = {}
        for c in (8, 10, 12, 13, 14, 15, 16, 17, 18):
            if c > lg + 2:
                continue
            ctx = m.MSMContext(1, 0, c)
            ctx.set_points(pts, n)
            ref = ctx.mult(d.data_ptr(), 255, on_device=True)
            reps = 5
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(reps):
                ctx.mult(d.data_ptr(), 255, on_device=True)
            row[c] = round((time.perf_counter() - t) / reps * 1e3, 4)
            ctx.close()
        pp = (ctypes.c_void_p * 2)(ctypes.cast(pts, ctypes.c_void_p), None)
        sp = (ctypes.c_void_p * 2)(ctypes.cast(sc, ctypes.c_void_p), None)
        r = (ctypes.c_uint8 * 144)()
        m.lib().blst_p1s_mult_pippenger(r, pp, n, sp, 255, None)
        t = time.perf_counter()
        for _ in range(5):
            m.lib().blst_p1s_mult_pippenger(r, pp, n, sp, 255, None)
        row["dropin"] = round((time.perf_counter() - t) / 5 * 1e3, 4)
        row["dropin_eq_ctx"] = m.compress(1, bytes(r)) == m.compress(1, ref)
        out[f"2^{lg}"] = row
        print(lg, row, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
