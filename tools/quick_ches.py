"""Quick CHES timing on one GPU: table build time, per-phase times, pairs/s."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import msm_blst_amd as m  # noqa: E402

group = int(sys.argv[1]) if len(sys.argv) > 1 else 1
log_n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n = 1 << log_n
t = time.time()
pts = m.fixed_points(group, n)
sc = m.gen_scalars(n, 1)
print(f"inputs {time.time() - t:.1f}s", flush=True)
ctx = m.CHESContext(group, 0, n_exp=log_n)
t = time.time()
ctx.build_table(pts, n)
print(f"table build {time.time() - t:.3f}s  |B|={ctx.bucket_count()}", flush=True)
r = ctx.mult(sc)
gold = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", f"msm_g{group}.json")))
want = [c for c in gold["cases"] if c["n"] == n and c["seed"] == 1 and c["case"] == "rand"]
print("parity", (m.compress(group, r).hex() == want[0]["compressed"]) if want else "n/a", flush=True)
ctx.set_profiling(True)
for k in range(5):
    t = time.perf_counter()
    ctx.mult(sc)
    dt = time.perf_counter() - t
    print(f"mult {dt * 1e3:.3f} ms  ({n / dt / 1e6:.1f} M pairs/s) phases", {k: round(v, 3) for k, v in ctx.phase_times().items()}, flush=True)
