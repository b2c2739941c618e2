"""Quick timing of the plain-Pippenger engine (development aid, not bench.py)."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import msm_blst_amd as m  # noqa: E402

for group, lg, c in [(1, 16, 13), (1, 16, 16), (1, 20, 16), (1, 20, 15), (1, 20, 17), (2, 16, 13)]:
    n = 1 << lg
    t = time.time()
    pts = m.fixed_points(group, n)
    sc = m.gen_scalars(n, 1)
    tgen = time.time() - t
    ctx = m.MSMContext(group, 0, c)
    ctx.set_points(pts, n)
    ctx.set_profiling(True)
    r = ctx.mult(sc)
    ts = []
    for _ in range(3):
        t = time.time()
        r = ctx.mult(sc)
        ts.append(time.time() - t)
    ph = ctx.phase_times()
    best = min(ts)
    print(f"G{group} n=2^{lg} c={c}: {best*1e3:.2f} ms wall -> {n/best/1e6:.2f} M pairs/s | phases(ms) "
          + " ".join(f"{k}={v:.3f}" for k, v in ph.items()) + f" | gen {tgen:.1f}s | {m.compress(group, r).hex()[:16]}",
          flush=True)
    ctx.close()
