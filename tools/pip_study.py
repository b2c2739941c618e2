#!/usr/bin/env python3
"""configs[1] study: plain-Pippenger batch (msm_ctx_mult_batch) at n = 2^16 over
windows and batch knobs.  Each knob setting runs in a child process (the
library reads MSM_* once per process); the child times K resident sets, best of
`reps`, and checks set 0 against the golden and the batch against sync MSMs.
usage: python tools/pip_study.py [--steps K] [--windows 13,14,15,16] [--envs "A=1 B=2;C=3"]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time
sys.path.insert(0, sys.argv[1])
import numpy as np, torch
import msm_blst_amd as m
K, reps, lg = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[5])
n = 1 << lg
gold = [c['compressed'] for c in json.load(open(sys.argv[1] + '/tests/golden/msm_g1.json'))['cases']
        if c['n'] == n and c['seed'] == 1 and c['case'] == 'rand' and c['nbits'] == 255]
raw = b''.join(m.gen_scalars(n, 1 if k == 0 else 100 + k) for k in range(K))
d = torch.tensor(np.frombuffer(raw, dtype=np.uint8), device='cuda:0')
pts = m.fixed_points(1, n)
for c in [int(x) for x in sys.argv[4].split(',')]:
    ctx = m.MSMContext(1, 0, c)
    ctx.set_points(pts, n)
    ctx.mult_batch(d.data_ptr(), K, 255, on_device=True)
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        got = ctx.mult_batch(d.data_ptr(), K, 255, on_device=True)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t) / K * 1e3
        best = el if best is None else min(best, el)
    sync = [ctx.mult(d.data_ptr() + k * 32 * n, 255, on_device=True) for k in (0, K - 1)]
    ok = m.compress(1, got[0]).hex() == gold[0] and [m.compress(1, x) for x in sync] == [m.compress(1, got[0]), m.compress(1, got[K - 1])]
    print(json.dumps({"c": c, "ms": round(best, 4), "Mpairs": round(n / best / 1e3, 1), "parity": ok}), flush=True)
    ctx.close()
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--windows", default="13,14,15,16")
    ap.add_argument("--envs", default="")
    a = ap.parse_args()
    for envs in (a.envs.split(";") if a.envs else [""]):
        env = dict(os.environ)
        for kv in envs.split():
            k, v = kv.split("=")
            env[k] = v
        r = subprocess.run([sys.executable, "-c", CHILD, REPO, str(a.steps), str(a.reps), a.windows, str(a.log_n)],
                           capture_output=True, text=True, env=env, timeout=300)
        for ln in r.stdout.splitlines():
            print(json.dumps(dict(json.loads(ln), env=envs)), flush=True)
        if r.returncode:
            print("child failed", envs, r.stderr[-2000:], flush=True)
            sys.exit(1)


if __name__ == "__main__":
    main()
