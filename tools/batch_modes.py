"""Time the CHES batch under each MSM_BATCH_MODE (bit 0: front k+1 issued before
head k; bit 1: reduction tails at the lowest stream priority).
usage: python tools/batch_modes.py [modes...]   (G1, n = 2^20, batches of 20)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import msm_blst_amd as m  # noqa: E402

modes = [int(a) for a in sys.argv[1:]] or [0, 1, 2, 3]
n = 1 << 20
pts = m.fixed_points(1, n)
sc = m.gen_scalars(n, 1)
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev)
d_sc = torch.frombuffer(bytearray(bytes(sc)), dtype=torch.uint8).to(dev)
for mode in modes:
    os.environ["MSM_BATCH_MODE"] = str(mode)
    ctx = m.CHESContext(1, 0, n_exp=20)
    ctx.build_table(pts, n, stream=stream.cuda_stream)
    want = m.compress(1, ctx.mult(d_sc.data_ptr(), 32, on_device=True, stream=stream.cuda_stream)).hex()
    ctx.mult_batch(d_sc.data_ptr(), 3, 32, set_stride=0, on_device=True, stream=stream.cuda_stream)
    best = 0
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        outs = ctx.mult_batch(d_sc.data_ptr(), 20, 32, set_stride=0, on_device=True, stream=stream.cuda_stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        best = max(best, 20 * n / dt)
        ok = all(m.compress(1, o).hex() == want for o in outs)
    print(f"mode {mode}: {best / 1e6:.1f} M pairs/s  parity {ok}", flush=True)
    del ctx
    torch.cuda.synchronize()
