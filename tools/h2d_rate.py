"""Pinned host -> HBM copy rate (hipMemcpyAsync via torch), 32 MiB and 640 MiB."""
import time

import torch

for mb in (32, 640):
    h = torch.empty(mb << 20, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(mb << 20, dtype=torch.uint8, device="cuda:0")
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
    print(f"H2D {mb} MiB: {el * 1e3:.3f} ms  {(mb << 20) / el / 1e9:.1f} GB/s", flush=True)
