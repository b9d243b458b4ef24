"""Pinned D2H bandwidth of this box (trip-list copy sizing)."""
import time
import torch
for mb in (8, 76, 256):
    d = torch.empty(mb << 20, dtype=torch.uint8, device="cuda")
    h = torch.empty(mb << 20, dtype=torch.uint8, pin_memory=True)
    h.copy_(d, non_blocking=True); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 5
    print("D2H %d MB: %.2f ms, %.1f GB/s" % (mb, dt * 1e3, (mb << 20) / dt / 1e9), flush=True)
