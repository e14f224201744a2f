#!/usr/bin/env python3
"""Write-only and read-only ceilings of 1 GiB on this GPU (torch fill_ / amax),
to price the RL decode (write-dominated) against them. GPU box."""
import torch

n = 1 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
y = torch.ones(n // 4, dtype=torch.int32, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, f in (("fill u8", lambda: x.fill_(7)), ("fill i32 view", lambda: x.view(torch.int32).fill_(7)),
                ("zero_", lambda: x.zero_()), ("amax read", lambda: torch.amax(y))):
    for _ in range(3):
        f()
    t = []
    for _ in range(10):
        e0.record()
        f()
        e1.record()
        e1.synchronize()
        t.append(e0.elapsed_time(e1))
    t.sort()
    print(f"{name:14s} median {t[5]:.4f} ms  {n / t[5] / 1e6:.0f} GB/s", flush=True)
