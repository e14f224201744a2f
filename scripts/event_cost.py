#!/usr/bin/env python3
"""Does recording timing events inside a step change the step time? FL encode +
decode of 1 GiB, 50 steps each: no events, 2 events (call brackets), and the
bench's 8 (incl. flrl_time_next_kernel pairs), interleaved over 3 rounds."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-rl-compression-mpi_amd"))
import torch  # noqa: E402

import flrl  # noqa: E402
from flrl.device import FLDevice, gen  # noqa: E402

n = 1 << 30
x = gen("u8", n, 42)
d = FLDevice(n)
out = torch.empty_like(x)
d.encode(x)
v = d.values_size()
s = torch.cuda.current_stream()
K = 50
ev = [[torch.cuda.Event(enable_timing=True) for _ in range(8)] for _ in range(K)]
for row in ev:
    for e in row:
        e.record(s)


def run(mode):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        e = ev[k]
        if mode >= 2:
            e[0].record(s)
        if mode == 8:
            flrl.time_next_kernel(e[4], e[5])
        d.encode(x)
        if mode >= 2:
            e[1].record(s)
        if mode == 8:
            e[2].record(s)
            flrl.time_next_kernel(e[6], e[7])
        d.decode(v, out=out)
        if mode == 8:
            e[3].record(s)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / K


for m in (0, 2, 8):
    run(m)
res = {0: [], 2: [], 8: []}
for _ in range(3):
    for m in (0, 2, 8):
        res[m].append(run(m))
for m, r in res.items():
    print(f"{m} events/step: ms/step {min(r):.4f} (all {[round(t, 4) for t in r]})", flush=True)
