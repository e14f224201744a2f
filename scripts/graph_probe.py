#!/usr/bin/env python3
"""Probe: capture one FL encode+decode step into a HIP graph (torch.cuda.graph)
and replay it, checking every replay's output and device error word against
the eager step. Usage: python scripts/graph_probe.py [bytes] [replays]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-rl-compression-mpi_amd"))
import torch  # noqa: E402

from flrl.device import FLDevice, gen  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256 << 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
x = gen("u8", n, 42)
d = FLDevice(n)
out = torch.empty_like(x)
d.encode(x)
v = d.values_size()
d.decode(v, out=out)
torch.cuda.synchronize()
assert d.error() == 0 and torch.equal(out[:n], x[:n])
bits0, vals0 = d.bits[: d.frames].clone(), d.values[:v].clone()
print("eager ok", flush=True)

side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):  # warm the capture stream
    for _ in range(3):
        d.encode(x)
        d.decode(v, out=out)
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    d.encode(x)
    d.decode(v, out=out)
torch.cuda.synchronize()
print("captured", flush=True)
for i in range(reps):
    out.zero_()  # every output cleared: a skipped kernel cannot pass on stale results
    d.bits.zero_()
    d.values.zero_()
    d.sizes[1] = 0
    g.replay()
    torch.cuda.synchronize()
    e = d.error()
    ok = e == 0 and torch.equal(out[:n], x[:n]) and torch.equal(d.bits[: d.frames], bits0) \
        and torch.equal(d.values[:v], vals0)
    if not ok:
        print("replay", i, "MISMATCH err", e, flush=True)
        sys.exit(1)
print("replays ok:", reps, flush=True)
# timing: eager vs graph, back to back
for label, fn in (("eager", lambda: (d.encode(x), d.decode(v, out=out))), ("graph", g.replay)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    print(label, "ms/step", round((time.perf_counter() - t0) * 1e3 / 50, 4), flush=True)
