#!/usr/bin/env python3
"""A/B timing of RL decode variants (FLRL_RL_DEC, read by a temporary switch in
flrl_rl_decode_device while an experiment is open; none is compiled in now, so
every variant runs the library's kernel), interleaved in one process on the
runs32 (or --kind) bench input; every variant's output must equal the input.
Used for the rank-decode decision (DESIGN.md §RL decode)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-rl-compression-mpi_amd"))
import torch  # noqa: E402

import flrl  # noqa: E402
from flrl.device import RLDevice, gen  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--bytes", type=int, default=1 << 30)
p.add_argument("--kind", default="runs32")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--variants", default="0,1")
p.add_argument("--ablation", action="store_true", help="variants may change the output")
a = p.parse_args()
n = a.bytes
x = (gen(a.kind, n, 42) if a.kind in ("u8", "lo4", "zero")
     else torch.from_numpy(flrl.gen_host(a.kind, n, 42)).cuda())
d = RLDevice(n, "cuda")
d.encode(x)
R = d.runs()
assert d.error() == 0
vs = [int(v) for v in a.variants.split(",")]
for v in vs:
    os.environ["FLRL_RL_DEC"] = str(v)
    d.out.fill_(0xA5)
    y = d.decode(R)
    torch.cuda.synchronize()
    ok = d.error() == 0 and torch.equal(y, x[:n])
    print(f"variant {v}: round trip {'ok' if ok else 'MISMATCH'} (R={R})", flush=True)
    assert ok or a.ablation
tot = {v: 0.0 for v in vs}
blk = {}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for v in vs:  # blocks of reps per variant (no interleaving)
    os.environ["FLRL_RL_DEC"] = str(v)
    d.decode(R)
    e0.record()
    for r in range(a.reps):
        d.decode(R)
    e1.record()
    e1.synchronize()
    blk[v] = e0.elapsed_time(e1) / a.reps
for v in vs:
    print(f"variant {v} ({a.kind}) block of {a.reps}: {blk[v]:.4f} ms", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(a.reps):
    for v in vs:
        os.environ["FLRL_RL_DEC"] = str(v)
        e0.record()
        d.decode(R)
        e1.record()
        e1.synchronize()
        if r:
            tot[v] += e0.elapsed_time(e1)
alg = n + 2 * R
for v in vs:
    ms = tot[v] / (a.reps - 1)
    print(f"variant {v} ({a.kind}): {ms:.4f} ms  {alg / ms / 1e6:.1f} GB/s alg", flush=True)
