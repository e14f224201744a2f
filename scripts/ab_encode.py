#!/usr/bin/env python3
"""A/B timing of FL encode variants, interleaved in one process on the 1 GiB
(or --bytes) bench input; each variant's output is checked against the first's.
Variants are selected through the FLRL_ENC_LW environment variable, read by a
temporary switch in flrl_fl_encode_device while an experiment is open (none is
compiled in now: every variant runs the library's kernel). Used for the
look-back-wave decision (DESIGN.md §FL encode)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-rl-compression-mpi_amd"))
import torch  # noqa: E402

from flrl.device import FLDevice, gen  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--bytes", type=int, default=1 << 30)
p.add_argument("--kind", default="u8")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--variants", default="0,1,2")
a = p.parse_args()
n = a.bytes
x = gen(a.kind, n, 42)
d = FLDevice(n, "cuda")
vs = [int(v) for v in a.variants.split(",")]
ref = None
for v in vs:
    os.environ["FLRL_ENC_LW"] = str(v)
    d.encode(x)
    torch.cuda.synchronize()
    vsz = d.values_size()
    assert d.error() == 0, (v, d.error())
    got = (d.bits[: d.frames].clone(), d.values[:vsz].clone())
    if ref is None:
        ref = got
    else:
        ok = torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])
        print(f"variant {v}: output {'== ' if ok else '!= '}variant {vs[0]}", flush=True)
        assert ok
tot = {v: 0.0 for v in vs}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(a.reps):
    for v in vs:
        os.environ["FLRL_ENC_LW"] = str(v)
        e0.record()
        d.encode(x)
        e1.record()
        e1.synchronize()
        if r:
            tot[v] += e0.elapsed_time(e1)
alg = n + d.frames + d.values_size()
for v in vs:
    ms = tot[v] / (a.reps - 1)
    print(f"variant {v}: {ms:.4f} ms  {alg / ms / 1e6:.1f} GB/s alg", flush=True)
