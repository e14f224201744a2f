#!/usr/bin/env python3
"""A/B two (or more) builds of libflrl.so in ONE process on the same device
buffers: each library is loaded by path with ctypes (separate code objects,
one HIP runtime), the chosen device entry point is timed with HIP events,
builds interleaved rep by rep, and every build's output is checked against the
first's. Usage (on the GPU box):

  python scripts/ab_libs.py --op fl_encode --libs scripts/ab_libs/libflrl_old.so,fl-rl-compression-mpi_amd/lib/libflrl.so

ops: fl_encode, fl_decode, rl_encode, rl_decode. Inputs: --kind u8|lo4|zero
(device generator), runs32|longruns (host generator) or uptoM (uniform runs of
1..M bytes), --bytes (default 1 GiB).
"""
import argparse
import ctypes
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-rl-compression-mpi_amd"))
import torch  # noqa: E402

import flrl  # noqa: E402
from flrl.device import FLDevice, RLDevice, gen  # noqa: E402

VP, SZ = ctypes.c_void_p, ctypes.c_size_t


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.flrl_fl_encode_device.argtypes = [VP, SZ, VP, VP, VP, VP, SZ, VP]
    lib.flrl_fl_decode_device.argtypes = [VP, SZ, VP, SZ, VP, SZ, VP, SZ, VP]
    lib.flrl_rl_encode_device.argtypes = [VP, SZ, VP, VP, VP, VP, SZ, VP]
    lib.flrl_rl_decode_device.argtypes = [VP, VP, SZ, VP, SZ, VP, SZ, VP]
    for f in ("flrl_fl_encode_device", "flrl_fl_decode_device", "flrl_rl_encode_device",
              "flrl_rl_decode_device"):
        getattr(lib, f).restype = ctypes.c_int
    return lib


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--op", default="fl_encode", choices=["fl_encode", "fl_decode", "rl_encode", "rl_decode"])
    p.add_argument("--libs", required=True)
    p.add_argument("--kind", default="")
    p.add_argument("--bytes", type=int, default=1 << 30)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--dirty", type=int, default=0,
                   help="bytes written by a fill kernel before every timed call (cache state of a real pipeline)")
    p.add_argument("--clean", type=int, default=0,
                   help="bytes read by a reduction before every timed call (evicts dirty cache lines)")
    p.add_argument("--nocheck", action="store_true",
                   help="timing-only builds: do not compare outputs with the first build's")
    a = p.parse_args()
    libs = [load(x) for x in a.libs.split(",")]
    n = a.bytes
    kind = a.kind or ("runs32" if a.op.startswith("rl") else "u8")
    if kind in ("u8", "lo4", "zero"):
        x = gen(kind, n, 42)
    elif kind in ("lo2", "lo1"):  # every FL frame of width 2 / 1 (and not all-zero)
        x = gen("u8", n, 42) & (3 if kind == "lo2" else 1)
    elif kind.startswith("upto"):  # uniform run lengths 1..M (M = the number after "upto")
        import numpy as np
        rng = np.random.default_rng(42)
        m = int(kind[4:])
        lens = rng.integers(1, m + 1, size=int(2.2 * n / (m + 1)) + 4096)
        vals = (np.cumsum(rng.integers(1, 255, size=lens.size)) % 256).astype(np.uint8)
        x = torch.from_numpy(np.repeat(vals, lens)[:n].copy()).cuda()
    else:
        x = torch.from_numpy(flrl.gen_host(kind, n, 42)).cuda()
    s = torch.cuda.current_stream().cuda_stream
    def roomy(d):
        """scratch with room for builds whose scratch layout is larger"""
        d.scratch_bytes = 2 * d.scratch_bytes + (1 << 24)
        d.scratch = torch.empty(d.scratch_bytes, dtype=torch.uint8, device="cuda")

    if a.op.startswith("fl"):
        d = FLDevice(n, "cuda")
        roomy(d)
        d.encode(x)
        V = d.values_size()

        def call(lib):
            if a.op == "fl_encode":
                return lib.flrl_fl_encode_device(x.data_ptr(), n, d.bits.data_ptr(), d.values.data_ptr(),
                                                 d.sizes.data_ptr() + 8, d.scratch.data_ptr(),
                                                 d.scratch_bytes, s)
            return lib.flrl_fl_decode_device(d.bits.data_ptr(), d.frames, d.values.data_ptr(), V,
                                             d.out.data_ptr(), n, d.scratch.data_ptr(), d.scratch_bytes, s)

        def result():
            if a.op == "fl_encode":
                return torch.cat([d.bits[: d.frames], d.values[: d.values_size()]])
            return d.out[:n].clone()
        alg = n + d.frames + V
    else:
        d = RLDevice(n, "cuda")
        roomy(d)
        d.encode(x)
        R = d.runs()

        def call(lib):
            if a.op == "rl_encode":
                return lib.flrl_rl_encode_device(x.data_ptr(), n, d.counts.data_ptr(), d.values.data_ptr(),
                                                 d.runs_t.data_ptr(), d.scratch.data_ptr(), d.scratch_bytes, s)
            return lib.flrl_rl_decode_device(d.counts.data_ptr(), d.values.data_ptr(), R, d.out.data_ptr(), n,
                                             d.scratch.data_ptr(), d.scratch_bytes, s)

        def result():
            if a.op == "rl_encode":
                r = d.runs()
                return torch.cat([d.counts[:r], d.values[:r]])
            return d.out[:n].clone()
        alg = n + 2 * R
    ref = None
    for i, lib in enumerate(libs):
        assert call(lib) == 0, flrl.last_error() if hasattr(flrl, "last_error") else "call failed"
        torch.cuda.synchronize()
        assert d.error() == 0
        r = result()
        if ref is None:
            ref = r
            if a.op.endswith("decode"):
                assert torch.equal(r, x[:n]), "round trip failed"
        elif not a.nocheck:
            assert torch.equal(ref, r), f"build {i} output differs from build 0"
    print(f"{a.op} {kind} n={n}: outputs of {len(libs)} builds identical", flush=True)
    tot = [0.0] * len(libs)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dirty = torch.empty(a.dirty, dtype=torch.uint8, device="cuda") if a.dirty else None
    clean = torch.ones(a.clean // 4, dtype=torch.int32, device="cuda") if a.clean else None
    for r in range(a.reps):
        # builds in a shuffled order per rep: the preceding call's cache state
        # moves a build's time by up to ~4 %, so no build keeps one predecessor
        order = list(range(len(libs)))
        random.Random(r).shuffle(order)
        for i in order:
            lib = libs[i]
            if dirty is not None:
                dirty.fill_(r & 0xFF)
            if clean is not None:
                torch.amax(clean)
            e0.record()
            call(lib)
            e1.record()
            e1.synchronize()
            if r:
                tot[i] += e0.elapsed_time(e1)
    for i, path in enumerate(a.libs.split(",")):
        ms = tot[i] / (a.reps - 1)
        print(f"  {os.path.basename(path):24s} {ms:.4f} ms  {alg / ms / 1e6:.1f} GB/s alg", flush=True)


if __name__ == "__main__":
    main()
