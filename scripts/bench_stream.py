#!/usr/bin/env python3
"""End-to-end FL file rates (file I/O + PCIe included), for DESIGN.md.

Compares, on one synthetic input file (u8 for FL, runs32 for RL):
  whole   read file -> flrl_fl_compress (host buffers: H2D, encode, D2H,
          synchronous, the reference gpuCompress shape) -> write .fl
  stream  flrl_fl_compress_file (chunked, pipelined; workers = 1 and = GPUs)
and the same for decompression, plus the host-buffer C API memory to memory
(flrl_fl_compress / flrl_fl_decompress through their pinned chunk pipelines,
timed around the raw C calls) next to the PCIe copy ceiling (torch copies of
the same bytes between pinned host memory and HBM). Prints one JSON line. Not
part of bench.py's metric (that one is device-resident).
Usage: bench_stream.py [--bytes N] [--kind u8] [--dir DIR] [--reps R] [--mem-only]
(the host pipelines' shape is compile-time: FLRL_HOST_* in csrc/flrl_tuning.hpp,
A/B by variant builds, scripts/build_variant.sh)
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fl-rl-compression-mpi_amd"))

import flrl  # noqa: E402


def best(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def mem_rates(n: int, kind: str, reps: int, ceiling: bool = True) -> dict:
    """flrl_fl_compress / flrl_fl_decompress memory to memory vs the PCIe ceiling."""
    import ctypes

    import numpy as np
    import torch
    kinds = {"u8": 0, "lo4": 1, "zero": 2}
    x = flrl.gen_host(kinds[kind], n, 42)
    lib = flrl._lib
    res = {"bytes": n, "kind": kind, "api": "flrl_fl_compress / flrl_fl_decompress (host buffers)"}

    def comp():
        b = flrl._FLBuf()
        flrl._check(lib.flrl_fl_compress(x.ctypes.data, n, ctypes.byref(b)))
        return b

    b = comp()
    bits = np.ctypeslib.as_array(ctypes.cast(b.bits, ctypes.POINTER(ctypes.c_uint8)), (b.bits_size,)).copy()
    vals = np.ctypeslib.as_array(ctypes.cast(b.values, ctypes.POINTER(ctypes.c_uint8)), (b.values_size,)).copy()
    flrl._libc.free(ctypes.cast(b.bits, ctypes.c_void_p).value)
    flrl._libc.free(ctypes.cast(b.values, ctypes.c_void_p).value)

    def decomp():
        o, on = flrl._u8p(), ctypes.c_size_t(0)
        flrl._check(lib.flrl_fl_decompress(n, bits.ctypes.data, bits.size, vals.ctypes.data, vals.size,
                                           ctypes.byref(o), ctypes.byref(on)))
        return o

    o = decomp()
    back = np.ctypeslib.as_array(ctypes.cast(o, ctypes.POINTER(ctypes.c_uint8)), (n,))
    res["roundtrip_ok"] = bool(np.array_equal(back, x))
    flrl._libc.free(ctypes.cast(o, ctypes.c_void_p).value)

    # The call alone (what the reference's [TIMER] brackets: main.cu times the
    # gpuCompress / gpuDecompress call, the caller frees later) and the call
    # plus the caller's free() of the outputs, best of `reps` each.
    def split(call, outs):
        tc_, tf_ = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = call()
            t1 = time.perf_counter()
            for p in outs(r):
                flrl._libc.free(ctypes.cast(p, ctypes.c_void_p).value)
            tc_.append(t1 - t0)
            tf_.append(time.perf_counter() - t0)
        return min(tc_), min(tf_)
    tc, tcf = split(comp, lambda b: (b.bits, b.values))
    td, tdf = split(decomp, lambda o: (o,))
    res["compress_GBps"] = n / tc / 1e9
    res["decompress_GBps"] = n / td / 1e9
    res["compress_moved_GBps"] = (n + bits.size + vals.size) / tc / 1e9
    res["decompress_moved_GBps"] = (n + bits.size + vals.size) / td / 1e9
    res["compress_with_free_GBps"] = n / tcf / 1e9
    res["decompress_with_free_GBps"] = n / tdf / 1e9
    def first_touch():
        y = np.empty(n, dtype=np.uint8)  # fresh pages: what a malloc'd output costs
        y.fill(1)
    res["host_first_touch_GBps"] = n / best(first_touch, reps) / 1e9
    if not ceiling:
        return {k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}
    # PCIe ceiling: one torch copy each way of n bytes, pinned and pageable host memory
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    g = torch.empty(n, dtype=torch.uint8, device="cuda")
    p = torch.from_numpy(x)

    def cp(dst, src):
        def f():
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
        return f
    res["pcie_h2d_pinned_GBps"] = n / best(cp(g, h), reps) / 1e9
    res["pcie_d2h_pinned_GBps"] = n / best(cp(h, g), reps) / 1e9
    res["pcie_h2d_pageable_GBps"] = n / best(cp(g, p), reps) / 1e9
    res["host_memcpy_1thread_GBps"] = n / best(lambda: h.copy_(p), reps) / 1e9
    # both directions at once (H2D on one stream, D2H on another; DMA copies):
    # moved bytes per second, against twice the one-way rate if they overlap
    h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    g2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def duplex():
        with torch.cuda.stream(sa):
            g.copy_(h, non_blocking=True)
        with torch.cuda.stream(sb):
            h2.copy_(g2, non_blocking=True)
        torch.cuda.synchronize()
    res["pcie_duplex_moved_GBps"] = 2 * n / best(duplex, reps) / 1e9

    return {k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--kind", default="u8")
    ap.add_argument("--dir", default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mem-only", action="store_true")
    a = ap.parse_args()
    if a.mem_only:
        print(json.dumps(mem_rates(a.bytes, a.kind, a.reps)))
        return
    kinds = {"u8": 0, "lo4": 1, "zero": 2}
    d = tempfile.mkdtemp(dir=a.dir)
    src, dst, back = (os.path.join(d, x) for x in ("in", "out.fl", "back"))
    data = flrl.gen_host(kinds[a.kind], a.bytes, 42)
    data.tofile(src)
    del data
    n = a.bytes
    res = {"bytes": n, "kind": a.kind, "devices": flrl.device_count()}

    def whole_c():
        x = open(src, "rb").read()
        c = flrl.fl_compress(x)
        with open(dst, "wb") as f:
            f.write(c.to_file_bytes())

    def whole_d():
        c = flrl.parse_fl_file(open(dst, "rb").read())
        out = flrl.fl_decompress(c.input_size, c.bits, c.values)
        out.tofile(back)

    whole_c()  # warm page cache and device
    res["whole_compress_GBps"] = n / best(whole_c, a.reps) / 1e9
    res["whole_decompress_GBps"] = n / best(whole_d, a.reps) / 1e9
    ref = open(dst, "rb").read()
    for w in sorted({1, 2, 4, max(1, flrl.device_count())}):
        res[f"stream_w{w}_compress_GBps"] = n / best(lambda: flrl.fl_compress_file(src, dst, w, 0), a.reps) / 1e9
        assert open(dst, "rb").read() == ref, "streamed file differs"
        res[f"stream_w{w}_decompress_GBps"] = n / best(lambda: flrl.fl_decompress_file(dst, back, w, 0), a.reps) / 1e9
    res["files_identical"] = True
    # RL on runs32 of the same size
    data = flrl.gen_host("runs32", n, 42)
    data.tofile(src)
    del data

    def rl_whole_c():
        x = open(src, "rb").read()
        c = flrl.rl_compress(x)
        with open(dst, "wb") as f:
            f.write(c.to_file_bytes())

    def rl_whole_d():
        c = flrl.parse_rl_file(open(dst, "rb").read())
        flrl.rl_decompress(c.input_size, c.counts, c.values).tofile(back)

    rl_whole_c()
    res["rl_whole_compress_GBps"] = n / best(rl_whole_c, a.reps) / 1e9
    res["rl_whole_decompress_GBps"] = n / best(rl_whole_d, a.reps) / 1e9
    ref = open(dst, "rb").read()
    for w in sorted({1, 2, max(1, flrl.device_count())}):
        res[f"rl_stream_w{w}_compress_GBps"] = n / best(lambda: flrl.rl_compress_file(src, dst, w, 0), a.reps) / 1e9
        assert open(dst, "rb").read() == ref, "streamed RL file differs"
        res[f"rl_stream_w{w}_decompress_GBps"] = n / best(lambda: flrl.rl_decompress_file(dst, back, w, 0), a.reps) / 1e9
    res["rl_files_identical"] = True
    for p in (src, dst, back):
        os.remove(p)
    os.rmdir(d)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
