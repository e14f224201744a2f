#!/usr/bin/env python3
"""End-to-end FL file rates (file I/O + PCIe included), for DESIGN.md.

Compares, on one synthetic input file (u8 for FL, runs32 for RL):
  whole   read file -> flrl_fl_compress (host buffers: H2D, encode, D2H,
          synchronous, the reference gpuCompress shape) -> write .fl
  stream  flrl_fl_compress_file (chunked, pipelined; workers = 1 and = GPUs)
and the same for decompression. Prints one JSON line. Not part of bench.py's
metric (that one is device-resident).
Usage: bench_stream.py [--bytes N] [--kind u8] [--dir DIR] [--reps R]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--kind", default="u8")
    ap.add_argument("--dir", default=None)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
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
