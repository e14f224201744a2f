#!/usr/bin/env python3
"""bench.py — FL encode+decode throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: FL encode of this rank's
shard (per-frame width scan -> look-back offset scan -> bit-pack, one kernel),
the multi-GPU size-scan (RCCL all-gather of {F_r, V_r} + exclusive scan; only
when N > 1), and FL decode of the shard back to bytes. Inputs are resident in
HBM before timing (device-generated, SURVEY.md §8(d) splitmix64 u8, seed 42,
rank r holding global bytes [r*B, (r+1)*B) of one N*B-byte buffer), so `value`
is whole-job input bytes / second through encode+decode, weak scaling.

Default workload = BASELINE.json configs[1]: FL encode/decode of 1 GiB of
uniform-random bytes per GPU, bit-exact against the reference fl-cpu (the
1 GiB output's sha256 is the reference's).

Every N-rank line (N > 1; at N = 1 with --force-scan) also carries `configs4`:
BASELINE configs[4], FL encode of 16 GiB uniform-random bytes per GPU through
flrl_fl_encode_rank (encode + the RCCL size exchange), 128 GiB at N = 8
(--configs4-bytes sets the per-GPU size). At N = 1 the same bytes without the
exchange are the `north_star` section.

Launch: python bench.py [--gpus N --steps K --warmup W]. For N > 1 the ranks
are started by this script (torch.distributed.run child, one rank per GPU)
unless it already runs under torch.distributed.run. The data-path exchange is
an RCCL communicator of the C ABI (flrl_comm_init_rank, xGMI); torch.distributed
(gloo) carries only the unique id, the barriers and the max-over-ranks timing.
"""
from __future__ import annotations

import argparse
import hashlib
import struct
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fl-rl-compression-mpi_amd"))


def _gpus_arg(argv) -> int:
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--gpus", type=int, default=1)
    return p.parse_known_args(argv)[0].gpus


def rank_launch_cmd(argv, env) -> list | None:
    """`python bench.py --gpus N` (N > 1) outside torch.distributed: the command
    that starts the N ranks (torch.distributed.run, one process per GPU,
    127.0.0.1 rendezvous on a free port), run as a child process by this
    process BEFORE anything touches the GPU (never an exec). None when this
    process is itself a rank (WORLD_SIZE set) or N == 1."""
    n = _gpus_arg(argv)
    if n <= 1 or "WORLD_SIZE" in env:
        return None
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


if __name__ == "__main__":
    _cmd = rank_launch_cmd(sys.argv[1:], os.environ)
    if _cmd is not None:
        sys.exit(subprocess.call(_cmd))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import flrl  # noqa: E402
from flrl.device import FLDevice, RLDevice, gen  # noqa: E402

METRIC = ("encode+decode GB/s (input bytes) at 1/2/4/8 GPUs; % HBM roofline; "
          "bit-exact round-trip")
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GOLDEN_1GIB_U8_SHA = "0512b67cd1f3940885e5c3043c4541c5d8105403eb1273be20cd3c87d5ecef78"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--bytes", type=int, default=1 << 30, help="input bytes per GPU (weak scaling, the default)")
    p.add_argument("--global-bytes", type=int, default=0,
                   help="strong scaling: a FIXED total split over the N ranks by the reference shard rule "
                        "(file_io.cu:46-51, flrl_shard_range: every shard but the last floor(B/(128N))*128 "
                        "bytes); the line reports scaling 'strong' and value = B / step time")
    p.add_argument("--kind", default="u8", choices=["u8", "lo4", "zero"])
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--cpu-sample", type=int, default=-1,
                   help="bytes of the workload the CPU oracle times (default: min(bytes, 1 GiB)); 0 = skip")
    p.add_argument("--traffic-json", default=None,
                   help="PMC summary (scripts/summarize_profile.py); default profiles/traffic_<kind>_<bytes>.json")
    p.add_argument("--no-north-star", action="store_true",
                   help="skip the 16 GiB u8 FL encode of the north star (N=1)")
    p.add_argument("--no-configs4", action="store_true",
                   help="skip the configs[4] section (16 GiB per GPU through flrl_fl_encode_rank)")
    p.add_argument("--configs4-bytes", type=int, default=16 << 30,
                   help="bytes per GPU of the configs[4] section (runs at N>1, and at N=1 with --force-scan)")
    p.add_argument("--no-configs3", action="store_true",
                   help="skip the configs[3] section (16 GiB and 1 GiB lo4 FL encode + decode, N=1)")
    p.add_argument("--no-rl-dense", action="store_true",
                   help="skip the random-bytes RL section (profiles average kernels per name)")
    p.add_argument("--no-rl", action="store_true",
                   help="skip the RL section (config #3: 1 GiB runs32), which runs at N=1 only")
    p.add_argument("--force-scan", action="store_true",
                   help="run the RCCL size exchange (flrl_fl_encode_rank, 1-rank comm) even at N = 1")
    return p.parse_args()


def file_sha(n, frames, bits: np.ndarray, values: np.ndarray) -> str:
    h = hashlib.sha256()
    h.update(np.array([n, frames, values.size], dtype="<u8").tobytes())
    h.update(bits.tobytes())
    h.update(values.tobytes())
    return h.hexdigest()


def host_info() -> dict:
    """The GPU box's host CPU (report nproc and the CPU model;
    the baselines use one core, like the reference fl-cpu)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "cpu_model": model}


def cpu_baseline(kind: str, seed: int, sample: int, gpu_bits, gpu_values):
    """Time the oracle (1 core, the reference fl-cpu's algorithm and loops) on
    the first `sample` bytes of the same workload; also compare its output with
    the GPU's for those bytes (128-aligned prefix => identical slices)."""
    import oracle
    a = oracle.gen(kind, sample, seed)
    t0 = time.perf_counter()
    bits, values = oracle.fl_compress(a)
    t1 = time.perf_counter()
    back = oracle.fl_decompress(sample, bits, values)
    t2 = time.perf_counter()
    ok = bool(np.array_equal(back, a))
    same = None
    if gpu_bits is not None and sample % 128 == 0:
        same = bool(np.array_equal(gpu_bits[: bits.size], bits)
                    and np.array_equal(gpu_values[: values.size], values))
    return {
        "value": round(sample / (t2 - t0) / 1e9, 4),
        "unit": "GB/s",
        "cores": 1,
        "host": host_info(),
        "kind": "port",
        "sample": f"{sample} bytes ({kind}, seed {seed}) = the first {sample} bytes of rank 0's "
                  f"workload; oracle/flrl_oracle.c encode {t1 - t0:.2f} s + decode {t2 - t1:.2f} s, "
                  f"single-threaded like the reference fl-cpu",
        "encode_s": round(t1 - t0, 3),
        "decode_s": round(t2 - t1, 3),
        "roundtrip_ok": ok,
        "gpu_bytes_equal_oracle": same,
    }


def rl_cpu_baseline(n: int, seed: int) -> dict:
    """The RL oracle (1 core) on n bytes of runs32 (BASELINE configs[2]'s
    input, the product generator): the rl-cpu figure for lines where the
    GPU RL section does not run (N > 1)."""
    import oracle
    a = flrl.gen_host("runs32", n, seed)
    t0 = time.perf_counter()
    counts, values = oracle.rl_compress(a)
    t1 = time.perf_counter()
    back = oracle.rl_decompress(counts, values, n)
    t2 = time.perf_counter()
    return {"value": round(n / (t2 - t0) / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"{n} bytes runs32 (seed {seed}); oracle rl encode {t1 - t0:.2f} s + decode {t2 - t1:.2f} s, "
                      f"single-threaded",
            "runs": int(counts.size), "roundtrip_ok": bool(np.array_equal(back, a))}


def line_cpu_baseline(rank: int, world: int, kind: str, seed: int, sample: int, gpu_bits=None, gpu_values=None):
    """The line's `cpu_baseline` (rank 0 only, any N; None when sample == 0):
    the FL oracle on the first `sample` bytes of rank 0's shard, and at N > 1
    the RL oracle as `rl` (at N = 1 the RL section carries its own)."""
    if rank != 0 or sample <= 0:
        return None
    cpu = cpu_baseline(kind, seed, sample, gpu_bits, gpu_values)
    if world > 1:
        cpu["rl"] = rl_cpu_baseline(sample, seed)
    return cpu


def rank_shard(per_gpu: int, global_bytes: int, world: int, rank: int) -> tuple[int, int, int]:
    """(start, length, job total) of rank's input bytes. Weak scaling (the
    default): `per_gpu` bytes per rank, rank r at r * per_gpu. Strong scaling
    (global_bytes > 0; on_cluster.sh:18-34 splits fixed 512/2048/3124 MB files
    over the mpirun ranks): the fixed total split by the reference shard rule
    (file_io.cu:46-51 via flrl_shard_range), every shard but the last
    floor(B / (128 N)) * 128 bytes, so only the last may be ragged."""
    if global_bytes > 0:
        if global_bytes < 128 * world:
            raise SystemExit("--global-bytes must give every rank at least one frame")
        start, n = flrl.shard_range(global_bytes, world, rank)
        return start, n, global_bytes
    if per_gpu % 128:
        raise SystemExit("--bytes must be a multiple of 128 (frame-aligned shards for weak scaling)")
    return rank * per_gpu, per_gpu, world * per_gpu


def workload_ref(n: int, kind: str, world: int) -> str:
    """Which BASELINE.json config (or north-star target) this FL workload is."""
    if kind == "u8" and n == 1 << 30:
        return "BASELINE configs[1]" + (f", weak-scaled x{world}" if world > 1 else "")
    if kind == "lo4" and n == 16 << 30 and world == 1:
        return "BASELINE configs[3]"
    if kind == "u8" and n == 16 << 30:
        return ("north-star target: 16 GiB uniform-random at 1 GPU" if world == 1
                else f"BASELINE configs[4]: 16 GiB per GPU x{world}")
    return "custom size"


def pmc_traffic(kind: str, n: int, kernel: str, path: str | None = None):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this
    exact workload (scripts/profile.sh + summarize_profile.py), else None."""
    path = path or os.path.join(ROOT, "profiles", f"traffic_{kind}_{n}.json")
    try:
        with open(path) as f:
            tj = json.load(f)
        if tj.get("bytes") == n and tj.get("kind") == kind:
            return tj["kernels"].get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError, KeyError, AttributeError):
        pass
    return None


def created_events(rows: int, cols: int, stream) -> list:
    """rows x cols timing events, each recorded once so its HIP event exists
    (flrl.time_next_kernel takes the raw handle)."""
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(cols)] for _ in range(rows)]
    for row in ev:
        for e in row:
            e.record(stream)
    return ev


def mean_ms(ev, a: int, b: int) -> float:
    return float(np.mean([e[a].elapsed_time(e[b]) for e in ev]))


def median_ms(ev, a: int, b: int) -> float:
    return float(np.median([e[a].elapsed_time(e[b]) for e in ev]))


def north_star_section(seed: int, steps: int, warmup: int, dev):
    """BASELINE north star: FL encode of 16 GiB uniform-random bytes on 1 GPU,
    target >= 70 % of HBM peak on algorithmic bytes. Encode and
    decode timed with HIP events; parity: device round trip, and the first
    1 GiB of the output (frame-aligned, so byte-identical to a 1 GiB encode,
    SURVEY.md fact 7) hashes to the reference fl-cpu's 1 GiB file."""
    n = 16 << 30
    x = gen("u8", n, seed, word_offset=0, device=dev)
    codec = FLDevice(n, dev)
    stream = torch.cuda.current_stream()
    for _ in range(max(1, warmup)):
        codec.encode(x)
    v = codec.values_size()
    ev = created_events(steps, 4, stream)  # call start/end, kernel start/end (separate passes)
    torch.cuda.synchronize()
    for k in range(steps):
        ev[k][0].record(stream)
        codec.encode(x)
        ev[k][1].record(stream)
    for k in range(steps):
        flrl.time_next_kernel(ev[k][2], ev[k][3])
        codec.encode(x)
    torch.cuda.synchronize()
    err = codec.error()
    enc_call_ms = mean_ms(ev, 0, 1)
    enc_ms = mean_ms(ev, 2, 3)
    f1 = (1 << 30) // 128
    v1 = int(codec.bits[:f1].to(torch.int64).sum().item()) * 16
    h = hashlib.sha256(struct.pack("<QQQ", 1 << 30, f1, v1))
    h.update(codec.bits[:f1].cpu().numpy().tobytes())
    h.update(codec.values[:v1].cpu().numpy().tobytes())
    prefix_ok = seed == 42 and h.hexdigest() == GOLDEN_1GIB_U8_SHA
    out = torch.empty_like(x)
    (d0, d1, k0, k1), = created_events(1, 4, stream)
    codec.decode(v, out=out)
    d0.record(stream)
    codec.decode(v, out=out)
    d1.record(stream)
    flrl.time_next_kernel(k0, k1)
    codec.decode(v, out=out)
    torch.cuda.synchronize()
    dec_call_ms = d0.elapsed_time(d1)
    dec_ms = k0.elapsed_time(k1)
    ok = bool(torch.equal(out, x)) and err == 0 and codec.error() == 0
    alg = n + codec.frames + v
    res = {
        "workload": f"FL encode of {n} u8 bytes (seed {seed}) on 1 GPU (BASELINE north star)",
        "timing": "kernel time (HIP events around the kernel, flrl_time_next_kernel); call = + scratch "
                  "zero-fill (decode: + the offsets pre-pass, skipped when valuesSize == n), timed in its own pass without the kernel events",
        "encode_ms": round(enc_ms, 4),
        "encode_median_ms": round(median_ms(ev, 2, 3), 4),
        "encode_call_ms": round(enc_call_ms, 4),
        "encode_alg_GBps": round(alg / (enc_ms * 1e-3) / 1e9, 1),
        "encode_input_GBps": round(n / (enc_ms * 1e-3) / 1e9, 1),
        "frac": round(alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "target_frac": 0.70,
        "algorithmic_bytes_per_launch": alg,
        "traffic": pmc_traffic("u8", n, "fl_encode"),
        "decode_ms": round(dec_ms, 4),
        "decode_call_ms": round(dec_call_ms, 4),
        "decode_alg_GBps": round(alg / (dec_ms * 1e-3) / 1e9, 1),
        "roundtrip": ok,
        "prefix_1GiB_matches_reference_fl_cpu": prefix_ok,
    }
    del x, out, codec
    torch.cuda.empty_cache()
    return res


def fl_kind_timed(kind: str, n: int, seed: int, steps: int, warmup: int, dev) -> dict:
    """FL encode and decode of n device-generated `kind` bytes on 1 GPU: the
    kernels alone (HIP events by flrl_time_next_kernel) and the whole calls
    (+ scratch zero-fill; decode + the offsets pre-pass, which runs unless
    valuesSize == n) in separate passes, means over `steps`; frac on the
    algorithmic bytes N + F + V; device round trip."""
    x = gen(kind, n, seed, word_offset=0, device=dev)
    codec = FLDevice(n, dev)
    stream = torch.cuda.current_stream()
    for _ in range(max(1, warmup)):
        codec.encode(x)
    v = codec.values_size()
    out = torch.empty_like(x)
    for _ in range(max(1, warmup)):
        codec.decode(v, out=out)
    ev = created_events(steps, 8, stream)
    torch.cuda.synchronize()
    for k in range(steps):
        ev[k][0].record(stream)
        codec.encode(x)
        ev[k][1].record(stream)
        codec.decode(v, out=out)
        ev[k][2].record(stream)
    for k in range(steps):
        flrl.time_next_kernel(ev[k][4], ev[k][5])
        codec.encode(x)
        flrl.time_next_kernel(ev[k][6], ev[k][7])
        codec.decode(v, out=out)
    torch.cuda.synchronize()
    ok = bool(torch.equal(out, x)) and codec.error() == 0
    alg = n + codec.frames + v
    enc_ms, dec_ms = mean_ms(ev, 4, 5), mean_ms(ev, 6, 7)
    enc_call, dec_call = mean_ms(ev, 0, 1), mean_ms(ev, 1, 2)

    def gbs(ms):
        return alg / (ms * 1e-3) / 1e9
    res = {
        "bytes": n, "kind": kind, "values_size": v, "algorithmic_bytes_per_launch": alg,
        "fl_encode": {"ms": round(enc_ms, 4), "call_ms": round(enc_call, 4), "alg_GBps": round(gbs(enc_ms), 1),
                      "frac": round(gbs(enc_ms) / HBM_PEAK_GBS, 4),
                      "traffic": pmc_traffic(kind, n, "fl_encode")},
        "fl_decode": {"ms": round(dec_ms, 4), "call_ms": round(dec_call, 4), "alg_GBps": round(gbs(dec_ms), 1),
                      "frac": round(gbs(dec_ms) / HBM_PEAK_GBS, 4),
                      "call_frac": round(gbs(dec_call) / HBM_PEAK_GBS, 4),
                      "traffic": pmc_traffic(kind, n, "fl_decode")},
        "roundtrip": ok,
    }
    del x, out, codec
    torch.cuda.empty_cache()
    return res


def configs3_section(seed: int, steps: int, warmup: int, dev) -> dict:
    """BASELINE configs[3]: FL encode of 16 GiB low-entropy bytes (values
    0-15: every frame at width 4, V = N/2) on 1 GPU against the HBM roofline,
    with the decode of the same data (the general decode: offsets pre-pass +
    LDS unpack, which the u8 headline never takes since valuesSize == n there),
    and the same at 1 GiB. `traffic` = PMC HBM bytes per launch from
    profiles/traffic_lo4_<bytes>.json when that summary exists."""
    return {
        "workload": "BASELINE configs[3]: FL encode (+ decode) of 17179869184 lo4 bytes (values 0-15, "
                    f"splitmix64 seed {seed}) on 1 GPU; also 1 GiB",
        "timing": "means over K launches; ms = the kernel alone (HIP events by flrl_time_next_kernel), "
                  "call_ms = the whole device call in a separate pass (decode: + the offsets pre-pass)",
        "16GiB": fl_kind_timed("lo4", 16 << 30, seed, steps, warmup, dev),
        "1GiB": fl_kind_timed("lo4", 1 << 30, seed, steps, warmup, dev),
    }


def _rl_timed(x, n: int, steps: int, warmup: int, dev):
    """RL encode + decode of x (n bytes in HBM): R, the round trip, and the
    MEDIAN whole-call / kernel-alone times of both over `steps` encode/decode
    pairs after `warmup` untimed pairs (HIP events; one measurement, so the
    line carries one RL encode figure: VERDICT r03 weak item 3)."""
    d = RLDevice(n, dev)
    stream = torch.cuda.current_stream()
    d.encode(x)
    R = d.runs()
    out = d.decode(R)
    ok = bool(torch.equal(out, x)) and d.error() == 0
    for _ in range(warmup):
        d.encode(x)
        d.decode(R)
    # calls: events 0-1-2 (one pass); kernels alone: 3-4 encode, 5-6 decode (a
    # second pass, so the call times hold no kernel-event records)
    ev = created_events(steps, 7, stream)
    torch.cuda.synchronize()
    for k in range(steps):
        ev[k][0].record(stream)
        d.encode(x)
        ev[k][1].record(stream)
        d.decode(R)
        ev[k][2].record(stream)
    for k in range(steps):
        flrl.time_next_kernel(ev[k][3], ev[k][4])
        d.encode(x)
        flrl.time_next_kernel(ev[k][5], ev[k][6])
        d.decode(R)
    torch.cuda.synchronize()
    if d.error():
        raise SystemExit(f"RL device error {d.error()} during the timed steps")
    t = (median_ms(ev, 0, 1), median_ms(ev, 1, 2), median_ms(ev, 3, 4), median_ms(ev, 5, 6))
    means = (mean_ms(ev, 3, 4), mean_ms(ev, 5, 6))
    return d, R, ok, t, means


def rl_dense_section(n: int, seed: int, steps: int, warmup: int, dev):
    """RL of n uniform-random bytes (mean run 1.004: the densest input; decode
    takes the wave-tile kernel): kernel and call times, device round trip."""
    from flrl.device import gen
    x = gen("u8", n, seed)
    d, R, ok, (enc_ms, dec_ms, enc_k, dec_k), _ = _rl_timed(x, n, steps, warmup, dev)
    alg = n + 2 * R
    res = {"workload": f"RL encode+decode of {n} uniform-random bytes (u8, seed {seed})", "runs": R,
           "rl_encode": {"ms": round(enc_k, 4), "call_ms": round(enc_ms, 4),
                         "alg_GBps": round(alg / (enc_k * 1e-3) / 1e9, 1)},
           "rl_decode": {"ms": round(dec_k, 4), "call_ms": round(dec_ms, 4),
                         "alg_GBps": round(alg / (dec_k * 1e-3) / 1e9, 1),
                         "call_alg_GBps": round(alg / (dec_ms * 1e-3) / 1e9, 1)},
           "roundtrip": ok}
    del x, d
    torch.cuda.empty_cache()
    return res


def rl_section(n: int, seed: int, steps: int, warmup: int, dev, cpu: bool):
    """BASELINE configs[2]: RL encode/decode of n bytes of runs32 (mean run 32).
    Input generated on the host by the product generator (runs32 is
    sequential), copied to HBM before timing."""
    x = torch.from_numpy(flrl.gen_host("runs32", n, seed)).to(dev)
    d, R, ok, (enc_ms, dec_ms, enc_k, dec_k), (enc_mean, dec_mean) = _rl_timed(x, n, steps, warmup, dev)
    out = d.out[:n]
    alg = n + 2 * R  # RL encode N+2R, decode 2R+N
    res = {
        "workload": f"RL encode+decode of {n} bytes runs32 (seed {seed}), BASELINE configs[2]",
        "runs": R,
        "value": round(n / ((enc_ms + dec_ms) * 1e-3) / 1e9, 2),
        "unit": "GB/s (input bytes, encode+decode)",
        "timing": f"median over {steps} encode/decode pairs after {warmup} warm-up pairs (HIP events); "
                  "mean_ms = the mean of the same samples; call_ms from a separate pass of {steps} pairs "
                  "without the kernel events".replace("{steps}", str(steps)),
        "rl_encode": {"ms": round(enc_k, 4), "mean_ms": round(enc_mean, 4), "call_ms": round(enc_ms, 4),
                      "alg_GBps": round(alg / (enc_k * 1e-3) / 1e9, 1),
                      "frac": round(alg / (enc_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "rl_decode": {"ms": round(dec_k, 4), "mean_ms": round(dec_mean, 4), "call_ms": round(dec_ms, 4),
                      "alg_GBps": round(alg / (dec_k * 1e-3) / 1e9, 1),
                      "frac": round(alg / (dec_k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                      "call_frac": round(alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
        "roundtrip": ok,
    }
    if cpu:
        import oracle
        a = x.cpu().numpy()
        t0 = time.perf_counter()
        counts, values = oracle.rl_compress(a)
        t1 = time.perf_counter()
        back = oracle.rl_decompress(counts, values, n)
        t2 = time.perf_counter()
        same = bool(counts.size == R and np.array_equal(d.counts[:R].cpu().numpy(), counts)
                    and np.array_equal(d.values[:R].cpu().numpy(), values))
        res["cpu_baseline"] = {
            "value": round(n / (t2 - t0) / 1e9, 4), "unit": "GB/s", "cores": 1, "host": host_info(),
            "kind": "port",
            "sample": f"the full {n}-byte runs32 input; oracle rl encode {t1 - t0:.2f} s + "
                      f"decode {t2 - t1:.2f} s, single-threaded",
            "roundtrip_ok": bool(np.array_equal(back, a)), "gpu_bytes_equal_oracle": same,
        }
    del x, d, out
    torch.cuda.empty_cache()
    return res


def _barrier(world: int):
    if world > 1:
        dist.barrier()


def _all_gather_obj(obj, world: int) -> list:
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def configs4_section(comm, rank: int, world: int, seed: int, steps: int, warmup: int, dev,
                     n: int = 16 << 30, rccl: dict | None = None):
    """BASELINE configs[4]: FL encode of 16 GiB uniform-random bytes per GPU
    (128 GiB at N = 8), rank r holding global bytes [r*n, (r+1)*n), through
    flrl_fl_encode_rank (encode + the RCCL all-gather of {F_r, V_r} + device
    scan). K uninstrumented steps between barriers, max over ranks; then K
    steps with HIP events around each rank's encode kernel. Parity: every
    rank's device round trip, every rank's exchange record against the ranks'
    sizes (recomputed by the shipped layout code, flrl_shard_scan), and rank
    0's first 1 GiB against the reference fl-cpu hash. At N = 1 (with
    --force-scan) the same path runs on a one-rank communicator."""
    x = gen("u8", n, seed, word_offset=rank * n // 8, device=dev)
    codec = FLDevice(n, dev)
    stream = torch.cuda.current_stream()
    for _ in range(max(1, warmup)):
        codec.encode_rank(comm, x)
    torch.cuda.synchronize()
    rec = [int(t) for t in codec.rank_sizes[:flrl.SZ_COUNT].cpu()]
    err = codec.error()
    _barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        codec.encode_rank(comm, x)
    torch.cuda.synchronize()
    _barrier(world)
    wall = time.perf_counter() - t0
    ev = created_events(steps, 2, stream)
    torch.cuda.synchronize()
    for k in range(steps):
        flrl.time_next_kernel(ev[k][0], ev[k][1])
        codec.encode_rank(comm, x)
    torch.cuda.synchronize()
    enc_ms = mean_ms(ev, 0, 1)
    v = rec[flrl.SZ_V]
    prefix_ok = None
    if rank == 0 and n >= 1 << 30:
        f1 = (1 << 30) // 128
        v1 = int(codec.bits[:f1].to(torch.int64).sum().item()) * 16
        h = hashlib.sha256(struct.pack("<QQQ", 1 << 30, f1, v1))
        h.update(codec.bits[:f1].cpu().numpy().tobytes())
        h.update(codec.values[:v1].cpu().numpy().tobytes())
        prefix_ok = seed == 42 and h.hexdigest() == GOLDEN_1GIB_U8_SHA
    out = torch.empty_like(x)
    codec.decode(v, out=out)
    ok = bool(torch.equal(out, x)) and err == 0 and codec.error() == 0
    del out
    alg = n + codec.frames + v
    mine = {"rank": rank, "wall": wall, "encode_ms": enc_ms, "F": rec[flrl.SZ_F], "V": v,
            "F_off": rec[flrl.SZ_F_OFF], "V_off": rec[flrl.SZ_V_OFF],
            "F_total": rec[flrl.SZ_F_TOTAL], "V_total": rec[flrl.SZ_V_TOTAL],
            "frac": alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "roundtrip": ok}
    allr = _all_gather_obj(mine, world)
    del x, codec
    torch.cuda.empty_cache()
    if rank != 0:
        return None
    Fs = [r["F"] for r in allr]
    Vs = [r["V"] for r in allr]
    gathered = np.zeros(2 * world, dtype=np.uint64)  # the exchange's slots, as RCCL filled them
    for i in range(world):
        s0 = flrl.shard_slot(i, world, world)
        gathered[s0], gathered[s0 + 1] = flrl.shard_size_word(n), Vs[i]
    scan_ok = all(r["F_off"] == sum(Fs[:i]) and r["V_off"] == sum(Vs[:i]) and r["F_total"] == sum(Fs)
                  and r["V_total"] == sum(Vs) and r["F"] == n // 128
                  and flrl.shard_scan(gathered, world, world, i) == [
                      r["F"], r["V"], r["F_off"], r["V_off"], r["F_total"], r["V_total"]]
                  for i, r in enumerate(allr))
    wall = max(r["wall"] for r in allr)
    return {
        "workload": f"{'BASELINE configs[4]' if n == 16 << 30 else 'configs[4] path, custom size'}: FL encode "
                    f"of {n} u8 bytes per GPU x{world} = {n * world} bytes (seed {seed}), flrl_fl_encode_rank "
                    f"(encode + RCCL size exchange)",
        "ranks_seen": rccl["comm_count"] if rccl else world,
        "rccl": rccl,
        "value": round(world * n / (wall / steps) / 1e9, 2),
        "unit": "GB/s (input bytes, whole job)",
        "ms_per_step": round(wall * 1e3 / steps, 4),
        "per_rank_encode_ms": [round(r["encode_ms"], 4) for r in allr],
        "per_rank_frac": [round(r["frac"], 4) for r in allr],
        "min_frac": round(min(r["frac"] for r in allr), 4),
        "size_scan_ok": scan_ok,
        "roundtrip": all(r["roundtrip"] for r in allr),
        "prefix_1GiB_matches_reference_fl_cpu": prefix_ok,
        "F_total": allr[0]["F_total"], "V_total": allr[0]["V_total"],
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    scan = world > 1 or args.force_scan
    comm = None
    if world > 1:
        # control plane only (unique id, barriers, max over ranks); the data
        # path's exchange is the C ABI's own RCCL communicator
        dist.init_process_group("gloo")
        uid = [flrl.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = flrl.Comm.rank(world, uid[0], rank)
    elif scan:
        comm = flrl.Comm.rank(1, flrl.comm_unique_id(), 0)
    # what RCCL itself saw: its rank count, and each rank's device + PCI bus id
    rccl = None
    if comm is not None:
        info = _all_gather_obj(comm.rccl_info(), world)
        rccl = {"comm_count": info[0]["count"],
                "counts_agree": all(i["count"] == info[0]["count"] for i in info),
                "user_ranks": [i["rank"] for i in info],
                "devices": [i["device"] for i in info],
                "pci_bus_ids": [i["pci_bus_id"] for i in info],
                "distinct_gpus": len({i["pci_bus_id"] for i in info})}
    ranks_seen = rccl["comm_count"] if rccl else world

    def barrier():
        if world > 1:
            dist.barrier()

    strong = args.global_bytes > 0
    start, n, total = rank_shard(args.bytes, args.global_bytes, world, rank)

    x = gen(args.kind, n, args.seed, word_offset=start // 8, device=dev)
    codec = FLDevice(n, dev)
    out = torch.empty_like(x)
    stream = torch.cuda.current_stream()

    def encode():
        if scan:
            codec.encode_rank(comm, x)
        else:
            codec.encode(x)

    # ---- correctness of this exact workload (outside the timed region) ----
    encode()
    torch.cuda.synchronize()
    v = int(codec.rank_sizes[flrl.SZ_V].item()) if scan else codec.values_size()
    err = codec.error()
    codec.decode(v, out=out)
    err |= codec.error()
    roundtrip = bool(torch.equal(out[:n], x[:n])) and err == 0
    parity = {"roundtrip": roundtrip, "device_error": err}
    gpu_bits = gpu_values = None
    if rank == 0:  # (N > 1: rank 0's shard, for the CPU baseline's comparison)
        gpu_bits = codec.bits[: codec.frames].cpu().numpy()
        gpu_values = codec.values[:v].cpu().numpy()
    if rank == 0 and world == 1:
        sha = file_sha(n, codec.frames, gpu_bits, gpu_values)
        parity["fl_sha256"] = sha
        if args.kind == "u8" and args.seed == 42 and n == 1 << 30:
            parity["fl_sha256_matches_reference_fl_cpu"] = sha == GOLDEN_1GIB_U8_SHA
    if scan:  # the exchange record, checked against every rank's sizes
        rec = [int(t) for t in codec.rank_sizes[:flrl.SZ_COUNT].cpu()]
        allv = [None] * world
        if world > 1:
            dist.all_gather_object(allv, (rec[flrl.SZ_F], rec[flrl.SZ_V]))
        else:
            allv = [(rec[flrl.SZ_F], rec[flrl.SZ_V])]
        parity["size_scan_ok"] = bool(
            rec[flrl.SZ_F] == codec.frames and rec[flrl.SZ_V] == v
            and rec[flrl.SZ_F_OFF] == sum(a[0] for a in allv[:rank])
            and rec[flrl.SZ_V_OFF] == sum(a[1] for a in allv[:rank])
            and rec[flrl.SZ_F_TOTAL] == sum(a[0] for a in allv)
            and rec[flrl.SZ_V_TOTAL] == sum(a[1] for a in allv))

    # One step: encode (+ the exchange when scan: flrl_fl_encode_rank runs the
    # RCCL all-gather of {F_r, V_r} and the scan on the same stream), decode.
    # Instrumented forms for the per-kernel breakdown: calls=True brackets the
    # two device calls with events 0-1 / 2-3; calls=False brackets the two
    # kernels alone with events 4-5 / 6-7 (flrl_time_next_kernel). Separate
    # passes, so no call time holds the ~4.6 us of the kernel events' records.
    def step(e=None, calls=True):
        if e is not None:
            if calls:
                e[0].record(stream)
            else:
                flrl.time_next_kernel(e[4], e[5])
        encode()
        if e is not None and calls:
            e[1].record(stream)
            e[2].record(stream)
        if e is not None and not calls:
            flrl.time_next_kernel(e[6], e[7])
        codec.decode(v, out=out)
        if e is not None and calls:
            e[3].record(stream)

    # ---- warmup ----
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- practical HBM ceiling on these buffers: a plain device copy (read N + write N)
    cp = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    for i in range(3):
        cp[2 * i].record(stream)
        out[:n].copy_(x[:n])
        cp[2 * i + 1].record(stream)
    torch.cuda.synchronize()
    copy_ms = min(cp[2 * i].elapsed_time(cp[2 * i + 1]) for i in range(3))
    copy_gbs = 2 * n / (copy_ms * 1e-3) / 1e9

    # ---- timed region: K uninstrumented steps (a timing event costs ~4.6 us of GPU
    # timeline, scripts/event_cost.py: 8 per step would add ~5 %) ----
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    # ---- per-kernel breakdown: K more steps with HIP events (not part of `value`) ----
    # 0-3: step phases (encode call incl. exchange, -, decode call); 4-7: encode / decode kernels alone
    ev = created_events(args.steps, 8, stream)
    torch.cuda.synchronize()
    for k in range(args.steps):
        step(ev[k], calls=True)
    for k in range(args.steps):
        step(ev[k], calls=False)
    torch.cuda.synchronize()
    enc_call_ms = mean_ms(ev, 0, 1)  # + scratch zero-fill (+ the exchange when scan)
    dec_call_ms = mean_ms(ev, 2, 3)  # + zero-fill, offsets pre-pass (none when valuesSize == n)
    enc_ms, dec_ms = mean_ms(ev, 4, 5), mean_ms(ev, 6, 7)  # the kernels alone
    if codec.error():
        raise SystemExit(f"device error {codec.error()} during the timed steps")

    ms_per_step = wall * 1e3 / args.steps
    value = total / (wall / args.steps) / 1e9

    # algorithmic bytes per launch: encode N+F+V, decode F+V+N
    alg = n + codec.frames + v
    enc_gbs = alg / (enc_ms * 1e-3) / 1e9
    dec_gbs = alg / (dec_ms * 1e-3) / 1e9
    dominant = "fl_encode" if enc_ms >= dec_ms else "fl_decode"
    achieved = enc_gbs if dominant == "fl_encode" else dec_gbs
    traffic = pmc_traffic(args.kind, n, dominant, args.traffic_json)

    if world > 1:
        for key in ("roundtrip", "size_scan_ok"):
            ok = torch.tensor([1 if parity[key] else 0])
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            parity[key] = bool(ok.item())
    del x, out, codec
    torch.cuda.empty_cache()

    c4 = None
    if scan and not args.no_configs4:
        if args.configs4_bytes <= 0 or args.configs4_bytes % 128:
            raise SystemExit("--configs4-bytes must be a positive multiple of 128")
        c4 = configs4_section(comm, rank, world, args.seed, args.steps, args.warmup, dev,
                              n=args.configs4_bytes, rccl=rccl)

    if rank == 0:
        # The CPU baseline runs on rank 0 at every N (north_star: "next to the
        # reference fl-cpu/rl-cpu ... in the same run"), after the timed region,
        # on the first min(n, 1 GiB) bytes of rank 0's shard (the shard starts
        # at byte 0 in both scaling modes, so the oracle's generator gives the
        # same bytes); at N > 1 it also times the RL oracle on runs32.
        sample = min(n, 1 << 30) if args.cpu_sample < 0 else args.cpu_sample
        cpu = line_cpu_baseline(rank, world, args.kind, args.seed, sample, gpu_bits, gpu_values)
        del gpu_bits, gpu_values
        ns = None
        if world == 1 and not args.no_north_star and not (n == 16 << 30 and args.kind == "u8"):
            ns = north_star_section(args.seed, args.steps, args.warmup, dev)
        rl = None
        if world == 1 and not args.no_rl:
            rl = rl_section(n, args.seed, args.steps, args.warmup, dev, cpu=sample > 0)
            if not args.no_rl_dense:
                rl["dense_u8"] = rl_dense_section(n, args.seed, args.steps, args.warmup, dev)
        # configs[3] last (16 + 1 GiB of lo4 buffers, released before it returns),
        # so the sections above run with the same memory as without it
        c3 = None
        if world == 1 and not args.no_configs3:
            c3 = configs3_section(args.seed, args.steps, args.warmup, dev)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic ({args.kind} splitmix64 seed {args.seed}, SURVEY.md §8(d), generated in HBM)",
            "config": {
                "workload": (f"FL encode+decode of {total} {args.kind} bytes in total, split over {world} GPU(s) "
                             f"by the reference shard rule (strong scaling)" if strong else
                             f"FL encode+decode of {n} {args.kind} bytes per GPU ({workload_ref(n, args.kind, world)})"),
                "bytes_per_gpu": n,
                "global_bytes": total,
                "parallelism": (f"dp{world}: 128-aligned shards, RCCL size exchange (flrl_fl_encode_rank)"
                                if world > 1 else "single GPU"),
                "ranks_seen": ranks_seen,
                "rccl": rccl,
                "values_size_per_gpu": v,
                "ratio": round((alg - n + 24) / n, 6),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dominant,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": alg,
            },
            "kernels": {
                "timing": "ms / median_ms = mean / median over K steps of the kernel alone (HIP events "
                          "recorded by flrl_time_next_kernel on the launch stream); call_ms = the whole "
                          "device call (+ scratch zero-fill; + the size exchange when N > 1; decode: "
                          "+ the offsets pre-pass unless valuesSize == n), timed in a separate pass of K steps without the kernel "
                          "events (each event record costs ~4.6 us of GPU timeline)",
                "fl_encode": {"ms": round(enc_ms, 4), "median_ms": round(median_ms(ev, 4, 5), 4),
                              "call_ms": round(enc_call_ms, 4),
                              "alg_GBps": round(enc_gbs, 1),
                              "input_GBps": round(n / (enc_ms * 1e-3) / 1e9, 1)},
                "fl_decode": {"ms": round(dec_ms, 4), "median_ms": round(median_ms(ev, 6, 7), 4),
                              "call_ms": round(dec_call_ms, 4),
                              "alg_GBps": round(dec_gbs, 1),
                              "output_GBps": round(n / (dec_ms * 1e-3) / 1e9, 1)},
                "device_copy_ceiling": {"ms": round(copy_ms, 4), "GBps": round(copy_gbs, 1),
                                        "note": "torch copy_ of the same N bytes (read N + write N)"},
            },
            "cpu_baseline": cpu,
            "parity": parity,
            "rl": rl,
            "north_star": ns,
            "configs3": c3,
            "configs4": c4,
            "sections_run": {"cpu_baseline": cpu is not None, "north_star": ns is not None, "rl": rl is not None,
                             "configs3": c3 is not None, "configs4": c4 is not None},
        }
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.destroy()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
