"""BASELINE configs[4] on one MI355X: FL encode of 128 GiB of uniform-random
bytes in eight 16 GiB shards (the 8-GPU weak-scaling workload), one shard
after another through the per-rank entry flrl_fl_encode_rank on a one-rank
RCCL communicator, plus bench.py's configs4 section run in a child process.

Shard r is global bytes [r * 16 GiB, (r + 1) * 16 GiB) of one generated
buffer (counter-based generator at word offset r * 2^31),
exactly what rank r of `bench.py --gpus 8` encodes. Checked per shard: the
device round trip, 128-aligned windows against the oracle (a window's encode
equals the matching slice of the whole-input output),
and the window across each shard boundary against the oracle's encode of the
joined input — so the concatenation of the eight outputs is the 128 GiB
whole-input encode there. Rank 0's first 1 GiB hashes to the reference fl-cpu
file. The eight {F_r, V_r} are placed by the shipped exchange arithmetic
(flrl_shard_scan, the size_scan_kernel's code). Reference: gpuNCCLCompress
(src/fl/fl_gpu.cu:76-287), loadFileMpi's shard rule (src/file_io.cu:46-51).
"""
import hashlib
import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

import flrl
import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN_1GIB_U8_SHA = "0512b67cd1f3940885e5c3043c4541c5d8105403eb1273be20cd3c87d5ecef78"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available() or flrl.device_count() == 0:
        pytest.fail("GPU tests need a HIP device")


def _oracle_window(gstart: int, frames: int):
    """Oracle encode of `frames` frames of the global buffer from byte gstart."""
    a = oracle.gen("u8", frames * 128, 42, word_offset=gstart // 8)
    return a, oracle.fl_compress(a)


def test_configs4_eight_16gib_shards():
    from flrl.device import FLDevice, gen
    n, P, W = 16 << 30, 8, 2048  # shard bytes, shards, window frames
    F = n // 128
    torch.cuda.set_device(0)
    comm = flrl.Comm.rank(1, flrl.comm_unique_id(), 0)
    d = FLDevice(n)
    rng = np.random.default_rng(4)
    Vs, tail = [], None
    try:
        for r in range(P):
            x = gen("u8", n, 42, word_offset=r * n // 8)
            d.encode_rank(comm, x)
            torch.cuda.synchronize()
            rec = [int(t) for t in d.rank_sizes[:flrl.SZ_COUNT].cpu()]
            assert d.error() == 0, r
            V = rec[flrl.SZ_V]
            assert rec == [F, V, 0, 0, F, V], (r, rec)
            bits = d.bits[:F]
            assert 1 <= int(bits.min()) and int(bits.max()) <= 8
            assert int(bits.to(torch.int64).sum()) * 16 == V
            # windows inside the shard (first, last, three random)
            for f0 in [0, F - W] + [int(s) for s in rng.integers(0, F - W, size=3)]:
                a, (ob, ov) = _oracle_window(r * n + f0 * 128, W)
                assert np.array_equal(x[f0 * 128:(f0 + W) * 128].cpu().numpy(), a), (r, f0)
                v0 = int(d.bits[:f0].to(torch.int64).sum()) * 16
                assert np.array_equal(bits[f0:f0 + W].cpu().numpy(), ob), (r, f0)
                assert np.array_equal(d.values[v0:v0 + ov.size].cpu().numpy(), ov), (r, f0)
            # the window across the boundary with shard r-1: the two shards'
            # outputs, joined, equal the oracle's encode of the joined input
            if tail is not None:
                tb, tv = tail
                hv = int(bits[:W].to(torch.int64).sum()) * 16
                _, (ob, ov) = _oracle_window(r * n - W * 128, 2 * W)
                assert np.array_equal(np.concatenate([tb, bits[:W].cpu().numpy()]), ob), r
                assert np.array_equal(np.concatenate([tv, d.values[:hv].cpu().numpy()]), ov), r
            tw = int(bits[F - W:].to(torch.int64).sum()) * 16
            tail = (bits[F - W:].cpu().numpy(), d.values[V - tw:V].cpu().numpy())
            if r == 0:  # rank 0's first GiB is the reference fl-cpu's 1 GiB file
                f1 = (1 << 30) // 128
                v1 = int(bits[:f1].to(torch.int64).sum()) * 16
                h = hashlib.sha256(struct.pack("<QQQ", 1 << 30, f1, v1))
                h.update(bits[:f1].cpu().numpy().tobytes())
                h.update(d.values[:v1].cpu().numpy().tobytes())
                assert h.hexdigest() == GOLDEN_1GIB_U8_SHA
            out = d.decode(V)
            assert d.error() == 0 and torch.equal(out, x[:n]), r
            Vs.append(V)
            del x, out, bits
    finally:
        comm.destroy()
        del d
        torch.cuda.empty_cache()
    # placement of the eight shards by the exchange's own arithmetic, as the
    # 8-rank all-gather would leave the slots
    gathered = np.zeros(2 * P, dtype=np.uint64)
    for r in range(P):
        s = flrl.shard_slot(r, P, P)
        gathered[s], gathered[s + 1] = flrl.shard_size_word(n), Vs[r]
    for r in range(P):
        assert flrl.shard_scan(gathered, P, P, r) == [F, Vs[r], r * F, sum(Vs[:r]), P * F, sum(Vs)]
    assert P * F == (128 << 30) // 128


def test_bench_configs4_section_at_one_gpu(tmp_path):
    """bench.py --force-scan at N = 1 runs the configs[4] section (through
    flrl_fl_encode_rank on a one-rank communicator), small."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
           "--bytes", str(1 << 24), "--configs4-bytes", str(1 << 26), "--force-scan", "--cpu-sample", "0",
           "--no-north-star", "--no-rl"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=str(tmp_path), env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    c4 = line["configs4"]
    assert c4 is not None and c4["ranks_seen"] == 1
    assert c4["size_scan_ok"] and c4["roundtrip"]
    assert line["parity"]["roundtrip"] and line["parity"]["size_scan_ok"]


def test_bench_strong_scaling_mode_at_one_gpu(tmp_path):
    """bench.py --global-bytes (strong scaling: a fixed total split over the
    ranks by the reference shard rule), at N = 1 through the exchange
    (--force-scan) on a total that is not whole frames: scaling 'strong',
    value = total / step time, round trip and size scan green."""
    B = (1 << 24) + 77
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
           "--global-bytes", str(B), "--force-scan", "--no-configs4", "--cpu-sample", "0",
           "--no-north-star", "--no-rl"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=str(tmp_path), env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["scaling"] == "strong"
    assert line["config"]["global_bytes"] == B and line["config"]["bytes_per_gpu"] == B
    assert line["parity"]["roundtrip"] and line["parity"]["size_scan_ok"]
    assert abs(line["value"] - B / (line["ms_per_step"] * 1e-3) / 1e9) < 0.02 * line["value"] + 0.01
