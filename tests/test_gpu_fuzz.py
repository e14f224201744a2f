"""Seeded structured-random parity sweep of the device paths against the oracle.

The fixed-shape tests elsewhere pin named edge cases; this sweep draws inputs
that mix the shapes the kernels branch on, within ONE buffer, at random sizes
up to a few MiB: constant runs of 1..2000 bytes (255-splits, runs crossing
tiles and windows), random bytes (dense RL records, FL width 8), low-entropy
stretches of every FL width 1..8, all-zero frames, alternating two-byte
patterns and ragged tails. Every input is checked both ways against the
oracle's restatement of the reference (oracle/flrl_oracle.c: fl_cpu.cu:9-147
for FL, IMPLEMENTATION-PLAN.md:81-179 for RL): FL bits/values and RL
counts/values bit-exact, and both round trips exact. The seeds are fixed, so a
failure reproduces.
"""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    import flrl
    if not torch.cuda.is_available() or flrl.device_count() == 0:
        pytest.fail(f"GPU tests need a HIP device (HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES')})")


def structured(seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    n = int(rng.choice([rng.integers(0, 4096), rng.integers(4096, 1 << 20), rng.integers(1 << 20, 6 << 20)]))
    parts, total = [], 0
    while total < n:
        kind = rng.integers(0, 6)
        size = int(min(n - total, rng.integers(1, 1 << int(rng.integers(1, 18)))))
        if kind == 0:  # constant runs of 1..2000 bytes
            lens = rng.integers(1, 2001, size=size // 500 + 2)
            vals = rng.integers(0, 256, size=lens.size).astype(np.uint8)
            seg = np.repeat(vals, lens)[:size]
        elif kind == 1:  # random bytes
            seg = rng.integers(0, 256, size=size).astype(np.uint8)
        elif kind == 2:  # one FL width 1..8
            w = int(rng.integers(1, 9))
            seg = rng.integers(0, 1 << w, size=size).astype(np.uint8)
        elif kind == 3:  # zeros
            seg = np.zeros(size, dtype=np.uint8)
        elif kind == 4:  # two alternating bytes (runs of 1)
            a, b = rng.integers(0, 256, size=2)
            seg = np.where(np.arange(size) % 2 == 0, a, b ^ (1 if a == b else 0)).astype(np.uint8)
        else:  # short runs (mean ~3)
            lens = rng.integers(1, 6, size=size // 3 + 2)
            vals = rng.integers(0, 256, size=lens.size).astype(np.uint8)
            seg = np.repeat(vals, lens)[:size]
        parts.append(seg)
        total += seg.size
    return np.concatenate(parts)[:n] if parts else np.zeros(0, dtype=np.uint8)


@pytest.mark.parametrize("seed", range(40))
def test_fl_structured_vs_oracle(seed):
    import flrl
    from flrl.device import FLDevice
    a = structured(1000 + seed)
    bits, values = oracle.fl_compress(a)
    if a.size == 0:
        c = flrl.fl_compress(a)
        assert c.bits.size == 0 and c.values.size == 0
        return
    x = torch.from_numpy(a.copy()).cuda()
    d = FLDevice(a.size)
    d.encode(x)
    v = d.values_size()
    assert d.error() == 0
    assert v == values.size
    assert np.array_equal(d.bits[: d.frames].cpu().numpy(), bits)
    assert np.array_equal(d.values[:v].cpu().numpy(), values)
    assert torch.equal(d.decode(v), x)
    assert d.error() == 0


@pytest.mark.parametrize("seed", range(40))
def test_rl_structured_vs_oracle(seed):
    import flrl
    from flrl.device import RLDevice
    a = structured(2000 + seed)
    counts, values = oracle.rl_compress(a)
    if a.size == 0:
        c = flrl.rl_compress(a)
        assert c.counts.size == 0 and c.values.size == 0
        return
    x = torch.from_numpy(a.copy()).cuda()
    d = RLDevice(a.size)
    d.encode(x)
    r = d.runs()
    assert d.error() == 0
    assert r == counts.size
    assert np.array_equal(d.counts[:r].cpu().numpy(), counts)
    assert np.array_equal(d.values[:r].cpu().numpy(), values)
    assert torch.equal(d.decode(r), x)
    assert d.error() == 0


@pytest.mark.parametrize("seed", range(12))
def test_file_paths_structured_vs_oracle(tmp_path, seed):
    """The streamed file paths (chunked pipelines; RL runs re-split across chunk
    boundaries by the in-order writer) on the same structured inputs, with a
    random chunk size and worker count per seed: the .fl file equals the
    oracle's bytes (the reference fl-cpu format), the RL file the oracle's
    records in the build's container, and both decompress back."""
    import flrl
    rng = np.random.default_rng(3000 + seed)
    a = structured(3000 + seed)
    src = tmp_path / "in"
    a.tofile(src)
    workers = int(rng.integers(1, 5))
    fl_chunk = int(rng.choice([0, 128 * int(rng.integers(1, 64)), 128 * int(rng.integers(64, 8192))]))
    rl_chunk = int(rng.choice([0, int(rng.integers(256, 5000)), int(rng.integers(5000, 1 << 20))]))
    enc, back = tmp_path / "out.fl", tmp_path / "back"
    flrl.fl_compress_file(str(src), str(enc), workers, fl_chunk)
    assert enc.read_bytes() == oracle.fl_file_bytes(a), (workers, fl_chunk)
    flrl.fl_decompress_file(str(enc), str(back), workers, fl_chunk)
    assert back.read_bytes() == a.tobytes()
    enc = tmp_path / "out.rl"
    flrl.rl_compress_file(str(src), str(enc), workers, rl_chunk)
    counts, values = oracle.rl_compress(a)
    assert enc.read_bytes() == flrl.rl_file_bytes(a.size, counts, values), (workers, rl_chunk)
    flrl.rl_decompress_file(str(enc), str(back), workers, rl_chunk)
    assert back.read_bytes() == a.tobytes()
