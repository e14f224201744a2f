"""RL parity on the MI355X: HIP path (through the C ABI) vs the CPU oracle.

The reference fork has no RL code, so the oracle is the
restatement of IMPLEMENTATION-PLAN.md:81-179, pinned only by the plan's worked
examples (tests/golden/golden.json "rl_kat"): RL parity is partially unpinned.
Bit-exact checks cover runs crossing 16-byte lanes, 1 KiB wave items, 16 KiB
wave sub-tiles and 128 KiB tiles, 255-splits of long runs starting anywhere
(including inside earlier tiles), and config #3 (1 GiB runs32) in full.
"""
import numpy as np
import pytest

import flrl
import oracle
from conftest import kat_input

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available() or flrl.device_count() == 0:
        pytest.fail("GPU tests need a HIP device")


def encode(a: np.ndarray):
    """RL records of `a` through the host API (flrl_rl_compress)."""
    r = flrl.rl_compress(a)
    assert r.input_size == a.size
    return r.counts, r.values


def check(a: np.ndarray):
    rc, rv = encode(a)
    counts, values = oracle.rl_compress(a)
    assert rc.size == counts.size, (rc.size, counts.size)
    assert np.array_equal(rc, counts)
    assert np.array_equal(rv, values)
    back = flrl.rl_decompress(a.size, rc, rv)
    assert np.array_equal(back, a)
    return flrl.RLCompressed(rc, rv, a.size)


def test_kats(golden):
    for case in golden["rl_kat"]:
        data = np.frombuffer(kat_input(case), np.uint8)
        c, v = encode(data)
        assert c.tolist() == case["counts"], case["name"]
        assert v.tolist() == case["values"], case["name"]
        assert flrl.rl_decompress(data.size, c, v).tobytes() == data.tobytes()


def test_empty():
    r = flrl.rl_compress(b"")
    assert r.counts.size == 0 and r.input_size == 0
    assert flrl.rl_decompress(0, r.counts, r.values).size == 0


SIZES = [1, 2, 15, 16, 17, 255, 256, 257, 1023, 1024, 1025, 16383, 16384, 16385,
         32767, 32768, 32769, 65535, 65536, 65537, 98303, 98304, 98305, 131071, 131072, 131073, 196609, 300_001, (1 << 20) + 7]


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("kind", ["runs32", "longruns", "u8", "zero"])
def test_sizes_vs_oracle(n, kind):
    check(oracle.gen(kind, n, 17))


@pytest.mark.parametrize("L", [254, 255, 256, 509, 510, 511, 16384 + 3, 131072 + 255, 400_000])
@pytest.mark.parametrize("start", [0, 1, 15, 16, 1023, 16380, 32767, 32768, 65535, 65536, 98304, 131070])
def test_long_run_splits(L, start):
    # one long run of 7s starting at `start` inside random data
    rng = np.random.default_rng(L + start)
    a = rng.integers(0, 256, size=start + L + 300, dtype=np.uint8)
    a[start:start + L] = 7
    if start > 0 and a[start - 1] == 7:
        a[start - 1] = 8
    if a[start + L] == 7:
        a[start + L] = 9
    check(a)


def test_runs_spanning_many_tiles():
    # alternating long runs of 1..3 tiles, so most tiles have no natural head
    parts = []
    rng = np.random.default_rng(3)
    v = 0
    total = 0
    while total < 3_000_000:
        L = int(rng.integers(1, 3 * 131072))
        parts.append(np.full(L, v, np.uint8))
        v = (v + 1 + int(rng.integers(0, 200))) % 256
        total += L
    check(np.concatenate(parts))


@pytest.fixture
def always_help():
    flrl.debug_lookback_help_us(0)
    yield
    flrl.debug_lookback_help_us(-1)


def _fallback_input(case: str) -> np.ndarray:
    rng = np.random.default_rng(11)
    if case == "tiles":  # runs of up to 3 tiles: most tiles have no natural head
        parts, v, total = [], 0, 0
        while total < 3_000_000:
            L = int(rng.integers(1, 3 * 131072))
            parts.append(np.full(L, v, np.uint8))
            v = (v + 1 + int(rng.integers(0, 200))) % 256
            total += L
        return np.concatenate(parts)
    if case == "late":  # the first natural head in the third tile
        a = rng.integers(0, 4, size=2_000_000, dtype=np.uint8)
        a[:2 * 131072 + 77] = 5
        a[2 * 131072 + 77] = 6
        return a
    return oracle.gen(case, 3 * 131072 * 4 + 12345, 23)


@pytest.mark.parametrize("case", ["runs32", "longruns", "u8", "zero", "tiles", "late"])
def test_lookback_fallback_bit_exact(case, always_help):
    """The decoupled fallback of the RL encode look-back (an unpublished
    predecessor's map computed from the input; here at the first unpublished
    poll, so most look-backs of a multi-tile launch take it) gives the
    oracle's records, which decode back to the input."""
    from flrl.device import RLDevice
    a = _fallback_input(case)
    d = RLDevice(a.size)
    d.encode(torch.from_numpy(a).cuda())
    R = d.runs()
    assert d.error() == 0
    counts, values = oracle.rl_compress(a)
    assert R == counts.size
    assert np.array_equal(d.counts[:R].cpu().numpy(), counts)
    assert np.array_equal(d.values[:R].cpu().numpy(), values)
    out = d.decode(R)
    assert d.error() == 0
    assert np.array_equal(out[:a.size].cpu().numpy(), a)


def test_lookback_fallback_1gib(always_help):
    from flrl.device import RLDevice
    n = 1 << 30
    d = RLDevice(n)
    x = torch.from_numpy(flrl.gen_host("runs32", n, 42)).cuda()
    d.encode(x)
    R = d.runs()
    assert d.error() == 0
    flrl.debug_lookback_help_us(-1)
    ref = RLDevice(n)
    ref.encode(x)
    assert ref.runs() == R and ref.error() == 0
    assert torch.equal(d.counts[:R], ref.counts[:R]) and torch.equal(d.values[:R], ref.values[:R])


def test_concurrent_large_encodes():
    """Two RL encodes whose grids exceed the GPU (3072 tiles each, 1280
    resident) on two streams at once: their workgroups interleave on the CUs,
    so a tile's predecessor may wait behind the other launch (the look-back's
    fallback covers that); outputs must equal the serial ones."""
    from flrl.device import RLDevice, gen
    n = 384 << 20
    xs = [torch.from_numpy(flrl.gen_host("runs32", n, 5)).cuda(), gen("lo4", n, 6)]
    ds = [RLDevice(n), RLDevice(n)]
    ref = []
    for d, x in zip(ds, xs):
        d.encode(x)
        R = d.runs()
        assert d.error() == 0
        ref.append((R, d.counts[:R].clone(), d.values[:R].clone()))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(2)]
    for rep in range(3):
        for d in ds:
            d.counts.zero_()
        torch.cuda.synchronize()
        for d, x, st in zip(ds, xs, streams):
            d.encode(x, stream=st)
        torch.cuda.synchronize()
        for i, (d, (R, c0, v0)) in enumerate(zip(ds, ref)):
            assert d.error() == 0 and d.runs() == R, (rep, i)
            assert torch.equal(d.counts[:R], c0) and torch.equal(d.values[:R], v0), (rep, i)


def test_debug_lookback_help_us_rejects_below_minus_one():
    with pytest.raises(flrl.FLRLError):
        flrl.debug_lookback_help_us(-2)


@pytest.mark.parametrize("quiet", [1, 32768 - 3, 32768 + 100, 65536 - 3, 98304 + 7, 131072 + 5])
def test_first_natural_head_late(quiet):
    # no natural head for `quiet` bytes (in the first 32 KiB sub-tile, at and
    # after sub-tile boundaries, in the last sub-tile, in the next tile), then
    # mixed data
    rng = np.random.default_rng(quiet)
    a = rng.integers(0, 4, size=quiet + 300_000, dtype=np.uint8)
    a[:quiet] = 5
    a[quiet] = 6
    check(a)


@pytest.mark.parametrize("maxrun", [6, 12, 20, 28, 40])
def test_medium_density(maxrun):
    # mean runs around the staging threshold (state-independent runs per tile
    # vs the LDS staging capacity): the staging overflows in the first, second,
    # third or last 32 KiB sub-tile of a tile, or not at all
    rng = np.random.default_rng(maxrun)
    lens = rng.integers(1, maxrun + 1, size=400_000)
    vals = (np.cumsum(rng.integers(1, 255, size=lens.size)) % 256).astype(np.uint8)
    check(np.repeat(vals, lens)[:2_000_003])


def _dense_sparse(pattern, seed):
    """4 KiB sub-chunks (one wave's 64 lanes x 64 B) after the pattern: 'd' random
    bytes (more records than the wave's staging: the piece emission), 'm' runs of
    1..3 bytes (the staging overflows part-way), 's' runs of 20..40 bytes, 'h'
    half a sub-chunk of random bytes then a 255-byte run."""
    rng = np.random.default_rng(seed)
    parts = []
    for c in pattern:
        if c == "d":
            parts.append(rng.integers(0, 256, size=4096, dtype=np.uint8))
        elif c == "h":
            parts.append(rng.integers(0, 256, size=2048, dtype=np.uint8))
            parts.append(np.full(255, rng.integers(0, 256), dtype=np.uint8))
        else:
            lo, hi = (1, 4) if c == "m" else (20, 41)
            lens = rng.integers(lo, hi, size=4096)
            vals = (np.cumsum(rng.integers(1, 255, size=lens.size)) % 256).astype(np.uint8)
            parts.append(np.repeat(vals, lens)[:4096])
    return np.concatenate(parts)


@pytest.mark.parametrize("pattern", ["d", "dd", "ds", "sd", "dsd", "dmd", "ddddddddd", "sdddddddsd",
                                     "hdhd", "dhs", "m" * 8 + "d" * 8, "d" * 40])
@pytest.mark.parametrize("tail", [0, 1, 15, 17, 1000, 4095])
def test_dense_pieces_carry(pattern, tail):
    """Dense sub-chunks store whole 16-byte chunks and carry a part's last partial
    chunk into the next part (RlWave::piece_flush): dense runs starting at the input's
    first byte (its first head ends no run), switching to and from sparse sub-chunks
    (the carry flushed before the staging is reused), crossing tiles, and ending
    in partial sub-chunks; bit-exact against the oracle, round trip exact."""
    a = _dense_sparse(pattern, len(pattern) * 7 + tail)
    if tail:
        a = np.concatenate([a, np.random.default_rng(tail).integers(0, 256, size=tail, dtype=np.uint8)])
    check(a)
    check(a[1:])  # every chunk alignment of the output shifted by one record


def test_decode_offsets_rounds():
    # random bytes: ~72M runs, more than 1024 x 65536, so the decode pre-pass
    # runs two rounds per workgroup with a partial last workgroup
    check(oracle.gen("u8", (72 << 20) + 999, 23))


def test_all_zero_large():
    a = np.zeros(5 * 131072 + 77, np.uint8)  # no natural head after byte 0
    r = check(a)
    assert r.counts.tolist()[:3] == [255, 255, 255]


def test_decode_rejects_malformed():
    with pytest.raises(flrl.FLRLError) as e:
        flrl.rl_decompress(5, np.array([2, 0, 3], np.uint8), np.array([1, 2, 3], np.uint8))
    assert e.value.code == flrl.E_FORMAT
    with pytest.raises(flrl.FLRLError):
        flrl.rl_decompress(6, np.array([2, 3], np.uint8), np.array([1, 2], np.uint8))
    with pytest.raises(flrl.FLRLError):
        flrl.rl_decompress(3, np.zeros(0, np.uint8), np.zeros(0, np.uint8))


def test_device_1gib_runs32():
    """Config #3: RL encode/decode of 1 GiB runs32 (mean run 32) — bit-exact vs
    the oracle over the full buffer and a device round trip."""
    from flrl.device import RLDevice
    n = 1 << 30
    a = oracle.gen("runs32", n, 42)
    counts, values = oracle.rl_compress(a)
    x = torch.from_numpy(a).cuda()
    d = RLDevice(n)
    d.encode(x)
    R = d.runs()
    assert d.error() == 0
    assert R == counts.size
    assert np.array_equal(d.counts[:R].cpu().numpy(), counts)
    assert np.array_equal(d.values[:R].cpu().numpy(), values)
    out = d.decode(R)
    assert d.error() == 0
    assert torch.equal(out, x)


# ---- rank decode: dense-path threshold (tile output <= 32 KiB), 64 KiB
# windows, chunks with 0..16 run starts, tiles starting mid-chunk -------------
@pytest.mark.parametrize("runlen", [7, 8, 9, 15, 16, 17, 24, 31, 33, 63, 64, 200, 239, 240, 241, 255])
def test_decode_fixed_run_lengths(runlen):
    # every tile of 4096 (8192) runs has output 4096 (8192) * runlen: at, below and
    # above the dense threshold and the 64 KiB window; run starts fall at every
    # offset within 16-byte chunks when runlen is odd; 239..241 straddle the
    # 512/256-thread block decode threshold (mean run 240)
    nruns = 3 * 8192 + 77
    vals = (np.arange(nruns) * 37 % 251 + 1).astype(np.uint8)
    a = np.repeat(vals, runlen)
    check(a[: a.size - 3])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_decode_mixed_tile_densities(seed):
    # tiles alternate between dense (runs of 1..4) and sparse (runs of 20..200)
    # stretches, so neighbouring tiles take different decode paths and a
    # window's first chunk is shared with a tile of the other kind
    rng = np.random.default_rng(seed)
    parts = []
    for k in range(24):
        lo, hi = (1, 5) if k % 2 == 0 else (20, 201)
        lens = rng.integers(lo, hi, size=int(rng.integers(1000, 9000)))
        vals = (np.cumsum(rng.integers(1, 255, size=lens.size)) % 256).astype(np.uint8)
        parts.append(np.repeat(vals, lens))
    check(np.concatenate(parts))


def test_decode_all_starts_in_chunk():
    # runs of exactly 1 byte for whole tiles (16 starts per chunk), then runs of
    # 2 and 3 (8 and 5-6 starts), in one input
    a = np.concatenate([(np.arange(70_000) % 2).astype(np.uint8),
                        np.repeat((np.arange(40_000) % 2 + 5).astype(np.uint8), 2),
                        np.repeat((np.arange(40_000) % 3 + 9).astype(np.uint8), 3)])
    check(a)


# ---- wave decode (mean run <= 12 bytes: one wave per 2048-run tile) --------
@pytest.mark.parametrize("runlen", [1, 2, 3, 11, 12, 13, 23, 24, 25])
def test_decode_wave_threshold(runlen):
    # mean run exactly at, below and above the wave-decode threshold
    nruns = 5 * 2048 + 31
    vals = (np.arange(nruns) * 29 % 253 + 1).astype(np.uint8)
    check(np.repeat(vals, runlen))


@pytest.mark.parametrize("seed", [4, 5, 6])
def test_decode_wave_long_runs_in_dense(seed):
    # mostly 1-byte runs with a few runs of 100..255 bytes: a dense input (wave
    # decode) whose tiles have one to six 8 KiB output windows
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(300_000) < 0.04, rng.integers(100, 256, 300_000), 1)
    vals = (np.cumsum(rng.integers(1, 255, size=lens.size)) % 256).astype(np.uint8)
    a = np.repeat(vals, lens)
    assert a.size <= 12 * lens.size
    check(a)


@pytest.mark.parametrize("at", [0, 4096 * 7 + 11, 300_000 - 200])
def test_decode_densest_with_long_stretch(at):
    # random bytes (mean run ~1: 4096-run wave tiles) with a stretch of 200
    # runs of 255 bytes, so one or two tiles need several 8 KiB windows
    rng = np.random.default_rng(at + 1)
    lens = np.ones(300_000, np.int64)
    lens[at:at + 200] = 255
    vals = (np.cumsum(rng.integers(1, 255, size=lens.size)) % 256).astype(np.uint8)
    a = np.repeat(vals, lens)
    assert a.size <= 2 * lens.size
    check(a)


def test_decode_wave_rejects_zero_count():
    # a zero count inside a dense input (and inside the last, partial tile)
    for pos in (1000, 4096 * 3 + 5):
        counts = np.ones(4096 * 3 + 100, np.uint8)
        counts[pos] = 0
        values = (np.arange(counts.size) % 250).astype(np.uint8)
        with pytest.raises(flrl.FLRLError) as e:
            flrl.rl_decompress(int(counts.sum()), counts, values)
        assert e.value.code == flrl.E_FORMAT


def test_device_more_than_2_32_runs():
    """64-bit run indices: ~4.27 GiB of random bytes has R > 2^32 runs (all
    shorter than 255). Device round trip; R against an independent torch count
    of run starts; and the records of three windows that start at run starts
    (the head, around record 2^32, the tail) bit-exact against the oracle."""
    from flrl.device import RLDevice, gen
    n = (1 << 32) + (1 << 28) + 12345
    x = gen("u8", n, 77)
    d = RLDevice(n)
    d.encode(x)
    R = d.runs()
    assert d.error() == 0
    changes = (x[1:n] != x[: n - 1])
    expect = int(changes.sum().item()) + 1
    assert R == expect and R > (1 << 32), (R, expect)

    def window(i0: int, length: int):
        """records of x[i0 : i0+length] (i0 moved to the next run start, the end
        moved back to a run end) and the index of its first record"""
        i0 = max(i0, 1)
        while bool(x[i0] == x[i0 - 1]):
            i0 += 1
        i1 = min(i0 + length, n)
        while i1 < n and bool(x[i1] == x[i1 - 1]):
            i1 -= 1
        k0 = int(changes[: i0 - 1].sum().item()) + 1  # runs starting before i0
        return k0, x[i0:i1].cpu().numpy()

    for k0, a in [(0, x[: 1 << 20].cpu().numpy())] + [window(i, 1 << 20) for i in
                                                        (int((1 << 32) * 256 / 255) - (1 << 19), n - (1 << 20))]:
        c, v = oracle.rl_compress(a)
        assert k0 + c.size <= R
        assert np.array_equal(d.counts[k0:k0 + c.size].cpu().numpy(), c), k0
        assert np.array_equal(d.values[k0:k0 + c.size].cpu().numpy(), v), k0
    del changes
    out = d.decode(R)
    assert d.error() == 0
    assert torch.equal(out[:n], x[:n])
