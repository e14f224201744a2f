"""FL parity on the MI355X: HIP path (through the C ABI) vs the CPU oracle.

Bit-exact on every case: golden vectors of the reference fl-cpu, seeded
inputs at oracle-checkable sizes (edges of frames, 16-byte lanes and 64 KiB
tiles; every width 1..8 inside one tile), and at full BASELINE sizes the
size-independent properties: golden sha256 of the 1 GiB configs, decode(encode)
round trips, and shard-equivalence against the oracle on sampled 128-aligned
windows of a 16 GiB input.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

import flrl
import oracle
from conftest import kat_input

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    avail, ndev = torch.cuda.is_available(), flrl.device_count()
    if not avail or ndev == 0:  # never silently skip on the GPU box
        pytest.fail(f"GPU tests need a HIP device (torch: {avail}, flrl: {ndev}, "
                    f"HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES')}, "
                    f"CUDA_VISIBLE_DEVICES={os.environ.get('CUDA_VISIBLE_DEVICES')}, "
                    f"ROCR_VISIBLE_DEVICES={os.environ.get('ROCR_VISIBLE_DEVICES')})")


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def mixed_width_input(n: int, seed: int) -> np.ndarray:
    """Every frame gets a random width in [1,8] (and some frames all-zero)."""
    rng = np.random.default_rng(seed)
    frames = (n + 127) // 128
    widths = rng.integers(0, 9, size=frames)
    hi = np.repeat((1 << widths) - 1, 128)[:n]
    a = (rng.integers(0, 256, size=n) & hi).astype(np.uint8)
    return a


def check_against_oracle(a: np.ndarray):
    c = flrl.fl_compress(a)
    bits, values = oracle.fl_compress(a)
    assert c.input_size == a.size
    assert np.array_equal(c.bits, bits)
    assert np.array_equal(c.values, values)
    back = flrl.fl_decompress(a.size, c.bits, c.values)
    assert np.array_equal(back, a)
    return c


def test_kats(golden):
    for case in golden["fl_kat"]:
        data = kat_input(case)
        c = flrl.fl_compress(data)
        assert c.bits.tobytes().hex() == case["bits_hex"], case["name"]
        assert c.values.tobytes().hex() == case["values_hex"], case["name"]
        assert flrl.fl_decompress(len(data), c.bits, c.values).tobytes() == data


def test_empty(golden):
    c = flrl.fl_compress(b"")
    assert c.bits.size == 0 and c.values.size == 0 and c.input_size == 0
    assert sha(c.to_file_bytes()) == golden["fl_empty_file_sha256"]
    assert flrl.fl_decompress(0, c.bits, c.values).size == 0


def test_bmp(golden, bmp_bytes):
    c = flrl.fl_compress(bmp_bytes)
    assert sha(c.to_file_bytes()) == golden["fl_bmp"]["fl_sha256"]
    assert flrl.fl_decompress(c.input_size, c.bits, c.values).tobytes() == bmp_bytes


@pytest.mark.parametrize("idx", range(7))
def test_generated_golden(golden, idx):
    g = golden["fl_generated"][idx]
    a = oracle.gen(g["kind"], g["n"], g["seed"])
    c = flrl.fl_compress(a)
    assert sha(c.to_file_bytes()) == g["fl_sha256"]
    assert np.array_equal(flrl.fl_decompress(a.size, c.bits, c.values), a)


SIZES = [1, 2, 7, 8, 15, 16, 17, 127, 128, 129, 255, 256, 1000, 4096, 4741, 65535, 65536,
         65537, 100003, 131071, 131072, 131073, 196607, 196609, 262144 + 4095, 327744,
         (1 << 20) + 13,
         90769, 253951]  # decode tiles are 64 KiB (8 KiB of frames per wave), encode tiles 128 KiB;
                         # the last two end inside a later wave of a decode tile


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("kind", ["u8", "lo4", "zero", "ff", "mixed"])
def test_sizes_vs_oracle(n, kind):
    if kind == "ff":
        a = np.full(n, 255, np.uint8)
    elif kind == "mixed":
        a = mixed_width_input(n, n)
    else:
        a = oracle.gen(kind, n, 11)
    check_against_oracle(a)


def test_every_width_in_one_tile():
    # width b in frame f = 1 + f % 8, max value present in each frame
    frames = 1024
    a = np.zeros(frames * 128, np.uint8)
    for f in range(frames):
        b = 1 + f % 8
        a[f * 128:(f + 1) * 128] = np.arange(128) % (1 << b)
        a[f * 128 + 5] = (1 << b) - 1
    c = check_against_oracle(a)
    assert c.bits.tolist() == [1 + f % 8 for f in range(frames)]


def test_raw_and_packed_decode_tiles():
    # decode tiles (64 KiB) whose widths are all 8 are copied from the load
    # registers; the others are unpacked through LDS. Alternate the two, with a
    # width-7 frame at a tile's first, middle and last frame, then a partial
    # last tile (never raw), through the host pipeline and the device API.
    tile = 65536
    n = 9 * tile + 5000
    a = oracle.gen("u8", n, 21).copy()
    for t, f in ((1, 0), (3, 255), (5, 511), (7, 100)):
        o = t * tile + f * 128
        a[o:o + 128] &= 0x7F
    c = check_against_oracle(a)
    assert [int(c.bits[t * 512:(t + 1) * 512].min()) for t in range(9)] == [8, 7, 8, 7, 8, 7, 8, 7, 8]
    from flrl.device import FLDevice
    x = torch.from_numpy(a).cuda()
    d = FLDevice(n)
    d.encode(x)
    v = d.values_size()
    assert v == c.values.size and d.error() == 0
    d.decode(v)
    assert d.error() == 0
    assert torch.equal(d.out[:n], x)


def test_many_tiles_random_widths():
    a = mixed_width_input(64 * 65536 + 777, 5)  # 65 tiles: look-back over > 64 tiles
    check_against_oracle(a)


# ------------------------------------------------------------- malformed input
def test_decode_rejects_bad_width():
    a = oracle.gen("lo4", 1000, 1)
    c = flrl.fl_compress(a)
    for bad in (0, 9, 255):
        bits = c.bits.copy()
        bits[3] = bad
        with pytest.raises(flrl.FLRLError) as e:
            flrl.fl_decompress(a.size, bits, c.values)
        assert e.value.code == flrl.E_FORMAT


def test_decode_rejects_size_mismatch():
    a = oracle.gen("u8", 5000, 1)
    c = flrl.fl_compress(a)
    with pytest.raises(flrl.FLRLError):
        flrl.fl_decompress(a.size, c.bits, c.values[:-1])
    with pytest.raises(flrl.FLRLError):
        flrl.fl_decompress(a.size + 128, c.bits, c.values)


def test_decode_reference_early_out():
    # fl_cpu.cu:94-97: valuesSize == 0 || bitsSize == 0 -> empty output
    assert flrl.fl_decompress(100, np.zeros(0, np.uint8), np.ones(4, np.uint8)).size == 0
    assert flrl.fl_decompress(100, np.ones(1, np.uint8), np.zeros(0, np.uint8)).size == 0


# ----------------------------------------------------- device API, full sizes
def test_device_api_errors():
    from flrl.device import FLDevice
    d = FLDevice(4096)
    x = torch.zeros(4096 + 32, dtype=torch.uint8, device="cuda")
    with pytest.raises(flrl.FLRLError) as e:
        flrl.fl_encode_device(x.data_ptr() + 1, 4096, d.bits.data_ptr(), d.values.data_ptr(),
                              d.sizes.data_ptr() + 8, d.scratch.data_ptr(), d.scratch_bytes)
    assert e.value.code == flrl.E_ARG
    with pytest.raises(flrl.FLRLError):
        flrl.fl_encode_device(x.data_ptr(), 4096, d.bits.data_ptr(), d.values.data_ptr(),
                              d.sizes.data_ptr() + 8, d.scratch.data_ptr(), 8)


def test_device_bad_width_flag():
    from flrl.device import FLDevice
    n = 300_000
    a = torch.from_numpy(oracle.gen("lo4", n, 2)).cuda()
    d = FLDevice(n)
    d.encode(a)
    v = d.values_size()
    assert d.error() == 0
    d.bits[1234] = 0
    d.decode(v)
    assert d.error() == flrl.E_FORMAT


def test_device_all8_decode_checks_widths():
    # valuesSize == n: the decode takes every frame as width 8 without the
    # offsets pre-pass and checks each width itself (the last frame: any width
    # whose packed size is its byte count)
    from flrl.device import FLDevice
    for n, last in ((2344 * 128 + 1, 0), (2344 * 128 + 2, None)):
        a = oracle.gen("u8", n, 4).copy()
        a[-1] = 200  # a 2-byte last frame of width 8
        if last is not None:
            a[-1] = last  # a 1-byte last frame of value 0: width 1, 1 packed byte
        x = torch.from_numpy(a).cuda()
        d = FLDevice(n)
        d.encode(x)
        v = d.values_size()
        assert v == n and d.error() == 0
        bits, values = oracle.fl_compress(a)
        assert np.array_equal(d.bits[:d.frames].cpu().numpy(), bits)
        assert np.array_equal(d.values[:v].cpu().numpy(), values)
        assert torch.equal(d.decode(v), x) and d.error() == 0
        for f, w in ((1234, 7), (1234, 0), (1234, 9), (d.frames - 1, 9), (d.frames - 1, 0)) + \
                (((d.frames - 1, 4),) if last is None else ()):
            bad = d.bits.clone()
            bad[f] = w
            d.decode(v, bits=bad)
            assert d.error() == flrl.E_FORMAT, (n, f, w)
        d.decode(v)
        assert d.error() == 0 and torch.equal(d.out[:n], x)


@pytest.mark.parametrize("kind", ["lo4", "u8"])
def test_stale_scratch_all8_decode(kind):
    """Past 1024 decode tiles the decode takes tickets; without the offsets
    pre-pass (u8: valuesSize == n) the decode itself flags a counter that was
    not reset (FLRL_E_ARG) instead of leaving tiles undecoded."""
    from flrl.device import FLDevice
    n = (96 << 20) + 5
    x = torch.from_numpy(oracle.gen(kind, n, 9)).cuda()
    d = FLDevice(n)
    d.encode(x)
    v = d.values_size()
    assert d.error() == 0 and (v == n) == (kind == "u8")
    d.decode(v)
    assert d.error() == 0 and torch.equal(d.out[:n], x)
    flrl.debug_skip_scratch_resets(1)
    d.decode(v)
    assert d.error() == flrl.E_ARG
    d.out.zero_()
    d.decode(v)
    assert d.error() == 0 and torch.equal(d.out[:n], x)


@pytest.mark.parametrize("n", [5000, (8 << 20) + 5])
def test_stale_scratch_raises(n):
    """A launch on scratch whose ticket was not reset (flrl_debug_skip_scratch_resets)
    flags FLRL_E_ARG in every ticketed kernel (FL encode included: it used to
    return silently when every first ticket was past the grid); the next
    normal call resets the scratch and runs bit-exact again."""
    from flrl.device import FLDevice, RLDevice
    a = oracle.gen("lo4", n, 9)
    x = torch.from_numpy(a).cuda()
    d = FLDevice(n)
    d.encode(x)
    v = d.values_size()
    assert d.error() == 0
    bits0, vals0 = d.bits[:d.frames].clone(), d.values[:v].clone()
    flrl.debug_skip_scratch_resets(1)
    d.encode(x)
    assert d.error() == flrl.E_ARG
    d.encode(x)
    assert d.error() == 0 and d.values_size() == v
    assert torch.equal(d.bits[:d.frames], bits0) and torch.equal(d.values[:v], vals0)
    assert torch.equal(d.decode(v), x) and d.error() == 0
    flrl.debug_skip_scratch_resets(1)
    d.decode(v)
    assert d.error() == flrl.E_ARG
    assert torch.equal(d.decode(v), x) and d.error() == 0

    r = RLDevice(n)
    r.encode(x)
    R = r.runs()
    assert r.error() == 0
    flrl.debug_skip_scratch_resets(1)
    r.encode(x)
    assert r.error() == flrl.E_ARG
    r.encode(x)
    assert r.error() == 0 and r.runs() == R
    assert torch.equal(r.decode(R), x) and r.error() == 0
    flrl.debug_skip_scratch_resets(1)
    r.decode(R)
    assert r.error() == flrl.E_ARG
    assert torch.equal(r.decode(R), x) and r.error() == 0
    flrl.debug_skip_scratch_resets(0)


@pytest.mark.parametrize("idx", [0, 1])
def test_device_1gib_golden(golden, idx):
    """Config #2 (u8) and the lo4 twin at 1 GiB: file sha256 == reference fl-cpu."""
    from flrl.device import FLDevice, gen
    g = golden["fl_generated_large"][idx]
    n = g["n"]
    x = gen(g["kind"], n, g["seed"])
    d = FLDevice(n)
    d.encode(x)
    v = d.values_size()
    assert d.error() == 0
    h = hashlib.sha256()
    h.update(np.array([n, d.frames, v], dtype="<u8").tobytes())
    h.update(d.bits[: d.frames].cpu().numpy().tobytes())
    h.update(d.values[:v].cpu().numpy().tobytes())
    assert h.hexdigest() == g["fl_sha256"]
    assert 24 + d.frames + v == g["fl_bytes"]
    xin = hashlib.sha256(x[:n].cpu().numpy().tobytes()).hexdigest()
    assert xin == g["input_sha256"]
    out = d.decode(v)
    assert d.error() == 0
    assert torch.equal(out, x[:n])


def test_device_16gib_lo4_shard_equivalence():
    """Config #4: 16 GiB lo4 on one GPU. Round trip on device, and 128-aligned
    windows of the input re-encoded by the oracle equal the matching slices of
    the GPU output."""
    from flrl.device import FLDevice, gen
    n = 16 << 30
    x = gen("lo4", n, 42)
    x[(12 << 30) + 77] = 0xF3  # a wide frame deep in the buffer
    d = FLDevice(n)
    d.encode(x)
    v = d.values_size()
    assert d.error() == 0
    bits = d.bits[: d.frames]
    assert int(bits.min()) >= 1 and int(bits.max()) <= 8
    pref = torch.cumsum(bits.to(torch.int64), 0) * 16  # byte end of each frame
    assert int(pref[-1]) == v
    rng = np.random.default_rng(0)
    starts = [0, ((12 << 30) + 77) // 128 * 128 - 100 * 128, (d.frames - 4096) * 128] + \
        [int(s) * 128 for s in rng.integers(0, d.frames - 4096, size=3)]
    for s in starts:
        L = 4096 * 128
        f0 = s // 128
        ob, ov = oracle.fl_compress(x[s:s + L].cpu().numpy())
        assert np.array_equal(bits[f0:f0 + 4096].cpu().numpy(), ob)
        v0 = 0 if f0 == 0 else int(pref[f0 - 1])
        assert np.array_equal(d.values[v0:v0 + ov.size].cpu().numpy(), ov)
    out = d.decode(v)
    assert d.error() == 0
    assert torch.equal(out, x[:n])
    del d, x, out
    torch.cuda.empty_cache()


def test_device_decode_offsets_rounds():
    """A ragged 2 GiB input: more than 1024 x 16384 frames, so the decode
    pre-pass runs two rounds per workgroup with a partial last workgroup; the
    offsets' width sum also equals valuesSize."""
    from flrl.device import FLDevice, gen
    n = (2 << 30) + 12345
    x = gen("lo4", n, 5)
    x[n - 1] = 0xFF  # a full-width last (partial) frame
    d = FLDevice(n)
    d.encode(x)
    v = d.values_size()
    assert d.error() == 0
    out = d.decode(v)
    assert d.error() == 0
    assert torch.equal(out, x[:n])
    del d, x, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kind", ["u8", "lo4"])
def test_device_repeat_stability(kind):
    """Back-to-back device encodes/decodes of the same 96 MiB + 77 input, every
    output compared with the first: persistent workgroups, tickets and LDS
    hand-offs must give identical results on every launch (catches
    intra-workgroup races on shared ticket/base slots)."""
    from flrl.device import FLDevice, gen
    n = (96 << 20) + 77
    x = gen(kind, n, 9)
    d = FLDevice(n)
    d.encode(x)
    v = d.values_size()
    bits0, vals0 = d.bits[: d.frames].clone(), d.values[:v].clone()
    out = torch.empty_like(x)
    for _ in range(30):
        d.encode(x)
        d.decode(v, out=out)
    torch.cuda.synchronize()
    assert d.error() == 0 and d.values_size() == v
    for i in range(30):
        d.encode(x)
        assert torch.equal(d.bits[: d.frames], bits0) and torch.equal(d.values[:v], vals0), i
        out.zero_()
        d.decode(v, out=out)
        assert torch.equal(out[:n], x[:n]), i
    assert d.error() == 0
    del d, x, out
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------- CLI
def test_cli_gpu_methods(golden, bmp_bytes, cli_path, tmp_path):
    src = tmp_path / "in.bmp"
    src.write_bytes(bmp_bytes)
    for method in ("fl", "fl-nccl", "fl-mpi", "fl-shmem"):
        out = tmp_path / f"o.{method}"
        subprocess.run([cli_path, "c", method, str(src), str(out)], check=True,
                       capture_output=True)
        assert sha(out.read_bytes()) == golden["fl_bmp"]["fl_sha256"], method
        back = tmp_path / f"b.{method}"
        subprocess.run([cli_path, "d", method, str(out), str(back)], check=True,
                       capture_output=True)
        assert back.read_bytes() == bmp_bytes


def test_cli_rl_gpu(bmp_bytes, cli_path, tmp_path):
    src = tmp_path / "in.bmp"
    src.write_bytes(bmp_bytes)
    subprocess.run([cli_path, "c", "rl", str(src), str(tmp_path / "o.rl")], check=True,
                   capture_output=True)
    subprocess.run([cli_path, "c", "rl-cpu", str(src), str(tmp_path / "o2.rl")], check=True,
                   capture_output=True)
    assert (tmp_path / "o.rl").read_bytes() == (tmp_path / "o2.rl").read_bytes()
    subprocess.run([cli_path, "d", "rl", str(tmp_path / "o.rl"), str(tmp_path / "b")], check=True,
                   capture_output=True)
    assert (tmp_path / "b").read_bytes() == bmp_bytes


@pytest.mark.gpu
def test_time_next_kernel_brackets_the_kernel():
    """flrl_time_next_kernel: the kernel window lies inside the call window
    (the call adds the scratch memset; decode also the offsets pre-pass), the
    pair is consumed by one call, and results are unaffected."""
    from flrl.device import FLDevice, RLDevice, gen
    n = (32 << 20) + 77
    x = gen("u8", n, 5)
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for e in ev:
        e.record(s)
    d = FLDevice(n)
    for call in (lambda: d.encode(x), lambda: d.decode(d.values_size())):
        call()
        torch.cuda.synchronize()
        ev[0].record(s)
        flrl.time_next_kernel(ev[2], ev[3])
        call()
        ev[1].record(s)
        torch.cuda.synchronize()
        whole, kern = ev[0].elapsed_time(ev[1]), ev[2].elapsed_time(ev[3])
        assert 0 < kern <= whole, (kern, whole)
        assert ev[0].elapsed_time(ev[2]) >= 0 and ev[3].elapsed_time(ev[1]) >= 0
    assert torch.equal(d.out[:n], x[:n]) and d.error() == 0
    # consumed: a further call leaves the events where they were
    t = ev[2].elapsed_time(ev[3])
    d.encode(x)
    torch.cuda.synchronize()
    assert ev[2].elapsed_time(ev[3]) == t
    r = RLDevice(n)
    ev[0].record(s)
    flrl.time_next_kernel(ev[2], ev[3])
    r.encode(x)
    ev[1].record(s)
    torch.cuda.synchronize()
    assert 0 < ev[2].elapsed_time(ev[3]) <= ev[0].elapsed_time(ev[1])
    flrl.time_next_kernel(ev[2], ev[3])
    flrl.time_next_kernel(None, None)  # cancel
    ev[0].record(s)
    r.decode(r.runs())
    ev[1].record(s)
    torch.cuda.synchronize()
    assert torch.equal(r.out[:n], x[:n]) and r.error() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1000003, (64 << 20) + 77])
def test_graph_capture_replays(n):
    """Device calls captured into a HIP graph (torch.cuda.graph) re-initialise
    their scratch on every replay: FL and RL encode + decode replayed with every
    output cleared in between stay bit-exact. (With hipMemsetAsync resets the
    second replay saw the first one's ticket and the encode did nothing.)"""
    from flrl.device import FLDevice, RLDevice, gen
    x = gen("lo4", n, 3)
    d, r = FLDevice(n), RLDevice(n)
    d.encode(x)
    v = d.values_size()
    r.encode(x)
    R = r.runs()
    bits0, vals0 = d.bits[: d.frames].clone(), d.values[:v].clone()
    c0, rv0 = r.counts[:R].clone(), r.values[:R].clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        d.encode(x)
        d.decode(v)
        r.encode(x)
        r.decode(R)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        d.encode(x)
        d.decode(v)
        r.encode(x)
        r.decode(R)
    for i in range(4):
        for t in (d.out, d.bits, d.values, r.out, r.counts, r.values):
            t.zero_()
        d.sizes[1] = 0
        r.runs_t.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert d.error() == 0 and r.error() == 0, i
        assert d.values_size() == v and r.runs() == R, i
        assert torch.equal(d.bits[: d.frames], bits0) and torch.equal(d.values[:v], vals0), i
        assert torch.equal(r.counts[:R], c0) and torch.equal(r.values[:R], rv0), i
        assert torch.equal(d.out[:n], x[:n]) and torch.equal(r.out[:n], x[:n]), i


@pytest.mark.gpu
def test_concurrent_streams():
    """Two FL and two RL codecs on four streams at once: the persistent grids
    compete for the CUs (workgroups dispatched late find every tile taken);
    every output must still equal the one from a serial run."""
    from flrl.device import FLDevice, RLDevice, gen
    sizes = [(48 << 20) + 5, (40 << 20) + 131, (32 << 20) + 7, (24 << 20) + 9]
    xs = [gen(k, n, 11 + i) for i, (k, n) in enumerate(zip(["u8", "lo4", "u8", "zero"], sizes))]
    fl = [FLDevice(sizes[0]), FLDevice(sizes[1])]
    rl = [RLDevice(sizes[2]), RLDevice(sizes[3])]
    ref = []
    for d, x in zip(fl, xs[:2]):
        d.encode(x)
        v = d.values_size()
        ref.append((v, d.bits[: d.frames].clone(), d.values[:v].clone()))
    for r, x in zip(rl, xs[2:]):
        r.encode(x)
        R = r.runs()
        ref.append((R, r.counts[:R].clone(), r.values[:R].clone()))
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(4)]
    for rep in range(5):
        for t in (fl[0].out, fl[1].out, rl[0].out, rl[1].out):
            t.zero_()
        torch.cuda.synchronize()
        for i in range(2):
            fl[i].encode(xs[i], stream=streams[i])
            fl[i].decode(ref[i][0], stream=streams[i])
            rl[i].encode(xs[2 + i], stream=streams[2 + i])
            rl[i].decode(ref[2 + i][0], stream=streams[2 + i])
        torch.cuda.synchronize()
        for i in range(2):
            v, b0, v0 = ref[i]
            assert fl[i].error() == 0 and fl[i].values_size() == v, (rep, i)
            assert torch.equal(fl[i].bits[: fl[i].frames], b0) and torch.equal(fl[i].values[:v], v0), (rep, i)
            assert torch.equal(fl[i].out[: sizes[i]], xs[i][: sizes[i]]), (rep, i)
            R, c0, rv0 = ref[2 + i]
            assert rl[i].error() == 0 and rl[i].runs() == R, (rep, i)
            assert torch.equal(rl[i].counts[:R], c0) and torch.equal(rl[i].values[:R], rv0), (rep, i)
            assert torch.equal(rl[i].out[: sizes[2 + i]], xs[2 + i][: sizes[2 + i]]), (rep, i)

