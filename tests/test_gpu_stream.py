"""Streamed FL file codec (flrl_fl_compress_file / flrl_fl_decompress_file, the
CLI's GPU FL path) against the oracle.

Frame-aligned chunks through several pipelines must give the same file as the
whole-input oracle encode (the concatenation identity):
chunk sizes from one frame up, more workers than GPUs (so the multi-worker
ordering logic runs on a 1-GPU box), ragged tails, the empty file, and the
reference's BMP through the CLI. Decompression must reject malformed files."""
import hashlib
import os
import struct
import subprocess

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

flrl = pytest.importorskip("flrl")


def _oracle_file(data: np.ndarray) -> bytes:
    return oracle.fl_file_bytes(data)


def _input(kind: str, n: int, seed: int = 7) -> np.ndarray:
    if kind == "mixed":
        a = oracle.gen("lo4", n, seed)
        a[::997] = 0xE1  # every width appears
        a[5000:9000] = 0
        return a
    return oracle.gen(kind, n, seed)


@pytest.mark.parametrize("n", [1, 127, 128, 129, 4096 * 3 + 17, (5 << 20) + 77])
@pytest.mark.parametrize("chunk,workers", [(128, 1), (4096, 3), (1 << 20, 2), (0, 1)])
def test_compress_file_matches_oracle(tmp_path, n, chunk, workers):
    if chunk == 128 and n > 100_000:
        pytest.skip("one-frame chunks: small inputs only (one H2D per 128 bytes)")
    data = _input("mixed", n)
    src, dst, back = tmp_path / "in", tmp_path / "out.fl", tmp_path / "back"
    data.tofile(src)
    flrl.fl_compress_file(str(src), str(dst), workers, chunk)
    assert dst.read_bytes() == _oracle_file(data)
    flrl.fl_decompress_file(str(dst), str(back), workers, chunk)
    assert back.read_bytes() == data.tobytes()


@pytest.mark.parametrize("kind", ["u8", "lo4", "runs32", "zero"])
def test_file_round_trip_kinds(tmp_path, kind):
    n = (24 << 20) + 333
    data = _input(kind, n, 11)
    src, dst, back = tmp_path / "in", tmp_path / "out.fl", tmp_path / "back"
    data.tofile(src)
    flrl.fl_compress_file(str(src), str(dst), 4, 5 << 20)
    assert hashlib.sha256(dst.read_bytes()).hexdigest() == hashlib.sha256(_oracle_file(data)).hexdigest()
    flrl.fl_decompress_file(str(dst), str(back), 3, 3 << 20)
    assert back.read_bytes() == data.tobytes()


def test_empty_file(tmp_path):
    src, dst, back = tmp_path / "in", tmp_path / "out.fl", tmp_path / "back"
    src.write_bytes(b"")
    flrl.fl_compress_file(str(src), str(dst), 2, 0)
    assert dst.read_bytes() == bytes(24)  # empty input -> 24 zero bytes
    flrl.fl_decompress_file(str(dst), str(back), 2, 0)
    assert back.read_bytes() == b""


def test_decode_chunking_independent_of_encode(tmp_path):
    data = _input("mixed", (3 << 20) + 5, 3)
    src, dst = tmp_path / "in", tmp_path / "out.fl"
    data.tofile(src)
    flrl.fl_compress_file(str(src), str(dst), 1, 1 << 20)
    for chunk, workers in ((128 * 7, 2), (1 << 16, 5), (0, 1)):
        back = tmp_path / f"back{chunk}"
        flrl.fl_decompress_file(str(dst), str(back), workers, chunk)
        assert back.read_bytes() == data.tobytes()


def _bad(tmp_path, blob: bytes, name: str):
    p = tmp_path / name
    p.write_bytes(blob)
    with pytest.raises(flrl.FLRLError) as e:
        flrl.fl_decompress_file(str(p), str(tmp_path / (name + ".out")), 2, 4096)
    return e.value


def test_malformed_files_rejected(tmp_path):
    data = _input("mixed", 10_000, 5)
    good = _oracle_file(data)
    n, F, V = struct.unpack_from("<QQQ", good)
    body = good[24:]
    assert _bad(tmp_path, good[:20], "short").code == 4
    assert _bad(tmp_path, struct.pack("<QQQ", n, F + 1, V) + body, "bits").code == 4
    assert _bad(tmp_path, struct.pack("<QQQ", n, F, V + 1) + body, "vals").code == 4
    assert _bad(tmp_path, good[:-1], "trunc").code == 4
    for w in (0, 9):
        b = bytearray(good)
        b[24 + 3] = w
        assert _bad(tmp_path, bytes(b), f"w{w}").code == 4
    # widths consistent with F but values one frame short: sizes disagree
    b = bytearray(good)
    b[24] = b[24] + 1 if b[24] < 8 else b[24] - 1
    assert _bad(tmp_path, bytes(b), "sum").code == 4


def test_missing_input(tmp_path):
    with pytest.raises(flrl.FLRLError):
        flrl.fl_compress_file(str(tmp_path / "nope"), str(tmp_path / "o"), 1, 0)


def test_cli_streamed_bmp(golden, bmp_bytes, cli_path, tmp_path):
    src = tmp_path / "in.bmp"
    src.write_bytes(bmp_bytes)
    env = dict(os.environ, FLRL_CHUNK_BYTES=str(128 * 1000), FLRL_WORKERS="3")
    for method in ("fl", "fl-nccl"):
        out, back = tmp_path / f"{method}.fl", tmp_path / f"{method}.bmp"
        r = subprocess.run([cli_path, "c", method, str(src), str(out)], env=env,
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        assert "[TIMER]" in r.stdout
        assert hashlib.sha256(out.read_bytes()).hexdigest() == golden["fl_bmp"]["fl_sha256"]
        r = subprocess.run([cli_path, "d", method, str(out), str(back)], env=env,
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        assert back.read_bytes() == bmp_bytes


def test_cli_streamed_error_removes_output(cli_path, tmp_path):
    bad = tmp_path / "bad.fl"
    bad.write_bytes(struct.pack("<QQQ", 1000, 3, 5) + bytes(8))
    out = tmp_path / "out"
    r = subprocess.run([cli_path, "d", "fl", str(bad), str(out)], capture_output=True, text=True)
    assert r.returncode == 2 and "[ERROR]" in r.stderr
    assert not out.exists()


@pytest.mark.parametrize("method", ["fl", "rl"])
def test_cli_streamed_read_failure_reported(cli_path, tmp_path, method):
    """A worker's read failure must wake the in-order writer and surface as an
    error (it used to leave the writer waiting forever). A directory opens and
    stats fine but every pread fails (EISDIR)."""
    src = tmp_path / "dir"
    src.mkdir()
    if os.stat(src).st_size == 0:
        pytest.skip("directory size 0 on this filesystem: no chunk to read")
    out = tmp_path / "out"
    env = dict(os.environ, FLRL_CHUNK_BYTES=str(128 * 8), FLRL_WORKERS="2")
    r = subprocess.run([cli_path, "c", method, str(src), str(out)], env=env, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode != 0 and "[ERROR]" in r.stderr, (r.returncode, r.stderr)
    assert "Cannot read file content" in r.stderr


def test_large_file_default_chunks(tmp_path):
    n = (300 << 20) + 4097  # 5 default 64 MiB chunks, ragged tail
    data = oracle.gen("u8", n, 42)
    src, dst, back = tmp_path / "in", tmp_path / "out.fl", tmp_path / "back"
    data.tofile(src)
    flrl.fl_compress_file(str(src), str(dst), 0, 0)
    bits, values = oracle.fl_compress(data)
    blob = dst.read_bytes()
    assert blob[:24] == struct.pack("<QQQ", n, bits.size, values.size)
    assert blob[24:24 + bits.size] == bits.tobytes()
    assert blob[24 + bits.size:] == values.tobytes()
    del blob
    flrl.fl_decompress_file(str(dst), str(back), 2, 0)
    assert back.read_bytes() == data.tobytes()


# ---- RL file path -------------------------------------------------------------

def _oracle_rl_file(data: np.ndarray) -> bytes:
    counts, values = oracle.rl_compress(data)
    return flrl.rl_file_bytes(data.size, counts, values)


def _rl_input(kind: str, n: int, seed: int = 9) -> np.ndarray:
    if kind == "spans":  # runs far longer than a chunk, some exact multiples of 255
        a = np.zeros(n, np.uint8)
        a[n // 3:] = 7
        a[n // 3 + 255 * 40: n // 3 + 255 * 80] = 9
        a[-1] = 1
        return a
    return oracle.gen(kind, n, seed)


@pytest.mark.parametrize("kind,n", [("runs32", 1), ("runs32", 255), ("runs32", 256), ("runs32", 100_003),
                                    ("longruns", 300_007), ("zero", 70_000), ("u8", 65_537),
                                    ("spans", 200_000)])
@pytest.mark.parametrize("chunk,workers", [(1000, 3), (4096, 1), (65536, 2), (0, 1)])
def test_rl_compress_file_matches_oracle(tmp_path, kind, n, chunk, workers):
    data = _rl_input(kind, n)
    src, dst, back = tmp_path / "in", tmp_path / "out.rl", tmp_path / "back"
    data.tofile(src)
    flrl.rl_compress_file(str(src), str(dst), workers, chunk)
    assert dst.read_bytes() == _oracle_rl_file(data)
    flrl.rl_decompress_file(str(dst), str(back), workers, chunk)
    assert back.read_bytes() == data.tobytes()


def test_rl_file_empty_and_one_chunk_per_byte(tmp_path):
    src, dst, back = tmp_path / "in", tmp_path / "out.rl", tmp_path / "back"
    src.write_bytes(b"")
    flrl.rl_compress_file(str(src), str(dst), 2, 0)
    assert dst.read_bytes() == bytes(16)
    flrl.rl_decompress_file(str(dst), str(back), 2, 0)
    assert back.read_bytes() == b""
    data = _rl_input("spans", 3000)
    data.tofile(src)
    flrl.rl_compress_file(str(src), str(dst), 3, 1)  # every byte its own chunk
    assert dst.read_bytes() == _oracle_rl_file(data)


def test_rl_file_large_default_chunks(tmp_path):
    n = (200 << 20) + 12345
    data = oracle.gen("runs32", n, 42)
    src, dst, back = tmp_path / "in", tmp_path / "out.rl", tmp_path / "back"
    data.tofile(src)
    flrl.rl_compress_file(str(src), str(dst), 2, 0)
    assert hashlib.sha256(dst.read_bytes()).digest() == hashlib.sha256(_oracle_rl_file(data)).digest()
    flrl.rl_decompress_file(str(dst), str(back), 3, 0)
    assert back.read_bytes() == data.tobytes()


def test_rl_malformed_files_rejected(tmp_path):
    data = _rl_input("runs32", 5000)
    good = _oracle_rl_file(data)
    n, R = struct.unpack_from("<QQ", good)

    def bad(blob, name):
        p = tmp_path / name
        p.write_bytes(blob)
        with pytest.raises(flrl.FLRLError) as e:
            flrl.rl_decompress_file(str(p), str(tmp_path / (name + ".out")), 2, 1024)
        return e.value.code

    assert bad(good[:10], "short") == 4
    assert bad(good[:-1], "trunc") == 4
    assert bad(struct.pack("<QQ", n + 1, R) + good[16:], "sum") == 4
    b = bytearray(good)
    b[16 + 5] = 0
    assert bad(bytes(b), "zero") == 4


def test_cli_rl_streamed(cli_path, tmp_path):
    data = _rl_input("longruns", 400_001, 3)
    src = tmp_path / "in"
    data.tofile(src)
    ref = tmp_path / "ref.rl"
    subprocess.run([cli_path, "c", "rl-cpu", str(src), str(ref)], check=True, capture_output=True)
    env = dict(os.environ, FLRL_CHUNK_BYTES="777", FLRL_WORKERS="3")
    out, back = tmp_path / "o.rl", tmp_path / "back"
    r = subprocess.run([cli_path, "c", "rl", str(src), str(out)], env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert out.read_bytes() == ref.read_bytes()
    r = subprocess.run([cli_path, "d", "rl", str(out), str(back)], env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert back.read_bytes() == data.tobytes()


@pytest.mark.parametrize("op", ["fl_c", "fl_d", "rl_c", "rl_d"])
@pytest.mark.parametrize("fail_at", [0, 5, 37])
def test_injected_chunk_failure(tmp_path, op, fail_at):
    """One pipeline fails (flrl_debug_fail_chunk) while the others and the
    in-order writer are busy: the call raises, frees every pinned buffer only
    after the writer has let go of it, and leaves an existing output alone."""
    n = (48 << 20) + 99
    data = _input("mixed", n, 4)
    src, enc, out = tmp_path / "in", tmp_path / "enc", tmp_path / "out"
    data.tofile(src)
    chunk = 1 << 20
    if op == "fl_d":
        flrl.fl_compress_file(str(src), str(enc), 2, chunk)
    elif op == "rl_d":
        flrl.rl_compress_file(str(src), str(enc), 2, chunk)
    out.write_bytes(b"keep me")
    fn, arg = {"fl_c": (flrl.fl_compress_file, src), "fl_d": (flrl.fl_decompress_file, enc),
               "rl_c": (flrl.rl_compress_file, src), "rl_d": (flrl.rl_decompress_file, enc)}[op]
    flrl.debug_fail_chunk(fail_at)
    try:
        with pytest.raises(flrl.FLRLError) as e:
            fn(str(arg), str(out), 4, chunk)
        assert "injected" in str(e.value)
    finally:
        flrl.debug_fail_chunk(-1)
    assert out.read_bytes() == b"keep me"
    assert sorted(p.name for p in tmp_path.iterdir()) == sorted(
        ["in", "out"] + (["enc"] if op.endswith("_d") else []))
    fn(str(arg), str(out), 4, chunk)  # and the next call works
    if op == "fl_c":
        assert out.read_bytes() == _oracle_file(data)
    elif op.endswith("_d"):
        assert out.read_bytes() == data.tobytes()


@pytest.mark.parametrize("method", ["fl", "fl-nccl", "rl"])
def test_cli_streamed_in_place(cli_path, tmp_path, method):
    """`compress c <m> f f` / `compress d <m> f f` (the streamed GPU paths read
    the input while writing: the output goes to a temporary renamed into place)."""
    data = _input("mixed", (3 << 20) + 11, 8)
    f = tmp_path / "f"
    f.write_bytes(data.tobytes())
    env = dict(os.environ, FLRL_CHUNK_BYTES=str(1 << 20), FLRL_WORKERS="2")
    for op in ("c", "d"):
        r = subprocess.run([cli_path, op, method, str(f), str(f)], env=env, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        if op == "c" and method != "rl":
            assert f.read_bytes() == _oracle_file(data)
    assert f.read_bytes() == data.tobytes()
    assert [p.name for p in tmp_path.iterdir()] == ["f"]


def test_cli_streamed_error_keeps_existing_output(cli_path, tmp_path):
    bad = tmp_path / "bad.fl"
    bad.write_bytes(struct.pack("<QQQ", 1000, 3, 5) + bytes(8))
    out = tmp_path / "out"
    out.write_bytes(b"old")
    for argv in (["d", "fl", str(bad), str(out)], ["c", "fl", str(tmp_path / "missing"), str(out)],
                 ["c", "rl", str(tmp_path / "missing"), str(out)]):
        r = subprocess.run([cli_path, *argv], capture_output=True, text=True)
        assert r.returncode == 2 and "[ERROR]" in r.stderr
        assert out.read_bytes() == b"old"
    assert sorted(p.name for p in tmp_path.iterdir()) == ["bad.fl", "out"]


@pytest.fixture
def ro_dir(tmp_path):
    """A read-only directory (mode 0555) holding a writable existing output
    'out'; OutFile can create no temporary there and writes in place. Root
    ignores directory permissions, so the case only exists for other users
    (the GPU box runs tests as an ordinary user)."""
    if os.geteuid() == 0:
        pytest.skip("root bypasses directory permissions")
    d = tmp_path / "ro"
    d.mkdir()
    out = d / "out"
    out.write_bytes(b"old")
    out.chmod(0o666)
    d.chmod(0o555)
    yield d
    d.chmod(0o755)


@pytest.mark.parametrize("method", ["fl", "rl"])
def test_cli_read_only_dir_in_place(cli_path, tmp_path, ro_dir, method):
    """the RL side file used to be created next to the output after
    the output was truncated in place, so `c rl` into a read-only directory
    destroyed the existing output and failed. It now falls back to $TMPDIR and
    is created first: both methods succeed and round-trip."""
    data = _input("mixed", (2 << 20) + 5, 12)
    src, back = tmp_path / "in", tmp_path / "back"
    data.tofile(src)
    env = dict(os.environ, FLRL_CHUNK_BYTES=str(1 << 19), FLRL_WORKERS="2", TMPDIR=str(tmp_path))
    out = ro_dir / "out"
    r = subprocess.run([cli_path, "c", method, str(src), str(out)], env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    if method == "fl":
        assert out.read_bytes() == _oracle_file(data)
    r = subprocess.run([cli_path, "d", method, str(out), str(back)], env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert back.read_bytes() == data.tobytes()
    assert [p.name for p in ro_dir.iterdir()] == ["out"]


def test_cli_read_only_dir_failures(cli_path, tmp_path, ro_dir):
    """Failures before the in-place open leave the output alone: a missing
    input, and the output being the input (never truncated while read). A
    failure after it leaves the output truncated or partial, as documented in
    flrl_outfile.hpp (the reference's fopen "wb" does the same)."""
    out = ro_dir / "out"
    for m in ("fl", "rl"):
        r = subprocess.run([cli_path, "c", m, str(tmp_path / "missing"), str(out)], capture_output=True, text=True)
        assert r.returncode == 2 and "[ERROR]" in r.stderr
        assert out.read_bytes() == b"old"
        r = subprocess.run([cli_path, "c", m, str(out), str(out)], capture_output=True, text=True)
        assert r.returncode == 2 and "[ERROR]" in r.stderr
        assert out.read_bytes() == b"old"
    data = _input("mixed", (3 << 20) + 1, 13)
    src = tmp_path / "in"
    data.tofile(src)
    flrl.debug_fail_chunk(1)
    try:
        with pytest.raises(flrl.FLRLError):
            flrl.rl_compress_file(str(src), str(out), 2, 1 << 20)
    finally:
        flrl.debug_fail_chunk(-1)
    assert out.read_bytes() != b"old"  # truncated at open: the documented exception
    flrl.rl_compress_file(str(src), str(out), 2, 1 << 20)  # and the next call works
    back = tmp_path / "back"
    flrl.rl_decompress_file(str(out), str(back), 2, 1 << 20)
    assert back.read_bytes() == data.tobytes()
    assert [p.name for p in ro_dir.iterdir()] == ["out"]


def test_alternating_host_calls_keep_their_staging():
    """the idle-pool cap (1 GiB) was just below one compress set
    plus one decompress set of all 8 pipelines (~1028 MiB), so every call of an
    alternating compress/decompress loop evicted and re-allocated a 64 MiB set.
    With the cap sized from the sets, the idle pool holds all 16 afterwards."""
    import flrl
    a = oracle.gen("lo4", (128 << 20) + 3, 21)  # 9 chunks: every pipeline busy
    flrl.release_staging()
    for _ in range(3):
        c = flrl.fl_compress(a)
        assert np.array_equal(flrl.fl_decompress(a.size, c.bits, c.values), a)
    freed = flrl.release_staging()
    # 2 directions x 8 pipelines x 2 slots x (two 16 MiB buffers + the bits)
    assert freed >= 2 * 8 * 2 * (32 << 20), freed


def test_alternating_file_calls_keep_larger_staging(tmp_path):
    """the file APIs take workers and chunk sizes at run time; with
    more pipelines or larger chunks than the host API's 8 x 16 MiB, the fixed
    idle-pool cap evicted and re-allocated pinned sets on every alternating
    compress/decompress call. The cap now grows to both directions of the
    largest shape leased, so the idle pool keeps them all."""
    import flrl
    W, C = 12, 24 << 20
    a = oracle.gen("lo4", W * C + 5, 23)
    src, enc, back = tmp_path / "in", tmp_path / "enc", tmp_path / "back"
    src.write_bytes(a.tobytes())
    flrl.release_staging()
    for _ in range(2):
        flrl.fl_compress_file(str(src), str(enc), W, C)
        flrl.fl_decompress_file(str(enc), str(back), W, C)
    assert back.read_bytes() == a.tobytes()
    freed = flrl.release_staging()
    # both directions x W pipelines x 2 slots x (two C-byte buffers at least)
    assert freed >= 2 * W * 2 * (2 * C), freed


def test_large_file_staging_leaves_the_pool_after_smaller_calls(tmp_path):
    """the idle-pool cap used to grow to twice the largest lease
    ever seen and never shrink, so one call with many pipelines or large
    chunks kept that much pinned host memory idle for the rest of the process.
    The cap now follows the last few busy periods only: after a large file call
    and a handful of host-API calls the idle pool is back within the host API's
    own bound (8 pipelines x 2 directions of 16 MiB-chunk sets + 64 MiB)."""
    import flrl
    W, C = 12, 32 << 20
    a = oracle.gen("lo4", W * C + 5, 29)
    src, enc, back = tmp_path / "in", tmp_path / "enc", tmp_path / "back"
    src.write_bytes(a.tobytes())
    flrl.release_staging()
    flrl.fl_compress_file(str(src), str(enc), W, C)
    flrl.fl_decompress_file(str(enc), str(back), W, C)
    assert back.read_bytes() == a.tobytes()
    small = oracle.gen("lo4", (128 << 20) + 3, 21)
    for _ in range(3):
        c = flrl.fl_compress(small)
        assert np.array_equal(flrl.fl_decompress(small.size, c.bits, c.values), small)
    freed = flrl.release_staging()
    host_bound = 2 * 8 * 2 * (2 * (16 << 20) + (16 << 20) // 128 + 16) + (64 << 20)
    assert 2 * 8 * 2 * (32 << 20) <= freed <= host_bound, freed


def test_release_staging_frees_idle_sets():
    """The host API keeps its pinned staging between calls (bounded); releasing
    it frees the idle sets, and the next call allocates afresh."""
    import flrl
    rng = np.random.default_rng(9)
    a = (rng.integers(0, 256, size=(40 << 20) + 77) >> 3).astype(np.uint8)
    ref_bits, ref_vals = oracle.fl_compress(a[:1 << 20])
    flrl.release_staging()
    c = flrl.fl_compress(a)
    assert np.array_equal(flrl.fl_decompress(a.size, c.bits, c.values), a)
    freed = flrl.release_staging()
    # 8 pipelines x 2 slots of (16 MiB in + 128 KiB bits + 16 MiB values) per direction,
    # as many pipelines as there are chunks (3 of 16 MiB here)
    assert freed >= 2 * 3 * 2 * (16 << 20)
    assert flrl.release_staging() == 0
    c2 = flrl.fl_compress(a[:1 << 20])
    assert np.array_equal(c2.bits, ref_bits) and np.array_equal(c2.values, ref_vals)
