"""Pin the CPU oracle to the reference's golden vectors.

The oracle (oracle/flrl_oracle.c) is the checker every GPU parity test uses, so
it is itself checked here against outputs of the reference's own fl-cpu path:
known-answer tests, sha256 of generated inputs (pins the generator) and of the
.fl files (pins codec + container), and the BMP example input.
"""
import hashlib

import numpy as np
import pytest

import oracle
from conftest import kat_input


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def test_clz8_matches_reference_definition():
    # fl_common.cuh:198-212: clz8(0) = 8; else leading zeros of an 8-bit value
    for v in range(256):
        expect = 8 if v == 0 else 8 - v.bit_length()
        assert oracle.clz8(v) == expect


def test_fl_kats(golden):
    for case in golden["fl_kat"]:
        data = kat_input(case)
        bits, values = oracle.fl_compress(np.frombuffer(data, np.uint8))
        assert bits.tobytes().hex() == case["bits_hex"], case["name"]
        assert values.tobytes().hex() == case["values_hex"], case["name"]
        back = oracle.fl_decompress(len(data), bits, values)
        assert back.tobytes() == data


def test_fl_plan_example_frame3():
    """The one reference-held FL vector (IMPLEMENTATION-PLAN.md:9-27): at frame
    length 3, input [0,2,1,5,5,7,10,1,13] has outputBits [2,3,4] and
    frameStartIndices [0,6,15]; outputValues is ceil((15 + 3*4)/8) = 4 bytes
    whose fields, read at bitsOffset = start[f] + k*b (plan :35-40), are the
    plan's binary strings 00_10_01---101_101_111---1010_0001_1101."""
    data = np.array([0, 2, 1, 5, 5, 7, 10, 1, 13], np.uint8)
    bits, starts, total = oracle.fl_widths_frame(data, 3)
    assert bits.tolist() == [2, 3, 4]
    assert starts.tolist() == [0, 6, 15]
    assert total == 27
    b2, values = oracle.fl_compress_frame(data, 3)
    assert b2.tolist() == [2, 3, 4] and values.size == 4
    stream = int.from_bytes(values.tobytes(), "little")
    fields = []
    for i in range(data.size):
        f, k = divmod(i, 3)
        off = int(starts[f]) + k * int(bits[f])
        fields.append(format((stream >> off) & ((1 << int(bits[f])) - 1), f"0{bits[f]}b"))
    rendered = "---".join("_".join(fields[3 * f:3 * f + 3]) for f in range(3))
    assert rendered == "00_10_01---101_101_111---1010_0001_1101"
    assert oracle.fl_decompress_frame(data.size, 3, bits, values).tolist() == data.tolist()
    # at the reference's frame length the same input is one frame of width 4
    b128, _ = oracle.fl_compress(data)
    assert b128.tolist() == [4]


def test_fl_frame_length_generic_matches_128():
    """orc_fl_compress is the frame-length-generic restatement at 128."""
    a = oracle.gen("lo4", 100_003, 9)
    a[::997] = 0xFF
    bits, values = oracle.fl_compress(a)
    b2, v2 = oracle.fl_compress_frame(a, 128)
    assert np.array_equal(bits, b2) and np.array_equal(values, v2)
    for L in (1, 3, 7, 200):
        b, v = oracle.fl_compress_frame(a, L)
        assert np.array_equal(oracle.fl_decompress_frame(a.size, L, b, v), a)


def test_fl_empty_file(golden):
    blob = oracle.fl_file_bytes(np.zeros(0, np.uint8))
    assert blob == bytes(24)
    assert sha(blob) == golden["fl_empty_file_sha256"]
    assert oracle.fl_decompress(0, np.zeros(0, np.uint8), np.zeros(0, np.uint8)).size == 0


def test_fl_bmp(golden, bmp_bytes):
    g = golden["fl_bmp"]
    assert sha(bmp_bytes) == g["input_sha256"]
    a = np.frombuffer(bmp_bytes, np.uint8)
    blob = oracle.fl_file_bytes(a)
    assert len(blob) == g["fl_bytes"]
    assert sha(blob) == g["fl_sha256"]
    bits, values = oracle.fl_compress(a)
    assert bits.size == g["frames"] and values.size == g["values_size"]
    hist = {str(k): int(v) for k, v in zip(*np.unique(bits, return_counts=True))}
    assert hist == g["width_hist"]
    assert oracle.fl_decompress(a.size, bits, values).tobytes() == bmp_bytes


@pytest.mark.parametrize("idx", range(7))
def test_fl_generated(golden, idx):
    g = golden["fl_generated"][idx]
    a = oracle.gen(g["kind"], g["n"], g["seed"])
    assert sha(a) == g["input_sha256"], "generator drifted from SURVEY.md §8(d)"
    blob = oracle.fl_file_bytes(a)
    assert len(blob) == g["fl_bytes"]
    assert sha(blob) == g["fl_sha256"]
    bits, values = oracle.fl_compress(a)
    assert np.array_equal(oracle.fl_decompress(a.size, bits, values), a)


def test_generator_word_offset_shards():
    # counter-based kinds: a shard starting at byte 8k equals bytes [8k, ...) of the whole
    whole = oracle.gen("u8", 4096, 42)
    for k in (0, 1, 17, 300):
        part = oracle.gen("u8", 1000, 42, word_offset=k)
        assert np.array_equal(part, whole[8 * k: 8 * k + 1000])


@pytest.mark.parametrize("n", [0, 1, 7, 8, 127, 128, 129, 255, 256, 1000, 4096, 4741, 100003])
@pytest.mark.parametrize("kind", ["u8", "lo4", "zero", "ff"])
def test_fl_roundtrip_edges(n, kind):
    a = np.full(n, 255, np.uint8) if kind == "ff" else oracle.gen(kind, n, 3)
    bits, values = oracle.fl_compress(a)
    assert bits.size == (n + 127) // 128
    if n == 0:
        assert values.size == 0
        return
    if kind == "zero":
        assert set(bits.tolist()) == {1}  # b >= 1 even for all-zero frames
    if kind == "ff":
        assert values.size == n
    assert np.array_equal(oracle.fl_decompress(n, bits, values), a)


def test_fl_shard_concat_identity():
    # 128-aligned shard outputs concatenate to the whole output
    a = oracle.gen("lo4", 50_000, 9)
    a[::977] = 200  # mixed widths
    bits, values = oracle.fl_compress(a)
    for cut in (128, 128 * 7, 128 * 300):
        b1, v1 = oracle.fl_compress(a[:cut])
        b2, v2 = oracle.fl_compress(a[cut:])
        assert np.array_equal(np.concatenate([b1, b2]), bits)
        assert np.array_equal(np.concatenate([v1, v2]), values)


def test_rl_kats(golden):
    for case in golden["rl_kat"]:
        data = np.frombuffer(kat_input(case), np.uint8)
        counts, values = oracle.rl_compress(data)
        assert counts.tolist() == case["counts"], case["name"]
        assert values.tolist() == case["values"], case["name"]
        assert np.array_equal(oracle.rl_decompress(counts, values, data.size), data)


@pytest.mark.parametrize("kind", ["runs32", "longruns", "u8", "zero"])
def test_rl_roundtrip(kind):
    a = oracle.gen(kind, 70_001, 5)
    counts, values = oracle.rl_compress(a)
    assert counts.min() >= 1 and counts.max() <= 255
    assert int(counts.astype(np.int64).sum()) == a.size
    assert np.array_equal(oracle.rl_decompress(counts, values, a.size), a)
    if kind == "zero":
        assert counts.tolist() == [255] * (a.size // 255) + [a.size % 255]


def test_rl_split_boundaries():
    for L in (254, 255, 256, 509, 510, 511, 765, 766):
        a = np.concatenate([np.full(L, 3, np.uint8), np.full(3, 4, np.uint8)])
        counts, values = oracle.rl_compress(a)
        expect = [255] * (L // 255) + ([L % 255] if L % 255 else []) + [3]
        assert counts.tolist() == expect
