"""oracle — ctypes access to the CPU restatement of the reference codec.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the parity checker / CPU baseline; never by the
product path (libflrl.so, the CLI, the flrl Python binding).

FL is pinned by the plan's frame-length-3 example (IMPLEMENTATION-PLAN.md:9-13)
and checked against the golden vectors of SURVEY.md §8(c) (tests/golden/), which
came from a stand-in build of fl-cpu and corroborate without pinning (FL parity
partially unpinned beyond the plan example); RL has no reference implementation
and is pinned only by IMPLEMENTATION-PLAN.md's worked examples (RL parity
partially unpinned).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

KINDS = {"u8": 0, "lo4": 1, "zero": 2, "runs32": 3, "longruns": 4}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


if not os.path.exists(LIB_PATH):
    build()

_lib = ctypes.CDLL(LIB_PATH)
_vp, _sz = ctypes.c_void_p, ctypes.c_size_t
_lib.orc_fl_frames.restype = _sz
_lib.orc_fl_frames.argtypes = [_sz]
_lib.orc_fl_compress.restype = _sz
_lib.orc_fl_compress.argtypes = [_vp, _sz, _vp, _vp]
_lib.orc_fl_decompress.restype = _sz
_lib.orc_fl_decompress.argtypes = [_sz, _vp, _sz, _vp, _sz, _vp]
_lib.orc_rl_compress.restype = _sz
_lib.orc_rl_compress.argtypes = [_vp, _sz, _vp, _vp]
_lib.orc_rl_decompress.restype = _sz
_lib.orc_rl_decompress.argtypes = [_vp, _vp, _sz, _vp, _sz]
_lib.orc_fl_widths_frame.restype = _sz
_lib.orc_fl_widths_frame.argtypes = [_vp, _sz, _sz, _vp]
_lib.orc_fl_frame_starts.restype = None
_lib.orc_fl_frame_starts.argtypes = [_vp, _sz, _sz, _vp]
_lib.orc_fl_compress_frame.restype = _sz
_lib.orc_fl_compress_frame.argtypes = [_vp, _sz, _sz, _vp, _vp]
_lib.orc_fl_decompress_frame.restype = _sz
_lib.orc_fl_decompress_frame.argtypes = [_sz, _sz, _vp, _sz, _vp, _sz, _vp]
_lib.orc_gen.restype = ctypes.c_int
_lib.orc_gen.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, _vp, _sz]
_lib.orc_clz8.restype = ctypes.c_uint8
_lib.orc_clz8.argtypes = [ctypes.c_uint8]


def _ptr(a: np.ndarray):
    return a.ctypes.data if a.size else None


def gen(kind: str, n: int, seed: int, word_offset: int = 0) -> np.ndarray:
    """SURVEY.md §8(d) synthetic input."""
    a = np.zeros(n, dtype=np.uint8)
    rc = _lib.orc_gen(KINDS[kind], seed, word_offset, _ptr(a), n)
    if rc:
        raise ValueError(f"orc_gen({kind}) failed")
    return a


def clz8(v: int) -> int:
    return int(_lib.orc_clz8(v))


def fl_compress(data) -> tuple[np.ndarray, np.ndarray]:
    """cpuCompress (src/fl/fl_cpu.cu:9-90) -> (bits, values)."""
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8).reshape(-1)
    n = a.size
    bits = np.zeros(_lib.orc_fl_frames(n), dtype=np.uint8)
    values = np.zeros(max(n, 1), dtype=np.uint8)
    v = _lib.orc_fl_compress(_ptr(a), n, _ptr(bits), values.ctypes.data)
    return bits, values[:v].copy()


def fl_widths_frame(data, frame_len: int) -> tuple[np.ndarray, np.ndarray, int]:
    """Width pass + frameStartIndices at any frame length (IMPLEMENTATION-PLAN.md:9-29)
    -> (bits, starts, total_bits)."""
    a = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    frames = (a.size + frame_len - 1) // frame_len
    bits = np.zeros(max(frames, 1), dtype=np.uint8)
    total = _lib.orc_fl_widths_frame(_ptr(a), a.size, frame_len, bits.ctypes.data)
    starts = np.zeros(max(frames, 1), dtype=np.uint64)
    _lib.orc_fl_frame_starts(bits.ctypes.data, frames, frame_len, starts.ctypes.data)
    return bits[:frames].copy(), starts[:frames].copy(), int(total)


def fl_compress_frame(data, frame_len: int) -> tuple[np.ndarray, np.ndarray]:
    """cpuCompress at any frame length -> (bits, values)."""
    a = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    frames = (a.size + frame_len - 1) // frame_len
    bits = np.zeros(max(frames, 1), dtype=np.uint8)
    values = np.zeros(max(a.size, 1), dtype=np.uint8)
    v = _lib.orc_fl_compress_frame(_ptr(a), a.size, frame_len, bits.ctypes.data, values.ctypes.data)
    return bits[:frames].copy(), values[:v].copy()


def fl_decompress_frame(output_size: int, frame_len: int, bits, values) -> np.ndarray:
    """cpuDecompress at any frame length."""
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    values = np.ascontiguousarray(values, dtype=np.uint8)
    out = np.zeros(max(output_size, 1), dtype=np.uint8)
    got = _lib.orc_fl_decompress_frame(output_size, frame_len, _ptr(bits), bits.size, _ptr(values),
                                       values.size, out.ctypes.data)
    return out[:got].copy()


def fl_decompress(output_size: int, bits: np.ndarray, values: np.ndarray) -> np.ndarray:
    """cpuDecompress (src/fl/fl_cpu.cu:92-147); empty on the reference's early-out."""
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    values = np.ascontiguousarray(values, dtype=np.uint8)
    out = np.zeros(max(output_size, 1), dtype=np.uint8)
    got = _lib.orc_fl_decompress(output_size, _ptr(bits), bits.size, _ptr(values), values.size,
                                 out.ctypes.data)
    return out[:got].copy()


def rl_compress(data) -> tuple[np.ndarray, np.ndarray]:
    a = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    n = a.size
    counts = np.zeros(max(n, 1), dtype=np.uint8)
    values = np.zeros(max(n, 1), dtype=np.uint8)
    r = _lib.orc_rl_compress(_ptr(a), n, counts.ctypes.data, values.ctypes.data)
    return counts[:r].copy(), values[:r].copy()


def rl_decompress(counts: np.ndarray, values: np.ndarray, out_cap: int) -> np.ndarray:
    counts = np.ascontiguousarray(counts, dtype=np.uint8)
    values = np.ascontiguousarray(values, dtype=np.uint8)
    out = np.zeros(max(out_cap, 1), dtype=np.uint8)
    got = _lib.orc_rl_decompress(_ptr(counts), _ptr(values), counts.size, out.ctypes.data, out_cap)
    if got == ctypes.c_size_t(-1).value:
        raise ValueError("RL counts exceed output capacity")
    return out[:got].copy()


def fl_file_bytes(data) -> bytes:
    """The reference fl-cpu's output file for `data` (file_io.cu:222-280)."""
    import struct
    a = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    bits, values = fl_compress(a)
    return struct.pack("<QQQ", a.size, bits.size, values.size) + bits.tobytes() + values.tobytes()
