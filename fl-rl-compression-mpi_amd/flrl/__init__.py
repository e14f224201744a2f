"""flrl — Python binding of the MI355X FL/RL codec C ABI (include/flrl.h).

The product is ``lib/libflrl.so`` (HIP kernels for gfx950 + host entry
points); this module is a thin ctypes layer over it for tests and bench.py. It
never falls back to a CPU implementation: if the library is missing, importing
this module raises ImportError, and GPU entry points raise FLRLError when no HIP
device is visible.

Host-buffer API (mirrors the reference's FixedLength::gpuCompress /
gpuDecompress, src/fl/fl_gpu.cuh:14-15):
    fl_compress(data) -> FLCompressed(bits, values, input_size)
    fl_decompress(input_size, bits, values) -> np.ndarray[uint8]
    fl_compress_sharded(data, nshards) -> FLCompressed (gpuNCCLCompress, :16)
Exchange layout (host form of the device scan): shard_range, shard_slot,
    shard_size_word, shard_scan.
Multi-GPU (RCCL size exchange; gpuNCCLCompress, fl_gpu.cu:76-287):
    Comm.local(ndev) / Comm.rank(nranks, comm_unique_id(), rank)
    Comm.encode_rank / Comm.compress_rank / Comm.encode_sharded
    rl_compress(data) -> RLCompressed(counts, values, input_size)
    rl_decompress(input_size, counts, values) -> np.ndarray[uint8]
Device API (raw device pointers as ints; mirrors gpuCompressDevice, :17):
    fl_encode_device / fl_decode_device / rl_encode_device / rl_decode_device,
    gen_device, scratch_error, plus *_scratch_bytes sizing helpers.
File formats: fl_file_bytes / parse_fl_file, rl_file_bytes / parse_rl_file.
"""
from __future__ import annotations

import ctypes
import os
import struct
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_DIR, "lib", "libflrl.so")
CLI_PATH = os.path.join(PKG_DIR, "bin", "compress")
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "flrl.h")

FRAME_LENGTH = 128

E_OK, E_ARG, E_HIP, E_NOMEM, E_FORMAT, E_TIMEOUT, E_NODEV, E_RCCL = range(8)
ERROR_NAMES = {
    E_ARG: "FLRL_E_ARG", E_HIP: "FLRL_E_HIP", E_NOMEM: "FLRL_E_NOMEM",
    E_FORMAT: "FLRL_E_FORMAT", E_TIMEOUT: "FLRL_E_TIMEOUT", E_NODEV: "FLRL_E_NODEV",
    E_RCCL: "FLRL_E_RCCL",
}

GEN_KINDS = {"u8": 0, "lo4": 1, "zero": 2, "runs32": 3, "longruns": 4}


class FLRLError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {message}")
        self.code = code


# torch-ROCm bundles its own libamdhip64.so.7 with the same soname as
# /opt/rocm's; whichever is loaded first serves the whole process. Load torch's
# first (when torch is installed) so device pointers and streams from torch and
# from libflrl.so belong to one HIP runtime; loading /opt/rocm's first leaves
# torch without a usable device.
try:
    import torch as _torch  # noqa: F401
except ImportError:
    _torch = None

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libflrl.so not found at {LIB_PATH}; build it with "
        f"`make -C {PKG_DIR}` (or __graft_entry__.build())")

_lib = ctypes.CDLL(LIB_PATH)

_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_u64 = ctypes.c_uint64


class _FLBuf(ctypes.Structure):
    _fields_ = [("bits", _u8p), ("bits_size", _sz), ("values", _u8p),
                ("values_size", _sz), ("input_size", _sz)]


class _RLBuf(ctypes.Structure):
    _fields_ = [("counts", _u8p), ("values", _u8p), ("runs", _sz), ("input_size", _sz)]


def _sig(name, restype, *argtypes):
    f = getattr(_lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)
    return f


_sig("flrl_last_error", ctypes.c_char_p)
_sig("flrl_version", ctypes.c_char_p)
_sig("flrl_device_count", ctypes.c_int)
_sig("flrl_fl_compress", ctypes.c_int, _vp, _sz, ctypes.POINTER(_FLBuf))
_sig("flrl_release_staging", _sz)
_sig("flrl_fl_compress_sharded", ctypes.c_int, _vp, _sz, ctypes.c_int, ctypes.POINTER(_FLBuf))
_sig("flrl_fl_decompress", ctypes.c_int, _sz, _vp, _sz, _vp, _sz,
     ctypes.POINTER(_u8p), ctypes.POINTER(_sz))
_sig("flrl_fl_compress_file", ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, _sz)
_sig("flrl_fl_decompress_file", ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, _sz)
_sig("flrl_rl_compress_file", ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, _sz)
_sig("flrl_rl_decompress_file", ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, _sz)
_sig("flrl_fl_scratch_bytes", _sz, _sz)
_sig("flrl_fl_values_capacity", _sz, _sz)
_sig("flrl_fl_encode_device", ctypes.c_int, _vp, _sz, _vp, _vp, _vp, _vp, _sz, _vp)
_sig("flrl_fl_decode_device", ctypes.c_int, _vp, _sz, _vp, _sz, _vp, _sz, _vp, _sz, _vp)
_sig("flrl_scratch_error", ctypes.c_int, _vp, _vp)
_sig("flrl_time_next_kernel", ctypes.c_int, _vp, _vp)
_sig("flrl_debug_skip_scratch_resets", ctypes.c_int, ctypes.c_int)
_sig("flrl_debug_lookback_help_us", ctypes.c_int, ctypes.c_int)
_sig("flrl_debug_fail_chunk", ctypes.c_int, ctypes.c_longlong)
_sig("flrl_debug_fail_rank_step", ctypes.c_int, ctypes.c_int)
_sig("flrl_rl_compress", ctypes.c_int, _vp, _sz, ctypes.POINTER(_RLBuf))
_sig("flrl_rl_decompress", ctypes.c_int, _sz, _vp, _vp, _sz,
     ctypes.POINTER(_u8p), ctypes.POINTER(_sz))
_sig("flrl_rl_scratch_bytes", _sz, _sz)
_sig("flrl_rl_encode_device", ctypes.c_int, _vp, _sz, _vp, _vp, _vp, _vp, _sz, _vp)
_sig("flrl_rl_decode_scratch_bytes", _sz, _sz)
_sig("flrl_rl_decode_device", ctypes.c_int, _vp, _vp, _sz, _vp, _sz, _vp, _sz, _vp)
_sig("flrl_gen_device", ctypes.c_int, ctypes.c_int, _u64, _u64, _vp, _sz, _vp)
_sig("flrl_gen_host", ctypes.c_int, ctypes.c_int, _u64, _u64, _vp, _sz)
_pp = ctypes.POINTER(_vp)
_sig("flrl_comm_init", ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int), _pp)
_sig("flrl_comm_unique_id", ctypes.c_int, _vp)
_sig("flrl_comm_init_rank", ctypes.c_int, ctypes.c_int, _vp, ctypes.c_int, _pp)
_sig("flrl_comm_wrap", ctypes.c_int, _vp, _pp)
_sig("flrl_comm_destroy", ctypes.c_int, _vp)
_sig("flrl_comm_query", ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_int),
     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))
_sig("flrl_comm_rccl_info", ctypes.c_int, _vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int)
_sig("flrl_fl_encode_rank", ctypes.c_int, _vp, _vp, _sz, _vp, _vp, _vp, _vp, _sz, _vp)
_sig("flrl_fl_compress_rank", ctypes.c_int, _vp, _vp, _sz, ctypes.POINTER(_FLBuf))
_sig("flrl_shard_range", ctypes.c_int, _sz, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_sz),
     ctypes.POINTER(_sz))
_sig("flrl_shard_slot", _sz, ctypes.c_int, ctypes.c_int, ctypes.c_int)
_sig("flrl_shard_size_word", _u64, _sz)
_sig("flrl_shard_failed_word", _u64)
_sig("flrl_shard_scan", ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp)
_sig("flrl_fl_encode_sharded", ctypes.c_int, _vp, ctypes.c_int, _pp, ctypes.POINTER(_sz), _pp, _pp,
     _pp, _pp, ctypes.POINTER(_sz), _pp)

UNIQUE_ID_BYTES = 128
# per-shard sizes record written by the exchange (include/flrl.h FLRL_SZ_*)
SZ_F, SZ_V, SZ_F_OFF, SZ_V_OFF, SZ_F_TOTAL, SZ_V_TOTAL, SZ_COUNT = range(7)

_libc = ctypes.CDLL(None)
_libc.free.argtypes = [_vp]
_libc.free.restype = None


def _check(rc: int):
    if rc != 0:
        raise FLRLError(rc, _lib.flrl_last_error().decode(errors="replace"))


def _as_u8(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(data, dtype=np.uint8)
    if isinstance(data, (list, tuple)):
        return np.asarray(data, dtype=np.uint8)
    a = np.ascontiguousarray(data)
    if a.dtype != np.uint8:
        a = a.view(np.uint8).reshape(-1)
    return a.reshape(-1)


def _take(ptr, n: int) -> np.ndarray:
    """Copy n bytes out of a malloc'd buffer and free it."""
    if not ptr:
        return np.zeros(0, dtype=np.uint8)
    addr = ctypes.cast(ptr, _vp).value
    out = np.empty(n, dtype=np.uint8)
    if n:
        ctypes.memmove(out.ctypes.data, addr, n)
    _libc.free(addr)
    return out


@dataclass
class FLCompressed:
    """Mirrors FixedLength::FLCompressed (src/fl/fl_common.cuh:11-34)."""
    bits: np.ndarray
    values: np.ndarray
    input_size: int

    def to_file_bytes(self) -> bytes:
        return fl_file_bytes(self.input_size, self.bits, self.values)


@dataclass
class RLCompressed:
    counts: np.ndarray
    values: np.ndarray
    input_size: int

    def to_file_bytes(self) -> bytes:
        return rl_file_bytes(self.input_size, self.counts, self.values)


def version() -> str:
    return _lib.flrl_version().decode()


def device_count() -> int:
    return int(_lib.flrl_device_count())


# ---------------------------------------------------------------- host API
def fl_compress(data) -> FLCompressed:
    a = _as_u8(data)
    buf = _FLBuf()
    _check(_lib.flrl_fl_compress(a.ctypes.data if a.size else None, a.size, ctypes.byref(buf)))
    return FLCompressed(_take(buf.bits, buf.bits_size), _take(buf.values, buf.values_size),
                        int(buf.input_size))


def fl_compress_sharded(data, nshards: int = 0) -> FLCompressed:
    """Whole input in `nshards` shards (<= 0: one per GPU); shard r on GPU r mod ndev."""
    a = _as_u8(data)
    buf = _FLBuf()
    _check(_lib.flrl_fl_compress_sharded(a.ctypes.data if a.size else None, a.size, nshards,
                                         ctypes.byref(buf)))
    return FLCompressed(_take(buf.bits, buf.bits_size), _take(buf.values, buf.values_size),
                        int(buf.input_size))


def shard_range(n: int, nshards: int, shard: int) -> tuple[int, int]:
    """(start, length) of `shard` by the reference rule (file_io.cu:46-51)."""
    a, b = _sz(), _sz()
    _check(_lib.flrl_shard_range(n, nshards, shard, ctypes.byref(a), ctypes.byref(b)))
    return a.value, b.value


def shard_slot(shard: int, nshards: int, ndev: int) -> int:
    """u64 index of shard's {F word, V} pair in the all-gathered exchange array."""
    s = int(_lib.flrl_shard_slot(shard, nshards, ndev))
    if s == ctypes.c_size_t(-1).value:
        raise ValueError(f"shard {shard} of {nshards} on {ndev} devices")
    return s


def shard_size_word(n: int) -> int:
    """The F word a shard of n bytes puts into its slot (bit 63: ragged)."""
    return int(_lib.flrl_shard_size_word(n))


def shard_failed_word() -> int:
    """The F word (V = 0) a rank that failed locally puts into its slot, so that
    every rank's scan reports FLRL_E_ARG instead of peers waiting forever."""
    return int(_lib.flrl_shard_failed_word())


def shard_scan(gather: np.ndarray, nshards: int, ndev: int, shard: int) -> list[int]:
    """shard's exchange record [F, V, F_off, V_off, F_total, V_total] from the
    all-gathered u64 array (the device scan's code); FLRLError(E_ARG) when a
    shard before the last is ragged."""
    g = np.ascontiguousarray(gather, dtype=np.uint64)
    rec = np.zeros(SZ_COUNT, dtype=np.uint64)
    _check(_lib.flrl_shard_scan(g.ctypes.data, nshards, ndev, shard, rec.ctypes.data))
    return [int(v) for v in rec]


def release_staging() -> int:
    """Free the host-buffer / file paths' idle pinned staging; returns the bytes."""
    return int(_lib.flrl_release_staging())


def comm_unique_id() -> bytes:
    """ncclGetUniqueId as FLRL_UNIQUE_ID_BYTES bytes (rank 0 distributes it)."""
    b = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    _check(_lib.flrl_comm_unique_id(b))
    return b.raw


class Comm:
    """flrl_comm: an RCCL communicator for the FL size exchange, created once.

    Comm.local(ndev)            one process driving ndev GPUs (ncclCommInitAll)
    Comm.rank(nranks, uid, r)   one process per GPU (ncclCommInitRank, current device)
    """

    def __init__(self, handle: int):
        self._h = handle

    @classmethod
    def local(cls, ndev: int = 0, devs=None) -> "Comm":
        h = _vp()
        arr = (ctypes.c_int * len(devs))(*devs) if devs else None
        _check(_lib.flrl_comm_init(len(devs) if devs else ndev, arr, ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def rank(cls, nranks: int, uid: bytes, rank: int) -> "Comm":
        if len(uid) != UNIQUE_ID_BYTES:
            raise ValueError(f"unique id must be {UNIQUE_ID_BYTES} bytes")
        h = _vp()
        _check(_lib.flrl_comm_init_rank(nranks, uid, rank, ctypes.byref(h)))
        return cls(h.value)

    @property
    def handle(self) -> int:
        if not self._h:
            raise ValueError("communicator destroyed")
        return self._h

    def query(self) -> tuple[int, int, int]:
        """(nranks, rank, local devices)."""
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(_lib.flrl_comm_query(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def rccl_info(self, local: int = 0) -> dict:
        """RCCL's own view of local device `local`: ncclCommCount, the user
        rank, the HIP device and its PCI bus id (flrl_comm_rccl_info)."""
        n, r, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        bus = ctypes.create_string_buffer(64)
        _check(_lib.flrl_comm_rccl_info(self.handle, local, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d),
                                        bus, 64))
        return {"count": n.value, "rank": r.value, "device": d.value, "pci_bus_id": bus.value.decode()}

    def encode_rank(self, d_in: int, n: int, d_bits: int, d_values: int, d_sizes: int,
                    d_scratch: int, scratch_bytes: int, stream: int = 0) -> None:
        _check(_lib.flrl_fl_encode_rank(self.handle, d_in, n, d_bits, d_values, d_sizes,
                                        d_scratch, scratch_bytes, stream or None))

    def compress_rank(self, data) -> FLCompressed:
        """gpuNCCLCompress twin: this rank's shard in, merged result on rank 0."""
        a = _as_u8(data)
        buf = _FLBuf()
        _check(_lib.flrl_fl_compress_rank(self.handle, a.ctypes.data if a.size else None, a.size,
                                          ctypes.byref(buf)))
        return FLCompressed(_take(buf.bits, buf.bits_size), _take(buf.values, buf.values_size),
                            int(buf.input_size))

    def encode_sharded(self, d_in, n, d_bits, d_values, d_sizes, d_scratch, scratch_bytes,
                       streams) -> None:
        P = len(d_in)
        if not all(len(x) == P for x in (n, d_bits, d_values, d_sizes, d_scratch, scratch_bytes,
                                         streams)):
            raise ValueError("encode_sharded: per-shard lists differ in length")

        def ptrs(xs):
            return (_vp * P)(*[x or None for x in xs])
        _check(_lib.flrl_fl_encode_sharded(self.handle, P, ptrs(d_in), (_sz * P)(*n), ptrs(d_bits),
                                           ptrs(d_values), ptrs(d_sizes), ptrs(d_scratch),
                                           (_sz * P)(*scratch_bytes), ptrs(streams)))

    def destroy(self) -> None:
        if self._h:
            _lib.flrl_comm_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()


def fl_compress_file(in_path: str, out_path: str, workers: int = 1, chunk_bytes: int = 0) -> None:
    """File -> .fl file streamed through the GPU(s) (include/flrl.h)."""
    _check(_lib.flrl_fl_compress_file(os.fsencode(in_path), os.fsencode(out_path), workers,
                                      chunk_bytes))


def fl_decompress_file(in_path: str, out_path: str, workers: int = 1, chunk_bytes: int = 0) -> None:
    """.fl file -> file streamed through the GPU(s); validates header and widths."""
    _check(_lib.flrl_fl_decompress_file(os.fsencode(in_path), os.fsencode(out_path), workers,
                                        chunk_bytes))


def rl_compress_file(in_path: str, out_path: str, workers: int = 1, chunk_bytes: int = 0) -> None:
    """File -> .rl file streamed through the GPU(s) (runs re-split across chunks)."""
    _check(_lib.flrl_rl_compress_file(os.fsencode(in_path), os.fsencode(out_path), workers,
                                      chunk_bytes))


def rl_decompress_file(in_path: str, out_path: str, workers: int = 1, chunk_bytes: int = 0) -> None:
    """.rl file -> file streamed through the GPU(s); validates header and counts."""
    _check(_lib.flrl_rl_decompress_file(os.fsencode(in_path), os.fsencode(out_path), workers,
                                        chunk_bytes))


def fl_decompress(input_size: int, bits, values) -> np.ndarray:
    b, v = _as_u8(bits), _as_u8(values)
    out, out_size = _u8p(), _sz()
    _check(_lib.flrl_fl_decompress(input_size, b.ctypes.data if b.size else None, b.size,
                                   v.ctypes.data if v.size else None, v.size,
                                   ctypes.byref(out), ctypes.byref(out_size)))
    return _take(out, out_size.value)


def rl_compress(data) -> RLCompressed:
    a = _as_u8(data)
    buf = _RLBuf()
    _check(_lib.flrl_rl_compress(a.ctypes.data if a.size else None, a.size, ctypes.byref(buf)))
    return RLCompressed(_take(buf.counts, buf.runs), _take(buf.values, buf.runs),
                        int(buf.input_size))


def rl_decompress(input_size: int, counts, values) -> np.ndarray:
    c, v = _as_u8(counts), _as_u8(values)
    out, out_size = _u8p(), _sz()
    _check(_lib.flrl_rl_decompress(input_size, c.ctypes.data if c.size else None,
                                   v.ctypes.data if v.size else None, c.size,
                                   ctypes.byref(out), ctypes.byref(out_size)))
    return _take(out, out_size.value)


# -------------------------------------------------------------- device API
def fl_scratch_bytes(n: int) -> int:
    return int(_lib.flrl_fl_scratch_bytes(n))


def fl_values_capacity(n: int) -> int:
    return int(_lib.flrl_fl_values_capacity(n))


def rl_scratch_bytes(n: int) -> int:
    return int(_lib.flrl_rl_scratch_bytes(n))


def rl_decode_scratch_bytes(runs: int) -> int:
    return int(_lib.flrl_rl_decode_scratch_bytes(runs))


def fl_encode_device(d_in: int, n: int, d_bits: int, d_values: int, d_values_size: int,
                     d_scratch: int, scratch_bytes: int, stream: int = 0) -> None:
    _check(_lib.flrl_fl_encode_device(d_in, n, d_bits, d_values, d_values_size, d_scratch,
                                      scratch_bytes, stream or None))


def fl_decode_device(d_bits: int, bits_size: int, d_values: int, values_size: int, d_out: int,
                     n: int, d_scratch: int, scratch_bytes: int, stream: int = 0) -> None:
    _check(_lib.flrl_fl_decode_device(d_bits, bits_size, d_values, values_size, d_out, n,
                                      d_scratch, scratch_bytes, stream or None))


def rl_encode_device(d_in: int, n: int, d_counts: int, d_values: int, d_runs: int,
                     d_scratch: int, scratch_bytes: int, stream: int = 0) -> None:
    _check(_lib.flrl_rl_encode_device(d_in, n, d_counts, d_values, d_runs, d_scratch,
                                      scratch_bytes, stream or None))


def rl_decode_device(d_counts: int, d_values: int, runs: int, d_out: int, n: int,
                     d_scratch: int, scratch_bytes: int, stream: int = 0) -> None:
    _check(_lib.flrl_rl_decode_device(d_counts, d_values, runs, d_out, n, d_scratch,
                                      scratch_bytes, stream or None))


def gen_device(kind, seed: int, word_offset: int, d_out: int, n: int, stream: int = 0) -> None:
    k = GEN_KINDS[kind] if isinstance(kind, str) else int(kind)
    _check(_lib.flrl_gen_device(k, seed, word_offset, d_out, n, stream or None))


def gen_host(kind, n: int, seed: int, word_offset: int = 0) -> np.ndarray:
    """SURVEY.md §8(d) synthetic input on the host (all kinds, incl. runs32)."""
    k = GEN_KINDS[kind] if isinstance(kind, str) else int(kind)
    out = np.empty(n, dtype=np.uint8)
    _check(_lib.flrl_gen_host(k, seed, word_offset, out.ctypes.data if n else None, n))
    return out


def time_next_kernel(start=None, stop=None) -> None:
    """Record two events (torch.cuda.Event or raw hipEvent_t ints; already
    created, i.e. recorded once) around the main kernel of this thread's next
    device call; see flrl_time_next_kernel in include/flrl.h."""
    def handle(e):
        if e is None:
            return None
        h = e.cuda_event if hasattr(e, "cuda_event") else int(e)
        if not h:
            raise ValueError("event not created yet: record it once first")
        return h
    _check(_lib.flrl_time_next_kernel(handle(start), handle(stop)))


def debug_skip_scratch_resets(calls: int) -> None:
    """Test hook: this thread's next `calls` device calls skip their scratch reset."""
    _check(_lib.flrl_debug_skip_scratch_resets(calls))


def debug_lookback_help_us(microseconds: int) -> None:
    """Test hook: RL encode look-backs compute an unpublished predecessor's map
    after `microseconds` (0: immediately) instead of 200 us; -1 restores."""
    _check(_lib.flrl_debug_lookback_help_us(microseconds))


def debug_fail_chunk(chunk: int) -> None:
    """Test hook: the streamed file paths fail at `chunk` (negative: never)."""
    _check(_lib.flrl_debug_fail_chunk(chunk))


DEBUG_RANK_SET_DEVICE, DEBUG_RANK_STREAM_WAIT, DEBUG_RANK_STAGE_WORD, DEBUG_RANK_READ_SUM = 1, 2, 3, 4


def debug_fail_rank_step(step: int) -> None:
    """Test hook: this thread's next per-rank call fails once at `step`
    (DEBUG_RANK_*; 0 cancels); see flrl_debug_fail_rank_step in include/flrl.h."""
    _check(_lib.flrl_debug_fail_rank_step(step))


def scratch_error(d_scratch: int, stream: int = 0) -> int:
    rc = _lib.flrl_scratch_error(d_scratch, stream or None)
    return int(rc)


# ------------------------------------------------------------ file formats
def fl_file_bytes(input_size: int, bits, values) -> bytes:
    """FL container, byte-identical to the reference (src/file_io.cu:222-280)."""
    b, v = _as_u8(bits), _as_u8(values)
    return struct.pack("<QQQ", input_size, b.size, v.size) + b.tobytes() + v.tobytes()


def parse_fl_file(blob: bytes) -> FLCompressed:
    n, fb, vb = struct.unpack_from("<QQQ", blob, 0)
    if 24 + fb + vb != len(blob):
        raise ValueError("FL file sizes do not match the header")
    a = np.frombuffer(blob, dtype=np.uint8)
    return FLCompressed(a[24:24 + fb].copy(), a[24 + fb:24 + fb + vb].copy(), n)


def rl_file_bytes(input_size: int, counts, values) -> bytes:
    """RL container (build-defined): u64 inputSize | u64 runs | counts | values."""
    c, v = _as_u8(counts), _as_u8(values)
    if c.size != v.size:
        raise ValueError(f"RL counts ({c.size}) and values ({v.size}) differ in length")
    return struct.pack("<QQ", input_size, c.size) + c.tobytes() + v.tobytes()


def parse_rl_file(blob: bytes) -> RLCompressed:
    n, r = struct.unpack_from("<QQ", blob, 0)
    if 16 + 2 * r != len(blob):
        raise ValueError("RL file size does not match the header")
    a = np.frombuffer(blob, dtype=np.uint8)
    return RLCompressed(a[16:16 + r].copy(), a[16 + r:16 + 2 * r].copy(), n)


def declared_symbols(header: str = HEADER_PATH) -> list[str]:
    """Every function the C ABI header declares."""
    import re
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(flrl_[a-z0-9_]+)\s*\(", txt)))


def lib_handle() -> ctypes.CDLL:
    return _lib
