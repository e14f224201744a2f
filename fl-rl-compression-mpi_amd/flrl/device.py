"""Device-resident FL / RL codecs over torch-allocated HBM buffers.

torch is used only as plumbing here (device memory, streams); all compute is
the HIP kernels in libflrl.so, called through the C ABI. Buffers are sized once
per input length and reused across calls, so a step does no allocation.
"""
from __future__ import annotations

import torch

import flrl

FRAME = flrl.FRAME_LENGTH


def _round16(n: int) -> int:
    return max(16, (n + 15) // 16 * 16)


def _check_input(x: torch.Tensor, n: int) -> None:
    """The kernels read n bytes from x's device pointer: u8, contiguous, >= n."""
    if x.dtype != torch.uint8 or not x.is_contiguous() or x.numel() < n or not x.is_cuda:
        raise ValueError(f"input must be a contiguous uint8 device tensor of >= {n} bytes "
                         f"(got {x.dtype}, {tuple(x.shape)}, contiguous={x.is_contiguous()}, {x.device})")


def _stream_handle(stream: torch.cuda.Stream | None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


class FLDevice:
    """FL encode/decode of an n-byte buffer, mirroring gpuCompressDevice
    (src/fl/fl_gpu.cu:425-535): outputs stay in HBM."""

    def __init__(self, n: int, device: str | torch.device = "cuda"):
        self.n = n
        self.frames = (n + FRAME - 1) // FRAME
        dev = torch.device(device)
        self.bits = torch.empty(_round16(self.frames), dtype=torch.uint8, device=dev)
        self.values = torch.empty(flrl.fl_values_capacity(n), dtype=torch.uint8, device=dev)
        # sizes = [F, V] on device: V is written by the encode kernel, so the
        # multi-rank size-scan can all-gather it without a host round trip
        self.sizes = torch.tensor([self.frames, 0], dtype=torch.int64, device=dev)
        self.scratch_bytes = flrl.fl_scratch_bytes(n)
        self.scratch = torch.empty(_round16(self.scratch_bytes), dtype=torch.uint8, device=dev)
        self.out = torch.empty(_round16(n), dtype=torch.uint8, device=dev)

    def encode(self, x: torch.Tensor, stream: torch.cuda.Stream | None = None) -> None:
        _check_input(x, self.n)
        flrl.fl_encode_device(x.data_ptr(), self.n, self.bits.data_ptr(), self.values.data_ptr(),
                              self.sizes.data_ptr() + 8, self.scratch.data_ptr(),
                              self.scratch_bytes, _stream_handle(stream))

    def encode_rank(self, comm: "flrl.Comm", x: torch.Tensor,
                    stream: torch.cuda.Stream | None = None) -> None:
        """Encode this rank's shard and run the size exchange (flrl_fl_encode_rank):
        self.rank_sizes (int64[FLRL_SZ_COUNT], device) then holds this shard's
        F, V, F_off, V_off and the totals, with no host round trip."""
        _check_input(x, self.n)
        if not hasattr(self, "rank_sizes"):
            self.rank_sizes = torch.zeros(8, dtype=torch.int64, device=self.bits.device)
        comm.encode_rank(x.data_ptr(), self.n, self.bits.data_ptr(), self.values.data_ptr(),
                         self.rank_sizes.data_ptr(), self.scratch.data_ptr(), self.scratch_bytes,
                         _stream_handle(stream))

    def decode(self, values_size: int, bits: torch.Tensor | None = None,
               values: torch.Tensor | None = None, out: torch.Tensor | None = None,
               stream: torch.cuda.Stream | None = None) -> torch.Tensor:
        bits = self.bits if bits is None else bits
        values = self.values if values is None else values
        out = self.out if out is None else out
        flrl.fl_decode_device(bits.data_ptr(), self.frames, values.data_ptr(), values_size,
                              out.data_ptr(), self.n, self.scratch.data_ptr(), self.scratch_bytes,
                              _stream_handle(stream))
        return out[: self.n]

    def values_size(self) -> int:
        return int(self.sizes[1].item())

    def error(self, stream: torch.cuda.Stream | None = None) -> int:
        return flrl.scratch_error(self.scratch.data_ptr(), _stream_handle(stream))

    def compressed(self) -> flrl.FLCompressed:
        v = self.values_size()
        return flrl.FLCompressed(self.bits[: self.frames].cpu().numpy(),
                                 self.values[:v].cpu().numpy(), self.n)


class RLDevice:
    """RL encode/decode of an n-byte buffer (build-defined format)."""

    def __init__(self, n: int, device: str | torch.device = "cuda"):
        self.n = n
        dev = torch.device(device)
        self.counts = torch.empty(_round16(n), dtype=torch.uint8, device=dev)
        self.values = torch.empty(_round16(n), dtype=torch.uint8, device=dev)
        self.runs_t = torch.zeros(2, dtype=torch.int64, device=dev)
        self.scratch_bytes = max(flrl.rl_scratch_bytes(n), flrl.rl_decode_scratch_bytes(n))
        self.scratch = torch.empty(_round16(self.scratch_bytes), dtype=torch.uint8, device=dev)
        self.out = torch.empty(_round16(n), dtype=torch.uint8, device=dev)

    def encode(self, x: torch.Tensor, stream: torch.cuda.Stream | None = None) -> None:
        _check_input(x, self.n)
        flrl.rl_encode_device(x.data_ptr(), self.n, self.counts.data_ptr(), self.values.data_ptr(),
                              self.runs_t.data_ptr(), self.scratch.data_ptr(), self.scratch_bytes,
                              _stream_handle(stream))

    def decode(self, runs: int, counts: torch.Tensor | None = None,
               values: torch.Tensor | None = None, out: torch.Tensor | None = None,
               stream: torch.cuda.Stream | None = None) -> torch.Tensor:
        counts = self.counts if counts is None else counts
        values = self.values if values is None else values
        out = self.out if out is None else out
        flrl.rl_decode_device(counts.data_ptr(), values.data_ptr(), runs, out.data_ptr(), self.n,
                              self.scratch.data_ptr(), self.scratch_bytes, _stream_handle(stream))
        return out[: self.n]

    def runs(self) -> int:
        return int(self.runs_t[0].item())

    def error(self, stream: torch.cuda.Stream | None = None) -> int:
        return flrl.scratch_error(self.scratch.data_ptr(), _stream_handle(stream))


def gen(kind: str, n: int, seed: int, word_offset: int = 0, device="cuda",
        stream: torch.cuda.Stream | None = None) -> torch.Tensor:
    """SURVEY.md §8(d) counter-based synthetic input generated on the device."""
    t = torch.empty(_round16(n), dtype=torch.uint8, device=device)
    flrl.gen_device(kind, seed, word_offset, t.data_ptr(), n, _stream_handle(stream))
    return t
