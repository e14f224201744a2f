"""Sharding and the one exchange step of the multi-GPU FL path.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on
ROCm, "gloo" for CPU tests). The input byte range is cut into 128-byte-aligned
shards by the reference rule (src/file_io.cu:46-51: every shard but the last is
floor(N/(128P))*128 bytes; size_t arithmetic here instead of the reference's
int). Each rank encodes its shard independently; the only collective is an
all-gather of {F_r, V_r} (16 bytes per rank) followed by an exclusive scan,
which places each shard's bits/values in the global output. Concatenating the
shard outputs in rank order is byte-identical to encoding the whole input
 — the reference's padded O(P*N) ncclAllGather of the
payloads (src/fl/fl_gpu.cu:144-238) is not needed.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

FRAME = 128


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """(start, length) of rank's shard of an n-byte input (file_io.cu:46-51)."""
    per = (n // (FRAME * world)) * FRAME
    start = rank * per
    length = n - (world - 1) * per if rank == world - 1 else per
    return start, length


_SCAN_BUFS: dict = {}


def _scan_buf(world: int, device) -> torch.Tensor:
    """int64[(world + 1) * 2] whose first row stays [0, 0]: the all-gather fills
    rows 1..world, so ONE cumsum yields every rank's exclusive offsets (rows
    0..world-1) and the totals (row world)."""
    key = (world, str(device))
    buf = _SCAN_BUFS.get(key)
    if buf is None:
        buf = torch.zeros((world + 1) * 2, dtype=torch.int64, device=device)
        _SCAN_BUFS[key] = buf
    return buf


def size_scan(sizes: torch.Tensor, group=None) -> tuple[torch.Tensor, torch.Tensor]:
    """All-gather each rank's int64 [F_r, V_r] and exclusive-scan them.

    `sizes` stays on its device (no host sync for a GPU tensor). Returns
    (offsets of this rank [F_off, V_off], totals [F, V]) as int64 tensors on
    the same device. Device work: the all-gather and one cumsum kernel.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = sizes.reshape(2).to(torch.int64)
    buf = _scan_buf(world, sizes.device)
    dist.all_gather_into_tensor(buf[2:], sizes, group=group)  # one buffer: no per-rank list + stack
    scan = torch.cumsum(buf.view(world + 1, 2), dim=0)
    return scan[rank], scan[world]
