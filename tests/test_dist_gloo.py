"""Multi-rank FL path on CPU (gloo): the reference shard rule
(src/file_io.cu:46-51) + the one exchange step (all-gather of {F_r, V_r},
exclusive scan) used by bench.py's N > 1 path. Each rank encodes its shard with
the oracle; placing the shards at the scanned offsets must reproduce the
whole-input output byte for byte."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "fl-rl-compression-mpi_amd"))
    import oracle
    from flrl.dist import shard_range, size_scan

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        whole = oracle.gen("lo4", n, 5)
        whole[::1777] = 0xC3  # mixed widths
        start, length = shard_range(n, rank, world)
        bits, values = oracle.fl_compress(whole[start:start + length])
        sizes = torch.tensor([bits.size, values.size], dtype=torch.int64)
        offs, totals = size_scan(sizes)
        parts = [None] * world
        dist.all_gather_object(parts, (int(offs[0]), int(offs[1]), bits.tobytes(), values.tobytes()))
        if rank == 0:
            F, V = int(totals[0]), int(totals[1])
            out_bits = bytearray(F)
            out_vals = bytearray(V)
            for fo, vo, b, v in parts:
                out_bits[fo:fo + len(b)] = b
                out_vals[vo:vo + len(v)] = v
            rb, rv = oracle.fl_compress(whole)
            q.put((bytes(out_bits) == rb.tobytes(), bytes(out_vals) == rv.tobytes(), F, V))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("n", [1_000_003, 128 * 3 + 5, 100])
def test_sharded_size_scan_matches_whole(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    bits_ok, vals_ok, F, V = q.get(timeout=10)
    assert bits_ok and vals_ok
    assert F == (n + 127) // 128


def test_shard_rule_edges():
    from flrl.dist import shard_range
    for n in (0, 1, 127, 128, 1000, 1 << 20, (1 << 34) + 5):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert sum(length for _, length in spans) == n
            pos = 0
            for r, (start, length) in enumerate(spans):
                assert start == pos
                if r < world - 1:
                    assert length % 128 == 0
                pos += length
