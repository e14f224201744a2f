"""The multi-GPU FL exchange on CPU, through the shipped layout code.

flrl_fl_encode_rank / flrl_fl_encode_sharded / flrl_fl_compress_rank
(csrc/flrl_shard.hip) place shard outputs with one exchange: every shard puts
{F word, V} into its slot (flrl_shard_slot), an in-place all-gather spreads the
slots, and each shard's record comes from shard_record
(csrc/flrl_shard_layout.hpp) — on the device in size_scan_kernel, on the host
in flrl_fl_compress_rank's rank-0 merge. The C ABI exports the same functions
(flrl_shard_range / _slot / _size_word / _scan), so these tests run the
shipped arithmetic, with gloo (2-4 processes) standing in for the RCCL
all-gather of the per-rank model (ndev = nranks, one slot each) and a
simulated per-device all-gather for the single-process model (ndev < P).
Shards are encoded by the oracle; the placed output must equal the
whole-input encode byte for byte (the reference's
gpuNCCLCompress, src/fl/fl_gpu.cu:76-287, and merge, fl_common.cuh:95-151)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import flrl


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, ragged_rank, q, failed_rank=None):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "fl-rl-compression-mpi_amd"))
    import flrl as fl
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        whole = oracle.gen("lo4", n, 5)
        whole[::1777] = 0xC3  # mixed widths
        start, length = fl.shard_range(n, world, rank)
        if ragged_rank is not None:  # a caller that ignores the shard rule
            start, length = (0, 200) if rank == ragged_rank else (200 + 128 * rank, 128)
        bits, values = oracle.fl_compress(whole[start:start + length])
        # the rank's slot pair, exactly as put_u64_kernel + the encode write it
        mine = np.array([fl.shard_size_word(length), values.size], dtype=np.uint64)
        if rank == failed_rank:  # a local failure still joins the exchange (flrl_fl_encode_rank)
            mine = np.array([fl.shard_failed_word(), 0], dtype=np.uint64)
        slot = fl.shard_slot(rank, world, world)
        gathered = torch.zeros(2 * world, dtype=torch.int64)
        dist.all_gather_into_tensor(gathered, torch.from_numpy(mine.view(np.int64)))
        g = gathered.numpy().view(np.uint64)
        assert np.array_equal(g[slot:slot + 2], mine)
        try:
            rec = fl.shard_scan(g, world, world, rank)
            err = 0
        except fl.FLRLError as e:
            rec, err = None, e.code
        parts = [None] * world
        dist.all_gather_object(parts, (rec, err, bits.tobytes(), values.tobytes()))
        if rank == 0:
            if ragged_rank is not None or failed_rank is not None:
                q.put([p[1] for p in parts])
                return
            F, V = parts[0][0][flrl.SZ_F_TOTAL], parts[0][0][flrl.SZ_V_TOTAL]
            out_bits, out_vals = bytearray(F), bytearray(V)
            for r, (rr, _, b, v) in enumerate(parts):
                assert rr[flrl.SZ_F] == len(b) and rr[flrl.SZ_V] == len(v)
                assert rr[flrl.SZ_F_TOTAL] == F and rr[flrl.SZ_V_TOTAL] == V
                # rank 0's merge (flrl_fl_compress_rank) recomputes every rank's
                # record from its own copy of the gathered slots
                assert fl.shard_scan(g, world, world, r) == rr
                out_bits[rr[flrl.SZ_F_OFF]:rr[flrl.SZ_F_OFF] + len(b)] = b
                out_vals[rr[flrl.SZ_V_OFF]:rr[flrl.SZ_V_OFF] + len(v)] = v
            rb, rv = oracle.fl_compress(whole)
            q.put((bytes(out_bits) == rb.tobytes(), bytes(out_vals) == rv.tobytes(), F, V))
    finally:
        dist.destroy_process_group()


def _run(world, n, ragged_rank=None, failed_rank=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, ragged_rank, q, failed_rank))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return q.get(timeout=10)


@pytest.mark.parametrize("world,n", [(2, 1_000_003), (3, 128 * 3 + 5), (3, 100), (4, 524_288 + 77)])
def test_rank_exchange_matches_whole(world, n):
    bits_ok, vals_ok, F, V = _run(world, n)
    assert bits_ok and vals_ok
    assert F == (n + 127) // 128


def test_rank_exchange_flags_ragged_shard():
    """A shard before the last that is not whole frames: every rank's scan
    reports FLRL_E_ARG (on the device: each rank's scratch error word)."""
    assert _run(3, 4096, ragged_rank=0) == [flrl.E_ARG] * 3


@pytest.mark.parametrize("world,failed", [(2, 1), (3, 0), (4, 2)])
def test_rank_exchange_flags_failed_rank(world, failed):
    """a rank whose encode fails locally (scratch too
    small, misaligned buffers) no longer returns before the all-gather, which
    left every peer waiting in it: it joins with flrl_shard_failed_word() in its
    slot, and every rank's scan (the device size_scan_kernel runs the same
    shard_record) reports FLRL_E_ARG."""
    assert _run(world, 1_000_003, failed_rank=failed) == [flrl.E_ARG] * world


def test_shard_scan_failed_word():
    ok = np.array([flrl.shard_size_word(256), 5, flrl.shard_size_word(300), 7], dtype=np.uint64)
    assert flrl.shard_scan(ok, 2, 2, 1) == [3, 7, 2, 5, 5, 12]
    for bad_slot in (0, 2):
        g = ok.copy()
        g[bad_slot], g[bad_slot + 1] = flrl.shard_failed_word(), 0
        for me in (0, 1):
            with pytest.raises(flrl.FLRLError) as e:
                flrl.shard_scan(g, 2, 2, me)
            assert e.value.code == flrl.E_ARG and "failed" in str(e.value)
    assert flrl.shard_failed_word() == 1 << 62
    assert flrl.shard_failed_word() & flrl.shard_size_word(1 << 40) == 0


def _whole_scan(F, V, r):
    return [F[r], V[r], sum(F[:r]), sum(V[:r]), sum(F), sum(V)]


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
def test_sharded_layout_all_gather(ndev):
    """flrl_fl_encode_sharded's layout: shard r on device r mod ndev writes its
    slot in that device's own segment of the gathered array; the in-place
    all-gather of every device's S slots then gives each device the same array,
    and every shard's record is the exclusive scan in shard order."""
    rng = np.random.default_rng(ndev)
    for P in sorted({1, 2, ndev, ndev + 1, 2 * ndev - 1, 17, 64 * ndev - 1, 64 * ndev}):
        if P < 1:
            continue
        S = -(-P // ndev)
        lens = [int(x) * 128 for x in rng.integers(0, 1 << 20, size=P)]
        lens[-1] += int(rng.integers(0, 128))  # the last shard may be ragged
        V = [int(x) for x in rng.integers(0, 1 << 40, size=P)]
        F = [(L + 127) // 128 for L in lens]
        local = [np.zeros(2 * S * ndev, dtype=np.uint64) for _ in range(ndev)]
        slots = set()
        for r in range(P):
            k = r % ndev
            s = flrl.shard_slot(r, P, ndev)
            assert s // (2 * S) == k and s % 2 == 0 and s not in slots
            slots.add(s)
            local[k][s] = flrl.shard_size_word(lens[r])
            local[k][s + 1] = V[r]
        # ncclAllGather(sendbuff = gather + k*S*2, recvbuff = gather, 2*S) on every device k
        gathered = np.concatenate([local[k][2 * S * k:2 * S * (k + 1)] for k in range(ndev)])
        for r in range(P):
            assert flrl.shard_scan(gathered, P, ndev, r) == _whole_scan(F, V, r), (P, r)


def test_shard_scan_ragged_and_args():
    g = np.array([flrl.shard_size_word(130), 5, flrl.shard_size_word(256), 7], dtype=np.uint64)
    with pytest.raises(flrl.FLRLError) as e:
        flrl.shard_scan(g, 2, 2, 1)
    assert e.value.code == flrl.E_ARG
    g[0] = flrl.shard_size_word(128)
    g[2] = flrl.shard_size_word(131)  # the last shard may be ragged
    assert flrl.shard_scan(g, 2, 2, 1) == [2, 7, 1, 5, 3, 12]
    assert flrl.shard_size_word(0) == 0 and flrl.shard_size_word(128) == 1
    assert flrl.shard_size_word(129) == (1 << 63) | 2
    for bad in ((g, 0, 1, 0), (g, 2, 0, 0), (g, 2, 2, 2), (g, 2, 2, -1)):
        with pytest.raises(flrl.FLRLError):
            flrl.shard_scan(*bad)
    with pytest.raises(ValueError):
        flrl.shard_slot(3, 3, 1)


def test_shard_rule_edges():
    for n in (0, 1, 127, 128, 1000, 1 << 20, (1 << 34) + 5, 128 << 30):
        for world in (1, 2, 3, 8):
            spans = [flrl.shard_range(n, world, r) for r in range(world)]
            assert sum(length for _, length in spans) == n
            per = (n // (128 * world)) * 128  # src/file_io.cu:46-51 (size_t here)
            pos = 0
            for r, (start, length) in enumerate(spans):
                assert start == pos
                if r < world - 1:
                    assert length == per and length % 128 == 0
                pos += length
    with pytest.raises(flrl.FLRLError):
        flrl.shard_range(10, 0, 0)
