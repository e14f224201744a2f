"""Multi-shard FL encode on the MI355X: the RCCL size exchange of
flrl_shard.hip (replaces gpuNCCLCompress, src/fl/fl_gpu.cu:76-287).

On a one-GPU box several shards share the device (shard r on device r mod
ndev, flrl_fl_encode_sharded), so the exchange, the scan and the placement run
with P > 1 here; the output placed at the exchanged offsets must equal the
reference fl-cpu's whole-input output (golden BMP sha, 1 GiB u8 sha) byte for
byte. The per-rank entry (flrl_fl_encode_rank,
flrl_fl_compress_rank) runs with a one-rank communicator: RCCL refuses two
ranks on one GPU, so its P > 1 case runs on the driver's 8-GPU node
(bench.py --gpus N); tests/test_dist_gloo.py runs the exchange's layout code
(flrl_shard_scan, shared with size_scan_kernel) with 2-4 gloo ranks, and
tests/test_gpu_configs4.py runs BASELINE configs[4]'s eight 16 GiB shards.
"""
import hashlib
import os

import numpy as np
import pytest

import flrl

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available() or flrl.device_count() == 0:
        pytest.fail(f"GPU tests need a HIP device (HIP_VISIBLE_DEVICES="
                    f"{os.environ.get('HIP_VISIBLE_DEVICES')})")


def file_sha(n, bits: bytes, values: bytes) -> str:
    h = hashlib.sha256(np.array([n, len(bits), len(values)], dtype="<u8").tobytes())
    h.update(bits)
    h.update(values)
    return h.hexdigest()


def shard_lengths(n: int, P: int) -> list[int]:
    per = (n // (128 * P)) * 128  # src/file_io.cu:46-51
    return [per] * (P - 1) + [n - (P - 1) * per]


@pytest.mark.parametrize("P", [1, 2, 3, 4, 8, 17])
def test_host_sharded_bmp_golden(golden, bmp_bytes, P):
    """flrl_fl_compress_sharded with P shards: file sha == reference fl-cpu."""
    c = flrl.fl_compress_sharded(bmp_bytes, P)
    g = golden["fl_bmp"]
    assert c.input_size == len(bmp_bytes)
    assert file_sha(c.input_size, c.bits.tobytes(), c.values.tobytes()) == g["fl_sha256"]


def test_host_sharded_ragged_and_tiny():
    """Inputs smaller than P frames (empty shards but the last), ragged tails."""
    rng = np.random.default_rng(3)
    for n in (1, 127, 128, 129, 1000, 128 * 5 + 3, 70001):
        a = (rng.integers(0, 256, size=n) >> rng.integers(0, 8, size=n)).astype(np.uint8)
        ref = flrl.fl_compress(a)
        for P in (2, 3, 8):
            c = flrl.fl_compress_sharded(a, P)
            assert np.array_equal(c.bits, ref.bits) and np.array_equal(c.values, ref.values), (n, P)
    empty = flrl.fl_compress_sharded(b"", 4)
    assert empty.bits.size == 0 and empty.values.size == 0 and empty.input_size == 0


def test_host_sharded_repeat_reuses_comm(bmp_bytes):
    """The cached communicator serves repeated calls (no per-call init)."""
    ref = flrl.fl_compress(bmp_bytes)
    for _ in range(25):
        c = flrl.fl_compress_sharded(bmp_bytes, 5)
        assert np.array_equal(c.bits, ref.bits) and np.array_equal(c.values, ref.values)


def test_host_sharded_too_many_shards(bmp_bytes):
    with pytest.raises(flrl.FLRLError) as e:
        flrl.fl_compress_sharded(bmp_bytes, 64 * flrl.device_count() + 1)
    assert e.value.code == flrl.E_ARG


class Shards:
    """Device buffers of P shards of one resident input (views, no copies)."""

    def __init__(self, x, n: int, P: int):
        self.P = P
        self.len = shard_lengths(n, P)
        self.off = [sum(self.len[:r]) for r in range(P)]
        self.x = x
        self.bits = [torch.empty(max(16, (L + 127) // 128 + 16), dtype=torch.uint8, device=x.device)
                     for L in self.len]
        self.vals = [torch.empty(flrl.fl_values_capacity(L), dtype=torch.uint8, device=x.device)
                     for L in self.len]
        self.sizes = [torch.zeros(8, dtype=torch.int64, device=x.device) for _ in range(P)]
        self.scr_b = [flrl.fl_scratch_bytes(L) for L in self.len]
        self.scr = [torch.empty(max(16, b), dtype=torch.uint8, device=x.device) for b in self.scr_b]
        self.streams = [torch.cuda.Stream(device=x.device) for _ in range(P)]

    def encode(self, comm):
        cur = torch.cuda.current_stream()
        for s in self.streams:
            s.wait_stream(cur)
        comm.encode_sharded([self.x.data_ptr() + o for o in self.off], self.len,
                            [b.data_ptr() for b in self.bits], [v.data_ptr() for v in self.vals],
                            [s.data_ptr() for s in self.sizes], [s.data_ptr() for s in self.scr],
                            self.scr_b, [int(s.cuda_stream) for s in self.streams])
        for s in self.streams:
            cur.wait_stream(s)

    def records(self):
        torch.cuda.synchronize()
        return [[int(t) for t in s[:flrl.SZ_COUNT].cpu()] for s in self.sizes]

    def errors(self):
        return [flrl.scratch_error(s.data_ptr()) for s in self.scr]

    def place(self):
        """Whole-input bits/values assembled on the device at the exchanged offsets."""
        rec = self.records()
        F, V = rec[0][flrl.SZ_F_TOTAL], rec[0][flrl.SZ_V_TOTAL]
        bits = torch.empty(F, dtype=torch.uint8, device=self.x.device)
        vals = torch.empty(V, dtype=torch.uint8, device=self.x.device)
        for r, q in enumerate(rec):
            assert q[flrl.SZ_F_TOTAL] == F and q[flrl.SZ_V_TOTAL] == V
            bits[q[flrl.SZ_F_OFF]:q[flrl.SZ_F_OFF] + q[flrl.SZ_F]] = self.bits[r][:q[flrl.SZ_F]]
            vals[q[flrl.SZ_V_OFF]:q[flrl.SZ_V_OFF] + q[flrl.SZ_V]] = self.vals[r][:q[flrl.SZ_V]]
        return rec, bits, vals


@pytest.fixture(scope="module")
def local_comm():
    c = flrl.Comm.local(flrl.device_count())
    yield c
    c.destroy()


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_device_sharded_1gib_golden(golden, local_comm, P):
    """BASELINE configs[1] input in P device-resident shards through
    flrl_fl_encode_sharded: the exchanged offsets are the exclusive scan of the
    shards' sizes, and the placed output hashes to the reference fl-cpu's."""
    from flrl.device import gen
    g = golden["fl_generated_large"][0]
    n = g["n"]
    x = gen(g["kind"], n, g["seed"])
    sh = Shards(x, n, P)
    sh.encode(local_comm)
    rec, bits, vals = sh.place()
    assert sh.errors() == [0] * P
    Fs = [q[flrl.SZ_F] for q in rec]
    Vs = [q[flrl.SZ_V] for q in rec]
    assert Fs == [(L + 127) // 128 for L in sh.len]
    for r, q in enumerate(rec):
        assert q[flrl.SZ_F_OFF] == sum(Fs[:r]) and q[flrl.SZ_V_OFF] == sum(Vs[:r])
    assert file_sha(n, bits.cpu().numpy().tobytes(), vals.cpu().numpy().tobytes()) == g["fl_sha256"]
    del sh, bits, vals, x
    torch.cuda.empty_cache()


def test_device_sharded_repeat(local_comm):
    """Repeated exchanges on one comm, alternating shard counts: stable records."""
    from flrl.device import gen
    n = (64 << 20) + 333
    x = gen("lo4", n, 11)
    x[12345] = 0xFF
    ref = flrl.fl_compress(x[:n].cpu().numpy())
    for P in (3, 5, 3, 8, 1):
        sh = Shards(x, n, P)
        for _ in range(4):
            sh.encode(local_comm)
        rec, bits, vals = sh.place()
        assert sh.errors() == [0] * P
        assert np.array_equal(bits.cpu().numpy(), ref.bits), P
        assert np.array_equal(vals.cpu().numpy(), ref.values), P


def test_device_sharded_wrong_device_buffers(local_comm):
    """Shard buffers must be device memory of the shard's GPU."""
    from flrl.device import gen
    n = 1 << 20
    x = gen("u8", n, 1)
    sh = Shards(x, n, 2)
    host = np.zeros(64, dtype=np.uint8)
    with pytest.raises(flrl.FLRLError) as e:
        local_comm.encode_sharded([x.data_ptr(), x.data_ptr() + sh.off[1]], sh.len,
                                  [b.data_ptr() for b in sh.bits], [v.data_ptr() for v in sh.vals],
                                  [sh.sizes[0].data_ptr(), host.ctypes.data],
                                  [s.data_ptr() for s in sh.scr], sh.scr_b,
                                  [int(s.cuda_stream) for s in sh.streams])
    assert e.value.code == flrl.E_ARG


def test_device_sharded_rejects_ragged_shard(local_comm):
    """Every shard but the last must be whole frames (file_io.cu:46-51): a
    ragged earlier shard would misplace its successors, so it is refused."""
    from flrl.device import gen
    n = 1 << 20
    x = gen("u8", n, 1)
    sh = Shards(x, n, 3)
    lens = [sh.len[0] + 5, sh.len[1] - 5, sh.len[2]]
    with pytest.raises(flrl.FLRLError) as e:
        local_comm.encode_sharded([x.data_ptr(), x.data_ptr() + lens[0], x.data_ptr() + sh.off[2]], lens,
                                  [b.data_ptr() for b in sh.bits], [v.data_ptr() for v in sh.vals],
                                  [s.data_ptr() for s in sh.sizes], [s.data_ptr() for s in sh.scr], sh.scr_b,
                                  [int(s.cuda_stream) for s in sh.streams])
    assert e.value.code == flrl.E_ARG
    sh.len[2] -= 3  # a ragged LAST shard is fine
    sh.encode(local_comm)
    rec, bits, vals = sh.place()
    assert sh.errors() == [0] * 3
    ref = flrl.fl_compress(x[:n - 3].cpu().numpy())
    assert np.array_equal(bits.cpu().numpy(), ref.bits) and np.array_equal(vals.cpu().numpy(), ref.values)


def test_comm_init_errors():
    nd = flrl.device_count()
    with pytest.raises(flrl.FLRLError) as e:
        flrl.Comm.local(devs=[0, 0])
    assert e.value.code == flrl.E_ARG
    with pytest.raises(flrl.FLRLError) as e:
        flrl.Comm.local(devs=[nd])
    assert e.value.code == flrl.E_ARG
    with pytest.raises(flrl.FLRLError):
        flrl.Comm.rank(2, b"\0" * flrl.UNIQUE_ID_BYTES, 5)


@pytest.fixture(scope="module")
def rank_comm():
    torch.cuda.set_device(0)
    c = flrl.Comm.rank(1, flrl.comm_unique_id(), 0)
    yield c
    c.destroy()


def test_rank_comm_query(rank_comm, local_comm):
    assert rank_comm.query() == (1, 0, 1)
    assert local_comm.query() == (flrl.device_count(), 0, flrl.device_count())


def test_encode_rank_record(rank_comm, golden):
    """One-rank flrl_fl_encode_rank on the BMP: the record is {F, V, 0, 0, F, V}
    and the payload equals the reference fl-cpu's."""
    from flrl.device import FLDevice
    g = golden["fl_bmp"]
    with open(os.path.join(os.path.dirname(__file__), "golden", g["file"]), "rb") as f:
        a = np.frombuffer(f.read(), dtype=np.uint8)
    x = torch.from_numpy(a.copy()).cuda()
    d = FLDevice(a.size)
    for _ in range(3):
        d.encode_rank(rank_comm, x)
    torch.cuda.synchronize()
    rec = [int(t) for t in d.rank_sizes[:flrl.SZ_COUNT].cpu()]
    assert rec == [g["frames"], g["values_size"], 0, 0, g["frames"], g["values_size"]]
    assert d.error() == 0
    v = rec[flrl.SZ_V]
    assert file_sha(a.size, d.bits[:d.frames].cpu().numpy().tobytes(),
                    d.values[:v].cpu().numpy().tobytes()) == g["fl_sha256"]


def test_encode_rank_local_error_still_exchanges(rank_comm):
    """an undersized scratch is a local argument error,
    found before any encode launch; the rank still runs the all-gather (with a
    failed slot, flrl_shard_failed_word) and the size scan, so its peers see
    FLRL_E_ARG instead of waiting in the collective. On a one-rank comm: the
    call raises FLRL_E_ARG, the scan still wrote this rank's record (the failed
    slot reads F = V = 0), and the comm keeps working."""
    from flrl.device import FLDevice
    n = 1 << 20
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    d = FLDevice(n)
    d.rank_sizes = torch.full((8,), -1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(flrl.FLRLError) as e:
        rank_comm.encode_rank(x.data_ptr(), n, d.bits.data_ptr(), d.values.data_ptr(), d.rank_sizes.data_ptr(),
                              d.scratch.data_ptr(), 64, torch.cuda.current_stream().cuda_stream)
    assert e.value.code == flrl.E_ARG and "scratch" in str(e.value)
    torch.cuda.synchronize()
    assert [int(t) for t in d.rank_sizes[:flrl.SZ_COUNT].cpu()] == [0] * flrl.SZ_COUNT
    d.encode_rank(rank_comm, x)  # the next call works
    torch.cuda.synchronize()
    rec = [int(t) for t in d.rank_sizes[:flrl.SZ_COUNT].cpu()]
    v = rec[flrl.SZ_V]
    assert rec == [n // 128, v, 0, 0, n // 128, v] and v > 0
    assert d.error() == 0
    assert torch.equal(d.decode(v), x)


@pytest.mark.parametrize("step", [flrl.DEBUG_RANK_SET_DEVICE, flrl.DEBUG_RANK_STREAM_WAIT])
def test_encode_rank_runtime_failure_still_exchanges(rank_comm, step):
    """a rank whose hipSetDevice or hipStreamWaitEvent
    fails (injected, flrl_debug_fail_rank_step) still enters the all-gather --
    from the comm's constant failed pair when it cannot reach its device, with
    a failed slot written on the comm's stream otherwise -- so its peers never
    wait in the collective. On a one-rank comm: the call returns FLRL_E_HIP,
    and the comm keeps working."""
    from flrl.device import FLDevice
    n = 1 << 20
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    d = FLDevice(n)
    d.encode_rank(rank_comm, x)  # a successful call first: the slot holds a real record
    torch.cuda.synchronize()
    flrl.debug_fail_rank_step(step)
    with pytest.raises(flrl.FLRLError) as e:
        d.encode_rank(rank_comm, x)
    assert e.value.code == flrl.E_HIP
    torch.cuda.synchronize()
    if step == flrl.DEBUG_RANK_STREAM_WAIT:  # the scan ran on the failed slot
        assert [int(t) for t in d.rank_sizes[:flrl.SZ_COUNT].cpu()] == [0] * flrl.SZ_COUNT
    d.encode_rank(rank_comm, x)  # the hook fired once; the next call works
    torch.cuda.synchronize()
    rec = [int(t) for t in d.rank_sizes[:flrl.SZ_COUNT].cpu()]
    assert rec[flrl.SZ_F] == n // 128 and d.error() == 0
    assert torch.equal(d.decode(rec[flrl.SZ_V]), x)


@pytest.mark.parametrize("step", [flrl.DEBUG_RANK_SET_DEVICE, flrl.DEBUG_RANK_STREAM_WAIT])
def test_encode_rank_failure_between_calls_without_sync(rank_comm, step):
    """a failed call whose slot could not be staged sends
    the comm's constant failed pair from the comm's stream, and that all-gather
    still RECEIVES into the gather array. Issued right behind a good call and
    right before another, with no host synchronisation in between, it must not
    overwrite the array while the earlier call's size scan is still pending on
    the caller's stream, nor after the next call's slot write: both good calls
    keep their records and their scratch error words stay 0. 256 MiB inputs
    keep the earlier call's scan queued behind its encode when the failed call
    is issued."""
    from flrl.device import FLDevice
    n = 256 << 20
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    a, f, b = FLDevice(n), FLDevice(n), FLDevice(n)
    torch.cuda.synchronize()
    for _ in range(3):
        a.encode_rank(rank_comm, x)
        flrl.debug_fail_rank_step(step)
        with pytest.raises(flrl.FLRLError) as e:
            f.encode_rank(rank_comm, x)
        assert e.value.code == flrl.E_HIP
        b.encode_rank(rank_comm, x)
        torch.cuda.synchronize()
        for name, d in (("first", a), ("next", b)):
            rec = [int(t) for t in d.rank_sizes[:flrl.SZ_COUNT].cpu()]
            assert rec == [n // 128, n, 0, 0, n // 128, n], (name, rec)
            assert d.error() == 0, name
    flrl.debug_fail_rank_step(0)


def test_comm_destroy_right_after_encode_rank():
    """A per-rank call's size scan runs on the caller's stream and reads the
    comm's gather array; destroying the comm right after the call (no host
    synchronisation) waits for that scan before freeing the array, so the
    record is still the right one."""
    from flrl.device import FLDevice
    torch.cuda.set_device(0)
    n = 256 << 20
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    d = FLDevice(n)
    torch.cuda.synchronize()
    for _ in range(2):
        c = flrl.Comm.rank(1, flrl.comm_unique_id(), 0)
        d.rank_sizes = torch.full((8,), -1, dtype=torch.int64, device="cuda")
        d.encode_rank(c, x)
        c.destroy()
        torch.cuda.synchronize()
        assert [int(t) for t in d.rank_sizes[:flrl.SZ_COUNT].cpu()] == [n // 128, n, 0, 0, n // 128, n]
        assert d.error() == 0


@pytest.mark.parametrize("step", [flrl.DEBUG_RANK_SET_DEVICE, flrl.DEBUG_RANK_STREAM_WAIT,
                                  flrl.DEBUG_RANK_STAGE_WORD, flrl.DEBUG_RANK_READ_SUM])
def test_compress_rank_runtime_failure_returns(rank_comm, golden, bmp_bytes, step):
    """flrl_fl_compress_rank with a failure injected at
    each collective step -- the exchange (device unreachable, stream order),
    staging the {size, failed} word (the constant {0, 1} is reduced instead),
    reading the reduced word back -- returns an error instead of hanging, and
    the next call on the same comm gives the reference result."""
    flrl.debug_fail_rank_step(step)
    with pytest.raises(flrl.FLRLError) as e:
        rank_comm.compress_rank(bmp_bytes)
    assert e.value.code == flrl.E_HIP
    c = rank_comm.compress_rank(bmp_bytes)
    assert file_sha(c.input_size, c.bits.tobytes(), c.values.tobytes()) == golden["fl_bmp"]["fl_sha256"]


def test_debug_fail_rank_step_rejects_unknown():
    with pytest.raises(flrl.FLRLError):
        flrl.debug_fail_rank_step(9)
    flrl.debug_fail_rank_step(0)


def test_encode_rank_rejects_sharded_comm(local_comm):
    from flrl.device import FLDevice
    if flrl.device_count() > 1:
        x = torch.zeros(256, dtype=torch.uint8, device="cuda")
        with pytest.raises(flrl.FLRLError) as e:
            FLDevice(256).encode_rank(local_comm, x)
        assert e.value.code == flrl.E_ARG


def test_compress_rank_one_rank(rank_comm, golden, bmp_bytes):
    """flrl_fl_compress_rank (gpuNCCLCompress twin) with one rank: rank 0 gets
    the whole result."""
    c = rank_comm.compress_rank(bmp_bytes)
    assert c.input_size == len(bmp_bytes)
    assert file_sha(c.input_size, c.bits.tobytes(), c.values.tobytes()) == golden["fl_bmp"]["fl_sha256"]
    e = rank_comm.compress_rank(b"")
    assert e.input_size == 0 and e.bits.size == 0 and e.values.size == 0
