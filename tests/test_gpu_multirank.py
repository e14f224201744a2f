"""flrl_fl_compress_rank across real ranks on two GPUs: the
reference's one-process-per-GPU call, gpuNCCLCompress (src/fl/fl_gpu.cu:76-287),
run by two processes over an RCCL communicator. One case checks the merged
result on rank 0 against the single-GPU encode of the whole input; the others
inject a failure on rank 1 at each collective step (flrl_debug_fail_rank_step)
and check that BOTH ranks return an error within a time limit instead of
waiting in a collective. FLRL_DEBUG_RANK_READ_SUM is deliberately not among
them: a device that fails after the {size, failed} all-reduce but before its
result reaches the host is the one documented non-collective case
(include/flrl.h, flrl_fl_compress_rank) -- its peers wait in the payload
send/recv, so that case would hang here by design. Needs two visible GPUs;
skipped otherwise (the round's
one-GPU box runs the same steps on a one-rank communicator in
tests/test_gpu_shard.py)."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import flrl

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, os.path.join(sys.argv[1], "fl-rl-compression-mpi_amd"))
    import numpy as np
    import flrl
    root, rank, world, step, tmp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    uid_path = os.path.join(tmp, "uid")
    if rank == 0:
        uid = flrl.comm_unique_id()
        with open(uid_path + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(uid_path + ".tmp", uid_path)
    else:
        for _ in range(600):
            if os.path.exists(uid_path):
                break
            time.sleep(0.1)
        uid = open(uid_path, "rb").read()
    import torch
    torch.cuda.set_device(rank)
    comm = flrl.Comm.rank(world, uid, rank)
    data = np.fromfile(os.path.join(tmp, "input"), dtype=np.uint8)
    start, n = flrl.shard_range(data.size, world, rank)
    if rank == 1 and step:
        flrl.debug_fail_rank_step(step)
    out = os.path.join(tmp, f"rank{rank}")
    try:
        c = comm.compress_rank(data[start:start + n])
        if rank == 0:
            np.save(out + "_bits.npy", c.bits)
            np.save(out + "_values.npy", c.values)
        open(out + ".ok", "w").write(str(c.input_size))
    except flrl.FLRLError as e:
        open(out + ".err", "w").write(str(e.code))
    comm.destroy()
""")


def _run_two_ranks(tmp_path, data: np.ndarray, step: int, timeout: float = 120.0):
    data.tofile(tmp_path / "input")
    procs = []
    for rank in range(2):
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER, ROOT, str(rank), "2", str(step), str(tmp_path)],
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=timeout)[0].decode(errors="replace"))
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        pytest.fail(f"a rank did not return within {timeout} s (step {step}): a collective left a peer waiting")
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-2000:]
    return [(tmp_path / f"rank{r}.ok").exists() for r in range(2)], [(tmp_path / f"rank{r}.err") for r in range(2)]


@pytest.fixture(scope="module", autouse=True)
def _two_gpus():
    if flrl.device_count() < 2:
        pytest.skip("needs two visible GPUs")


def test_compress_rank_two_ranks_matches_single(tmp_path):
    rng = np.random.default_rng(5)
    data = (rng.integers(0, 256, size=(8 << 20) + 77, dtype=np.uint8) >> 2).astype(np.uint8)
    ok, _ = _run_two_ranks(tmp_path, data, 0)
    assert ok == [True, True]
    whole = flrl.fl_compress(data)
    assert np.array_equal(np.load(tmp_path / "rank0_bits.npy"), whole.bits)
    assert np.array_equal(np.load(tmp_path / "rank0_values.npy"), whole.values)


@pytest.mark.parametrize("step", [flrl.DEBUG_RANK_SET_DEVICE, flrl.DEBUG_RANK_STREAM_WAIT,
                                  flrl.DEBUG_RANK_STAGE_WORD])
def test_compress_rank_failure_on_one_rank_fails_both(tmp_path, step):
    rng = np.random.default_rng(6)
    data = rng.integers(0, 256, size=(4 << 20) + 5, dtype=np.uint8)
    ok, err = _run_two_ranks(tmp_path, data, step)
    assert ok == [False, False], "both ranks must report the failure"
    assert all(e.exists() for e in err)
