"""bench.py's rank launcher (CPU): `python bench.py --gpus N` with N > 1 and no
torch.distributed environment starts the N ranks itself, as a child
torch.distributed.run (never an exec), before anything touches the GPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_single_gpu_runs_in_process():
    assert bench.rank_launch_cmd([], {}) is None
    assert bench.rank_launch_cmd(["--gpus", "1", "--steps", "3"], {}) is None


def test_already_a_rank_does_not_relaunch():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert bench.rank_launch_cmd(["--gpus", "8"], env) is None


def test_launch_command_shape():
    argv = ["--gpus", "8", "--steps", "7", "--warmup", "2"]
    cmd = bench.rank_launch_cmd(argv, {})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert len(port) == 1 and 0 < int(port[0].split("=")[1]) < 65536
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv  # the ranks see the same arguments
    assert bench.rank_launch_cmd(["--gpus=4"], {})[4] == "--nproc-per-node=4"


def test_launcher_end_to_end_help():
    """The parent spawns 2 ranks that parse their own arguments (--help exits
    before any device work) and returns their exit status."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--help"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("usage:") == 2  # each rank printed its usage


def test_rank_shard_weak_and_strong():
    """--bytes (weak): fixed bytes per rank; --global-bytes (strong, VERDICT r03
    missing item 2): a fixed total split by the reference rule, shards
    frame-aligned but the last, covering the total exactly."""
    assert bench.rank_shard(1 << 30, 0, 4, 3) == (3 << 30, 1 << 30, 4 << 30)
    for B, N in ((16 << 30, 8), (512_000_000, 3), ((1 << 24) + 77, 2), (128 * 5, 5), (1000, 1)):
        parts = [bench.rank_shard(0, B, N, r) for r in range(N)]
        assert all(t == B for _, _, t in parts)
        assert parts[0][0] == 0 and sum(n for _, n, _ in parts) == B
        for (s0, n0, _), (s1, _, _) in zip(parts, parts[1:]):
            assert s1 == s0 + n0 and n0 % 128 == 0 and s1 % 8 == 0
    try:
        bench.rank_shard(0, 100, 2, 0)
        raise AssertionError("a rank without a frame must be refused")
    except SystemExit:
        pass


def test_cpu_baseline_on_every_line():
    """VERDICT r05 missing item 2: north_star asks for the fl-cpu / rl-cpu
    figure "in the same run" at 1, 2, 4 and 8 GPUs, so rank 0 of an N > 1 line
    carries `cpu_baseline` too (FL on the first bytes of its shard, plus the RL
    oracle, which at N = 1 the RL section times itself); other ranks carry none,
    and --cpu-sample 0 skips it."""
    n = 1 << 20
    for world in (1, 2, 8):
        cpu = bench.line_cpu_baseline(0, world, "u8", 42, n)
        assert cpu is not None and cpu["value"] > 0 and cpu["cores"] == 1 and cpu["kind"] == "port"
        assert cpu["roundtrip_ok"]
        assert ("rl" in cpu) == (world > 1)
        if world > 1:
            assert cpu["rl"]["value"] > 0 and cpu["rl"]["roundtrip_ok"] and cpu["rl"]["runs"] > n // 64
        assert bench.line_cpu_baseline(1, world, "u8", 42, n) is None
    assert bench.line_cpu_baseline(0, 2, "u8", 42, 0) is None
