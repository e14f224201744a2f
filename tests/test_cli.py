"""The `compress` CLI (reference src/main.cu, src/args_parser.cu) on host-only
methods: fl-cpu output is byte-identical to the reference's fl-cpu (golden
sha256), rl-cpu round-trips and matches the oracle, usage errors exit 1,
malformed files are rejected."""
import hashlib
import subprocess

import numpy as np
import pytest

import flrl
import oracle


def run(cli, *args, check=True):
    return subprocess.run([cli, *map(str, args)], capture_output=True, text=True, check=check)


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def test_fl_cpu_bmp_matches_reference(cli_path, golden, bmp_bytes, tmp_path):
    src = tmp_path / "in.bmp"
    src.write_bytes(bmp_bytes)
    r = run(cli_path, "c", "fl-cpu", src, tmp_path / "o.fl")
    assert '[TIMER] Step: "Compression"' in r.stdout
    assert sha((tmp_path / "o.fl").read_bytes()) == golden["fl_bmp"]["fl_sha256"]
    run(cli_path, "d", "fl-cpu", tmp_path / "o.fl", tmp_path / "back.bin")
    assert (tmp_path / "back.bin").read_bytes() == bmp_bytes


@pytest.mark.parametrize("idx", range(7))
def test_fl_cpu_generated(cli_path, golden, tmp_path, idx):
    g = golden["fl_generated"][idx]
    a = oracle.gen(g["kind"], g["n"], g["seed"])
    (tmp_path / "in").write_bytes(a.tobytes())
    run(cli_path, "c", "fl-cpu", tmp_path / "in", tmp_path / "o.fl")
    assert sha((tmp_path / "o.fl").read_bytes()) == g["fl_sha256"]


def test_fl_cpu_empty(cli_path, golden, tmp_path):
    (tmp_path / "e").write_bytes(b"")
    run(cli_path, "c", "fl-cpu", tmp_path / "e", tmp_path / "e.fl")
    assert sha((tmp_path / "e.fl").read_bytes()) == golden["fl_empty_file_sha256"]
    run(cli_path, "d", "fl-cpu", tmp_path / "e.fl", tmp_path / "e.out")
    assert (tmp_path / "e.out").read_bytes() == b""


@pytest.mark.parametrize("kind", ["runs32", "longruns", "u8", "zero"])
def test_rl_cpu_roundtrip_matches_oracle(cli_path, tmp_path, kind):
    a = oracle.gen(kind, 200_003, 8)
    (tmp_path / "in").write_bytes(a.tobytes())
    run(cli_path, "c", "rl-cpu", tmp_path / "in", tmp_path / "o.rl")
    blob = (tmp_path / "o.rl").read_bytes()
    counts, values = oracle.rl_compress(a)
    assert blob == flrl.rl_file_bytes(a.size, counts, values)
    run(cli_path, "d", "rl-cpu", tmp_path / "o.rl", tmp_path / "back")
    assert (tmp_path / "back").read_bytes() == a.tobytes()


def test_rl_cpu_kats(cli_path, golden, tmp_path):
    from conftest import kat_input
    for case in golden["rl_kat"]:
        data = kat_input(case)
        (tmp_path / "in").write_bytes(data)
        run(cli_path, "c", "rl-cpu", tmp_path / "in", tmp_path / "o.rl")
        r = flrl.parse_rl_file((tmp_path / "o.rl").read_bytes())
        assert r.counts.tolist() == case["counts"] and r.values.tolist() == case["values"]


@pytest.mark.parametrize("argv", [[], ["c"], ["x", "fl", "a", "b"], ["c", "zz", "a", "b"],
                                  ["c", "fl", "a", "b", "extra"]])
def test_usage_errors_exit_1(cli_path, argv):
    r = run(cli_path, *argv, check=False)
    assert r.returncode == 1
    assert "USAGE" in r.stderr


def test_missing_input_reports_error(cli_path, tmp_path):
    r = run(cli_path, "c", "fl-cpu", tmp_path / "nope", tmp_path / "o", check=False)
    assert r.returncode == 2 and "[ERROR]:" in r.stderr
    assert not (tmp_path / "o").exists()


def test_malformed_fl_files_rejected(cli_path, tmp_path):
    a = oracle.gen("lo4", 3000, 1)
    good = oracle.fl_file_bytes(a)
    cases = {
        "truncated_header": good[:20],
        "truncated_values": good[:-3],
        "bad_width": good[:24] + bytes([0]) + good[25:],
        "width9": good[:24] + bytes([9]) + good[25:],
        "bits_size_lies": (3000).to_bytes(8, "little") + (5).to_bytes(8, "little") + good[16:],
    }
    for name, blob in cases.items():
        (tmp_path / name).write_bytes(blob)
        r = run(cli_path, "d", "fl-cpu", tmp_path / name, tmp_path / "out", check=False)
        assert r.returncode == 2, name
        assert "[ERROR]:" in r.stderr, name


def test_malformed_rl_files_rejected(cli_path, tmp_path):
    blob = flrl.rl_file_bytes(5, [2, 0], [1, 1])  # zero count / wrong sum
    (tmp_path / "bad.rl").write_bytes(blob)
    r = run(cli_path, "d", "rl-cpu", tmp_path / "bad.rl", tmp_path / "o", check=False)
    assert r.returncode == 2


@pytest.mark.parametrize("method", ["fl", "fl-nccl", "rl"])
def test_gpu_methods_fail_loudly_without_device(cli_path, tmp_path, method):
    if flrl.device_count() > 0:
        pytest.skip("a HIP device is visible")
    src, out = tmp_path / "in", tmp_path / "out"
    src.write_bytes(bytes(range(200)))
    r = subprocess.run([cli_path, "c", method, str(src), str(out)], capture_output=True, text=True)
    assert r.returncode == 2 and "[ERROR]" in r.stderr
    assert not out.exists()


@pytest.mark.parametrize("method", ["fl-cpu", "rl-cpu"])
def test_failed_run_keeps_existing_output(cli_path, tmp_path, method):
    """A run that fails (missing input, malformed input) leaves a pre-existing
    output byte-for-byte alone and no temporary file behind."""
    out = tmp_path / "old.out"
    out.write_bytes(b"precious")
    r = run(cli_path, "c", method, tmp_path / "missing.bin", out, check=False)
    assert r.returncode == 2 and "[ERROR]:" in r.stderr
    assert out.read_bytes() == b"precious"
    (tmp_path / "bad").write_bytes(b"\x01\x02")  # truncated header
    r = run(cli_path, "d", method, tmp_path / "bad", out, check=False)
    assert r.returncode == 2
    assert out.read_bytes() == b"precious"
    assert sorted(p.name for p in tmp_path.iterdir()) == ["bad", "old.out"]


@pytest.mark.parametrize("method", ["fl-cpu", "rl-cpu"])
def test_input_may_be_output(cli_path, tmp_path, method):
    """`compress c <m> f f` then `compress d <m> f f` restores f (the reference
    loads the whole input before saving, so in == out works there too)."""
    a = oracle.gen("lo4", 100_003, 5)
    f = tmp_path / "f"
    f.write_bytes(a.tobytes())
    run(cli_path, "c", method, f, f)
    if method == "fl-cpu":
        assert f.read_bytes() == oracle.fl_file_bytes(a)
    run(cli_path, "d", method, f, f)
    assert f.read_bytes() == a.tobytes()
    assert [p.name for p in tmp_path.iterdir()] == ["f"]


def test_output_mode_follows_umask(cli_path, tmp_path):
    import os
    import stat
    (tmp_path / "in").write_bytes(b"abc" * 100)
    old = os.umask(0o027)
    try:
        run(cli_path, "c", "fl-cpu", tmp_path / "in", tmp_path / "o.fl")
    finally:
        os.umask(old)
    assert stat.S_IMODE((tmp_path / "o.fl").stat().st_mode) == 0o640


def test_output_to_dev_null(cli_path, tmp_path):
    (tmp_path / "in").write_bytes(b"abc" * 100)
    run(cli_path, "c", "fl-cpu", tmp_path / "in", "/dev/null")


def test_existing_output_keeps_mode_and_symlink(cli_path, tmp_path):
    """Replacing an existing output keeps its mode; a symlinked output's target
    is replaced and the link stays a link (as fopen "wb" would)."""
    import os
    import stat
    src = tmp_path / "in"
    a = oracle.gen("lo4", 5000, 2)
    src.write_bytes(a.tobytes())
    out = tmp_path / "o.fl"
    out.write_bytes(b"old")
    os.chmod(out, 0o600)
    run(cli_path, "c", "fl-cpu", src, out)
    assert stat.S_IMODE(out.stat().st_mode) == 0o600
    assert out.read_bytes() == oracle.fl_file_bytes(a)
    sub = tmp_path / "sub"
    sub.mkdir()
    target = sub / "target.fl"
    target.write_bytes(b"old")
    os.chmod(target, 0o640)
    link = tmp_path / "link.fl"
    link.symlink_to(target)
    run(cli_path, "c", "fl-cpu", src, link)
    assert link.is_symlink() and os.readlink(link) == str(target)
    assert target.read_bytes() == oracle.fl_file_bytes(a)
    assert stat.S_IMODE(target.stat().st_mode) == 0o640
    assert sorted(p.name for p in sub.iterdir()) == ["target.fl"]
