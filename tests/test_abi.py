"""The C-ABI library loads and exports every symbol include/flrl.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import os
import subprocess

import pytest

import flrl


def test_exports_every_declared_symbol():
    syms = flrl.declared_symbols()
    assert len(syms) >= 18
    lib = flrl.lib_handle()
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, f"declared but not exported: {missing}"


def test_exports_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", flrl.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in flrl.declared_symbols():
        assert s in exported, s


def test_gfx950_code_object(tmp_path):
    # llvm-objdump --offloading extracts the code objects next to its input:
    # run it on a copy so nothing lands beside the shipped library
    import shutil
    lib = tmp_path / "libflrl.so"
    shutil.copy(flrl.LIB_PATH, lib)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    if "gfx950" not in text:  # older objdump: fall back to the bundle string
        with open(flrl.LIB_PATH, "rb") as f:
            assert b"gfx950" in f.read()


def test_sizing_functions_are_pure():
    assert flrl.fl_values_capacity(0) == 16
    assert flrl.fl_values_capacity(17) == 32
    s1 = flrl.fl_scratch_bytes(1)
    s2 = flrl.fl_scratch_bytes(1 << 30)
    assert s1 >= 24 and s2 > s1 and s2 % 16 == 0
    assert flrl.version().startswith("flrl")


def test_no_silent_cpu_fallback_without_device():
    if flrl.device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(flrl.FLRLError) as e:
        flrl.fl_compress(b"abc")
    assert e.value.code == flrl.E_NODEV
    # empty input never needs the device (fl_gpu.cu:291-294)
    assert flrl.fl_compress(b"").input_size == 0


def test_file_format_helpers():
    import numpy as np
    blob = flrl.fl_file_bytes(5, np.array([3], np.uint8), np.array([1, 2], np.uint8))
    assert blob[:24] == (5).to_bytes(8, "little") + (1).to_bytes(8, "little") + (2).to_bytes(8, "little")
    c = flrl.parse_fl_file(blob)
    assert c.input_size == 5 and c.bits.tolist() == [3] and c.values.tolist() == [1, 2]
    r = flrl.parse_rl_file(flrl.rl_file_bytes(4, [1, 3], [9, 8]))
    assert r.input_size == 4 and r.counts.tolist() == [1, 3] and r.values.tolist() == [9, 8]
    with pytest.raises(ValueError):
        flrl.parse_fl_file(blob[:-1])


def test_file_codec_needs_device(tmp_path):
    if flrl.device_count() > 0:
        pytest.skip("a HIP device is visible")
    src = tmp_path / "in"
    src.write_bytes(b"abc")
    for fn in (flrl.fl_compress_file, flrl.fl_decompress_file):
        with pytest.raises(flrl.FLRLError) as e:
            fn(str(src), str(tmp_path / "out"), 1, 0)
        assert e.value.code == flrl.E_NODEV


def test_time_next_kernel_arguments():
    """The measurement hook takes both events or neither (no GPU work)."""
    f = flrl.lib_handle().flrl_time_next_kernel
    assert f(ctypes.c_void_p(16), None) == flrl.E_ARG
    assert f(None, ctypes.c_void_p(16)) == flrl.E_ARG
    assert f(None, None) == flrl.E_OK
    with pytest.raises(ValueError):
        flrl.time_next_kernel(0, 0)  # a not-yet-created event handle


def test_scratch_sizes_monotone():
    # callers size scratch once for an upper bound (RLDevice: runs <= n; the
    # streamed decode: runs <= chunk), so a smaller count must never need more
    k = 32768 * 1024  # decode pre-pass: one more round per workgroup past this many runs
    pts = sorted({1, 2, 2047, 2048, 2049, 4096, 32767, 32768, 32769, 10 ** 6}
                 | {m * k + d for m in (1, 2, 3, 7) for d in (-32769, -1, 0, 1, 32768, 10 ** 6)})
    for f in (flrl.rl_decode_scratch_bytes, flrl.rl_scratch_bytes, flrl.fl_scratch_bytes):
        sizes = [f(x) for x in pts]
        assert sizes == sorted(sizes), f.__name__


def test_rl_encode_scratch_small():
    # the single-pass encode needs only its tile states (one 128-byte status
    # line per 128 KiB tile): under 1 % of n, growing with n
    pts = [1, 4096, 131072, 131073, 10 ** 6, 1 << 30]
    sizes = [flrl.rl_scratch_bytes(x) for x in pts]
    assert sizes == sorted(sizes)
    big = flrl.rl_scratch_bytes(1 << 30)
    assert big < (1 << 30) // 100
    assert big == flrl.lib_handle().flrl_rl_scratch_bytes(1 << 30)


def test_three_pass_form_removed():
    # round 4: the scan/state/emit form and its entry points are gone
    import ctypes
    lib = ctypes.CDLL(flrl.LIB_PATH)
    for sym in ("flrl_rl_encode_device_form", "flrl_rl_scratch_bytes_form"):
        assert not hasattr(lib, sym), sym


def test_tuning_overrides_need_the_tuning_build(tmp_path):
    """A kernel-shape override (-DFLRL_RL_STAGE=..., any FLRL_* knob of
    csrc/flrl_tuning.hpp) is a compile error unless FLRL_TUNING_BUILD is also
    defined, so a stray -D cannot change the shipped library; the shipped
    defaults compile clean."""
    inc = os.path.join(os.path.dirname(flrl.LIB_PATH), "..", "csrc")
    src = tmp_path / "t.cpp"
    src.write_text('#include "flrl_tuning.hpp"\nint main() { return FLRL_RL_STAGE > 0 ? 0 : 1; }\n')

    def cc(*defs):
        return subprocess.run(["g++", "-fsyntax-only", "-I", inc, *defs, str(src)], capture_output=True, text=True)

    assert cc().returncode == 0
    bad = cc("-DFLRL_RL_STAGE=1024")
    assert bad.returncode != 0 and "FLRL_TUNING_BUILD" in bad.stderr
    assert cc("-DFLRL_RL_STAGE=1024", "-DFLRL_TUNING_BUILD").returncode == 0
