"""The CPU oracle under AddressSanitizer + UBSan (oracle/asan_check.c).

Builds the oracle together with a driver that calls every orc_* entry point
on small seeded inputs and edge shapes (one row, K = n - 1, all-NA columns,
8/16-bit codes, the SNN capacity query) with exactly sized buffers, and runs
it: any out-of-bounds access, use after free or undefined arithmetic in the
checker aborts the run.  CPU only."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


def test_oracle_is_memory_safe(tmp_path):
    if shutil.which("gcc") is None or shutil.which("make") is None:
        pytest.skip("gcc/make not available")
    exe = tmp_path / "asan_check"
    b = subprocess.run(["make", "-s", "-C", ORACLE, "asan", f"ASAN_OUT={exe}"], capture_output=True, text=True)
    if b.returncode != 0 and "sanitize" in (b.stderr or ""):
        pytest.skip("toolchain without AddressSanitizer: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="2")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ok" in r.stdout
