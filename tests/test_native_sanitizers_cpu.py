"""Host native code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 race detection /
sanitizers).  The host runtime (csrc/host_data.cpp) is compiled together with a C++ harness
(tests/native/host_data_check.cpp) with ``-fsanitize=address,undefined`` and run as its own
process: any out-of-bounds access, overflow or UB aborts it.  GPU kernels are not built with
sanitizers (not available on the GPU pool); their bounds are covered by the numerics tests."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "distributed_training_compare_jax_amd", "csrc", "host_data.cpp")
HARNESS = os.path.join(ROOT, "tests", "native", "host_data_check.cpp")


def _cxx():
    return os.environ.get("CXX") or shutil.which("g++") or shutil.which("clang++")


@pytest.mark.skipif(_cxx() is None, reason="no host C++ compiler")
def test_host_data_asan_ubsan(tmp_path):
    exe = str(tmp_path / "host_data_check")
    flags = ["-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=all"]
    r = subprocess.run([_cxx(), *flags, HARNESS, SRC, "-o", exe], capture_output=True, text=True)
    if r.returncode != 0 and "asan" in (r.stderr or "").lower():
        pytest.skip(f"sanitizer runtime unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert run.returncode == 0, (run.stdout + run.stderr)[-3000:]
    assert "ok" in run.stdout
