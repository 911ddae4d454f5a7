"""Native host unit tests (csrc/tests/test_host.cpp), plain and under the
host sanitizers: ASan+UBSan and ThreadSanitizer (SURVEY §5 race detection:
the reference only had a valgrind script, unitest/valgrind.sh).  GPU code is
not in this binary (no GPU sanitizer runs on this pool)."""
import shutil
import subprocess

import pytest


@pytest.mark.parametrize("variant", ["plain", "asan", "tsan"])
def test_host_cpp_suite(variant):
    if shutil.which("g++") is None:
        pytest.skip("no host C++ compiler")
    from swiftsnails_amd._build import build_cpp_tests

    exe = build_cpp_tests(variant)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "0 failed expectations" in r.stdout
    assert "ThreadSanitizer" not in out and "AddressSanitizer" not in out, out[-4000:]
    assert "runtime error" not in out, out[-4000:]  # UBSan
