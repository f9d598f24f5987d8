"""Sanitizer builds of the native host code: the TCP/File stores and a
multi-threaded stress driver compiled with AddressSanitizer+UBSan and with ThreadSanitizer."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "distributeddataparallel_amd", "csrc")
SRCS = [os.path.join(CSRC, "store", "tcp_store.cpp"), os.path.join(CSRC, "store", "file_store.cpp"),
        os.path.join(CSRC, "tests", "store_stress.cpp")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_store_stress_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "store_stress")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-I", CSRC, *SRCS,
           "-o", exe, "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "store_stress OK" in r.stdout, (r.stdout[-2000:], r.stderr[-6000:])
