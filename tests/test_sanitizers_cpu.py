"""Sanitizer builds of the native host code: the TCP/File stores and a
multi-threaded stress driver compiled with AddressSanitizer+UBSan and with ThreadSanitizer, and the
whole extension's host code (Reducer, communicators, bindings) under both, driving W=2 DDP
scenarios (``_san_scenarios.py``)."""
import os
import shutil
import subprocess
import sys

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


_SCENARIOS = ["collectives", "parity_and_no_sync", "find_unused_and_static", "join_uneven"]
_BUILT: dict = {}  # sanitizer -> instrumented package root (one build per session)


def _san_env(tmp_path_factory, san, **extra):
    from distributeddataparallel_amd import _build

    try:
        rt = _build.sanitizer_runtime(san)
    except FileNotFoundError as e:
        pytest.skip(str(e))
    if san not in _BUILT:
        out = tmp_path_factory.mktemp("san_" + san.replace(",", "_"))
        _build.build_sanitized(san, out)
        _BUILT[san] = out
    pre = os.environ.get("LD_PRELOAD")  # the runtime must come first; keep anything already preloaded
    env = dict(os.environ, XDDP_PKG_ROOT=str(_BUILT[san]), LD_PRELOAD=f"{rt}:{pre}" if pre else str(rt),
               OMP_NUM_THREADS="1",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0:report_mutex_bugs=0:suppressions="
                            + os.path.join(REPO, "tests", "tsan_suppressions.txt"))
    env.pop("XDDP_TSAN_CANARY", None)
    env.update(extra)
    return env


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_reducer_and_cpu_backend_under_sanitizer(tmp_path_factory, san):
    """The Reducer (autograd hooks, bucket launches, rebuild, finalize callback, no_sync,
    find_unused_parameters, static graph, join) and the CPU ring backend's worker thread, built
    with ASan+UBSan / TSan (``_build.build_sanitized``: host code instrumented, device objects of
    the regular build), W=2 ranks, halt_on_error. TSan runs with NO race suppressions
    (``tsan_suppressions.txt`` is empty; torch / python are uninstrumented, so only xddp's own
    accesses can be reported) and mutex-misuse reports off (torch's own locking is uninstrumented)."""
    env = _san_env(tmp_path_factory, san)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "_san_driver.py"), *_SCENARIOS],
                       capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode == 0 and "sanitizer scenarios OK" in r.stdout, (r.stdout[-2000:], r.stderr[-8000:])
    assert "Sanitizer" not in r.stderr, r.stderr[-8000:]


def test_tsan_reports_reducer_canary_race(tmp_path_factory):
    """The TSan run can fail: XDDP_TSAN_CANARY=1 makes the Reducer race a plain counter between a
    hook-side thread (as the autograd engine's device threads run the hooks of GPU parameters) and
    prepare_for_backward. The same build, options and suppression file as the clean run must
    report it — a data race naming xddp::Reducer — and the run must fail."""
    env = _san_env(tmp_path_factory, "thread", XDDP_TSAN_CANARY="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "_san_driver.py"), "parity_and_no_sync"],
                       capture_output=True, text=True, env=env, timeout=900)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "WARNING: ThreadSanitizer: data race" in r.stderr, r.stderr[-6000:]
    assert "xddp::Reducer::prepare_for_backward" in r.stderr and "xddp::Reducer::autograd_hook" in r.stderr, \
        r.stderr[-6000:]
