"""Host-side race / memory-error detection for the native C++ TCP rendezvous store (csrc/store_core.h): the
stress driver csrc/tests/store_stress.cpp (server acceptor + per-connection threads, blocking GETs on a
condition variable, ADD counters, barriers, timeouts, teardown with a blocked waiter; 8 client threads) built
and run under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer (SURVEY §5 race
detection).  CPU only: g++ with the sanitizer runtimes."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "tests", "store_stress.cpp")
GXX = shutil.which("g++")


def _build_run(tmp_path, flags, env):
    exe = str(tmp_path / "store_stress")
    b = subprocess.run([GXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", *flags,
                        f"-I{os.path.join(ROOT, 'csrc')}", SRC, "-o", exe], capture_output=True, text=True)
    if b.returncode != 0 and "cannot find" in b.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {b.stderr[-300:]}")
    assert b.returncode == 0, b.stderr[-3000:]
    r = subprocess.run([exe, "8", "20"], capture_output=True, text=True, timeout=300, env=dict(os.environ, **env))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "0 errors" in out
    return out


@pytest.mark.skipif(GXX is None, reason="needs g++")
def test_store_under_asan_ubsan(tmp_path):
    out = _build_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                     {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert "AddressSanitizer" not in out and "runtime error" not in out


@pytest.mark.skipif(GXX is None, reason="needs g++")
def test_store_under_tsan(tmp_path):
    out = _build_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})
    assert "ThreadSanitizer" not in out
