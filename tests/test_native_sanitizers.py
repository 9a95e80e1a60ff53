"""Tier T1: the host C++ runtime built with sanitizers.

tests/native/runtime_selftest.cpp drives the process supervisor (spawn,
pidfd/epoll exit events, kill, two concurrent waiters) and the A/B
shared-memory checkpoint store (commits racing a reader) — compiled together
with csrc/runtime/{supervisor,shm_store}.cpp under AddressSanitizer +
UndefinedBehaviorSanitizer, and under ThreadSanitizer.  Host code only (GPU
sanitizers are not available on the MI355X pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
SRCS = [os.path.join(ROOT, "tests", "native", "runtime_selftest.cpp"),
        os.path.join(ROOT, "csrc", "runtime", "supervisor.cpp"),
        os.path.join(ROOT, "csrc", "runtime", "shm_store.cpp")]


def _build_and_run(tmp_path, flags, env_extra):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "selftest")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, "-D__HIP_PLATFORM_AMD__",
           f"-I{ROCM}/include", *SRCS, "-o", exe, f"-L{ROCM}/lib", "-lamdhip64", "-lpthread", "-ldl",
           f"-Wl,-rpath,{ROCM}/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "runtime selftest OK" in r.stdout
    return r


def test_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
                   {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0", "UBSAN_OPTIONS": "halt_on_error=1"})


def test_runtime_tsan(tmp_path):
    r = _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1:report_signal_unsafe=0"})
    assert "ThreadSanitizer" not in r.stderr
