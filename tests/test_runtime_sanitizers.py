"""Host-side race detection and memory checking of the native runtime.

The token-loader core (csrc/runtime/token_loader_core.h: mmap'd .npy shards + a producer thread) is
built standalone with ThreadSanitizer and with AddressSanitizer + UndefinedBehaviorSanitizer and its
self-test (csrc/runtime/token_loader_selftest.cc) must pass with no sanitizer report.  GPU-side
sanitizers (xnack+, device ASan) are not available on the MI355X pool; the HIP kernels are instead
covered by the determinism tests (bitwise-equal reruns) in tests/test_kernels_gpu.py.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "mamba_distributed_amd", "csrc", "runtime")
CXX = shutil.which("g++") or shutil.which("clang++")


def _build_and_run(tmp_path, flags, env_extra):
    exe = str(tmp_path / "selftest")
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-pthread", *flags, "-I", RT,
           os.path.join(RT, "token_loader_selftest.cc"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0:
        pytest.skip(f"sanitizer toolchain unavailable: {b.stderr[-500:]}")
    data = tmp_path / "data"
    data.mkdir()
    env = dict(os.environ, **env_extra)
    r = subprocess.run([exe, str(data)], capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0 and "unexpected memory mapping" in r.stderr:
        # TSan's shadow layout vs a high-entropy ASLR kernel: retry with ASLR off for this process
        setarch = shutil.which("setarch")
        if setarch:
            r = subprocess.run([setarch, os.uname().machine, "-R", exe, str(data)], capture_output=True, text=True,
                               timeout=300, env=env)
        if r.returncode != 0 and "unexpected memory mapping" in r.stderr:
            pytest.skip("ThreadSanitizer cannot map its shadow memory on this kernel")
    return r


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
def test_token_loader_threadsanitizer(tmp_path):
    r = _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"})
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
def test_token_loader_address_ub_sanitizer(tmp_path):
    r = _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                                  "-fno-omit-frame-pointer"],
                       {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
