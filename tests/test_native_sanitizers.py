"""Host-side sanitizer runs of the native runtime (SURVEY.md §5.2 race detection / sanitizers).

The token loader core (``csrc/runtime/token_loader.h``: mmap, worker-thread pool, buffer ring,
condition-variable hand-off) is built stand-alone with its stress driver
(``csrc/runtime/tests/token_loader_stress.cpp``) under AddressSanitizer + UndefinedBehaviorSanitizer
and under ThreadSanitizer, and run over several ranks, full and aborted epochs, 16- and 32-bit token
files.  Any sanitizer report fails the run (halt_on_error).  CPU only: GPU sanitizers are not
available on the MI355X pool, and the kernels are covered by the numerics tests instead.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "runtime", "tests", "token_loader_stress.cpp")
CXX = shutil.which("g++")

pytestmark = pytest.mark.skipif(CXX is None, reason="no host C++ compiler")


def _build(tmp_path, flags, name):
    exe = str(tmp_path / name)
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", *flags, SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {r.stderr[-400:]}")
    return exe


def _run(exe, path, itemsize, env):
    r = subprocess.run([exe, path, str(itemsize), "127", "4", "3", "4", "3", "6"], capture_output=True, text=True,
                       timeout=240, env={**os.environ, **env})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("OK"), r.stdout
    assert "ERROR" not in r.stderr and "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]


@pytest.fixture(scope="module")
def token_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("tok")
    p16, p32 = str(d / "t16.bin"), str(d / "t32.bin")
    (np.arange(150_000, dtype=np.int64) * 7919 % 65521).astype(np.uint16).tofile(p16)
    (np.arange(150_000, dtype=np.int64) * 104729 % 128256).astype(np.uint32).tofile(p32)
    return {2: p16, 4: p32}


@pytest.mark.parametrize("itemsize", [2, 4])
def test_token_loader_asan_ubsan(tmp_path, token_files, itemsize):
    exe = _build(tmp_path, ["-fsanitize=address,undefined"], "tls_asan")
    _run(exe, token_files[itemsize], itemsize,
         {"ASAN_OPTIONS": "detect_leaks=1:verify_asan_link_order=0:halt_on_error=1",
          "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})


@pytest.mark.parametrize("itemsize", [2, 4])
def test_token_loader_tsan(tmp_path, token_files, itemsize):
    exe = _build(tmp_path, ["-fsanitize=thread"], "tls_tsan")
    _run(exe, token_files[itemsize], itemsize, {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
