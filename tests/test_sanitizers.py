"""Host-code sanitizers. The host C++ runtime (multithreaded loaders, CPU
samplers) is rebuilt under AddressSanitizer + UBSan and under ThreadSanitizer and the
workload script drives every entry point in a child process with the sanitizer runtime
preloaded. A deliberate heap overflow checks that ASan is really active. GPU code is not
sanitized (no GPU ASan / xnack on this pool)."""
import os
import subprocess
import sys

import pytest

from harp_amd.ops.build import ROOT, build_runtime_sanitized

RT = {"asan": "libasan.so", "tsan": "libtsan.so"}


def _preload(kind):
    try:
        p = subprocess.run(["gcc", f"-print-file-name={RT[kind]}"], capture_output=True, text=True, check=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


def _run(kind, code=None):
    pre = _preload(kind)
    if pre is None:
        pytest.skip(f"{RT[kind]} not available")
    lib = build_runtime_sanitized(kind)
    env = dict(os.environ, LD_PRELOAD=pre, HARP_RUNTIME_LIB=lib, ASAN_OPTIONS="detect_leaks=0",
               TSAN_OPTIONS="halt_on_error=1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "sanitize_workload.py")] if code is None else \
        [sys.executable, "-c", code]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_runtime_clean_under_sanitizer(kind):
    r = _run(kind)
    assert r.returncode == 0 and "sanitize workload ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "Sanitizer" not in r.stderr or "ERROR" not in r.stderr, r.stderr[-4000:]


def test_asan_catches_an_overflow():
    code = """
import ctypes, os, sys, tempfile
import numpy as np
sys.path.insert(0, os.getcwd())
from harp_amd.utils import datasets as D
rt = D._native()
fn = os.path.join(tempfile.mkdtemp(), 'x.csv')
open(fn, 'w').write('1,2,3\\n4,5,6\\n')
h = rt.harp_text_open(fn.encode(), 1)
out = np.zeros(5)  # one element short of 2 x 3
rt.harp_dense_fill(h, b',', out.ctypes.data, 3)
print('not caught')
"""
    r = _run("asan", code)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr, (r.stdout, r.stderr[-3000:])
