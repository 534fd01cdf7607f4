"""In-tree build of the native libraries.

* ``harp_amd/_native/libharp_kernels.so`` — every ``csrc/*.hip`` kernel family, compiled
  by hipcc for gfx950 only (``--offload-arch=gfx950``), exporting ``extern "C"``
  launchers that take raw device pointers + a ``hipStream_t``.
* ``harp_amd/_native/libharp_runtime.so`` — host-side C++ runtime pieces
  (``csrc/host/*.cpp``: multithreaded text loaders, exact sequential CPU samplers / SGD
  used on CPU workers and as GPU-kernel oracles), built with g++.
* ``build/sanitize/libharp_runtime_{asan,tsan}.so`` (``--sanitize asan|tsan``, not shipped)
  — the same host sources under AddressSanitizer + UBSan or ThreadSanitizer, for
  ``tests/test_sanitizers.py`` (host code only: GPU sanitizers are not used).

Both are loaded with ctypes *after* ``import torch`` so the kernels launch through the
HIP runtime torch already loaded (same soname ``libamdhip64.so.7``).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
NATIVE = os.path.join(ROOT, "harp_amd", "_native")
OBJ = os.path.join(ROOT, "build", "obj")
KERNEL_LIB = os.path.join(NATIVE, "libharp_kernels.so")
RUNTIME_LIB = os.path.join(NATIVE, "libharp_runtime.so")

ARCH = os.environ.get("HARP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-I" + CSRC]
CXX = os.environ.get("CXX", "g++")
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-I" + CSRC]


def _stale(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    os.makedirs(NATIVE, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    if not force and not _stale(KERNEL_LIB, srcs + headers):
        return KERNEL_LIB  # shipped/up-to-date library (object files need not exist)
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _stale(o, [s] + headers):
            todo.append([HIPCC] + HIP_FLAGS + ["-c", s, "-o", o])
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for fut in [ex.submit(_run, c) for c in todo]:
                fut.result()
        if verbose:
            print(f"[harp build] compiled {len(todo)} HIP source(s)", file=sys.stderr)
    if force or todo or _stale(KERNEL_LIB, objs):
        tmp = f"{KERNEL_LIB}.{os.getpid()}.tmp"
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp] + objs)
        os.replace(tmp, KERNEL_LIB)  # atomic: concurrent loaders never see a partial file
    return KERNEL_LIB


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(NATIVE, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    headers = glob.glob(os.path.join(CSRC, "host", "*.h"))
    if not srcs:
        return ""
    if force or _stale(RUNTIME_LIB, srcs + headers):
        tmp = f"{RUNTIME_LIB}.{os.getpid()}.tmp"
        _run([CXX] + CXX_FLAGS + ["-shared", "-o", tmp] + srcs)
        os.replace(tmp, RUNTIME_LIB)
        if verbose:
            print(f"[harp build] linked {RUNTIME_LIB}", file=sys.stderr)
    return RUNTIME_LIB


SANITIZE_DIR = os.path.join(ROOT, "build", "sanitize")
_SAN_FLAGS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}


def build_runtime_sanitized(kind: str = "asan", force: bool = False) -> str:
    """Host runtime under a sanitizer (loaded with the sanitizer runtime LD_PRELOADed)."""
    os.makedirs(SANITIZE_DIR, exist_ok=True)
    out = os.path.join(SANITIZE_DIR, f"libharp_runtime_{kind}.so")
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    headers = glob.glob(os.path.join(CSRC, "host", "*.h"))
    if force or _stale(out, srcs + headers):
        flags = [f for f in CXX_FLAGS if f != "-O3"] + ["-O1", "-g"] + _SAN_FLAGS[kind]
        tmp = f"{out}.{os.getpid()}.tmp"
        _run([CXX] + flags + ["-shared", "-o", tmp] + srcs)
        os.replace(tmp, out)
    return out


def build_all(force: bool = False, verbose: bool = True) -> None:
    build_kernels(force=force, verbose=verbose)
    build_runtime(force=force, verbose=verbose)


if __name__ == "__main__":
    if "--sanitize" in sys.argv:
        print(build_runtime_sanitized(sys.argv[sys.argv.index("--sanitize") + 1], force="--force" in sys.argv))
    else:
        build_all(force="--force" in sys.argv)
