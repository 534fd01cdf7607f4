"""ctypes binding of ``libharp_kernels.so`` (hand-written gfx950 HIP kernels).

Contract: on a GPU device the native path is mandatory — :func:`kernels` raises if the
library is missing or fails to load, it never silently falls back to PyTorch. CPU
tensors use the reference PyTorch implementations in each ops module (the gloo test
path), which double as the fp32 numerics oracles for the GPU tests.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from .build import KERNEL_LIB, RUNTIME_LIB

_lock = threading.Lock()
_kern = None
_rt = None

c_int, c_long, c_float, c_void_p, c_ulonglong, c_double = (
    ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_double)

# name -> argtypes (restype is always c_int status)
_SIGNATURES = {
    "harp_kmeans_points_per_block": [c_int],
    "harp_kmeans_assign": [c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                           c_void_p, c_void_p, c_int, c_void_p],
    # X, ldx, Cm2, N, dp, kswept, kp, d, keys, variant, stream
    "harp_kmeans_assign_wide": [c_void_p, c_long, c_void_p, c_long, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                c_void_p],
    "harp_kmeans_wide_finish": [c_void_p, c_long, c_void_p, c_void_p, c_void_p, c_void_p],
    "harp_kmeans_normalize": [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p],
    "harp_kmeans_prepare": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "harp_uniform_rows_bf16": [c_void_p, c_long, c_int, c_int, c_float, c_float, c_ulonglong, c_long, c_int,
                               c_void_p],
}


class NativeUnavailable(RuntimeError):
    pass


def _bind(lib, sigs):
    for name, args in sigs.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            continue
        fn.argtypes = args
        fn.restype = c_int


def register(signatures: dict) -> None:
    """Let an ops module declare the argtypes of its launchers."""
    _SIGNATURES.update(signatures)
    if _kern is not None:
        _bind(_kern, signatures)


def kernels():
    """The loaded kernel library; raises :class:`NativeUnavailable` if absent."""
    global _kern
    if _kern is not None:
        return _kern
    with _lock:
        if _kern is None:
            path = os.environ.get("HARP_KERNEL_LIB", KERNEL_LIB)
            if not os.path.exists(path):
                raise NativeUnavailable(
                    f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                    "or `python -m harp_amd.ops.build`")
            try:
                lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            except OSError as e:
                raise NativeUnavailable(f"cannot load {path}: {e}") from e
            _bind(lib, _SIGNATURES)
            _kern = lib
    return _kern


def runtime():
    """Host C++ runtime library (text loaders, exact CPU samplers / SGD oracles) or None.
    ``HARP_RUNTIME_LIB`` selects another build of it (e.g. the sanitizer build)."""
    global _rt
    path = os.environ.get("HARP_RUNTIME_LIB", RUNTIME_LIB)
    if _rt is None and os.path.exists(path):
        with _lock:
            if _rt is None:
                _rt = ctypes.CDLL(path)
    return _rt


def available() -> bool:
    try:
        kernels()
        return True
    except NativeUnavailable:
        return False


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def check(status: int, what: str) -> None:
    if status != 0:
        names = {1: "bad argument", 2: "launch failure", 3: "unsupported shape"}
        raise RuntimeError(f"{what}: native kernel returned {status} ({names.get(status, '?')})")


def use_native(t: torch.Tensor) -> bool:
    """True for HIP device tensors (native path mandatory), False for CPU tensors."""
    if t.device.type == "cuda":
        kernels()  # raise loudly if missing
        return True
    return False
