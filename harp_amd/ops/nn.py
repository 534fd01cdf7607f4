"""Fused MLP epilogues (``csrc/nn.hip``): bias + activation, softmax-cross-entropy
forward + backward with the bias gradient, activation derivative + bias gradient. The
GEMMs between them stay on hipBLASLt (``torch.mm``)."""
from __future__ import annotations

import torch

from . import _lib

ACT = {"sigmoid": 0, "tanh": 1, "relu": 2, "none": 3}

_lib.register({
    "harp_nn_bias_act": [_lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_int, _lib.c_void_p],
    "harp_nn_softmax_xent": [_lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_float, _lib.c_void_p,
                             _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    "harp_nn_dact_bgrad": [_lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_int, _lib.c_void_p,
                           _lib.c_void_p],
})


def available(t: torch.Tensor) -> bool:
    return t.device.type == "cuda" and t.dtype == torch.float32 and _lib.use_native(t)


def bias_act_(z: torch.Tensor, b: torch.Tensor | None, act: str) -> torch.Tensor:
    """In place: z = act(z + b) ([rows, N] fp32, contiguous)."""
    assert z.is_contiguous() and z.dtype == torch.float32
    assert b is None or (b.is_contiguous() and b.numel() >= z.shape[1])
    _lib.check(_lib.kernels().harp_nn_bias_act(z.data_ptr(), _lib.ptr(b), z.shape[0], z.shape[1], ACT[act],
                                               _lib.stream_ptr(z.device)), "nn_bias_act")
    return z


def softmax_xent(z: torch.Tensor, labels: torch.Tensor, scale: float, delta: torch.Tensor,
                 dbias: torch.Tensor | None = None) -> torch.Tensor:
    """delta = (softmax(z) - onehot(labels)) * scale; dbias += column sums of delta;
    returns the summed cross-entropy loss (0-dim device tensor)."""
    B, C = z.shape
    assert z.is_contiguous() and delta.is_contiguous() and labels.dtype == torch.int32
    assert delta.shape == z.shape and labels.numel() >= B and (dbias is None or dbias.numel() >= C)
    loss = torch.zeros(1, dtype=torch.float32, device=z.device)
    _lib.check(_lib.kernels().harp_nn_softmax_xent(z.data_ptr(), B, C, labels.data_ptr(), float(scale),
                                                   delta.data_ptr(), loss.data_ptr(), _lib.ptr(dbias),
                                                   _lib.stream_ptr(z.device)), "nn_softmax_xent")
    return loss[0]


def dact_bgrad_(delta: torch.Tensor, a: torch.Tensor, act: str, dbias: torch.Tensor | None = None) -> torch.Tensor:
    """In place: delta *= act'(a) (a = activation values); dbias += column sums."""
    B, N = delta.shape
    assert delta.is_contiguous() and a.is_contiguous() and a.shape == delta.shape
    assert dbias is None or dbias.numel() >= N
    _lib.check(_lib.kernels().harp_nn_dact_bgrad(delta.data_ptr(), a.data_ptr(), B, N, ACT[act], _lib.ptr(dbias),
                                                 _lib.stream_ptr(delta.device)), "nn_dact_bgrad")
    return delta
