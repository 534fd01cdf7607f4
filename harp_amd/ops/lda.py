"""LDA collapsed-Gibbs device ops (``csrc/lda.hip``) with the native CPU sampler as oracle."""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib

_lib.register({
    "harp_lda_cgs": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_int,
                     _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_float,
                     _lib.c_float, _lib.c_ulonglong, _lib.c_int, _lib.c_void_p],
    "harp_lda_count": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_int, _lib.c_int,
                       _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p],
})


# csrc/lda.hip harp_lda_cgs variants: 0 = compiler occupancy (4 waves/SIMD at K=1000),
# 1 = next token's doc row prefetched, 2..5 = variant 0 forced to 1..4 more waves per SIMD.
# Default 3 (6 waves, a few VGPRs spilled): 1.47e9 vs 1.17e9 tokens/s at 1M x 1M x 1000
# (profiles/r1_lda/occupancy) — more resident waves hide the random doc-row fetch best.
SAMPLER_VARIANT = int(os.environ.get("HARP_LDA_VARIANT", "3"))


def padded_topics(K: int) -> int:
    if K <= 256:
        return 256
    if K <= 512:
        return 512
    if K <= 1024:
        return 1024
    raise NotImplementedError("LDA sampler supports K <= 1024")


def build_chunks(words: torch.Tensor, max_chunk: int = 2048) -> torch.Tensor:
    """Chunk boundaries (int64 [nchunks+1]) of a word-sorted token array: a chunk is a run
    of one word of at most ``max_chunk`` tokens."""
    n = words.numel()
    if n == 0:
        return torch.zeros(1, dtype=torch.int64, device=words.device)
    idx = torch.arange(n, device=words.device)
    new_word = torch.ones(n, dtype=torch.bool, device=words.device)
    new_word[1:] = words[1:] != words[:-1]
    run_start = torch.where(new_word, idx, torch.zeros_like(idx))
    run_start = torch.cummax(run_start, 0).values
    start = new_word | ((idx - run_start) % max_chunk == 0)
    b = torch.nonzero(start).reshape(-1)
    return torch.cat([b, torch.tensor([n], device=words.device)]).to(torch.int64)


def doc_topic_dtype(device, max_doc_len: int) -> torch.dtype:
    """Doc-topic count storage: packed 16-bit on the GPU when every doc has < 32768
    tokens (halves the per-token row read that bounds the sampler), else int32."""
    return torch.int16 if device.type == "cuda" and max_doc_len < 32768 else torch.int32


def _bits(ndk) -> int:
    return 16 if ndk is not None and ndk.dtype == torch.int16 else 32


def count(tdoc, tword, tz, ndk=None, nwk=None, nk=None) -> None:
    n = tz.numel()
    dev = tz.device
    if _lib.use_native(tz):
        st = _lib.kernels().harp_lda_count(_lib.ptr(tdoc), _lib.ptr(tword), tz.data_ptr(), n, _lib.ptr(ndk),
                                           ndk.stride(0) if ndk is not None else 0, _bits(ndk), _lib.ptr(nwk),
                                           nwk.stride(0) if nwk is not None else 0, _lib.ptr(nk), _lib.stream_ptr(dev))
        _lib.check(st, "lda_count")
        return
    one = torch.ones(n, dtype=torch.int32)
    z = tz.long()
    if ndk is not None:
        ndk.index_put_((tdoc.long(), z), one.to(ndk.dtype), accumulate=True)
    if nwk is not None:
        nwk.index_put_((tword.long(), z), one, accumulate=True)
    if nk is not None:
        nk.index_add_(0, z, one)


def cgs_sample(tdoc, tword, tz, chunks, ndk, nwk, nk, K: int, alpha: float, beta: float, vbeta: float,
               seed: int) -> torch.Tensor:
    """One Gibbs sweep over the given (word-sorted) tokens. Returns the topic-count delta
    [K_pad] int32 of this sweep (nk itself is read, not written, on the GPU; the CPU
    sampler updates a private copy exactly)."""
    dev = tz.device
    Kp = ndk.shape[1]
    if _lib.use_native(tz):
        inv = torch.zeros(Kp, dtype=torch.float32, device=dev)
        inv[:K] = 1.0 / (nk[:K].float() + vbeta)
        delta = torch.zeros(Kp, dtype=torch.int32, device=dev)
        st = _lib.kernels().harp_lda_cgs(tdoc.data_ptr(), tword.data_ptr(), tz.data_ptr(), chunks.data_ptr(),
                                         chunks.numel() - 1, ndk.data_ptr(), ndk.stride(0), _bits(ndk), nwk.data_ptr(),
                                         nwk.stride(0), inv.data_ptr(), delta.data_ptr(), K, float(alpha), float(beta),
                                         seed & 0xFFFFFFFFFFFFFFFF, SAMPLER_VARIANT, _lib.stream_ptr(dev))
        _lib.check(st, "lda_cgs")
        return delta
    rt = _lib.runtime()
    if rt is None:
        raise _lib.NativeUnavailable("libharp_runtime.so not built")
    fn = rt.harp_lda_cgs_cpu
    fn.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_uint64]
    fn.restype = None
    work = nk.clone()
    fn(tdoc.data_ptr(), tword.data_ptr(), tz.data_ptr(), tz.numel(), ndk.data_ptr(), ndk.stride(0), nwk.data_ptr(),
       nwk.stride(0), work.data_ptr(), K, float(alpha), float(beta), float(vbeta), seed & 0xFFFFFFFFFFFFFFFF)
    return work - nk


def loglik_terms(counts: torch.Tensor, prior: float, K: int) -> torch.Tensor:
    """sum_k lgamma(c + prior) - lgamma(prior) over the first K columns, and
    sum_rows lgamma(row_total + K prior) terms: returns (entry_sum, row_sum) fp64."""
    c = counts[:, :K].double()
    if counts.dtype == torch.int16:  # packed unsigned 16-bit counts
        c = torch.where(c < 0, c + 65536.0, c)
    ent = (torch.lgamma(c + prior) - torch.lgamma(torch.tensor(prior, dtype=torch.float64))).sum()
    tot = c.sum(1)
    rows = (torch.lgamma(torch.tensor(K * prior, dtype=torch.float64)) - torch.lgamma(tot + K * prior)).sum()
    return torch.stack([ent, rows])
