"""LDA collapsed-Gibbs device ops (``csrc/lda.hip``) with the native CPU sampler as oracle."""
from __future__ import annotations

import ctypes
import os
import weakref
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib

_lib.register({
    # ..., seed, variant, lpt (longest-first chunk bounds or null), stream
    "harp_lda_cgs": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_int,
                     _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_float,
                     _lib.c_float, _lib.c_ulonglong, _lib.c_int, _lib.c_void_p, _lib.c_void_p],
    # tspan, tword, tz, chunks, nchunks, order, work, tpos, zdoc, nwk, ldw, inv_nk, nk_delta, K, alpha, beta,
    # seed, waves, stream
    "harp_lda_cgs_sparse_span": [_lib.c_void_p] * 4 + [_lib.c_long] + [_lib.c_void_p] * 5 + [
        _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_float, _lib.c_float, _lib.c_ulonglong,
        _lib.c_int, _lib.c_void_p],
    # tspan, tword, tz, chunks, nchunks, order, work, tpos, zdoc, inv, delta, K, alpha, beta, seed, waves,
    # pbuf, poff, pcap, qbuf, qoff, qcap, overflow, stream
    "harp_lda_cgs_sparse_span_ps": [_lib.c_void_p] * 4 + [_lib.c_long] + [_lib.c_void_p] * 6 + [
        _lib.c_int, _lib.c_float, _lib.c_float, _lib.c_ulonglong, _lib.c_int] + [_lib.c_void_p] * 8,
    "harp_lda_cgs_sparse": [_lib.c_void_p] * 4 + [_lib.c_long] + [_lib.c_void_p] * 6 + [
        _lib.c_int, _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_float,
        _lib.c_float, _lib.c_ulonglong, _lib.c_int, _lib.c_void_p],
    # tdoc, tword, tz, chunks, nchunks, ndk, ldd, ndk_bits, inv_nk, nk_delta, K, alpha, beta, seed, variant,
    # pull buf / off / cap, push buf / off / cap, overflow, lpt, stream
    "harp_lda_cgs_ps": [_lib.c_void_p] * 4 + [_lib.c_long, _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p,
                                              _lib.c_void_p, _lib.c_int, _lib.c_float, _lib.c_float, _lib.c_ulonglong,
                                              _lib.c_int] + [_lib.c_void_p] * 9,
    "harp_lda_count": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_long, _lib.c_void_p, _lib.c_int, _lib.c_int,
                       _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p],
})


# csrc/lda.hip harp_lda_cgs variants: 0 = six waves per SIMD, 3 = seven (the default: 67
# VGPRs and 20.5 KB of LDS per workgroup since the inverse topic sums are read from global
# memory; 8-share 5.44 -> 5.33 ms, profiles/r5_lda_waves7). More resident waves hide the
# per-token doc-row fetch (round 5 before: five -> six waves, 8.72 -> 8.06 ms).
SAMPLER_VARIANT = int(os.environ.get("HARP_LDA_VARIANT", "3"))


# Sampler choice: "dense" = register-row kernel (K <= 1024), "sparse" = doc-token-list
# kernel (any K <= 32768, see csrc/lda.hip lda_cgs_sparse_kernel), "auto" = sparse for
# K > 1024 or corpora of >= SPARSE_MIN_TOKENS tokens, dense otherwise. Measured at
# 1M docs x 1M words x 1000 topics (1e8 tokens, profiles/r1_lda/sparse): sparse 1.56e9
# tokens/s and log-likelihood -1.676e9 after 4 iterations vs dense 1.48e9 and -1.688e9;
# on 1e5-token corpora (tens of tokens per word) the sparse sampler's workgroup-wide
# sampling of one word loses ~10% of the per-iteration likelihood gain, the dense one
# (a wave per word) does not.
SAMPLER = os.environ.get("HARP_LDA_SAMPLER", "auto")
SPARSE_WAVES = int(os.environ.get("HARP_LDA_SPARSE_WAVES", "0"))  # 0: by K (csrc launcher)
SPARSE_MIN_TOKENS = 1 << 24
MAX_TOPICS = 32768      # GPU sparse sampler: the word's qw row in LDS (csrc/lda.hip kSparseMaxK)
MAX_TOPICS_GPU_HOST = 65535  # GPU workers above MAX_TOPICS: the exact host sampler (uint16 doc-order topics)


def use_sparse(K: int, n_tokens: int = 0, max_doc_len: Optional[int] = None) -> bool:
    """Sampler choice (identical on every worker: by the tokens ONE worker samples and the
    corpus's longest document). auto: the dense sampler for K <= 1024 -- since round 5 (packed
    uint8 doc rows with the next row prefetched, longest-first chunk schedule, chunks of up to
    32768 tokens) it is faster AND mixes better per sweep at the full BASELINE #5 size (3.11e9
    vs 2.63e9 tokens/s, log-likelihood -1.443e9 vs -1.466e9 after 6 sweeps,
    profiles/r5_lda_chunks) -- except on corpora of >= SPARSE_MIN_TOKENS tokens whose
    documents reach 256 tokens (no packed uint8 rows: 2-4 KB doc-row reads per token)."""
    if SAMPLER not in ("auto", "dense", "sparse"):
        raise ValueError(f"HARP_LDA_SAMPLER={SAMPLER!r}: expected auto, dense or sparse")
    if K > 1024 or SAMPLER == "sparse":
        return True
    if SAMPLER == "dense" or n_tokens < SPARSE_MIN_TOKENS:
        return False
    return max_doc_len is None or max_doc_len >= 256


def padded_topics(K: int) -> int:
    if K <= 256:
        return 256
    if K <= 512:
        return 512
    if K <= 1024:
        return 1024
    return (K + 127) // 128 * 128  # any K (GPU workers: see cgs_sample for K > MAX_TOPICS)


@dataclass
class DocIndex:
    """Doc-order view of the topic assignments for the sparse sampler:
    ``zdoc[doc_off[d]:doc_off[d+1]]`` are the topics (uint16 bits in int16) of doc d's
    tokens and ``tpos[i]`` is token i's position in ``zdoc``; the sampler keeps ``zdoc``
    and ``tz`` in step."""

    zdoc: torch.Tensor     # [n] int16
    doc_off: torch.Tensor  # [n_docs + 1] int64
    tpos: torch.Tensor     # [n] int64
    span: Optional[torch.Tensor] = None  # [n] int64: doc_off[doc] | (doc length << 40), token order

    @staticmethod
    def build(tdoc: torch.Tensor, tz: torch.Tensor, n_docs: int) -> "DocIndex":
        from .sorting import argsort_small_keys

        order = argsort_small_keys(tdoc, n_docs)  # any length (chunked past INT_MAX tokens)
        zdoc = tz[order].to(torch.int16)
        tpos = torch.empty_like(order)
        tpos[order] = torch.arange(order.numel(), device=order.device)
        del order
        off = torch.zeros(n_docs + 1, dtype=torch.int64, device=tdoc.device)
        off[1:] = torch.cumsum(torch.bincount(tdoc, minlength=n_docs)[:n_docs], 0)
        span = None
        if tdoc.device.type == "cuda" and SPAN:  # built in pieces: no int64 temporaries of n
            span = torch.empty(tdoc.numel(), dtype=torch.int64, device=tdoc.device)
            for a in range(0, tdoc.numel(), 1 << 27):
                d = tdoc[a:a + (1 << 27)].long()
                lo = off[d]
                span[a:a + d.numel()] = lo | ((off[d + 1] - lo) << 40)
                del d, lo
        return DocIndex(zdoc, off, tpos, span)

    def sync(self, tz: torch.Tensor, tpos: Optional[torch.Tensor] = None) -> None:
        """Copy assignments ``tz`` (tokens ``tpos``, default all) into the doc-order view."""
        self.zdoc[self.tpos if tpos is None else tpos] = tz.to(torch.int16)


def _span_slice(doc_index: "DocIndex", tdoc: torch.Tensor, tpos: torch.Tensor) -> torch.Tensor:
    """The per-token doc spans of the tokens ``tpos`` (a slice of ``doc_index.tpos``: the
    matching slice of ``doc_index.span``; otherwise computed from ``tdoc``)."""
    full = doc_index.tpos
    o = (tpos.data_ptr() - full.data_ptr()) // full.element_size()
    if (doc_index.span is not None and tpos.untyped_storage().data_ptr() == full.untyped_storage().data_ptr()
            and tpos.is_contiguous() and 0 <= o and o + tpos.numel() <= full.numel()):
        return doc_index.span[o:o + tpos.numel()]
    d = tdoc.long()
    off = doc_index.doc_off
    return (off[d] | ((off[d + 1] - off[d]) << 40)).contiguous()


def build_chunks(words: torch.Tensor, max_chunk: int = 2048) -> torch.Tensor:
    """Chunk boundaries (int64 [nchunks+1]) of a word-sorted token array: a chunk is a run
    of one word of at most ``max_chunk`` tokens. Word-run boundaries are found in pieces of
    2^28 tokens (no token-length temporaries: a clueweb1 share is 3.7e9 tokens, past what
    torch's nonzero / cumsum index), then runs are split on the (few) run boundaries."""
    n = words.numel()
    dev = words.device
    if n == 0:
        return torch.zeros(1, dtype=torch.int64, device=dev)
    piece = 1 << 28
    starts = [torch.zeros(1, dtype=torch.int64, device=dev)]
    for a in range(1, n, piece):
        b = min(n, a + piece)
        ch = torch.nonzero(words[a:b] != words[a - 1:b - 1]).reshape(-1)
        if ch.numel():
            starts.append(ch + a)
    rs = torch.cat(starts)  # word-run starts
    re = torch.cat([rs[1:], torch.tensor([n], dtype=torch.int64, device=dev)])
    per = (re - rs + max_chunk - 1) // max_chunk  # chunks per run
    cs = torch.repeat_interleave(rs, per)
    first = torch.cumsum(per, 0) - per
    cs = cs + (torch.arange(cs.numel(), device=dev) - torch.repeat_interleave(first, per)) * max_chunk
    return torch.cat([cs, torch.tensor([n], dtype=torch.int64, device=dev)])


def max_chunk(requested: int, sparse: bool, n_tokens: int = 0) -> int:
    """Tokens per word chunk: ``requested`` if set; the sparse sampler 65536 (a workgroup
    per chunk, longest first: a word split over several workgroups is sampled against
    several stale copies of its row -- 1.83e9 vs 1.86e9 log-likelihood after 4 iterations
    at K = 10,000, profiles/r1_lda/sparse); the dense sampler (a wave per chunk, chunks
    dealt longest first to the resident waves) n_tokens / 3072 within [2048, 32768]: long
    enough that a frequent word is not sampled against many stale copies of its row (full
    BASELINE #5 size: 2048 -> 32768 tokens moves the log-likelihood after 6 sweeps from
    -1.554e9 to -1.443e9 and the sweep from 33.6 to 32.2 ms), short enough that the longest
    chunk stays within about twice a wave's share of the sweep."""
    if requested:
        return requested
    if sparse:
        return 65536
    return int(min(32768, max(2048, n_tokens // 3072)))


def chunk_order(chunks: torch.Tensor) -> torch.Tensor:
    """Chunk processing order for the sparse sampler: longest first (int32), so the
    workgroups that draw the last chunks from the work counter get short ones."""
    if os.environ.get("HARP_LDA_ORDER", "lpt") == "identity":
        return torch.arange(chunks.numel() - 1, dtype=torch.int32, device=chunks.device)
    return torch.argsort(chunks[1:] - chunks[:-1], descending=True).to(torch.int32)


_LPT: dict = {}


# HARP_LDA_SOLE=0: no chunk is marked the sole chunk of its word (every push slot reserved
# by an atomic, as before the flag existed)
SOLE = os.environ.get("HARP_LDA_SOLE", "1") != "0"


def lpt_desc(chunks: torch.Tensor, tword: torch.Tensor, slots=None) -> Optional[torch.Tensor]:
    """The dense sampler's chunk schedule: one descriptor per chunk, longest first (int64
    [n, 4]: start, length | sole << 31 | word << 32 (sole: the word's only chunk, whose push
    slot then needs no reservation atomic), the word's pull-slot and push-slot offsets when
    ``slots`` (fused rows) are given, else 0), dealt to the resident waves in snake order by
    the kernel. Cached per (chunks, tword, slots) (the layouts are static across sweeps).
    None with HARP_LDA_ORDER=identity (the static word-order stride)."""
    if os.environ.get("HARP_LDA_ORDER", "lpt") == "identity" or chunks.numel() < 2:
        return None
    # (a rotation slice passes a new view of the same token array every call: keyed by its
    # address and length; entries hold weak references, so a cached schedule never keeps a
    # model's arrays alive, and a hit needs the same, still-live chunk tensor)
    # The descriptors embed the slot offsets the kernel stores to, so a hit also needs the
    # SAME slot tensors (weak references): a rebuilt parameter-server layout that the
    # allocator placed at the old addresses is a miss, never stale offsets.
    key = (id(chunks), chunks.data_ptr(), chunks.numel(), tword.data_ptr(), tword.numel(),
           None if slots is None else tuple(x.data_ptr() for x in slots))
    hit = _LPT.get(key)
    if hit is not None and hit[0]() is chunks and (
            slots is None or (len(hit[2]) == len(slots) and all(r() is x for r, x in zip(hit[2], slots)))):
        return hit[1]
    order = torch.argsort(chunks[1:] - chunks[:-1], descending=True)
    a = chunks[:-1][order]
    n = chunks[1:][order] - a
    w = tword[a].long()
    sole = (torch.bincount(w)[w] == 1).long() * int(SOLE)
    d = torch.zeros((order.numel(), 4), dtype=torch.int64, device=chunks.device)
    d[:, 0] = a
    d[:, 1] = n | (sole << 31) | (w << 32)
    if slots is not None:
        d[:, 2] = slots[0][w]
        d[:, 3] = slots[2][w]
    for k in [k for k, v in _LPT.items() if v[0]() is None]:  # entries of freed layouts
        del _LPT[k]
    if len(_LPT) >= 16:
        _LPT.pop(next(iter(_LPT)))
    _LPT[key] = (weakref.ref(chunks), d.contiguous(), tuple(weakref.ref(x) for x in slots) if slots is not None else ())
    return _LPT[key][1]


DOC_TOPIC_8BIT = os.environ.get("HARP_LDA_NDK8", "1") != "0"
# sparse sampler without a doc-topic table: per-token doc spans instead of doc ids (one
# independent load for the next token's doc range instead of ids -> doc_off)
SPAN = os.environ.get("HARP_LDA_SPAN", "1") != "0"


def doc_topic_dtype(device, max_doc_len: int) -> torch.dtype:
    """Doc-topic count storage on the GPU: packed uint8 when every doc has < 256 tokens,
    packed 16-bit when < 32768 (each halves the per-token doc-row read that bounds the
    dense sampler: 1 KB instead of 2 KB at K_pad = 1024), else int32; int32 on the CPU."""
    if device.type != "cuda":
        return torch.int32
    if DOC_TOPIC_8BIT and max_doc_len < 256:
        return torch.uint8
    return torch.int16 if max_doc_len < 32768 else torch.int32


def _bits(ndk) -> int:
    if ndk is None:
        return 32
    return {torch.int16: 16, torch.uint8: 8}.get(ndk.dtype, 32)


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
               seed: int, doc_index: Optional[DocIndex] = None, tpos: Optional[torch.Tensor] = None,
               order: Optional[torch.Tensor] = None, deterministic: bool = False) -> torch.Tensor:
    """One Gibbs sweep over the given (word-sorted) tokens. Returns the topic-count delta
    [K_pad] int32 of this sweep (nk itself is read, not written, on the GPU; the CPU
    sampler updates a private copy exactly). ``doc_index`` (+ ``tpos``, the tokens'
    positions in it; default all of it) selects the sparse sampler and is kept in step;
    ``order`` is its chunk order (default :func:`chunk_order`). ``deterministic``: on the
    GPU, ONE wave samples every chunk in order -- bit-reproducible and independent of the
    word-row numbering (a test mode; the CPU sampler is always sequential)."""
    dev = tz.device
    Kp = nwk.shape[1]  # ndk may be None (sparse sampler on the GPU: no dense doc-topic table)
    if doc_index is None and use_sparse(K):
        raise ValueError(f"K={K} needs the sparse sampler: pass doc_index (DocIndex.build)")
    if doc_index is not None and tpos is None:
        tpos = doc_index.tpos
    if _lib.use_native(tz) and K > MAX_TOPICS:
        return _host_sweep(tdoc, tword, tz, ndk, nwk, nk, K, alpha, beta, vbeta, seed, doc_index, tpos)
    if _lib.use_native(tz):
        inv = torch.zeros(Kp, dtype=torch.float32, device=dev)
        inv[:K] = 1.0 / (nk[:K].float() + vbeta)
        if doc_index is not None:
            delta = torch.zeros(Kp, dtype=torch.int32, device=dev)
            assert tpos.dtype == torch.int64 and tpos.numel() == tz.numel() and tpos.is_contiguous()
            if order is None:
                order = chunk_order(chunks)
            assert order.dtype == torch.int32 and order.numel() == chunks.numel() - 1
            work = torch.zeros(1, dtype=torch.int32, device=dev)
            if ndk is None and SPAN:  # doc ranges from per-token spans: no dependent doc_off load
                span = _span_slice(doc_index, tdoc, tpos)
                st = _lib.kernels().harp_lda_cgs_sparse_span(
                    span.data_ptr(), tword.data_ptr(), tz.data_ptr(), chunks.data_ptr(), chunks.numel() - 1,
                    order.data_ptr(), work.data_ptr(), tpos.data_ptr(), doc_index.zdoc.data_ptr(), nwk.data_ptr(),
                    nwk.stride(0), inv.data_ptr(), delta.data_ptr(), K, float(alpha), float(beta),
                    seed & 0xFFFFFFFFFFFFFFFF, -1 if deterministic else SPARSE_WAVES, _lib.stream_ptr(dev))
                _lib.check(st, "lda_cgs_sparse_span")
                return delta
            st = _lib.kernels().harp_lda_cgs_sparse(
                tdoc.data_ptr(), tword.data_ptr(), tz.data_ptr(), chunks.data_ptr(), chunks.numel() - 1,
                order.data_ptr(), work.data_ptr(), tpos.data_ptr(), doc_index.doc_off.data_ptr(), doc_index.zdoc.data_ptr(), _lib.ptr(ndk),
                ndk.stride(0) if ndk is not None else 0, _bits(ndk), nwk.data_ptr(), nwk.stride(0), inv.data_ptr(),
                delta.data_ptr(), K, float(alpha), float(beta), seed & 0xFFFFFFFFFFFFFFFF, -1 if deterministic else SPARSE_WAVES,
                _lib.stream_ptr(dev))
            _lib.check(st, "lda_cgs_sparse")
            return delta
        delta = torch.zeros(Kp, dtype=torch.int32, device=dev)
        st = _lib.kernels().harp_lda_cgs(tdoc.data_ptr(), tword.data_ptr(), tz.data_ptr(), chunks.data_ptr(),
                                         chunks.numel() - 1, ndk.data_ptr(), ndk.stride(0), _bits(ndk), nwk.data_ptr(),
                                         nwk.stride(0), inv.data_ptr(), delta.data_ptr(), K, float(alpha), float(beta),
                                         seed & 0xFFFFFFFFFFFFFFFF,
                                         SAMPLER_VARIANT | (0x200 if deterministic == "lpt" else 0x100 if deterministic else 0),
                                         _lib.ptr(lpt_desc(chunks, tword) if deterministic in (False, "lpt") else None),
                                         _lib.stream_ptr(dev))
        _lib.check(st, "lda_cgs")
        return delta
    delta = _cpu_sweep(tdoc, tword, tz, ndk, nwk, nk, K, alpha, beta, vbeta, seed)
    if doc_index is not None:
        doc_index.sync(tz, tpos)
    return delta


def _cpu_sweep(tdoc, tword, tz, ndk, nwk, nk, K, alpha, beta, vbeta, seed) -> torch.Tensor:
    """The native sequential sampler (csrc/host/lda_cpu.cpp) on host tensors: updates tz,
    ndk, nwk in place and returns the topic-count delta."""
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


def _host_sweep(tdoc, tword, tz, ndk, nwk, nk, K, alpha, beta, vbeta, seed, doc_index, tpos):
    """GPU worker, K > :data:`MAX_TOPICS` (the sparse kernel's LDS word row does not fit):
    the exact sequential collapsed-Gibbs sweep of the native host sampler
    (``csrc/host``, the reference's per-token order, LDAMPTask.java:85-330) on host copies,
    results copied back. Correct at any K, not fast -- a documented capacity path, not a
    throughput one. The doc-topic counts are rebuilt on the host from the doc-order topic
    lists when the worker keeps no dense table (the sparse sampler's setting)."""
    if K > MAX_TOPICS_GPU_HOST:
        raise ValueError(f"GPU LDA workers support K <= {MAX_TOPICS_GPU_HOST} (uint16 doc-order topic lists); "
                         f"run K = {K} on CPU workers")
    dev = tz.device
    h_doc, h_word, h_tz = tdoc.cpu().int().contiguous(), tword.cpu().int().contiguous(), tz.cpu().int().contiguous()
    Kp = nwk.shape[1]
    h_nwk = nwk.cpu().contiguous()
    h_nk = nk.cpu().int().contiguous()
    if ndk is not None:
        h_ndk = ndk.cpu().int()
        if ndk.dtype == torch.int16:
            h_ndk = h_ndk & 0xFFFF
        h_ndk = h_ndk.contiguous()
        delta = _cpu_sweep(h_doc, h_word, h_tz, h_ndk, h_nwk, h_nk, K, alpha, beta, vbeta, seed)
    else:
        delta = _host_sweep_doc_batches(h_doc, h_word, h_tz, h_nwk, h_nk, Kp, K, alpha, beta, vbeta, seed, doc_index)
    tz.copy_(h_tz.to(dev))
    nwk.copy_(h_nwk.to(dev))
    if ndk is not None:
        ndk.copy_(h_ndk.to(ndk.dtype).to(dev))
    if doc_index is not None:
        doc_index.sync(tz, tpos)
    return delta.to(dev)


# host bytes one dense doc-topic batch of the GPU worker's host sampler may take (K > 32768)
HOST_NDK_BYTES = int(os.environ.get("HARP_LDA_HOST_NDK_BYTES", str(1 << 30)))


def _host_sweep_doc_batches(h_doc, h_word, h_tz, h_nwk, h_nk, Kp, K, alpha, beta, vbeta, seed, doc_index):
    """The host sweep of a worker that keeps no dense doc-topic table: the docs of this sweep
    are taken in batches whose dense [docs, Kp] int32 rows fit HOST_NDK_BYTES, each batch's
    counts rebuilt from the doc-order topic lists (EVERY token of those docs, not only this
    sweep's), and the batch's tokens (in their word order) sampled sequentially against the
    shared word-topic rows and topic totals carried from batch to batch. Every token is
    resampled once from its exact collapsed conditional, so the sweep stays a systematic-scan
    Gibbs sweep whatever the batching; with one batch it is the plain sequential sweep."""
    off = doc_index.doc_off.cpu()
    lens = off[1:] - off[:-1]
    zdoc = doc_index.zdoc.cpu().long() & 0xFFFF
    docs = torch.unique(h_doc.long())
    per = max(1, HOST_NDK_BYTES // (Kp * 4))
    delta = torch.zeros_like(h_nk)
    nk_cur = h_nk.clone()
    tdoc_l = h_doc.long()
    for q, s0 in enumerate(range(0, docs.numel(), per)):
        bd = docs[s0:s0 + per]
        if docs.numel() <= per:
            idx = None
            local = torch.searchsorted(bd, tdoc_l)
        else:
            idx = torch.isin(tdoc_l, bd).nonzero().squeeze(1)
            local = torch.searchsorted(bd, tdoc_l[idx])
        bl = lens[bd]
        pos = torch.arange(int(bl.sum())) + torch.repeat_interleave(off[bd] - (torch.cumsum(bl, 0) - bl), bl)
        b_ndk = torch.zeros((bd.numel(), Kp), dtype=torch.int32)
        b_ndk.index_put_((torch.repeat_interleave(torch.arange(bd.numel()), bl), zdoc[pos]),
                         torch.ones(pos.numel(), dtype=torch.int32), accumulate=True)
        b_tz = h_tz if idx is None else h_tz[idx].contiguous()
        b_word = h_word if idx is None else h_word[idx].contiguous()
        d = _cpu_sweep(local.int().contiguous(), b_word, b_tz, b_ndk, h_nwk, nk_cur, K, alpha, beta, vbeta,
                       seed + 0x9E3779B9 * q)
        nk_cur += d
        delta += d
        if idx is not None:
            h_tz[idx] = b_tz
    return delta


def cgs_sample_ps(tdoc, tword, tz, chunks, ndk, nk, K: int, alpha: float, beta: float, vbeta: float, seed: int,
                  pull_buf, push_buf, slots, overflow, deterministic: bool = False,
                  doc_index: Optional[DocIndex] = None, order: Optional[torch.Tensor] = None) -> torch.Tensor:
    """:func:`cgs_sample` on the GPU with the word rows read from the pull payload and the
    word-row deltas written into the (zeroed) push payload -- no dense local table
    (``parallel.sparse_ps.SparseRowPS.row_slots`` gives ``slots``). Dense sampler (``ndk``,
    K <= 1024), or with ``doc_index`` (and no ``ndk``) the sparse doc-span sampler
    (K <= :data:`MAX_TOPICS`). Returns the topic-count delta. ``deterministic``: True -- one
    wave, chunks in index order; "lpt" (dense sampler) -- one wave walking the production
    longest-first chunk descriptors in order (sole-chunk flags and slot offsets included)."""
    dev = tz.device
    poff, pcap, qoff, qcap = slots
    if doc_index is not None:
        if not _lib.use_native(tz) or K > MAX_TOPICS or ndk is not None:
            raise ValueError("fused push-pull rows with the sparse sampler need the GPU doc-span kernel")
        Kp = nk.shape[0]
        inv = torch.zeros(Kp, dtype=torch.float32, device=dev)
        inv[:K] = 1.0 / (nk[:K].float() + vbeta)
        delta = torch.zeros(Kp, dtype=torch.int32, device=dev)
        tpos = doc_index.tpos
        assert tpos.numel() == tz.numel()
        if order is None:
            order = chunk_order(chunks)
        work = torch.zeros(1, dtype=torch.int32, device=dev)
        span = _span_slice(doc_index, tdoc, tpos)
        st = _lib.kernels().harp_lda_cgs_sparse_span_ps(
            span.data_ptr(), tword.data_ptr(), tz.data_ptr(), chunks.data_ptr(), chunks.numel() - 1, order.data_ptr(),
            work.data_ptr(), tpos.data_ptr(), doc_index.zdoc.data_ptr(), inv.data_ptr(), delta.data_ptr(), K,
            float(alpha), float(beta), seed & 0xFFFFFFFFFFFFFFFF, -1 if deterministic else SPARSE_WAVES,
            pull_buf.data_ptr(), poff.data_ptr(), pcap.data_ptr(), push_buf.data_ptr(), qoff.data_ptr(),
            qcap.data_ptr(), overflow.data_ptr(), _lib.stream_ptr(dev))
        _lib.check(st, "lda_cgs_sparse_span_ps")
        return delta
    Kp = ndk.shape[1]
    if not _lib.use_native(tz) or K > 1024:
        raise ValueError("fused push-pull rows need the GPU dense sampler (K <= 1024)")
    inv = torch.zeros(Kp, dtype=torch.float32, device=dev)
    inv[:K] = 1.0 / (nk[:K].float() + vbeta)
    delta = torch.zeros(Kp, dtype=torch.int32, device=dev)
    st = _lib.kernels().harp_lda_cgs_ps(
        tdoc.data_ptr(), tword.data_ptr(), tz.data_ptr(), chunks.data_ptr(), chunks.numel() - 1, ndk.data_ptr(),
        ndk.stride(0), _bits(ndk), inv.data_ptr(), delta.data_ptr(), K, float(alpha), float(beta),
        seed & 0xFFFFFFFFFFFFFFFF, SAMPLER_VARIANT | (0x200 if deterministic == "lpt" else 0x100 if deterministic else 0),
        pull_buf.data_ptr(), poff.data_ptr(), pcap.data_ptr(), push_buf.data_ptr(), qoff.data_ptr(), qcap.data_ptr(),
        overflow.data_ptr(),
        _lib.ptr(lpt_desc(chunks, tword, slots) if deterministic in (False, "lpt") else None), _lib.stream_ptr(dev))
    _lib.check(st, "lda_cgs_ps")
    return delta


def doc_loglik_terms(doc_index: DocIndex, prior: float, K: int, block_tokens: int = 1 << 26) -> torch.Tensor:
    """:func:`loglik_terms` of the doc-topic counts, from the sparse sampler's doc-order
    topic lists instead of a dense [docs, K_pad] table (which at K = 10,000 would take
    20 KB per document): each doc block's (doc, topic) pairs are counted by ``unique``."""
    off, z = doc_index.doc_off, doc_index.zdoc
    dev = z.device
    n_docs = off.numel() - 1
    lg_p = torch.lgamma(torch.tensor(prior, dtype=torch.float64))
    lg_kp = torch.lgamma(torch.tensor(K * prior, dtype=torch.float64))
    out = torch.zeros(2, dtype=torch.float64, device=dev)
    lens = off[1:] - off[:-1]
    out[1] = (lg_kp - torch.lgamma(lens.double() + K * prior)).sum()
    # doc blocks of ~block_tokens tokens (at least one doc each)
    cuts = torch.searchsorted(off, torch.arange(0, int(off[-1]) + 1, block_tokens, device=dev)).cpu().tolist()
    edges = sorted(set([0, n_docs] + [min(c, n_docs) for c in cuts]))
    for d0, d1 in zip(edges[:-1], edges[1:]):
        a, b = int(off[d0]), int(off[d1])
        if b == a:
            continue
        doc = torch.repeat_interleave(torch.arange(d1 - d0, device=dev), lens[d0:d1])
        key = doc * 65536 + (z[a:b].long() & 0xFFFF)
        c = torch.unique(key, return_counts=True)[1].double()
        out[0] += (torch.lgamma(c + prior) - lg_p).sum()
    return out


def loglik_terms(counts: torch.Tensor, prior: float, K: int) -> torch.Tensor:
    """sum_k lgamma(c + prior) - lgamma(prior) over the first K columns, and
    sum_rows lgamma(row_total + K prior) terms: returns (entry_sum, row_sum) fp64."""
    lg_p = torch.lgamma(torch.tensor(prior, dtype=torch.float64))
    lg_kp = torch.lgamma(torch.tensor(K * prior, dtype=torch.float64))
    out = torch.zeros(2, dtype=torch.float64, device=counts.device)
    step = max(1, (1 << 26) // max(K, 1))  # row blocks: fp64 temporaries stay ~0.5 GB at large K
    for r in range(0, counts.shape[0], step):
        c = counts[r:r + step, :K].double()
        if counts.dtype == torch.int16:  # packed unsigned 16-bit counts
            c = torch.where(c < 0, c + 65536.0, c)
        out[0] += (torch.lgamma(c + prior) - lg_p).sum()
        out[1] += (lg_kp - torch.lgamma(c.sum(1) + K * prior)).sum()
    return out
