"""Sparse codec for rotating count slabs (``csrc/slabcodec.hip``).

A rotating LDA word-topic block is an int32 count matrix [rows, cols] whose rows are
mostly zero. A row with t tokens has at most min(cols, t) nonzero topics. The codec packs
a slab into ONE fixed-size uint8 payload::

    [row offsets (rows + 1) int32][counts cap int32][topics cap uint16]

``cap`` = sum over rows of min(cols, tokens(row)) is computed by every worker from the
per-word token totals. Those totals do not change during sampling, so a sender and its
receiver agree on the payload size without exchanging it. Encode and decode are
stream-ordered device work: no host sync sits between the sampler and the send. The
reference rotates dense ``TopicCountList`` rows
(ml/java/src/main/java/edu/iu/lda/LDAMPCollectiveMapper.java, dymoro/Rotator.java).

GPU tensors use the HIP kernels (mandatory there). CPU tensors use the PyTorch
implementation below, which is also the oracle of the GPU tests.
"""
from __future__ import annotations

import torch

from . import _lib

_lib.register({
    "harp_slab_nnz": [_lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_long, _lib.c_void_p, _lib.c_void_p],
    "harp_slab_pack": [_lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_long, _lib.c_void_p, _lib.c_long, _lib.c_void_p,
                       _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    "harp_slab_unpack": [_lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_long, _lib.c_void_p, _lib.c_long,
                         _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
})


def _align(n: int, a: int = 16) -> int:
    return (n + a - 1) // a * a


def capacity(row_tokens: torch.Tensor, cols: int) -> int:
    """Entries a slab can hold: sum over rows of min(cols, tokens of the row)."""
    return int(row_tokens.clamp(max=cols).sum().item())


class SlabCodec:
    """Encode / decode int32 [rows, cols] count slabs into fixed ``nbytes`` payloads."""

    def __init__(self, rows: int, cols: int, cap: int, device: torch.device):
        if cols > 65536:
            raise ValueError(f"topic ids travel as uint16: cols {cols} > 65536")
        self.rows, self.cols, self.cap = int(rows), int(cols), max(int(cap), 0)
        if self.cap >= 2**31 - 1:
            raise ValueError(f"slab codec capacity {self.cap} does not fit the int32 row offsets")
        # a slab with >= 2^31 cells could hold more nonzeros than int32 offsets count when its
        # counts break the token bound: such slabs sum the row counts in int64 and clamp at cap
        self.wide = self.rows * self.cols >= 2**31
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.o_counts = _align(4 * (self.rows + 1))
        self.o_topics = self.o_counts + _align(4 * self.cap)
        self.nbytes = self.o_topics + _align(2 * self.cap)
        self._nnz = torch.empty(self.rows, dtype=torch.int32, device=self.device)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=self.device)

    def dense_nbytes(self) -> int:
        return 4 * self.rows * self.cols

    def empty_payload(self) -> torch.Tensor:
        return torch.empty(self.nbytes, dtype=torch.uint8, device=self.device)

    def _views(self, buf: torch.Tensor):
        off = buf[: 4 * (self.rows + 1)].view(torch.int32)
        counts = buf[self.o_counts: self.o_counts + 4 * self.cap].view(torch.int32)
        topics = buf[self.o_topics: self.o_topics + 2 * self.cap].view(torch.int16)
        return off, counts, topics

    def _check(self, slab: torch.Tensor, buf: torch.Tensor) -> None:
        assert slab.dtype == torch.int32 and slab.dim() == 2 and tuple(slab.shape) == (self.rows, self.cols), slab.shape
        assert slab.stride(1) == 1 and buf.dtype == torch.uint8 and buf.numel() >= self.nbytes and buf.is_contiguous()
        assert slab.device == buf.device == self.device

    def encode(self, slab: torch.Tensor, buf: torch.Tensor) -> torch.Tensor:
        self._check(slab, buf)
        off, counts, topics = self._views(buf)
        if _lib.use_native(slab):
            lib, st = _lib.kernels(), _lib.stream_ptr(self.device)
            _lib.check(lib.harp_slab_nnz(slab.data_ptr(), self.rows, self.cols, slab.stride(0), self._nnz.data_ptr(), st),
                       "slab_nnz")
            off[0].zero_()
            if self.wide:
                c64 = torch.cumsum(self._nnz, 0, dtype=torch.int64)
                torch.maximum(self.overflow, (c64[-1:] > self.cap).to(torch.int32), out=self.overflow)
                off[1:].copy_(c64.clamp_max(self.cap))
            else:
                torch.cumsum(self._nnz, 0, dtype=torch.int32, out=off[1:])
            _lib.check(lib.harp_slab_pack(slab.data_ptr(), self.rows, self.cols, slab.stride(0), off.data_ptr(),
                                          self.cap, counts.data_ptr(), topics.data_ptr(), self.overflow.data_ptr(), st),
                       "slab_pack")
            return buf
        nz = slab != 0
        off[0] = 0
        off[1:] = torch.cumsum(nz.sum(1, dtype=torch.int64), 0).clamp_max(self.cap).to(torch.int32)
        r, c = nz.nonzero(as_tuple=True)  # row-major: column order within a row
        n = r.numel()
        if n > self.cap:
            self.overflow.fill_(1)
            r, c, n = r[: self.cap], c[: self.cap], self.cap
        counts[:n] = slab[r, c]
        topics[:n] = c.to(torch.int16)  # uint16 bit pattern (cols <= 65536)
        return buf

    def decode(self, buf: torch.Tensor, slab: torch.Tensor) -> torch.Tensor:
        self._check(slab, buf)
        off, counts, topics = self._views(buf)
        if _lib.use_native(slab):
            _lib.check(_lib.kernels().harp_slab_unpack(slab.data_ptr(), self.rows, self.cols, slab.stride(0),
                                                       off.data_ptr(), self.cap, counts.data_ptr(), topics.data_ptr(),
                                                       _lib.stream_ptr(self.device)), "slab_unpack")
            return slab
        slab.zero_()
        o = off.long().clamp(0, self.cap)
        lens = (o[1:] - o[:-1]).clamp_min(0)
        rows = torch.repeat_interleave(torch.arange(self.rows, device=slab.device), lens)
        first = torch.cumsum(lens, 0) - lens  # position of each row's first entry in `rows`
        idx = torch.repeat_interleave(o[:-1] - first, lens) + torch.arange(rows.numel(), device=slab.device)
        cols = topics[idx].long() & 0xFFFF
        keep = cols < self.cols
        slab[rows[keep], cols[keep]] = counts[idx][keep]
        return slab

    def check_overflow(self) -> None:
        """Raise if an encode dropped entries (cap was not a bound: counts inconsistent)."""
        if int(self.overflow.item()):
            raise RuntimeError("slab codec overflow: a slab held more nonzeros than its token bound")
