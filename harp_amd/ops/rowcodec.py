"""Sparse row codec for parameter-server push / pull (``csrc/rowcodec.hip``).

Count-table rows (LDA word-topic) travel as fixed-size per-row SLOTS whose capacity is a
token bound that never changes while sampling, so sender and receiver derive the same
layout once and every call is a fixed-size all-to-all with no size exchange (no host
sync). A slot is ``[int32 nnz][int32 counts cap][uint16 topics cap]`` or, when that is
not smaller, the dense row (``cap = -1``); every slot starts 16-byte aligned.

Reference: contrib/src/main/java/edu/iu/lda/LDAMapperDyn.java (push :380, pull :429)
moving sparse ``TopicCountList`` rows (ml/java/src/main/java/edu/iu/lda/LDAUtil.java:159-213).

GPU tensors use the HIP kernels (mandatory on a GPU); CPU tensors use the PyTorch
implementation below, which is also the oracle of the GPU tests.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _lib

_lib.register({
    "harp_rowcodec_encode": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p,
                             _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                             _lib.c_void_p],
    "harp_rowcodec_decode": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p,
                             _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p],
    # narrow (uint16 counts held in int16) global tables: encode from / add slots into
    "harp_rowcodec_encode16": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p,
                               _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    "harp_rowcodec_decode_add16": [_lib.c_void_p, _lib.c_long, _lib.c_int, _lib.c_void_p, _lib.c_int, _lib.c_void_p,
                                   _lib.c_void_p, _lib.c_void_p, _lib.c_void_p],
    "harp_rowcodec_copy_slots": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                                 _lib.c_int, _lib.c_int, _lib.c_void_p],
    "harp_rowcodec_merge": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_int,
                            _lib.c_void_p, _lib.c_int, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int,
                            _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_void_p,
                            _lib.c_int, _lib.c_void_p, _lib.c_void_p],
    "harp_rowcodec_merge_meta_bytes": [],
    "harp_rowcodec_merge_bounds": [_lib.c_void_p],
    "harp_rowcodec_reset": [_lib.c_void_p, _lib.c_void_p, _lib.c_void_p, _lib.c_int, _lib.c_int, _lib.c_void_p],
})

ALIGN = 16
MAX_K = 16384  # LDS row limit of the kernels (one 64 KB workgroup row)


def slot_caps(bound: torch.Tensor, K: int) -> torch.Tensor:
    """Per-row slot capacity from a nonzero bound: min(K, bound), or -1 (dense slot) when
    the sparse slot would not be smaller than the dense row."""
    c = bound.clamp(min=0, max=K).to(torch.int64)
    return torch.where(4 + 6 * c >= 4 * K, torch.full_like(c, -1), c)


def slot_sizes(caps: torch.Tensor, K: int) -> torch.Tensor:
    """Bytes of each slot (16-aligned)."""
    raw = torch.where(caps < 0, torch.full_like(caps, 4 * K), 4 + 6 * caps.clamp_min(0))
    return (raw + ALIGN - 1) // ALIGN * ALIGN


def layout(caps: torch.Tensor, K: int, base: int = 0) -> Tuple[torch.Tensor, int]:
    """(slot byte offsets from ``base``, total bytes) of consecutive slots."""
    sz = slot_sizes(caps, K)
    off = torch.cumsum(sz, 0) - sz + base
    return off, int(sz.sum().item())


def _check_args(t: torch.Tensor, K: int, narrow_ok: bool = False) -> None:
    ok = t.dtype == torch.int32 or (narrow_ok and t.dtype == torch.int16)
    if not ok or t.dim() != 2 or t.shape[1] < K or t.stride(1) != 1:
        raise ValueError(f"rowcodec needs an int32 [rows, >=K] table, got {tuple(t.shape)} {t.dtype}")
    if K <= 0 or K % 4 or K > MAX_K or (t.dtype == torch.int16 and (K % 8 or t.stride(0) % 8)):
        raise ValueError(f"rowcodec needs 0 < K <= {MAX_K}, K % 4 == 0 (K % 8 and a row stride % 8 for a "
                         f"narrow table; got K={K})")


def narrow_ok(max_count: int) -> bool:
    """A global count table may be narrow (uint16 counts stored in int16: half the bytes of
    every pull encode) when no count can reach 65536 -- every count of a word row is at
    most the word's token total."""
    return max_count < 65536


def widen(t: torch.Tensor) -> torch.Tensor:
    """int32 counts of a table (narrow int16 tables hold uint16 counts)."""
    return t.to(torch.int32) & 0xFFFF if t.dtype == torch.int16 else t


def _dense_rows(buf: torch.Tensor, off: torch.Tensor, cap: torch.Tensor, K: int) -> torch.Tensor:
    """Decode every slot into dense rows [n, K] (CPU oracle)."""
    n = off.numel()
    out = torch.zeros((n, K), dtype=torch.int32, device=buf.device)
    if n == 0:
        return out
    w32 = buf.view(torch.int32)
    w16 = buf.view(torch.int16)
    dense = cap < 0
    if bool(dense.any()):
        d = torch.nonzero(dense).flatten()
        idx = (off[d] // 4)[:, None] + torch.arange(K, device=buf.device)[None, :]
        out[d] = w32[idx]
    sp = torch.nonzero(~dense).flatten()
    if sp.numel():
        o, c = off[sp], cap[sp]
        nnz = w32[o // 4].to(torch.int64).clamp(min=0)
        nnz = torch.minimum(nnz, c)
        rows = torch.repeat_interleave(sp, nnz)
        first = torch.cumsum(nnz, 0) - nnz
        e = torch.arange(int(nnz.sum()), device=buf.device) - torch.repeat_interleave(first, nnz)
        ro, rc = torch.repeat_interleave(o, nnz), torch.repeat_interleave(c, nnz)
        cnt = w32[(ro + 4 + 4 * e) // 4]
        top = w16[(ro + 4 + 4 * rc + 2 * e) // 2].to(torch.int64) & 0xFFFF
        ok = top < K
        out.index_put_((rows[ok], top[ok]), cnt[ok], accumulate=True)  # repeated topics add up
    return out


def encode(src: torch.Tensor, K: int, rows: torch.Tensor, off: torch.Tensor, cap: torch.Tensor, out: torch.Tensor,
           overflow: torch.Tensor, before: Optional[torch.Tensor] = None, b_off: Optional[torch.Tensor] = None,
           b_cap: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Slot j of ``out`` := row ``src[rows[j], :K]`` (minus the row decoded from slot j of
    ``before`` when given: a count delta against the pulled snapshot). Entries past a
    slot's capacity are dropped and flag ``overflow``. ``rows`` int32, ``off`` int64
    byte offsets, ``cap`` int32 (-1 = dense slot). ``src`` may be a narrow table (int16
    holding uint16 counts; no ``before``)."""
    _check_args(src, K, narrow_ok=before is None)
    n = rows.numel()
    if n == 0:
        return out
    if src.dtype == torch.int16 and _lib.use_native(src):
        for t in (rows, off, cap, out, overflow):
            assert t.device == src.device and t.is_contiguous()
        assert rows.dtype == torch.int32 and off.dtype == torch.int64 and cap.dtype == torch.int32
        st = _lib.kernels().harp_rowcodec_encode16(
            src.data_ptr(), src.stride(0), K, rows.data_ptr(), n, off.data_ptr(), cap.data_ptr(), out.data_ptr(),
            overflow.data_ptr(), _lib.stream_ptr(src.device))
        _lib.check(st, "rowcodec_encode16")
        return out
    if src.dtype == torch.int16:  # CPU oracle of the narrow table
        src = widen(src)
    if _lib.use_native(src):
        for t in (rows, off, cap, out, overflow) + ((before, b_off, b_cap) if before is not None else ()):
            assert t.device == src.device and t.is_contiguous()
        assert rows.dtype == torch.int32 and off.dtype == torch.int64 and cap.dtype == torch.int32
        st = _lib.kernels().harp_rowcodec_encode(
            src.data_ptr(), src.stride(0), K, rows.data_ptr(), n, off.data_ptr(), cap.data_ptr(), out.data_ptr(),
            _lib.ptr(before), _lib.ptr(b_off), _lib.ptr(b_cap), overflow.data_ptr(), _lib.stream_ptr(src.device))
        _lib.check(st, "rowcodec_encode")
        return out
    vals = src[rows.long(), :K]
    if before is not None:
        vals = vals - _dense_rows(before, b_off.long(), b_cap.long(), K)
    off, cap = off.long(), cap.long()
    w32, w16 = out.view(torch.int32), out.view(torch.int16)
    dense = cap < 0
    if bool(dense.any()):
        d = torch.nonzero(dense).flatten()
        w32[(off[d] // 4)[:, None] + torch.arange(K)[None, :]] = vals[d]
    sp = torch.nonzero(~dense).flatten()
    if sp.numel():
        v = vals[sp]
        nz = v != 0
        nnz = nz.sum(1)
        pos = torch.cumsum(nz.to(torch.int64), 1) - 1
        r, t = torch.nonzero(nz, as_tuple=True)
        p = pos[r, t]
        c = cap[sp][r]
        keep = p < c
        if not bool(keep.all()):
            overflow.fill_(1)
        r, t, p, c = r[keep], t[keep], p[keep], c[keep]
        o = off[sp][r]
        w32[(o + 4 + 4 * p) // 4] = v[r, t]
        w16[(o + 4 + 4 * c + 2 * p) // 2] = t.to(torch.int16)
        w32[off[sp] // 4] = torch.minimum(nnz, cap[sp]).to(torch.int32)
    return out


def decode(dst: torch.Tensor, K: int, rows: torch.Tensor, off: torch.Tensor, cap: torch.Tensor, inp: torch.Tensor,
           add: bool = False) -> torch.Tensor:
    """Row ``dst[rows[j], :K]`` := slot j of ``inp`` (``add``: += instead; rows may repeat
    and then all add). ``dst`` may be a narrow table (int16 holding uint16 counts) when
    ``add``."""
    _check_args(dst, K, narrow_ok=add)
    n = rows.numel()
    if n == 0:
        return dst
    if dst.dtype == torch.int16:
        if _lib.use_native(dst):
            for t in (rows, off, cap, inp):
                assert t.device == dst.device and t.is_contiguous()
            assert rows.dtype == torch.int32 and off.dtype == torch.int64 and cap.dtype == torch.int32
            st = _lib.kernels().harp_rowcodec_decode_add16(dst.data_ptr(), dst.stride(0), K, rows.data_ptr(), n,
                                                           off.data_ptr(), cap.data_ptr(), inp.data_ptr(),
                                                           _lib.stream_ptr(dst.device))
            _lib.check(st, "rowcodec_decode_add16")
            return dst
        vals = _dense_rows(inp, off.long(), cap.long(), K)
        wide = widen(dst[:, :K]).index_add_(0, rows.long(), vals)
        dst[:, :K] = wide.to(torch.int16)  # two's complement: uint16 counts round-trip
        return dst
    if _lib.use_native(dst):
        for t in (rows, off, cap, inp):
            assert t.device == dst.device and t.is_contiguous()
        assert rows.dtype == torch.int32 and off.dtype == torch.int64 and cap.dtype == torch.int32
        st = _lib.kernels().harp_rowcodec_decode(dst.data_ptr(), dst.stride(0), K, rows.data_ptr(), n, off.data_ptr(),
                                                 cap.data_ptr(), inp.data_ptr(), 1 if add else 0,
                                                 _lib.stream_ptr(dst.device))
        _lib.check(st, "rowcodec_decode")
        return dst
    vals = _dense_rows(inp, off.long(), cap.long(), K)
    r = rows.long()
    if add:
        dst[:, :K].index_add_(0, r, vals)
    else:
        dst[r, :K] = vals
    return dst


def copy_slots(inp: torch.Tensor, src_off: torch.Tensor, out: torch.Tensor, dst_off: torch.Tensor,
               cap: torch.Tensor, K: int) -> torch.Tensor:
    """Slot j of ``out`` (at ``dst_off[j]``) := the slot at ``src_off[j]`` of ``inp`` (same
    capacity ``cap[j]``): the header and used entries of a sparse slot, the whole dense row."""
    n = cap.numel()
    if n == 0:
        return out
    if _lib.use_native(out):
        for t in (inp, src_off, dst_off, cap):
            assert t.device == out.device and t.is_contiguous()
        assert src_off.dtype == torch.int64 and dst_off.dtype == torch.int64 and cap.dtype == torch.int32
        st = _lib.kernels().harp_rowcodec_copy_slots(inp.data_ptr(), src_off.data_ptr(), out.data_ptr(),
                                                     dst_off.data_ptr(), cap.data_ptr(), n, K,
                                                     _lib.stream_ptr(out.device))
        _lib.check(st, "rowcodec_copy_slots")
        return out
    sz = slot_sizes(cap.long(), K)
    for a, d, b in zip(src_off.tolist(), dst_off.tolist(), sz.tolist()):
        out[d:d + b] = inp[a:a + b]
    return out


# csrc/rowcodec.hip kTinyBound / kSmallBound / kHashBound: rows with at most this many entries
# merge in an LDS hash, 4 / 2 / 1 rows per wave; larger rows in a K-wide accumulator
MERGE_BOUNDS = (64, 256, 512)


def merge_classes(c_cap: torch.Tensor, src_ptr: torch.Tensor, src_idx: torch.Tensor, in_cap: torch.Tensor,
                  K: int) -> Tuple[torch.Tensor, ...]:
    """(tiny, small, hash, big) row lists (int32) for :func:`merge` from the static slot
    capacities: a row's entry bound is its canonical capacity plus its delta slots' (K for a
    dense slot)."""
    n = c_cap.numel()
    dsz = torch.where(in_cap < 0, torch.full_like(in_cap, K), in_cap).to(torch.int64)
    per = dsz[src_idx.long()] if src_idx.numel() else torch.zeros(0, dtype=torch.int64, device=c_cap.device)
    owner = torch.repeat_interleave(torch.arange(n, device=c_cap.device), (src_ptr[1:] - src_ptr[:-1]).long())
    bound = torch.where(c_cap < 0, torch.full_like(c_cap, K), c_cap).to(torch.int64)
    bound = bound.index_add(0, owner, per)
    cls = torch.full_like(bound, 3)
    for i, b in reversed(list(enumerate(MERGE_BOUNDS))):
        cls = torch.where((bound <= b) & (c_cap >= 0), torch.full_like(cls, i), cls)
    return tuple(torch.nonzero(cls == i).flatten().to(torch.int32).contiguous() for i in range(4))


def merge_plan(c_off: torch.Tensor, c_cap: torch.Tensor, src_ptr: torch.Tensor, src_idx: torch.Tensor,
               in_off: torch.Tensor, in_cap: torch.Tensor, K: int) -> dict:
    """The static part of :func:`merge` (layouts never change while sampling): the row classes
    and, for the lane-group classes, one 32-byte metadata row per canonical row (csrc/rowcodec.hip
    ``MergeMeta``: slot offsets, capacities, the first delta slot inlined, the delta range), so
    the kernels issue a row's loads together and the next row's under the current one."""
    tiny, small, hsh, big = merge_classes(c_cap, src_ptr, src_idx, in_cap, K)
    dev = c_cap.device
    q0, q1 = src_ptr[:-1].long(), src_ptr[1:].long()
    has = q1 > q0
    if src_idx.numel():
        first = src_idx.long()[q0.clamp(max=src_idx.numel() - 1)]
        doff = torch.where(has, in_off.long()[first], torch.zeros_like(q0))
        dcap = torch.where(has, in_cap.long()[first], torch.zeros_like(q0))
    else:
        doff = dcap = torch.zeros_like(q0)

    def meta(rows: torch.Tensor) -> torch.Tensor:
        r = rows.long()
        m = torch.empty((r.numel(), 4), dtype=torch.int64, device=dev)
        m[:, 0] = c_off.long()[r]
        m[:, 1] = doff[r]
        m[:, 2] = (c_cap.long()[r] & 0xFFFFFFFF) | (dcap[r] << 32)
        m[:, 3] = (q0[r] & 0xFFFFFFFF) | (q1[r] << 32)
        return m.contiguous()

    si = src_idx.long()
    return {"meta": [meta(tiny), meta(small), meta(hsh)], "big": big,
            "qoff": in_off.long()[si].contiguous() if si.numel() else torch.zeros(1, dtype=torch.int64, device=dev),
            "qcap": in_cap[si].to(torch.int32).contiguous() if si.numel() else torch.zeros(1, dtype=torch.int32,
                                                                                          device=dev)}


def merge(canon: torch.Tensor, c_off: torch.Tensor, c_cap: torch.Tensor, src_ptr: torch.Tensor,
          src_idx: torch.Tensor, inp: torch.Tensor, in_off: torch.Tensor, in_cap: torch.Tensor, K: int,
          overflow: torch.Tensor, plan: Optional[dict] = None) -> torch.Tensor:
    """Owner table held as slots (no dense table): canonical slot u := slot u + the delta
    slots ``src_idx[src_ptr[u]:src_ptr[u + 1]]`` of ``inp``, written back in place without
    zero counts (unique topics, in no fixed order; a dense slot stays dense). ``plan``:
    :func:`merge_plan` (built here when omitted). ``overflow`` |= 1 when a row exceeds
    its capacity, |= 2 when a count goes negative."""
    n = c_cap.numel()
    if n == 0:
        return canon
    if K <= 0 or K % 4 or K > MAX_K:
        raise ValueError(f"rowcodec merge needs 0 < K <= {MAX_K}, K % 4 == 0 (got {K})")
    if _lib.use_native(canon):
        for t in (c_off, c_cap, src_ptr, src_idx, inp, in_off, in_cap, overflow):
            assert t.device == canon.device and t.is_contiguous()
        assert c_off.dtype == torch.int64 and in_off.dtype == torch.int64
        assert c_cap.dtype == torch.int32 and in_cap.dtype == torch.int32
        assert src_ptr.dtype == torch.int32 and src_idx.dtype == torch.int32 and src_ptr.numel() == n + 1
        if plan is None:
            plan = merge_plan(c_off, c_cap, src_ptr, src_idx, in_off, in_cap, K)
        (mt, ms, mh), br = plan["meta"], plan["big"]
        st = _lib.kernels().harp_rowcodec_merge(canon.data_ptr(), inp.data_ptr(), mt.data_ptr(), mt.shape[0],
                                                ms.data_ptr(), ms.shape[0], mh.data_ptr(), mh.shape[0],
                                                plan["qoff"].data_ptr(), plan["qcap"].data_ptr(), br.data_ptr(),
                                                br.numel(), c_off.data_ptr(), c_cap.data_ptr(), src_ptr.data_ptr(),
                                                src_idx.data_ptr(), in_off.data_ptr(), in_cap.data_ptr(), K,
                                                overflow.data_ptr(), _lib.stream_ptr(canon.device))
        _lib.check(st, "rowcodec_merge")
        return canon
    # CPU oracle: dense rows, add, re-encode
    rows = _dense_rows(canon, c_off.long(), c_cap.long(), K)
    if src_idx.numel():
        d = _dense_rows(inp, in_off.long(), in_cap.long(), K)
        owner = torch.repeat_interleave(torch.arange(n), (src_ptr[1:] - src_ptr[:-1]).long())
        rows.index_add_(0, owner, d[src_idx.long()])
    if bool((rows < 0).any()):
        overflow.view(-1)[0] |= 2
    flag = torch.zeros_like(overflow)
    encode(rows, K, torch.arange(n, dtype=torch.int32), c_off, c_cap, canon, flag)
    overflow |= flag
    return canon


def reset_slots(buf: torch.Tensor, off: torch.Tensor, cap: torch.Tensor, K: int) -> torch.Tensor:
    """Empty every slot for a kernel to fill (nnz = 0, dense rows zeroed) without clearing
    the whole payload."""
    n = cap.numel()
    if n == 0:
        return buf
    if _lib.use_native(buf):
        for t in (off, cap):
            assert t.device == buf.device and t.is_contiguous()
        assert off.dtype == torch.int64 and cap.dtype == torch.int32
        _lib.check(_lib.kernels().harp_rowcodec_reset(buf.data_ptr(), off.data_ptr(), cap.data_ptr(), n, K,
                                                      _lib.stream_ptr(buf.device)), "rowcodec_reset")
        return buf
    w32 = buf.view(torch.int32)
    o, c = off.long(), cap.long()
    w32[o[c >= 0] // 4] = 0
    d = torch.nonzero(c < 0).flatten()
    if d.numel():
        w32[(o[d] // 4)[:, None] + torch.arange(K, device=buf.device)[None, :]] = 0
    return buf
