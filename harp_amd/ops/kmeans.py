"""K-means device ops: padded point layout, assign+accumulate, normalize, prepare.

GPU tensors run the gfx950 kernels in ``csrc/kmeans.hip``; CPU tensors run the PyTorch
fp32 reference of the same op (also the numerics oracle in the GPU tests).

Layouts (chosen for the MFMA kernel):
  * points  ``X  [n, dp]`` bf16 (GPU) / fp32 (CPU), ``dp = round_up(d + 4, 16)``;
    columns ``d..d+3`` hold 1.0 (column d makes the accumulated row carry the count,
    d+1..d+3 pick up the three bf16 terms of ||c||^2 folded into the GEMM), rest 0;
  * centroids (master copy) ``c [K, d]`` fp32;
  * kernel operand ``Cm2 [Kp, dp]`` bf16: cols [0,d) = -2*bf16(c), col d = 0, cols
    d+1..d+3 = hi/mid/lo bf16 split of ||bf16(c)||^2; ``cn [Kp]`` the same norm in fp32;
    padded to ``Kp = round_up(K, 128)`` rows that can never win (norm = 1e38);
  * partial sums ``S [K, dp]`` fp32: columns ``0..d-1`` = sum of x, column ``d`` = count
    — the reference's centroid row (count + d values,
    KMeansCollectiveMapper.java:213-237) in a device-friendly order.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib

KP_ALIGN = 128
ONES = 4  # X columns d..d+3 hold 1.0
# (G4, W8, RG4, pipelined; 1024 points per workgroup) with static VALU priority for waves 4-7
# (15; 14 without it: 0.2 % slower, profiles/r3_setprio)
DEFAULT_VARIANT = 15


NARROW_MAX_DP = 256  # the register-resident assign kernel (X fragments live for the sweep)
WIDE_ALIGN = 64      # wider rows: the feature-staged kernel's stage width
WIDE_VARIANT = int(os.environ.get("HARP_KMEANS_WIDE_VARIANT", "0"))  # 0: the kernel default (LDS-staged, 8 waves: 6)


def padded_dim(d: int) -> int:
    dp = (d + ONES + 15) // 16 * 16
    return dp if dp <= NARROW_MAX_DP else (d + ONES + WIDE_ALIGN - 1) // WIDE_ALIGN * WIDE_ALIGN


def padded_k(k: int) -> int:
    return (k + KP_ALIGN - 1) // KP_ALIGN * KP_ALIGN


def row_stride(dp: int) -> int:
    """GPU row stride of the point matrix: dp rounded up to 128 bf16 = 256 B, so every row
    is whole 128-B lines. The MFMA k-range stays dp (the padding is never read by the
    assign); the bucketed gather-sum then fetches 2 lines per row instead of ~2.5."""
    return (dp + 127) // 128 * 128


def pack_points(x: torch.Tensor, device: torch.device | str | None = None) -> torch.Tensor:
    """[n, d] -> padded [n, dp] (bf16 on GPU, fp32 on CPU) with the count column. On the
    GPU the result is a [n, dp] view of rows laid out at :func:`row_stride`."""
    device = torch.device(device) if device is not None else x.device
    n, d = x.shape
    dp = padded_dim(d)
    dt = torch.bfloat16 if device.type == "cuda" else torch.float32
    ld = row_stride(dp) if device.type == "cuda" else dp
    out = torch.zeros((n, ld), dtype=dt, device=device)
    out[:, :d] = x.to(device=device, dtype=dt)
    out[:, d:d + ONES] = 1.0
    return out[:, :dp]


def generate_points(n: int, d: int, lo: float = 0.0, hi: float = 1000.0, seed: int = 0,
                    device: torch.device | str = "cpu", row0: int = 0) -> torch.Tensor:
    """Synthetic U[lo, hi) points in the padded layout, generated on the device
    (the reference's DataGenRunnable writes U[0,1000) doubles, KMUtil.java:112-178)."""
    device = torch.device(device)
    dp = padded_dim(d)
    if device.type == "cuda" and _lib.use_native(torch.empty(0, device=device)):
        ld = row_stride(dp)
        Xs = torch.empty((n, ld), dtype=torch.bfloat16, device=device)
        _lib.check(_lib.kernels().harp_uniform_rows_bf16(Xs.data_ptr(), n, d, ld, float(lo), float(hi),
                                                         seed & 0xFFFFFFFFFFFFFFFF, row0, 1,
                                                         _lib.stream_ptr(device)), "uniform_rows")
        return Xs[:, :dp]
    g = torch.Generator().manual_seed(seed * 1000003 + row0)
    x = torch.rand((n, d), generator=g, dtype=torch.float32) * (hi - lo) + lo
    return pack_points(x, device)


_SIDE: dict = {}


def pipeline_chunks(n: int, ppb: int) -> int:
    """Chunks the bucketed assign is split into (env HARP_KMEANS_CHUNKS, default 1 = one
    assign then one bucket + gather-sum). Small inputs always run unchunked."""
    c = int(os.environ.get("HARP_KMEANS_CHUNKS", "1"))
    return max(1, min(c, n // (ppb * 256)))  # every chunk still fills the chip


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(dev)
    return s


@dataclass
class CentroidOperand:
    Cm2: torch.Tensor  # [Kp, dp]
    cn: torch.Tensor   # [Kp]
    K: int
    d: int


def prepare(c: torch.Tensor, dp: int, out: Optional[CentroidOperand] = None) -> CentroidOperand:
    """Build the kernel operand (-2*bf16(c), ||bf16(c)||^2) from fp32 centroids."""
    K, d = c.shape
    Kp = padded_k(K)
    dev = c.device
    if out is None:
        dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
        out = CentroidOperand(torch.empty((Kp, dp), dtype=dt, device=dev), torch.empty(Kp, dtype=torch.float32, device=dev), K, d)
    if _lib.use_native(c):
        cc = c.contiguous().float()
        _lib.check(_lib.kernels().harp_kmeans_prepare(cc.data_ptr(), K, d, Kp, dp, out.Cm2.data_ptr(),
                                                      out.cn.data_ptr(), _lib.stream_ptr(dev)), "kmeans_prepare")
        return out
    out.Cm2.zero_()
    out.Cm2[:K, :d] = -2.0 * c
    out.cn.fill_(1e38)
    out.cn[:K] = (c.double() ** 2).sum(1).float()
    return out


def swept_k(op: "CentroidOperand") -> int:
    """Centroid rows the assign kernel sweeps: K rounded up to one 32-row MFMA group (the
    kernel skips the rest of the 128-row padding; K = 1e4 sweeps 10,016 of 10,112 rows)."""
    return min(op.Cm2.shape[0], (op.K + 31) // 32 * 32)


def _assign_wide(X, op, sums, labels, want_objective, obj_partial, min_dist):
    """dp > 256 (any d): the feature-staged kernel (csrc/kmeans.hip kmeans_assign_wide_kernel)
    merges per-centroid-block minima with 64-bit atomics, then the bucketed gather-sum."""
    n, dp = X.shape
    dev = X.device
    lib = _lib.kernels()
    assert X.dtype == torch.bfloat16 and X.stride(1) == 1 and X.stride(0) % 8 == 0 and op.Cm2.shape[1] == dp
    assert dp % WIDE_ALIGN == 0, f"wide rows need dp % {WIDE_ALIGN} == 0 (pack with padded_dim)"
    keys = torch.full((n,), -1, dtype=torch.int64, device=dev)  # all ones: +inf distance
    _lib.check(lib.harp_kmeans_assign_wide(X.data_ptr(), X.stride(0), op.Cm2.data_ptr(), n, dp, swept_k(op),
                                           op.Cm2.shape[0], op.d, keys.data_ptr(), WIDE_VARIANT, _lib.stream_ptr(dev)),
               "kmeans_assign_wide")
    nblk = (n + 255) // 256
    if want_objective and (obj_partial is None or obj_partial.numel() < nblk):
        obj_partial = torch.empty(nblk, dtype=torch.float32, device=dev)
    _lib.check(lib.harp_kmeans_wide_finish(keys.data_ptr(), n, labels.data_ptr(),
                                           obj_partial.data_ptr() if want_objective else None,
                                           min_dist.data_ptr() if min_dist is not None else None,
                                           _lib.stream_ptr(dev)), "kmeans_wide_finish")
    if sums is not None:
        from . import segment

        assert sums.dtype == torch.float32 and sums.shape[1] >= op.d + 1 and sums.is_contiguous()
        assert sums.shape[0] >= op.Cm2.shape[0], "sums needs Kp (padded) rows"
        assert sums.device == dev
        perm, start = segment.bucket_labels(labels, op.Cm2.shape[0])
        segment.bucket_rowsum(X, perm, start, sums)
    obj = obj_partial[:nblk].double().sum() if want_objective else None
    return labels, obj


def assign(X: torch.Tensor, op: CentroidOperand, sums: Optional[torch.Tensor] = None,
           labels: Optional[torch.Tensor] = None, want_objective: bool = True, variant: int = DEFAULT_VARIANT,
           obj_partial: Optional[torch.Tensor] = None, accumulate: str = "bucket",
           min_dist: Optional[torch.Tensor] = None):
    """Assign every point to its nearest centroid; optionally accumulate (x, 1) into
    ``sums`` [Kp, dp] and return the sum of squared distances (0-dim fp64 tensor).

    ``accumulate``: "bucket" (labels -> counting sort -> per-centroid row gather-sum,
    deterministic) or "atomic" (fused fp32 atomics in the assign kernel).
    ``min_dist`` (fp32 [n], optional) receives each point's squared distance to its
    centroid (used to merge partial argmins across centroid blocks under rotation).
    Returns (labels, objective)."""
    n, dp = X.shape
    dev = X.device
    if labels is None:
        labels = torch.empty(n, dtype=torch.int32, device=dev)
    if _lib.use_native(X):
        lib = _lib.kernels()
        if dp > NARROW_MAX_DP:
            if accumulate == "atomic":
                raise ValueError("accumulate='atomic' is only fused into the narrow kernel (dp <= "
                                 f"{NARROW_MAX_DP}); the wide path (dp = {dp}) accumulates by bucket")
            return _assign_wide(X, op, sums, labels, want_objective, obj_partial, min_dist)
        if dp > 128:
            variant = 4  # the only instantiation for 9..16 k-steps
        elif variant in (14, 15) and dp // 16 == 5:
            # the default tiling spills 22 VGPRs at 5 k-steps (d = 61..76); its RG=2 neighbour
            # does not: 112.1 vs 128.5 ms per assign at N = 1e8, d = 64 (profiles/r2_ktail)
            variant = 13
        ppb = lib.harp_kmeans_points_per_block(variant)
        if ppb <= 0:
            raise ValueError(f"unknown kmeans kernel variant {variant}")
        nblk = (n + ppb - 1) // ppb
        if want_objective and (obj_partial is None or obj_partial.numel() < nblk):
            obj_partial = torch.empty(nblk, dtype=torch.float32, device=dev)
        if sums is not None:
            assert sums.dtype == torch.float32 and sums.shape[1] >= op.d + 1 and sums.is_contiguous()
            assert sums.shape[0] >= op.Cm2.shape[0], "sums needs Kp (padded) rows"
            assert sums.device == dev
        assert X.dtype == torch.bfloat16 and X.stride(1) == 1 and X.stride(0) % 8 == 0 and op.Cm2.shape[1] == dp
        fused = sums if accumulate == "atomic" else None
        bucket = sums is not None and fused is None
        chunks = pipeline_chunks(n, ppb) if bucket else 1
        per = max(1, (nblk + chunks - 1) // chunks) * ppb  # rows per chunk, whole workgroups
        side = _side_stream(dev) if chunks > 1 else None
        main = torch.cuda.current_stream(dev)
        for r0 in range(0, n, per):
            r1 = min(n, r0 + per)
            b0 = r0 // ppb
            st = lib.harp_kmeans_assign(X[r0].data_ptr(), X.stride(0), op.Cm2.data_ptr(), r1 - r0, dp,
                                        swept_k(op), op.d,
                                        labels[r0].data_ptr(), _lib.ptr(fused),
                                        fused.stride(0) if fused is not None else 0,
                                        obj_partial[b0].data_ptr() if want_objective else None,
                                        min_dist[r0].data_ptr() if min_dist is not None else None, variant,
                                        _lib.stream_ptr(dev))
            _lib.check(st, "kmeans_assign")
            if not bucket:
                continue
            from . import segment

            if side is None:
                perm, start = segment.bucket_labels(labels, op.Cm2.shape[0])
                segment.bucket_rowsum(X, perm, start, sums)
                continue
            # bucket + gather-sum of this chunk on the side stream while the next chunk's
            # assign runs: the memory-bound row sums fill the gaps of the MFMA-bound assign
            side.wait_stream(main)
            with torch.cuda.stream(side):
                perm, start = segment.bucket_labels(labels[r0:r1], op.Cm2.shape[0])
                segment.bucket_rowsum(X[r0:r1], perm, start, sums)
        if side is not None:
            main.wait_stream(side)
        obj = obj_partial[:nblk].double().sum() if want_objective else None
        return labels, obj
    # CPU reference (fp32)
    Xf = X.float()
    d = op.d
    x = Xf[:, :d]
    C = -0.5 * op.Cm2[: op.K, :d].float()
    dist = op.cn[: op.K].unsqueeze(0) - 2.0 * (x @ C.t())
    lab = dist.argmin(1)
    labels.copy_(lab.to(labels.dtype))
    if min_dist is not None:
        min_dist.copy_((dist.gather(1, lab[:, None])[:, 0] + (x * x).sum(1)).to(min_dist.dtype))
    if sums is not None:
        sums[:, : d + 1].index_add_(0, lab, Xf[:, : d + 1])
    obj = None
    if want_objective:
        xs = (x.double() ** 2).sum(1)
        obj = (dist.gather(1, lab[:, None])[:, 0].double() + xs).clamp_min(0).sum()
    return labels, obj


def normalize(sums: torch.Tensor, c: torch.Tensor, d: int, counts: Optional[torch.Tensor] = None) -> torch.Tensor:
    """c[k] = sums[k, :d] / sums[k, d] where the count is > 0 (empty clusters keep c)."""
    Kr = c.shape[0]
    if _lib.use_native(c):
        assert sums.is_contiguous() and c.is_contiguous()
        _lib.check(_lib.kernels().harp_kmeans_normalize(sums.data_ptr(), sums.stride(0), c.data_ptr(), Kr, d,
                                                        _lib.ptr(counts), _lib.stream_ptr(c.device)),
                   "kmeans_normalize")
        return c
    cnt = sums[:, d]
    m = cnt > 0
    c[m] = sums[m, :d] / cnt[m, None]
    if counts is not None:
        counts.copy_(cnt)
    return c
