"""Stable argsort of small-range integer keys at any length.

torch sorts at most INT_MAX elements per call; an 8-GPU rank's share of the reference's
clueweb1 LDA run (29.9B tokens / 8 = 3.7e9 tokens, SURVEY §6 / BASELINE row 5) is past
that. Keys in [0, nkeys) (word ids, doc ids) are sorted in input-order chunks and each
chunk's key runs are placed after the earlier chunks' runs of the same key: the result is
the global stable order (the same scheme as ops.graph.build_csr's chunked CSR build).
"""
from __future__ import annotations

import torch

SORT_CHUNK = 1 << 30


def argsort_small_keys(keys: torch.Tensor, nkeys: int, chunk: int = 0) -> torch.Tensor:
    """int64 permutation ``order`` with ``keys[order]`` ascending and ties in input order
    (``chunk``: elements per sort call, default SORT_CHUNK)."""
    chunk = chunk if chunk > 0 else SORT_CHUNK
    E = keys.numel()
    dev = keys.device
    if E <= chunk:
        return torch.sort(keys, stable=True).indices
    bounds = list(range(0, E, chunk)) + [E]
    counts = [torch.bincount(keys[a:b].long(), minlength=nkeys)[:nkeys] for a, b in zip(bounds[:-1], bounds[1:])]
    total = torch.stack(counts).sum(0)
    start = torch.cumsum(total, 0) - total  # each key's first position in the output
    del total
    order = torch.empty(E, dtype=torch.int64, device=dev)
    before = torch.zeros(nkeys, dtype=torch.int64, device=dev)  # this key's tokens in earlier chunks
    for (a, b), cnt in zip(zip(bounds[:-1], bounds[1:]), counts):
        ks, o = torch.sort(keys[a:b], stable=True)
        ks = ks.long()
        seg = torch.cumsum(cnt, 0) - cnt  # each key's first position in the sorted chunk
        dest = start[ks] + before[ks] + (torch.arange(b - a, device=dev) - seg[ks])
        order[dest] = o + a
        before += cnt
        del ks, o, dest
    return order
