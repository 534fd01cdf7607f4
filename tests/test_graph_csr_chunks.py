"""CSR build past torch's sort limit: input-order chunks, each stable-sorted, placed after
the earlier chunks' segments of the same row, give exactly the single-sort CSR."""
import torch

from harp_amd.ops import graph as G


def test_chunked_csr_equals_single_sort(monkeypatch):
    g = torch.Generator().manual_seed(0)
    rows = torch.randint(0, 300, (20000,), generator=g)
    cols = torch.randint(0, 1000, (20000,), generator=g)
    ref = G.build_csr(rows, cols, 300)
    for chunk in (1, 97, 4096, 19999):
        monkeypatch.setattr(G, "SORT_CHUNK", chunk)
        got = G.build_csr(rows, cols, 300)
        assert torch.equal(ref.rowptr, got.rowptr) and torch.equal(ref.col, got.col), chunk
