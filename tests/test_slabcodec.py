"""Sparse slab codec for the LDA rotation (harp_amd/ops/slabcodec.py, csrc/slabcodec.hip):
lossless round trips, the token bound, and a 2-worker rotation that gives exactly the
dense rotation's result."""
import pytest
import torch

from harp_amd.models.lda import LDAConfig, run_lda, synthetic_corpus
from harp_amd.ops.slabcodec import SlabCodec, capacity
from harp_amd.runtime.launcher import launch


def _random_counts(rows, cols, max_tokens, seed, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(0, max_tokens, (rows,), generator=g)
    tok[0] = 0                 # an empty row
    if rows > 1:
        tok[1] = 4 * cols      # a row denser than its topic count
    slab = torch.zeros(rows, cols, dtype=torch.int32)
    for r in range(rows):
        t = int(tok[r])
        if t:
            slab[r].index_add_(0, torch.randint(0, cols, (t,), generator=g), torch.ones(t, dtype=torch.int32))
    return slab.to(device)


@pytest.mark.parametrize("rows,cols", [(1, 64), (37, 100), (200, 1024)])
def test_roundtrip_cpu(rows, cols):
    slab = _random_counts(rows, cols, 50, seed=rows)
    c = SlabCodec(rows, cols, capacity(slab.sum(1), cols), "cpu")
    buf = c.encode(slab, c.empty_payload())
    out = torch.full_like(slab, -5)
    c.decode(buf, out)
    assert torch.equal(out, slab)
    assert int(c.overflow) == 0
    c.check_overflow()


def test_strided_slab_and_payload_size():
    big = _random_counts(64, 300, 20, seed=3)
    view = big[:, :256]
    c = SlabCodec(64, 256, capacity(view.sum(1), 256), "cpu")
    out = torch.zeros(64, 300, dtype=torch.int32)
    c.decode(c.encode(view, c.empty_payload()), out[:, :256])
    assert torch.equal(out[:, :256], view) and int(out[:, 256:].abs().sum()) == 0
    # sparse rows: the payload is far below the dense slab
    assert 4 * c.nbytes < c.dense_nbytes()


def test_overflow_is_flagged():
    slab = _random_counts(16, 64, 30, seed=4)
    nnz = int((slab != 0).sum())
    c = SlabCodec(16, 64, nnz - 3, "cpu")
    c.encode(slab, c.empty_payload())
    with pytest.raises(RuntimeError, match="overflow"):
        c.check_overflow()


def _job(comm, cfg, nd, V, toks):
    return run_lda(comm, cfg, nd, V, toks)


@pytest.mark.parametrize("P", [2, 3])
def test_lda_rotation_codec_matches_dense(P):
    """P = 3 rotates its two slices on different ring strides (1 and 2)."""
    corpus = synthetic_corpus(300, 2000, 8, 40, seed=2)
    base = dict(num_topics=64, alpha=0.1, beta=0.01, iterations=6, print_interval=2, num_slices=2)
    dense = launch(_job, P, args=(LDAConfig(rotate_codec="off", **base), 300, 2000, corpus), timeout=300)
    sparse = launch(_job, P, args=(LDAConfig(rotate_codec="on", **base), 300, 2000, corpus), timeout=300)
    assert dense[0]["rotate_payload_bytes"] == 0 and sparse[0]["rotate_payload_bytes"] > 0
    assert dense[0]["loglik"] == sparse[0]["loglik"], (dense[0]["loglik"], sparse[0]["loglik"])


def test_capacity_beyond_int32_offsets_is_refused():
    """offsets are int32; a cap past 2^31 would wrap them silently."""
    with pytest.raises(ValueError):
        SlabCodec(1 << 20, 4096, 2**31, torch.device("cpu"))
    c = SlabCodec(1 << 20, 4096, 1000, torch.device("cpu"))  # >= 2^31 cells: int64 row sums
    assert c.wide and not SlabCodec(64, 64, 100, torch.device("cpu")).wide
