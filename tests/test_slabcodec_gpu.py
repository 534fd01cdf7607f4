"""HIP slab codec (csrc/slabcodec.hip) against the PyTorch oracle: identical payloads and
lossless decode, strided slabs, and a corrupted payload that must not write out of row."""
import pytest
import torch

from harp_amd.ops.slabcodec import SlabCodec, capacity

def _random_counts(rows, cols, max_tokens, seed):
    g = torch.Generator().manual_seed(seed)
    tok = torch.randint(0, max_tokens, (rows,), generator=g)
    tok[0] = 0
    slab = torch.zeros(rows, cols, dtype=torch.int32)
    for r in range(rows):
        t = int(tok[r])
        if t:
            slab[r].index_add_(0, torch.randint(0, cols, (t,), generator=g), torch.ones(t, dtype=torch.int32))
    return slab


pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,cols", [(1, 64), (200, 1024), (333, 1000), (64, 4096)])
def test_gpu_payload_matches_cpu(cuda, rows, cols):
    slab = _random_counts(rows, cols, 3 * cols // 2, seed=rows + cols)
    cap = capacity(slab.sum(1), cols)
    cc, gc = SlabCodec(rows, cols, cap, "cpu"), SlabCodec(rows, cols, cap, cuda)
    pc = cc.encode(slab, torch.zeros(cc.nbytes, dtype=torch.uint8))
    pg = gc.encode(slab.to(cuda), torch.zeros(gc.nbytes, dtype=torch.uint8, device=cuda))
    nnz = int((slab != 0).sum())
    oc, kc, tc = cc._views(pc)
    og, kg, tg = gc._views(pg.cpu())
    assert torch.equal(oc, og) and int(og[-1]) == nnz
    assert torch.equal(kc[:nnz], kg[:nnz]) and torch.equal(tc[:nnz], tg[:nnz])
    out = torch.full((rows, cols), 9, dtype=torch.int32, device=cuda)
    gc.decode(pg, out)
    assert torch.equal(out.cpu(), slab)
    gc.check_overflow()


def test_gpu_strided_and_corrupt_payload(cuda):
    big = _random_counts(128, 320, 40, seed=5).to(cuda)
    view = big[:, :256]
    c = SlabCodec(128, 256, capacity(view.sum(1), 256), cuda)
    buf = c.encode(view, c.empty_payload())
    out = torch.zeros(128, 320, dtype=torch.int32, device=cuda)
    c.decode(buf, out[:, :256])
    assert torch.equal(out[:, :256], view) and int(out[:, 256:].abs().sum()) == 0
    # topic ids past the row and offsets past cap are ignored, never written
    _, _, topics = c._views(buf)
    topics[:5] = 300
    out2 = torch.zeros(128, 320, dtype=torch.int32, device=cuda)
    c.decode(buf, out2[:, :256])
    torch.cuda.synchronize()
    assert int(out2[:, 256:].abs().sum()) == 0


def test_gpu_overflow_flag(cuda):
    slab = _random_counts(16, 64, 30, seed=4).to(cuda)
    nnz = int((slab != 0).sum())
    c = SlabCodec(16, 64, nnz - 3, cuda)
    c.encode(slab, c.empty_payload())
    with pytest.raises(RuntimeError, match="overflow"):
        c.check_overflow()
