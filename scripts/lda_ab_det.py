"""A/B of two builds of the sparse LDA sampler in the deterministic one-wave mode: the
in-tree kernel (harp_amd/_native/libharp_kernels.so) against another build of csrc/lda.hip
(argv[1], e.g. the previous commit's), same inputs, same seed: token topics, doc-order
lists, word rows and topic deltas must be bit-identical (a refactor that keeps the
sampler's semantics)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from harp_amd.models.lda import synthetic_corpus  # noqa: E402
from harp_amd.ops import _lib  # noqa: E402
from harp_amd.ops import lda as L  # noqa: E402


def run(lib, K, seed, dev):
    doc, word = synthetic_corpus(3000, 4000, 20, 60, seed=4, device=dev)
    order = torch.argsort(word, stable=True)
    tdoc, tword = doc[order].int().contiguous(), word[order].int().contiguous()
    g = torch.Generator(device=dev).manual_seed(1)
    tz = torch.randint(0, K, (tdoc.numel(),), generator=g, device=dev, dtype=torch.int32)
    Kp = L.padded_topics(K)
    nwk = torch.zeros((4000, Kp), dtype=torch.int32, device=dev)
    nk = torch.zeros(Kp, dtype=torch.int32, device=dev)
    L.count(tdoc, tword, tz, None, nwk, nk)
    di = L.DocIndex.build(tdoc, tz, 3000)
    chunks = L.build_chunks(tword, 65536)
    ordc = L.chunk_order(chunks)
    span = di.span
    inv = torch.zeros(Kp, dtype=torch.float32, device=dev)
    inv[:K] = 1.0 / (nk[:K].float() + 4000 * 0.01)
    delta = torch.zeros(Kp, dtype=torch.int32, device=dev)
    work = torch.zeros(1, dtype=torch.int32, device=dev)
    f = lib.harp_lda_cgs_sparse_span
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_long] + [ctypes.c_void_p] * 5 + [ctypes.c_int] + [
        ctypes.c_void_p] * 2 + [ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_ulonglong, ctypes.c_int,
                                ctypes.c_void_p]
    st = f(span.data_ptr(), tword.data_ptr(), tz.data_ptr(), chunks.data_ptr(), chunks.numel() - 1, ordc.data_ptr(),
           work.data_ptr(), di.tpos.data_ptr(), di.zdoc.data_ptr(), nwk.data_ptr(), nwk.stride(0), inv.data_ptr(),
           delta.data_ptr(), K, 0.05, 0.01, seed, -1, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert st == 0, st
    return tz.cpu(), di.zdoc.cpu(), nwk.cpu(), delta.cpu()


def main():
    dev = torch.device("cuda", 0)
    new = _lib.kernels()
    old = ctypes.CDLL(sys.argv[1])
    for K in (1000, 2000, 5000):
        a = run(new, K, 77, dev)
        b = run(old, K, 77, dev)
        same = [torch.equal(x, y) for x, y in zip(a, b)]
        moved = int((a[0] != run(new, K, 78, dev)[0]).sum())
        print(f"K={K}: identical tz/zdoc/nwk/delta {same}; tokens {a[0].numel()}, seed-sensitivity {moved}")
        assert all(same)


if __name__ == "__main__":
    main()
