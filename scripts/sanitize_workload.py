#!/usr/bin/env python3
"""Exercise every host C++ entry point of libharp_runtime on CPU tensors: the
multithreaded loaders (dense CSV split over many ranges, COO with comments, libsvm, a
malformed file), the sequential MF-SGD update + SSE and the LDA Gibbs sampler. Run under a
sanitizer build by tests/test_sanitizers.py (HARP_RUNTIME_LIB + LD_PRELOAD of the
sanitizer runtime); prints "sanitize workload ok" on success."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from harp_amd.ops import _lib  # noqa: E402
from harp_amd.ops import lda as L  # noqa: E402
from harp_amd.ops import mf as MF  # noqa: E402
from harp_amd.utils import datasets as D  # noqa: E402


def main() -> int:
    want = os.environ.get("HARP_RUNTIME_LIB")
    assert D._native() is not None, "runtime not loadable"
    if want:
        assert _lib.runtime()._name == want, (_lib.runtime()._name, want)
    g = np.random.default_rng(0)
    with tempfile.TemporaryDirectory() as td:
        A = g.uniform(-5, 5, size=(20000, 9))
        fn = os.path.join(td, "a.csv")
        np.savetxt(fn, A, delimiter=",", fmt="%.6f")
        for th in (1, 5, 16):
            X = D.load_dense_csv(fn, threads=th)
            assert X.shape == A.shape and np.allclose(X.numpy(), A, atol=1e-6)
        fn = os.path.join(td, "r.mm")
        with open(fn, "w") as f:
            f.write("% header\n")
            for _ in range(30000):
                f.write(f"{g.integers(1, 900)} {g.integers(1, 300)} {g.uniform(1, 5):.4f}\n")
        r, c, v = D.load_coo(fn)
        assert r.numel() == 30000 and int(r.min()) >= 0
        fn = os.path.join(td, "s.svm")
        with open(fn, "w") as f:
            for i in range(5000):
                f.write(f"{i % 2} " + " ".join(f"{j}:{g.uniform(0.5, 1):.3f}" for j in sorted(g.choice(40, 5, replace=False) + 1))
                        + "\n")
        Xs, ys = D.load_libsvm(fn)
        assert Xs.shape[0] == 5000 and (Xs != 0).sum() == 25000
        fn = os.path.join(td, "bad.csv")
        with open(fn, "w") as f:
            f.write("1,2\n3,x\n")
        try:
            D.load_dense_csv(fn)
            raise AssertionError("malformed file accepted")
        except ValueError:
            pass
    # MF-SGD sequential update + SSE (also the blocked cell schedule)
    nu, ni, n, rk = 300, 120, 20000, 32
    rows = torch.randint(0, nu, (n,), dtype=torch.int32)
    cols = torch.randint(0, ni, (n,), dtype=torch.int32)
    vals = torch.rand(n) * 4 + 1
    W, H = torch.rand(nu, rk) * 0.3, torch.rand(ni, rk) * 0.3
    e0 = MF.sse(rows, cols, vals, W, H).item()
    for _ in range(3):
        MF.sgd_update(rows, cols, vals, W, H, 0.01, 0.05)
    assert MF.sse(rows, cols, vals, W, H).item() < e0
    cid = MF.cell_layout(rows, cols, nu, ni)
    o = torch.argsort(cid)
    off = torch.zeros(65, dtype=torch.int64)
    off[1:] = torch.cumsum(torch.bincount(cid, minlength=64), 0)
    MF.sgd_update_blocked(rows[o].contiguous(), cols[o].contiguous(), vals[o].contiguous(), off, W, H, 0.01, 0.05)
    # LDA collapsed Gibbs sweep
    D_, V, K, T = 50, 80, 16, 4000
    tdoc = torch.randint(0, D_, (T,), dtype=torch.int32)
    tword = torch.sort(torch.randint(0, V, (T,), dtype=torch.int32)).values
    tz = torch.randint(0, K, (T,), dtype=torch.int32)
    ndk = torch.zeros((D_, K), dtype=torch.int32)
    nwk = torch.zeros((V, K), dtype=torch.int32)
    nk = torch.zeros(K, dtype=torch.int32)
    L.count(tdoc, tword, tz, ndk, nwk, nk)
    for sweep in range(3):
        delta = L.cgs_sample(tdoc, tword, tz, None, ndk, nwk, nk, K, 0.1, 0.01, V * 0.01, seed=sweep)
        nk += delta
        assert int(nk.sum()) == T and int(ndk.sum()) == T and int(nwk.sum()) == T
    print("sanitize workload ok", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
