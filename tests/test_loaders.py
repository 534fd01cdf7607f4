"""Native multithreaded text loaders (csrc/host/loaders.cpp) vs the Python parsers.

The reference's MTReader/ReadDenseCSVTask/ReadCOOTask (HarpDAALDataSource.java:198-333)
parse with String.split + Double.parseDouble; here the native path must give exactly the
same arrays as the Python fallback on edge-case files, on files large enough to be split
over many threads, and on the reference's own daal_* fixtures (read as text)."""
import os

import numpy as np
import pytest
import torch

from harp_amd.utils import datasets as D

pytestmark = pytest.mark.skipif(D._native() is None, reason="libharp_runtime.so not built")


def _python(monkeypatch, fn, *a, **kw):
    monkeypatch.setenv("HARP_NATIVE_LOADERS", "0")
    try:
        return fn(*a, **kw)
    finally:
        monkeypatch.delenv("HARP_NATIVE_LOADERS")


def test_dense_edge_cases(tmp_path, monkeypatch):
    p = tmp_path / "a.csv"
    p.write_text("1,2,3\n\n4.5, -6e2 ,7,\r\n  \n8,9\n+1,nan,inf\n1e-300,2.5E+3,-0")
    nat = D.load_dense_csv(str(p))
    py = _python(monkeypatch, D.load_dense_csv, str(p))
    assert nat.shape == py.shape == (5, 3)
    assert torch.equal(torch.nan_to_num(nat, nan=-123.0), torch.nan_to_num(py, nan=-123.0))
    assert nat[2].tolist() == [8.0, 9.0, 0.0]  # short rows are zero-padded


def test_dense_many_ranges_matches_numpy(tmp_path):
    g = np.random.default_rng(0)
    A = g.uniform(-1e3, 1e3, size=(60000, 7))
    fn = tmp_path / "big.csv"
    np.savetxt(fn, A, delimiter=",", fmt="%.17g")
    assert os.path.getsize(fn) > 1 << 20  # split over several threads
    for threads in (1, 3, 8, 64):
        X = D.load_dense_csv(str(fn), threads=threads)
        assert X.shape == A.shape and np.array_equal(X.numpy(), A)


def test_dense_directory_in_file_order(tmp_path):
    files = D.generate_dense_csv(str(tmp_path / "d"), 1000, 5, files=3, seed=1)
    X = D.load_dense_csv(str(tmp_path / "d"))
    ref = np.concatenate([np.loadtxt(f, delimiter=",", ndmin=2) for f in sorted(files)])
    assert np.array_equal(X.numpy(), ref)


def test_coo_matches_python(tmp_path, monkeypatch):
    g = np.random.default_rng(2)
    lines = ["%%MatrixMarket matrix coordinate real general", "% comment"]
    for _ in range(50000):
        lines.append(f"{g.integers(1, 5000)} {g.integers(1, 900)} {g.uniform(1, 5):.6f}")
    lines.insert(100, "")
    lines.insert(200, "12,34,2.5")
    fn = tmp_path / "r.mm"
    fn.write_text("\n".join(lines) + "\n")
    nat = D.load_coo(str(fn))
    py = _python(monkeypatch, D.load_coo, str(fn))
    for a, b in zip(nat, py):
        assert a.dtype == b.dtype and torch.equal(a, b)
    assert int(nat[0][197]) == 11 and int(nat[1][197]) == 33  # 1-based -> 0-based


def test_libsvm_matches_python(tmp_path, monkeypatch):
    fn = tmp_path / "s.svm"
    fn.write_text("1 1:0.5 3:2\n-1 2:1.5\n\n+1 4:-3e-1 1:7\n")
    Xn, yn = D.load_libsvm(str(fn))
    Xp, yp = _python(monkeypatch, D.load_libsvm, str(fn))
    assert torch.equal(Xn, Xp) and torch.equal(yn.double(), yp.double())
    assert Xn.shape == (3, 4) and Xn[2, 3] == -0.3


def test_malformed_field_raises(tmp_path):
    fn = tmp_path / "bad.csv"
    fn.write_text("1,2\n3,abc\n")
    with pytest.raises(ValueError):
        D.load_dense_csv(str(fn))


REF = "/root/reference/datasets"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference datasets not present")
@pytest.mark.parametrize("sub", ["daal_reg/train", "daal_dtree/train", "daal_svm/multidense/train", "daal_em/batchdense/train",
                                 "daal_kmeans/densedistri"])
def test_reference_fixtures_native_equals_python(sub, monkeypatch):
    path = os.path.join(REF, sub)
    if not os.path.exists(path):
        pytest.skip(f"{sub} absent")
    files = [f for f in D.list_files(path) if f.endswith(".csv")] or D.list_files(path)
    for f in files[:3]:
        nat = D.load_dense_csv(f)
        py = _python(monkeypatch, D.load_dense_csv, f)
        assert nat.shape == py.shape and torch.equal(nat, py), f
