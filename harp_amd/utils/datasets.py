"""Data sources: CSV / CSR / COO / libsvm loaders and synthetic generators.

Reference: core/harp-daal-interface/.../datasource/HarpDAALDataSource.java:76-775
(multithreaded dense CSV -> HomogenNumericTable, CSR files -> CSRNumericTable, COO
lists, regroupCOOList) and data_gen/DataGenerator.java:56-249 (synthetic dense / label
CSV generators).

Text parsing is host work done natively: ``csrc/host/loaders.cpp`` (in
``libharp_runtime.so``) mmaps each file, splits it into line-aligned byte ranges and
parses every range on its own thread straight into the numpy buffer (the reference's
MTReader runs one Java thread per *file*). The pure-Python parsers below are the fallback
when the runtime library is not built (or ``HARP_NATIVE_LOADERS=0``) and the oracle of the
loader tests.
"""
from __future__ import annotations

import ctypes
import os
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


_I64P = ctypes.POINTER(ctypes.c_int64)


def _native():
    """The host runtime with the loader symbols bound, or None (then Python parsing)."""
    if os.environ.get("HARP_NATIVE_LOADERS", "1") == "0":
        return None
    from ..ops import _lib

    rt = _lib.runtime()
    if rt is None or not hasattr(rt, "harp_text_open"):
        return None
    if not getattr(rt, "_loaders_bound", False):
        vp, c = ctypes.c_void_p, ctypes.c_char
        rt.harp_text_open.argtypes, rt.harp_text_open.restype = [ctypes.c_char_p, ctypes.c_int], vp
        rt.harp_text_close.argtypes, rt.harp_text_close.restype = [vp], None
        rt.harp_dense_shape.argtypes = [vp, c, _I64P, _I64P]
        rt.harp_dense_fill.argtypes = [vp, c, vp, ctypes.c_int64]
        rt.harp_coo_count.argtypes = [vp, _I64P]
        rt.harp_coo_fill.argtypes = [vp, c, vp, vp, vp]
        rt.harp_libsvm_count.argtypes = [vp, _I64P, _I64P, _I64P]
        rt.harp_libsvm_fill.argtypes = [vp, vp, vp, vp, vp]
        for f in ("harp_dense_shape", "harp_dense_fill", "harp_coo_count", "harp_coo_fill", "harp_libsvm_count",
                  "harp_libsvm_fill"):
            getattr(rt, f).restype = ctypes.c_int
        rt._loaders_bound = True
    return rt


class _Text:
    """mmap'ed, range-split text file of the native loader."""

    def __init__(self, rt, path: str, threads: int):
        self.rt = rt
        self.h = rt.harp_text_open(os.fsencode(path), int(threads))
        if not self.h:
            raise OSError(f"cannot open {path}")

    def __enter__(self):
        return self.h

    def __exit__(self, *exc):
        self.rt.harp_text_close(self.h)


def _check(st: int, path: str) -> None:
    if st != 0:
        raise ValueError(f"{path}: malformed numeric field")


def _native_dense(rt, path: str, threads: int, sep: str = ",") -> np.ndarray:
    with _Text(rt, path, threads) as h:
        r, c = ctypes.c_int64(0), ctypes.c_int64(0)
        rt.harp_dense_shape(h, sep.encode(), ctypes.byref(r), ctypes.byref(c))
        out = np.zeros((r.value, c.value), dtype=np.float64)
        if out.size:
            _check(rt.harp_dense_fill(h, sep.encode(), out.ctypes.data, c.value), path)
    return out


def _parse_dense(path: str) -> np.ndarray:
    rows = []
    with open(path) as f:
        for ln in f:
            ln = ln.strip().rstrip(",")
            if ln:
                rows.append([float(x) for x in ln.replace(" ", "").split(",") if x != ""])
    width = max((len(r) for r in rows), default=0)
    out = np.zeros((len(rows), width), dtype=np.float64)
    for i, r in enumerate(rows):
        out[i, :len(r)] = r
    return out


def list_files(path: str) -> List[str]:
    if os.path.isdir(path):
        return sorted(os.path.join(path, f) for f in os.listdir(path) if not f.startswith("."))
    return [path]


def load_dense_csv(path: str, threads: int = 8) -> torch.Tensor:
    """All files of ``path`` (a file or a directory), rows concatenated in file order."""
    files = list_files(path)
    rt = _native()
    if rt is not None:
        parts = [_native_dense(rt, f, threads) for f in files]
    else:
        with ThreadPoolExecutor(max_workers=max(1, min(threads, len(files)))) as ex:
            parts = list(ex.map(_parse_dense, files))
    parts = [p for p in parts if p.size]
    return torch.from_numpy(np.concatenate(parts)) if parts else torch.zeros((0, 0), dtype=torch.float64)


def load_features_labels(path: str, n_labels: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """DAAL example layout: the last ``n_labels`` columns are the dependent variables."""
    A = load_dense_csv(path)
    return A[:, :-n_labels].contiguous(), A[:, -n_labels:].squeeze(1) if n_labels == 1 else A[:, -n_labels:]


def load_daal_csr(path: str, n_cols: Optional[int] = None) -> torch.Tensor:
    """DAAL CSR text: line 1 row offsets, line 2 column indices, line 3 values (1-based).
    A file whose column indices contain 0 is read as zero-based columns (the reference's
    daal_kernelfunc/csrbatch fixture mixes 1-based offsets with 0-based columns)."""
    with open(path) as f:
        lines = [ln.strip().rstrip(",") for ln in f if ln.strip()]
    ro = np.array([int(x) for x in lines[0].split(",")], dtype=np.int64) - 1
    ci = np.array([int(x) for x in lines[1].split(",")], dtype=np.int64)
    ci = ci - (0 if ci.size and ci.min() == 0 else 1)
    va = np.array([float(x) for x in lines[2].split(",")], dtype=np.float64)
    nc = n_cols or int(ci.max()) + 1
    return torch.sparse_csr_tensor(torch.from_numpy(ro), torch.from_numpy(ci), torch.from_numpy(va),
                                   size=(len(ro) - 1, nc))


def load_coo(path: str, one_based: bool = True, sep: Optional[str] = None, threads: int = 8):
    """``row col value`` lines (Matrix Market body / Harp MF input) -> (rows, cols, vals)."""
    off = 1 if one_based else 0
    rt = _native()
    if rt is not None and (sep is None or len(sep) == 1):
        rs, cs, vs = [], [], []
        for fn in list_files(path):
            with _Text(rt, fn, threads) as h:
                n = ctypes.c_int64(0)
                rt.harp_coo_count(h, ctypes.byref(n))
                R = np.empty(n.value, dtype=np.int64)
                C = np.empty(n.value, dtype=np.int64)
                V = np.empty(n.value, dtype=np.float64)
                if n.value:
                    _check(rt.harp_coo_fill(h, (sep or ",").encode(), R.ctypes.data, C.ctypes.data, V.ctypes.data), fn)
            rs.append(R)
            cs.append(C)
            vs.append(V)
        cat = (lambda xs, dt: torch.from_numpy(np.concatenate(xs)) if xs else torch.zeros(0, dtype=dt))
        return cat(rs, torch.long) - off, cat(cs, torch.long) - off, cat(vs, torch.float64)
    r, c, v = [], [], []
    for fn in list_files(path):
        with open(fn) as f:
            for ln in f:
                if not ln.strip() or ln.startswith("%"):
                    continue
                t = ln.replace(",", " ").split() if sep is None else ln.split(sep)
                r.append(int(t[0]))
                c.append(int(t[1]))
                v.append(float(t[2]))
    return (torch.tensor(r, dtype=torch.long) - off, torch.tensor(c, dtype=torch.long) - off,
            torch.tensor(v, dtype=torch.float64))


def load_libsvm(path: str, n_features: Optional[int] = None, threads: int = 8) -> Tuple[torch.Tensor, torch.Tensor]:
    """libsvm ``label idx:val ...`` rows -> (dense X, y)."""
    rt = _native()
    if rt is not None:
        parts = []
        for fn in list_files(path):
            with _Text(rt, fn, threads) as h:
                r, z, m = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
                _check(rt.harp_libsvm_count(h, ctypes.byref(r), ctypes.byref(z), ctypes.byref(m)), fn)
                y = np.empty(r.value, dtype=np.float64)
                ip = np.zeros(r.value + 1, dtype=np.int64)
                ix = np.empty(z.value, dtype=np.int64)
                va = np.empty(z.value, dtype=np.float64)
                _check(rt.harp_libsvm_fill(h, y.ctypes.data, ip.ctypes.data, ix.ctypes.data, va.ctypes.data), fn)
            parts.append((y, ip, ix, va, m.value))
        d = n_features or max((p[4] for p in parts), default=0)
        Xs = []
        for y, ip, ix, va, _ in parts:
            X = torch.zeros((y.size, d), dtype=torch.float64)
            rows = torch.repeat_interleave(torch.arange(y.size), torch.from_numpy(np.diff(ip)))
            X[rows, torch.from_numpy(ix)] = torch.from_numpy(va)
            Xs.append(X)
        return (torch.cat(Xs) if Xs else torch.zeros((0, d), dtype=torch.float64),
                torch.from_numpy(np.concatenate([p[0] for p in parts])) if parts else torch.zeros(0))
    ys, rows = [], []
    for fn in list_files(path):
        with open(fn) as f:
            for ln in f:
                t = ln.split()
                if not t:
                    continue
                ys.append(float(t[0]))
                rows.append([(int(a) - 1, float(b)) for a, b in (x.split(":") for x in t[1:])])
    d = n_features or (max((j for r in rows for j, _ in r), default=-1) + 1)
    X = torch.zeros((len(rows), d), dtype=torch.float64)
    for i, r in enumerate(rows):
        for j, v in r:
            X[i, j] = v
    return X, torch.tensor(ys)


def load_term_count_docs(files: List[str], metadata: Optional[str] = None):
    """Contrib LDA-CVB input (datasets/tutorial/lda-cvb, contrib lda/LDAMapper.java): one
    document per line as ``termId:count`` pairs; the metadata file's lines
    ``<file name> <first doc index>`` place each file's documents in the global numbering
    (files it does not name keep the order given). Returns global (doc, term, count)."""
    import os

    start = {}
    if metadata:
        with open(metadata) as f:
            for ln in f:
                t = ln.split()
                if len(t) >= 2:
                    start[t[0]] = int(t[1])
    docs, terms, cnts = [], [], []
    nxt = 0
    for path in files:
        d0 = start.get(os.path.basename(path), nxt)
        n = 0
        with open(path) as f:
            for ln in f:
                t = ln.split()
                if not t:
                    continue
                for pair in t:
                    w, c = pair.split(":")
                    if int(c) > 0:
                        docs.append(d0 + n)
                        terms.append(int(w))
                        cnts.append(float(c))
                n += 1
        nxt = max(nxt, d0 + n)
    return (torch.tensor(docs, dtype=torch.long), torch.tensor(terms, dtype=torch.long),
            torch.tensor(cnts, dtype=torch.float64))


def shard(n: int, rank: int, world: int) -> slice:
    """Contiguous row block of this worker."""
    return slice(rank * n // world, (rank + 1) * n // world)


# ---------------------------------------------------------------- generators (DataGenerator)
def generate_dense_csv(path: str, n: int, d: int, files: int = 1, seed: int = 0, lo: float = 0.0,
                       hi: float = 1.0, label_classes: int = 0) -> List[str]:
    """Write ``files`` CSV shards of uniform rows (optionally with an integer label column)."""
    os.makedirs(path, exist_ok=True)
    g = np.random.default_rng(seed)
    out = []
    for k in range(files):
        m = n // files + (1 if k < n % files else 0)
        A = g.uniform(lo, hi, size=(m, d))
        if label_classes:
            A = np.concatenate([A, g.integers(0, label_classes, size=(m, 1)).astype(np.float64)], 1)
        fn = os.path.join(path, f"data_{k:05d}.csv")
        np.savetxt(fn, A, delimiter=",", fmt="%.6f")
        out.append(fn)
    return out


ML10M_TEXT = "/root/reference/datasets/daal_als"  # the reference's movielens-{train,test} (read-only text)
ML10M_PACKED = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                            "data", "ml10m", "ml10m.npz")  # the same split: u int32, i uint16, 2 x rating uint8


def load_ml10m():
    """The reference's MF-SGD gate split (ml/java/test_scripts/mfsgd.sh:64): train / test
    (user, item, rating) triples, 0-based int64 ids and float32 ratings, plus (n_users,
    n_items). From the reference's text files when the checkout is present, else from the
    packed copy shipped in-tree (plain arrays, no pickle). Returns None if neither exists."""
    if os.path.isdir(ML10M_TEXT):
        u, i, v = load_coo(os.path.join(ML10M_TEXT, "movielens-train"), sep=" ")
        tu, ti, tv = load_coo(os.path.join(ML10M_TEXT, "movielens-test"), sep=" ")
        v, tv = v.float(), tv.float()
    elif os.path.exists(ML10M_PACKED):
        z = np.load(ML10M_PACKED)
        col = lambda k, dt: torch.from_numpy(z[k].astype(dt))  # noqa: E731
        u, i, v = col("train_u", np.int64), col("train_i", np.int64), col("train_v2", np.float32) / 2
        tu, ti, tv = col("test_u", np.int64), col("test_i", np.int64), col("test_v2", np.float32) / 2
    else:
        return None
    nu, ni = int(max(u.max(), tu.max())) + 1, int(max(i.max(), ti.max())) + 1
    return (u, i, v), (tu, ti, tv), nu, ni
