"""Data sources: CSV / CSR / COO / libsvm loaders and synthetic generators.

Reference: core/harp-daal-interface/.../datasource/HarpDAALDataSource.java:76-775
(multithreaded dense CSV -> HomogenNumericTable, CSR files -> CSRNumericTable, COO
lists, regroupCOOList) and data_gen/DataGenerator.java:56-249 (synthetic dense / label
CSV generators). Text parsing is host work: files are parsed with numpy (no pickle),
split across a thread pool per file, and returned as tensors ready to move to the GPU.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


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
    with ThreadPoolExecutor(max_workers=max(1, min(threads, len(files)))) as ex:
        parts = list(ex.map(_parse_dense, files))
    parts = [p for p in parts if p.size]
    return torch.from_numpy(np.concatenate(parts)) if parts else torch.zeros((0, 0), dtype=torch.float64)


def load_features_labels(path: str, n_labels: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """DAAL example layout: the last ``n_labels`` columns are the dependent variables."""
    A = load_dense_csv(path)
    return A[:, :-n_labels].contiguous(), A[:, -n_labels:].squeeze(1) if n_labels == 1 else A[:, -n_labels:]


def load_daal_csr(path: str, n_cols: Optional[int] = None) -> torch.Tensor:
    """DAAL CSR text: line 1 row offsets, line 2 column indices, line 3 values (1-based)."""
    with open(path) as f:
        lines = [ln.strip().rstrip(",") for ln in f if ln.strip()]
    ro = np.array([int(x) for x in lines[0].split(",")], dtype=np.int64) - 1
    ci = np.array([int(x) for x in lines[1].split(",")], dtype=np.int64) - 1
    va = np.array([float(x) for x in lines[2].split(",")], dtype=np.float64)
    nc = n_cols or int(ci.max()) + 1
    return torch.sparse_csr_tensor(torch.from_numpy(ro), torch.from_numpy(ci), torch.from_numpy(va),
                                   size=(len(ro) - 1, nc))


def load_coo(path: str, one_based: bool = True, sep: Optional[str] = None):
    """``row col value`` lines (Matrix Market body / Harp MF input) -> (rows, cols, vals)."""
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
    off = 1 if one_based else 0
    return (torch.tensor(r, dtype=torch.long) - off, torch.tensor(c, dtype=torch.long) - off,
            torch.tensor(v, dtype=torch.float64))


def load_libsvm(path: str, n_features: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """libsvm ``label idx:val ...`` rows -> (dense X, y)."""
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
