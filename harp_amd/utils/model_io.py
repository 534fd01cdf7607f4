"""Text model dumps in the reference's formats.

* factor rows (MF-SGD ``W-<worker>`` / ``H-<worker>``, SGDCollectiveMapper.java:737-818):
  one line per row, ``<id> : v1 v2 ... vr``;
* LDA word model (``tmp_word_model/<iter>/<worker>``, LDAMPCollectiveMapper.java:593-628):
  one line per word, ``<wordID> topic:count topic:count ...`` over the non-zero topics;
* MDS embedding (XFileUtil.java:39-80 storeXOnMaster): one line per point,
  ``<id>\t<x1>\t...\t<xd>\t<label>`` with up to 10 decimals (label 1 by default);
* scalar evaluation files (``evaluation``: test RMSE / log-likelihood on one line).

Rows are copied device->host once per file and formatted with numpy.
"""
from __future__ import annotations

import os
from typing import Sequence

import numpy as np
import torch


def _ids(ids) -> np.ndarray:
    return (ids.detach().cpu().numpy() if torch.is_tensor(ids) else np.asarray(list(ids))).astype(np.int64)


def write_factor_rows(path: str, ids, F: torch.Tensor) -> str:
    ids = _ids(ids)
    M = F.detach().double().cpu().numpy()
    assert M.shape[0] == ids.shape[0], (M.shape, ids.shape)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        for i, row in zip(ids.tolist(), M):
            f.write(f"{i} : " + " ".join(repr(float(x)) for x in row) + "\n")
    os.replace(tmp, path)
    return path


def read_factor_rows(path: str):
    ids, rows = [], []
    with open(path) as f:
        for ln in f:
            if ":" not in ln:
                continue
            a, b = ln.split(":", 1)
            ids.append(int(a))
            rows.append([float(x) for x in b.split()])
    return torch.tensor(ids, dtype=torch.int64), torch.tensor(rows, dtype=torch.float64)


def write_topic_counts(path: str, ids, counts: torch.Tensor, num_topics: int) -> str:
    ids = _ids(ids)
    C = counts[:, :num_topics].detach().cpu().numpy()
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        for w, row in zip(ids.tolist(), C):
            nz = np.nonzero(row)[0]
            f.write(str(w) + "".join(f" {int(t)}:{int(row[t])}" for t in nz) + "\n")
    os.replace(tmp, path)
    return path


def read_topic_counts(path: str) -> dict:
    out = {}
    with open(path) as f:
        for ln in f:
            t = ln.split()
            if t:
                out[int(t[0])] = {int(a): int(b) for a, b in (x.split(":") for x in t[1:])}
    return out


def write_scalar(path: str, value: float) -> str:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        f.write(f"{value!r}\n")
    return path


def write_rows_text(path: str, rows: Sequence[Sequence[float]]) -> str:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        for r in rows:
            f.write(" ".join(repr(float(x)) for x in r) + "\n")
    return path


def _dec10(x: float) -> str:
    t = f"{x:.10f}".rstrip("0").rstrip(".")
    return "0" if t in ("", "-0") else t


def write_mds_points(path: str, X: torch.Tensor, labels=None) -> str:
    M = X.detach().double().cpu().numpy()
    lab = [1] * M.shape[0] if labels is None else [int(v) for v in labels]
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        for i, row in enumerate(M):
            f.write(f"{i}\t" + "".join(_dec10(float(v)) + "\t" for v in row) + f"{lab[i]}\n")
    os.replace(tmp, path)
    return path


def read_mds_points(path: str):
    ids, rows, labels = [], [], []
    with open(path) as f:
        for ln in f:
            t = ln.split("\t")
            if len(t) < 3:
                continue
            ids.append(int(t[0]))
            rows.append([float(v) for v in t[1:-1]])
            labels.append(int(t[-1]))
    return torch.tensor(ids, dtype=torch.int64), torch.tensor(rows, dtype=torch.float64), labels
