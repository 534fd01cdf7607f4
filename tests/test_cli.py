"""Reference-compatible CLI: positional launcher args + named flags, run end to end on
2 gloo workers (spawned by the CLI itself)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from harp_amd import cli

REF = "/root/reference/datasets"


def _run(args, timeout=600):
    env = dict(os.environ)
    out = subprocess.run([sys.executable, "-m", "harp_amd.cli", *args], capture_output=True, text=True,
                         timeout=timeout, env=env, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)["result"]


def test_parse_positional_and_named():
    cfg = cli.parse("kmeans", ["1000", "10", "10", "2", "2", "16", "5", "/w", "/l", "--iterations", "7",
                               "--strategy", "allreduce"])
    assert cfg["num_points"] == 1000 and cfg["num_centroids"] == 10 and cfg["files_per_worker"] == 2
    assert cfg["iterations"] == 7 and cfg["strategy"] == "allreduce" and cfg["work_dir"] == "/w"
    cfg = cli.parse("sgd", ["--rank", "8", "--input", "x"])
    assert cfg["rank"] == 8 and cfg["lam"] == 0.05


def test_cli_kmeans(tmp_path):
    res = _run(["kmeans", "1000", "10", "10", "2", "2", "1", "20", str(tmp_path / "work"), str(tmp_path / "pts"),
                "true", "--strategy", "allreduce"])
    obj = res["objective"]
    assert len(obj) == 20 and obj[-1] <= obj[0]
    c = np.loadtxt(tmp_path / "work" / "centroids" / "out")
    assert c.shape == (10, 10)
    assert len(os.listdir(tmp_path / "pts")) == 4  # filesPerWorker * maps


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference datasets not present")
def test_cli_sgd_movielens_slice(tmp_path):
    train = os.path.join(REF, "daal_als", "movielens-train")
    test = os.path.join(REF, "daal_als", "movielens-test")
    files = sorted(os.listdir(train))[:2]
    os.makedirs(tmp_path / "tr")
    for f in files:
        os.symlink(os.path.join(train, f), tmp_path / "tr" / f)
    res = _run(["sgd", str(tmp_path / "tr"), "16", "0.05", "0.01", "6", "100", "2", "1", "1.0", "0",
                str(tmp_path / "work"), test])
    rm = res["rmse"]
    assert rm[-1][1] < 1.2  # train RMSE after a few epochs on 1-5 star ratings
    assert os.path.exists(tmp_path / "work" / "evaluation")


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference datasets not present")
def test_cli_pagerank_reference_input():
    res = _run(["pagerank", os.path.join(REF, "tutorial", "simplepagerank", "input5K-2partitions"), "5000", "10", "2"])
    assert "pagerank" not in res  # tensors are not printed; the run succeeded


def test_cli_lda_ccd_subgraph_mds_daal(tmp_path):
    g = torch.Generator().manual_seed(0)
    # lda docs: "docName w w w"
    os.makedirs(tmp_path / "docs")
    for part in range(2):
        with open(tmp_path / "docs" / f"d{part}", "w") as f:
            for d in range(20):
                t = (d + part) % 3
                ws = torch.randint(t * 10, t * 10 + 10, (15,), generator=g).tolist()
                f.write(f"doc{part}_{d} " + " ".join(map(str, ws)) + "\n")
    res = _run(["lda", str(tmp_path / "docs"), "3", "0.1", "0.01", "4", "0", "0", "2", "1", "1.0", "0",
                str(tmp_path / "lda"), "false"])
    assert len(res["loglik"]) >= 1
    # ccd: COO "row col val"
    os.makedirs(tmp_path / "mf")
    u = torch.randint(0, 30, (400,), generator=g)
    i = torch.randint(0, 20, (400,), generator=g)
    with open(tmp_path / "mf" / "part0", "w") as f:
        for a, b in sorted(set(zip(u.tolist(), i.tolist()))):
            f.write(f"{a} {b} {1 + (a * b) % 5}\n")
    res = _run(["ccd", str(tmp_path / "mf"), "4", "0.1", "3", "2", "1", "2", str(tmp_path / "ccd"), ""])
    assert res["history"][-1]["train_rmse"] < res["history"][0]["train_rmse"] + 1e-9
    # subgraph: template + adjacency graph
    with open(tmp_path / "u3.template", "w") as f:
        f.write("3\n2\n0 1\n1 2\n")
    os.makedirs(tmp_path / "graph")
    with open(tmp_path / "graph" / "g0", "w") as f:
        for v in range(30):
            f.write(f"{v}\t{(v + 1) % 30},{(v + 7) % 30}\n")
    res = _run(["subgraph", "2", "true", str(tmp_path / "u3.template"), str(tmp_path / "graph"), str(tmp_path / "sc"),
                "1", "1", "x", "1", "0", "0", "false", "3"])
    assert res["estimate"] > 0
    # mds: big-endian int16 row blocks + ids file
    Y = torch.rand(24, 3, generator=g, dtype=torch.float64)
    D = torch.cdist(Y, Y)
    q = np.round(D.numpy() / D.max().item() * 32767).astype(">i2")
    os.makedirs(tmp_path / "mds")
    with open(tmp_path / "mds" / "ids", "w") as f:
        for b in range(2):
            q[b * 12:(b + 1) * 12].tofile(str(tmp_path / "mds" / f"distance_{b}"))
            f.write(f"{b}\t12\t24\t{b}\t{b * 12}\n")
    res = _run(["mds", "2", str(tmp_path / "mds"), "distance_", "w_", "v_", str(tmp_path / "mds" / "ids"), "",
                "1e-7", "3", "0.9", "24", "20", "1", "--work-dir", str(tmp_path / "mdsout")])
    assert res["stress"] < 1e-3
    with open(tmp_path / "mdsout" / "X") as f:
        lines = f.read().splitlines()
    assert len(lines) == 24 and lines[5].split("\t")[0] == "5" and lines[5].endswith("\t1")
    # daal-style pca on dense CSV files
    os.makedirs(tmp_path / "pca")
    X = torch.randn(200, 5, generator=g, dtype=torch.float64) @ torch.randn(5, 5, generator=g, dtype=torch.float64)
    for k in range(2):
        np.savetxt(tmp_path / "pca" / f"p{k}.csv", X[k * 100:(k + 1) * 100].numpy(), delimiter=",")
    _run(["daal", "pca", "2", "1", "0", "1", str(tmp_path / "pca"), str(tmp_path / "pcaout")])
    ev = np.loadtxt(tmp_path / "pcaout" / "pca_eigenvalues.csv", delimiter=",")
    ref = np.sort(np.linalg.eigvalsh(np.corrcoef(X.numpy().T)))[::-1]
    assert np.allclose(np.sort(ev.reshape(-1))[::-1], ref, atol=1e-8)
