"""Reference-compatible command line: ``python -m harp_amd.cli <app> [positional args] [--flags]``.

Every app accepts the reference launcher's POSITIONAL argument order (drop-in) and the
same parameters as named flags (which win when both are given):

  kmeans    <N> <K> <d> <filesPerWorker> <maps> <threads> <iters> <workDir> <localDir> [regen]
            (ml/java kmeans/regroupallgather/KMeansLauncher.java:52-78)      [--strategy]
  sgd       <in> <r> <lambda> <epsilon> <iters> <trainRatio> <maps> <threads> <schedRatio>
            <memMB> <workDir> <test>                   (ml/java sgd/SGDLauncher.java:64-77)
  ccd       <in> <r> <lambda> <iters> <maps> <threads> <numModelSlices> <workDir> <test>
            (ml/java ccd/CCDLauncher.java:64-79)
  lda       <docDir> <K> <alpha> <beta> <iters> <minBound> <maxBound> <maps> <threads>
            <schedRatio> <memMB> <workDir> <printModel>   (ml/java lda/LDALauncher.java:64-79)
  mds       <maps> <inputFolder> <inputPrefix> <weightPrefix> <vPrefix> <idsFile> <labelsFile>
            <threshold> <d> <alpha> <n> <cgIter> <threads>  (ml/java wdamds/MDSLauncher.java:83-95)
  subgraph  <maps> <useLocalMultiThread> <template> <graphDir> <outDir> <threads> <cores>
            <affinity> <tpc> <memMB> <sendArrayLimit> <rotationPipeline> <iters>
            (ml/java subgraph/SCLauncher.java:76-88)                       [--strategy]
  ldacvb    <inputDir> <metafile> <outputDir> <numTerms> <numTopics> <numDocs> <maps> <iters>
            <threads> <mode>                 (contrib lda/LdaMapCollective.java, ldacvb.sh)
  pagerank  <inputDir> <numUrls> <iters> <maps>   (contrib simplepagerank)
  daal      <algo> <maps> <threads> <memMB> <iters> <inputDir> <workDir> [algo args]
            (harp-daal-interface data_aux/Initialize.java:97-130 common prefix)

``maps`` = number of workers. Outside torchrun the CLI spawns ``maps`` local worker
processes (RCCL on GPUs when ``maps`` <= visible GPUs, else gloo on CPU); under torchrun
each rank runs its share. ``threads`` / ``memMB`` are accepted for compatibility (the
grid and the caching allocator replace them). Outputs go to ``workDir`` like the
reference (centroids, W/H, word model, X, counts, PR values).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

# (name, type, default) — positional order of the reference launcher
SPECS: Dict[str, List[Tuple[str, type, Any]]] = {
    "kmeans": [("num_points", int, 1000), ("num_centroids", int, 10), ("dim", int, 10), ("files_per_worker", int, 1),
               ("maps", int, 2), ("threads", int, 1), ("iterations", int, 10), ("work_dir", str, "harp-work/kmeans"),
               ("local_dir", str, "harp-work/kmeans-points"), ("regen", str, "true")],
    "sgd": [("input", str, ""), ("rank", int, 40), ("lam", float, 0.05), ("epsilon", float, 0.002),
            ("iterations", int, 10), ("train_ratio", int, 100), ("maps", int, 2), ("threads", int, 1),
            ("sched_ratio", float, 1.0), ("mem", int, 0), ("work_dir", str, "harp-work/sgd"), ("test", str, "")],
    "ccd": [("input", str, ""), ("rank", int, 16), ("lam", float, 0.1), ("iterations", int, 10), ("maps", int, 2),
            ("threads", int, 1), ("num_model_slices", int, 2), ("work_dir", str, "harp-work/ccd"), ("test", str, ""),
            ("mode", str, "allgather")],
    "lda": [("doc_dir", str, ""), ("num_topics", int, 100), ("alpha", float, 0.01), ("beta", float, 0.01),
            ("iterations", int, 10), ("min_bound", int, 0), ("max_bound", int, 0), ("maps", int, 2), ("threads", int, 1),
            ("sched_ratio", float, 1.0), ("mem", int, 0), ("work_dir", str, "harp-work/lda"), ("print_model", str, "false")],
    "mds": [("maps", int, 2), ("input_folder", str, ""), ("input_prefix", str, "distance_"),
            ("weight_prefix", str, "weight_"), ("v_prefix", str, "v_"), ("ids_file", str, ""), ("labels_file", str, ""),
            ("threshold", float, 1e-6), ("d", int, 3), ("alpha", float, 0.95), ("n", int, 0), ("cg_iter", int, 20),
            ("threads", int, 1)],
    "subgraph": [("maps", int, 2), ("use_local_multithread", str, "true"), ("template", str, ""), ("graph_dir", str, ""),
                 ("out_dir", str, "harp-work/subgraph"), ("threads", int, 1), ("cores", int, 1), ("affinity", str, ""),
                 ("tpc", int, 1), ("mem", int, 0), ("send_array_limit", int, 0), ("rotation_pipeline", str, "false"),
                 ("iterations", int, 1)],
    "ldacvb": [("input_dir", str, ""), ("metafile", str, ""), ("output_dir", str, "harp-work/ldacvb"),
               ("num_terms", int, 0), ("num_topics", int, 10), ("num_docs", int, 0), ("maps", int, 2),
               ("iterations", int, 5), ("threads", int, 1), ("mode", int, 1)],
    "pagerank": [("input_dir", str, ""), ("num_urls", int, 0), ("iterations", int, 10), ("maps", int, 2)],
    "daal": [("algo", str, "pca"), ("maps", int, 2), ("threads", int, 1), ("mem", int, 0), ("iterations", int, 10),
             ("input_dir", str, ""), ("work_dir", str, "harp-work/daal")],
}
EXTRA = {  # named-only flags
    "kmeans": [("strategy", str, "regroup_allgather")],
    "subgraph": [("strategy", str, "allgather"), ("seed", int, 0)],
    "lda": [("vocab", int, 0)],
    "ldacvb": [("strategy", str, "allreduce"), ("init", str, "random"), ("alpha", float, 1e-3), ("eta", float, 0.0),
               ("gamma_iters", int, 29)],
    "sgd": [("num_users", int, 0), ("num_items", int, 0)],
    "ccd": [("num_users", int, 0), ("num_items", int, 0)],
    "daal": [("k", int, 0), ("method", str, ""), ("label_cols", int, 1)],
    "mds": [("work_dir", str, "harp-work/mds"), ("checkpoint_every", int, 0)],
}


def _bool(s) -> bool:
    return str(s).lower() in ("1", "true", "yes", "y")


def parse(app: str, argv: Sequence[str]) -> Dict[str, Any]:
    spec = SPECS[app] + EXTRA.get(app, [])
    ap = argparse.ArgumentParser(prog=f"harp_amd.cli {app}")
    ap.add_argument("positional", nargs="*")
    for name, typ, _ in spec:
        ap.add_argument("--" + name.replace("_", "-"), dest=name, type=typ, default=None)
    ap.add_argument("--backend", default=None)
    a, extra = ap.parse_known_args(list(argv))
    cfg = {name: default for name, _, default in spec}
    for (name, typ, _), val in zip(SPECS[app], a.positional):
        cfg[name] = typ(val)
    cfg["extra_args"] = list(a.positional[len(SPECS[app]):]) + extra
    for name, _, _ in spec:
        v = getattr(a, name)
        if v is not None:
            cfg[name] = v
    cfg["backend"] = a.backend
    return cfg


# ------------------------------------------------------------------ helpers
def _files(path: str) -> List[str]:
    from .utils.datasets import list_files

    return list_files(path) if path else []


def _my_files(comm, path: str) -> List[str]:
    from .runtime.inputformat import multi_file_splits

    return multi_file_splits(_files(path), comm.world_size, seed=0)[comm.rank]


def _allmax(comm, v: int) -> int:
    from .core.combiner import Operation
    from .models.common import reduce_partials

    return int(reduce_partials(comm, {"m": torch.tensor([float(v)])}, op=Operation.MAX)["m"][0])


def _coo(files: Sequence[str]):
    from .utils.datasets import load_coo

    parts = [load_coo(f, one_based=False) for f in files]
    if not parts:
        z = torch.zeros(0, dtype=torch.long)
        return z, z.clone(), torch.zeros(0, dtype=torch.float64)
    return tuple(torch.cat(x) for x in zip(*parts))


def _write(path: str, text: str) -> None:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        f.write(text)


# ------------------------------------------------------------------ app runners (one rank)
def run_app(comm, app: str, cfg: Dict[str, Any]) -> Dict[str, Any]:
    return globals()["_run_" + app](comm, cfg)


def _run_kmeans(comm, cfg):
    from .models.kmeans import KMeansCollectiveMapper, KMeansConfig
    from .runtime.mapper import Context, KeyValReader

    P, me = comm.world_size, comm.rank
    files = sorted(_files(cfg["local_dir"])) if os.path.isdir(cfg["local_dir"]) else []
    if _bool(cfg["regen"]) or not files:
        # KMUtil.generatePoints: filesPerWorker*maps text files of U[0,1000) points
        nf = cfg["files_per_worker"] * P
        if me == 0:
            from .utils.datasets import generate_dense_csv

            import shutil
            shutil.rmtree(cfg["local_dir"], ignore_errors=True)
            paths = generate_dense_csv(cfg["local_dir"], cfg["num_points"], cfg["dim"], nf, seed=0, lo=0, hi=1000)
            for p in paths:  # space-separated like the reference's point files
                with open(p) as f:
                    txt = f.read().replace(",", " ")
                with open(p, "w") as f:
                    f.write(txt)
        comm.barrier()
        files = sorted(_files(cfg["local_dir"]))
    mine = [f for i, f in enumerate(files) if i % P == me]
    kc = KMeansConfig(num_points=0, num_centroids=cfg["num_centroids"], dim=cfg["dim"], iterations=cfg["iterations"],
                      strategy=cfg["strategy"], objective_every=1)
    m = KMeansCollectiveMapper(comm, kc)
    m.run(KeyValReader([(i, f) for i, f in enumerate(mine)]), Context(cfg))
    if comm.rank == 0:
        c = m.centroids.cpu()
        _write(os.path.join(cfg["work_dir"], "centroids", "out"),
               "\n".join(" ".join(f"{v:.6f}" for v in row.tolist()) for row in c) + "\n")
    return {"objective": m.objective, "work_dir": cfg["work_dir"]}


def _mf_data(comm, cfg):
    u, i, v = _coo(_my_files(comm, cfg["input"]))
    nu = cfg.get("num_users") or _allmax(comm, int(u.max()) + 1 if u.numel() else 0)
    ni = cfg.get("num_items") or _allmax(comm, int(i.max()) + 1 if i.numel() else 0)
    test = None
    if cfg.get("test"):
        test = _coo(_files(cfg["test"]))
        nu, ni = max(nu, int(test[0].max()) + 1), max(ni, int(test[1].max()) + 1)
    return u, i, v, nu, ni, test


def _run_sgd(comm, cfg):
    from .models.mf_common import shuffle_coo
    from .models.sgd_mf import SGDConfig, row_owner, run_sgd

    u, i, v, nu, ni, test = _mf_data(comm, cfg)
    sc = SGDConfig(rank=cfg["rank"], lam=cfg["lam"], lr=cfg["epsilon"], epochs=cfg["iterations"],
                   train_fraction=min(1.0, max(cfg["train_ratio"], 1) / 100.0))
    u, i, v = shuffle_coo(comm, row_owner(u, comm.world_size, sc.seed), u, i, v.float())
    if test is not None:
        tu, ti, tv = test
        tm = row_owner(tu, comm.world_size, sc.seed) == comm.rank
        test = (tu[tm], ti[tm], tv[tm].float())
    res = run_sgd(comm, sc, nu, ni, (u.cpu(), i.cpu(), v.cpu()), test)
    if comm.rank == 0:
        _write(os.path.join(cfg["work_dir"], "evaluation"),
               "\n".join(f"iteration {e} train-rmse {a:.6f} test-rmse {b:.6f}" for e, a, b in res["rmse"]) + "\n")
    return res


def _run_ccd(comm, cfg):
    from .models.ccd import CCDConfig, train_ccd

    u, i, v, nu, ni, test = _mf_data(comm, cfg)
    res = train_ccd(comm, u, i, v, nu, ni, CCDConfig(rank=cfg["rank"], lam=cfg["lam"], iterations=cfg["iterations"],
                                                     mode=cfg.get("mode", "allgather"),
                                                     slices_per_rank=max(1, cfg["num_model_slices"]),
                                                     model_dir=cfg["work_dir"]), test=test)
    return {"history": res["history"]}


def _run_lda(comm, cfg):
    from .models.lda import LDAConfig, run_lda
    from .models.mf_common import shuffle_coo

    docs, words = [], []
    files = _my_files(comm, cfg["doc_dir"])
    n_local = 0
    for fn in files:
        with open(fn) as f:
            for ln in f:
                t = ln.split()
                if not t:
                    continue
                for w in t[1:]:
                    docs.append(n_local)
                    words.append(int(w))
                n_local += 1
    counts = comm.all_gather_ints([n_local])[:, 0].tolist()
    off = sum(counts[:comm.rank])
    doc = torch.tensor(docs, dtype=torch.long) + off
    word = torch.tensor(words, dtype=torch.long)
    vocab = cfg.get("vocab") or _allmax(comm, int(word.max()) + 1 if word.numel() else 0)
    n_docs = sum(counts)
    doc, word = shuffle_coo(comm, doc % comm.world_size, doc, word)
    # minBound / maxBound (LDAMPCollectiveMapper.java:98-118): a band below 100 % turns on the
    # timer-bounded steps, starting at the reference's 1 s step and retuned every iteration
    lo, hi = cfg["min_bound"], cfg["max_bound"]
    tune = (lo > 0 or hi > 0) and hi != 100
    lc = LDAConfig(num_topics=cfg["num_topics"], alpha=cfg["alpha"], beta=cfg["beta"], iterations=cfg["iterations"],
                   print_interval=max(1, cfg["iterations"]), time_budget_ms=1000.0 if tune else 0.0,
                   min_bound=lo if tune else 0, max_bound=hi if tune else 0)
    res = run_lda(comm, lc, n_docs, vocab, (doc.cpu(), word.cpu()))
    if comm.rank == 0:
        _write(os.path.join(cfg["work_dir"], "likelihood"), "\n".join(f"{i} {v}" for i, v in res["loglik"]) + "\n")
    return res


def _run_ldacvb(comm, cfg):
    """Variational LDA on term-count documents (contrib LdaMapCollective: input dir, HDFS
    metafile of ``<file> <first doc>`` lines, output dir, terms, topics, docs, maps,
    iterations, threads, mode). Writes ``likelihood`` (iteration, bound, seconds) and
    ``alpha`` to the output dir."""
    from .models.lda_vb import LDAVBConfig, train_lda_vb
    from .utils.datasets import load_term_count_docs

    meta = cfg["metafile"]
    if meta and not os.path.isabs(meta) and not os.path.exists(meta):
        meta = os.path.join(cfg["input_dir"], meta)
    meta_name = os.path.basename(meta) if meta else ""
    files = [f for f in _my_files(comm, cfg["input_dir"]) if os.path.basename(f) != meta_name]
    doc, word, cnt = load_term_count_docs(sorted(files), meta if meta and os.path.exists(meta) else None)
    docs, local = torch.unique(doc, return_inverse=True)
    vocab = cfg["num_terms"] or _allmax(comm, int(word.max()) + 1 if word.numel() else 0)
    # the reference's settings: alpha 1e-3 (LDAMapper.java:99-106), maximum-likelihood beta
    # (no smoothing), 29 gamma passes per document (Constants.MAX_GAMMA_ITERATIONS = 30);
    # --init uniform also starts from its uniform beta (which keeps every topic identical)
    vc = LDAVBConfig(num_topics=cfg["num_topics"], iterations=cfg["iterations"], strategy=cfg["strategy"],
                     alpha=cfg["alpha"], eta=cfg["eta"], gamma_iters=cfg["gamma_iters"], gamma_tol=0.0,
                     init=cfg["init"])
    res = train_lda_vb(comm, local, word, cnt, docs.numel(), vocab, vc)
    if comm.rank == 0:
        _write(os.path.join(cfg["output_dir"], "likelihood"),
               "".join(f"{h['iter']} {h['elbo']} {h['time_s']}\n" for h in res["history"]))
        _write(os.path.join(cfg["output_dir"], "alpha"), " ".join(f"{a:.9g}" for a in res["alpha"].tolist()) + "\n")
    return {"history": res["history"], "num_docs": int(docs.numel()), "vocab": vocab}


def load_mds_block(folder: str, prefix: str, ids_file: str):
    """Reference WDA-MDS row blocks: file ``<prefix><i>`` holds ``height x width``
    big-endian int16 distances (value / Short.MAX_VALUE); ``ids_file`` lines are
    ``fileIdx height width rowIdx rowOffset``."""
    import numpy as np

    blocks = []
    with open(ids_file) as f:
        for ln in f:
            t = ln.split()
            if len(t) >= 5:
                blocks.append(tuple(int(x) for x in t[:5]))
    out = []
    for fi, h, w, _, off in blocks:
        raw = np.fromfile(os.path.join(folder, f"{prefix}{fi}"), dtype=">i2", count=h * w)
        out.append((off, torch.from_numpy(raw.astype(np.float64).reshape(h, w) / 32767.0)))
    return out


def _run_mds(comm, cfg):
    from .models.mds import MDSConfig, wda_mds

    blocks = load_mds_block(cfg["input_folder"], cfg["input_prefix"], cfg["ids_file"])
    n = cfg["n"] or sum(b.shape[0] for _, b in blocks)
    # contiguous row blocks per worker (the reference assigns row files to mappers)
    a, b = comm.rank * n // comm.world_size, (comm.rank + 1) * n // comm.world_size
    rows = torch.zeros((b - a, n), dtype=torch.float64)
    for off, blk in blocks:
        lo, hi = max(a, off), min(b, off + blk.shape[0])
        if lo < hi:
            rows[lo - a:hi - a] = blk[lo - off:hi - off, :n]
    every = cfg["checkpoint_every"] or 0
    res = wda_mds(comm, rows, torch.ones_like(rows), a, n,
                  MDSConfig(d=cfg["d"], alpha=cfg["alpha"], threshold=cfg["threshold"], cg_iter=cfg["cg_iter"],
                            checkpoint_dir=os.path.join(cfg["work_dir"], "checkpoints") if every > 0 else "",
                            checkpoint_every=every))
    if comm.rank == 0 and cfg["work_dir"]:
        from .utils.model_io import write_mds_points

        labels = None
        if cfg["labels_file"]:  # "<id> <label>" lines (the reference's label file)
            lab = {}
            with open(cfg["labels_file"]) as f:
                for ln in f:
                    t = ln.split()
                    if len(t) >= 2:
                        lab[int(t[0])] = int(t[1])
            labels = [lab.get(i, 1) for i in range(n)]
        write_mds_points(os.path.join(cfg["work_dir"], "X"), res["X"], labels)
    return {"stress": res["stress"], "smacof_iters": res["smacof_iters"], "X": res["X"].cpu()}


def load_template(path: str):
    from .models.graph import Template

    with open(path) as f:
        tok = [ln.split() for ln in f if ln.strip()]
    k = int(tok[0][0])
    edges = [(int(a), int(b)) for a, b in tok[2:]]
    return Template(k, edges)


def load_adjacency_graph(files: Sequence[str]):
    """``v<TAB>n1,n2,...`` adjacency (daal_subgraph) or ``v n1 n2 ...`` lines -> undirected
    edge arrays (both directions) and the vertex count."""
    src, dst = [], []
    nmax = -1
    for fn in files:
        with open(fn) as f:
            for ln in f:
                t = ln.replace(",", " ").split()
                if not t:
                    continue
                v = int(t[0])
                nmax = max(nmax, v)
                for x in t[1:]:
                    x = int(x)
                    nmax = max(nmax, x)
                    if x != v:
                        src.append(v)
                        dst.append(x)
    s, d = torch.tensor(src, dtype=torch.long), torch.tensor(dst, dtype=torch.long)
    s, d = torch.cat([s, d]), torch.cat([d, s])
    key = torch.unique(s * (nmax + 1) + d)
    return key // (nmax + 1), key % (nmax + 1), nmax + 1


def _run_subgraph(comm, cfg):
    from .models.graph import count_subgraphs

    T = load_template(cfg["template"])
    s, d, n = load_adjacency_graph(_files(cfg["graph_dir"]))
    res = count_subgraphs(comm, T, s, d, n, iterations=cfg["iterations"], seed=cfg["seed"], strategy=cfg["strategy"])
    if comm.rank == 0:
        _write(os.path.join(cfg["out_dir"], "count"), f"{res['estimate']}\n")
    return res


def _run_pagerank(comm, cfg):
    from .models.graph import pagerank, parse_adjacency

    lines = []
    for fn in _my_files(comm, cfg["input_dir"]):
        with open(fn) as f:
            lines += f.readlines()
    s, d, nodes = parse_adjacency(lines)
    n = cfg["num_urls"] or _allmax(comm, int(max(s.max() if s.numel() else -1, d.max() if d.numel() else -1,
                                                 nodes.max() if nodes.numel() else -1)) + 1)
    pr = pagerank(comm, s, d, nodes, n, iterations=cfg["iterations"])
    return {"pagerank": pr.cpu()}


def _run_daal(comm, cfg):
    """DAAL-family apps on dense CSV input (last ``label_cols`` columns = labels where
    the algorithm is supervised); each worker loads its share of the files."""
    from .models import naive_bayes as NB
    from .models import regression as RG
    from .models import stats as ST
    from .utils.datasets import load_dense_csv

    import numpy as np

    files = _my_files(comm, cfg["input_dir"])
    A = torch.cat([load_dense_csv(f) for f in files]) if files else torch.zeros((0, 0), dtype=torch.float64)
    algo = cfg["algo"]
    lc = cfg["label_cols"]
    out: Dict[str, Any] = {}
    if algo in ("cov", "covariance"):
        out = ST.covariance(A, comm)
    elif algo in ("mom", "moments"):
        out = ST.low_order_moments(A, comm)
    elif algo == "pca":
        out = ST.pca(A, comm, cfg["method"] or "correlation")
    elif algo == "svd":
        out = ST.svd(A, comm)
    elif algo == "qr":
        out = ST.tsqr(A, comm)
    elif algo in ("linreg", "ridge"):
        out = RG.train_linear(A[:, :-lc], A[:, -lc:], comm, ridge=1.0 if algo == "ridge" else 0.0,
                              method=cfg["method"] or "normal")
    elif algo in ("naive", "nb"):
        y = A[:, -1].long()
        out = NB.train(A[:, :-1], y, cfg["k"] or _allmax(comm, int(y.max()) + 1), comm)
    elif algo == "kmeans":
        from .models.kmeans_csr import kmeans_init, kmeans_sparse

        C0 = kmeans_init(A, cfg["k"] or 10, comm, method=cfg["method"] or "first")
        out = kmeans_sparse(A, C0, cfg["iterations"], comm)
    else:
        raise ValueError(f"unknown daal algo {algo}")
    if comm.rank == 0:
        os.makedirs(cfg["work_dir"], exist_ok=True)
        for k, v in (out.items() if isinstance(out, dict) else []):
            if isinstance(v, torch.Tensor):
                np.savetxt(os.path.join(cfg["work_dir"], f"{algo}_{k}.csv"), v.detach().cpu().double().reshape(
                    v.shape[0] if v.dim() else 1, -1).numpy(), delimiter=",")
    return {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in out.items()} if isinstance(out, dict) else out


# ------------------------------------------------------------------ entry
def _target(comm, app, cfg):
    return run_app(comm, app, cfg)


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in SPECS:
        print(__doc__)
        return 2
    app = argv[0]
    cfg = parse(app, argv[1:])
    maps = int(cfg.get("maps", 1) or 1)
    if "WORLD_SIZE" in os.environ:
        from .runtime.launcher import init_distributed, shutdown

        comm = init_distributed(cfg["backend"])
        res = run_app(comm, app, cfg)
        rank = comm.rank
        shutdown()
    else:
        from .runtime.launcher import launch

        backend = cfg["backend"] or ("nccl" if torch.cuda.is_available() and maps <= torch.cuda.device_count()
                                     else "gloo")
        res = launch(_target, maps, args=(app, cfg), backend=backend, timeout=24 * 3600)[0]
        rank = 0
    if rank == 0:
        summary = {k: v for k, v in (res or {}).items() if not isinstance(v, torch.Tensor)}
        print(json.dumps({"app": app, "result": summary}, default=str))
    return 0


if __name__ == "__main__":
    sys.exit(main())
