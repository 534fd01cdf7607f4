"""PageRank iteration time on one GPU: the pull kernel (``csrc/graph.hip``) vs the
scatter formulation (fp64 ``index_add_`` over the edge list, the previous path).
Synthetic web-like graph (skewed in-degree), default 2e7 pages x 16 out-links."""
import argparse
import json
import sys
import time
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from harp_amd.models import graph as G
from harp_amd.parallel.comm import Communicator


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pages", type=float, default=5e6)
    ap.add_argument("--degree", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = int(a.pages)
    m = n * a.degree
    g = torch.Generator(device=dev).manual_seed(0)
    src = torch.randint(0, n - n // 20, (m,), device=dev, generator=g)
    dst = (torch.rand(m, device=dev, generator=g) ** 2 * n).long().clamp_max(n - 1)
    nodes = torch.arange(n, device=dev)
    comm = Communicator(device=dev)
    print("graph built", flush=True)
    G.pagerank(comm, src, dst, nodes, n, iterations=2)
    torch.cuda.synchronize()
    print("pull warm", flush=True)
    t0 = time.perf_counter()
    G.pagerank(comm, src, dst, nodes, n, iterations=1)
    torch.cuda.synchronize()
    t_setup1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    pr = G.pagerank(comm, src, dst, nodes, n, iterations=a.iters + 1)
    torch.cuda.synchronize()
    t_pull = (time.perf_counter() - t0 - t_setup1) / a.iters

    # scatter formulation (previous implementation)
    def scatter(iters):
        outdeg = torch.zeros(n, dtype=torch.float64, device=dev)
        outdeg.index_add_(0, src, torch.ones(m, dtype=torch.float64, device=dev))
        dang = outdeg == 0
        p = torch.full((n,), 1.0 / n, dtype=torch.float64, device=dev)
        for _ in range(iters):
            c = torch.zeros(n, dtype=torch.float64, device=dev)
            c.index_add_(0, dst, p[src] / outdeg[src])
            c += p[dang].sum() / n
            p = 0.85 * c + 0.15 / n
        return p
    print("pull timed %.4f s/iter" % t_pull, flush=True)
    scatter(1)
    torch.cuda.synchronize()
    print("scatter warm", flush=True)
    t0 = time.perf_counter()
    scatter(1)
    torch.cuda.synchronize()
    s1 = time.perf_counter() - t0
    t0 = time.perf_counter()
    ps = scatter(a.iters + 1)
    torch.cuda.synchronize()
    t_scatter = (time.perf_counter() - t0 - s1) / a.iters
    diff = float((pr - ps).abs().max())
    print(json.dumps({"metric": "PageRank s/iteration (pull kernel)", "value": t_pull, "unit": "s/iter",
                      "scatter_s_per_iter": t_scatter, "speedup": t_scatter / t_pull, "pages": n, "edges": m,
                      "edges_per_s": m / t_pull, "max_abs_diff_vs_scatter": diff, "n_gpus": 1}), flush=True)


if __name__ == "__main__":
    main()
