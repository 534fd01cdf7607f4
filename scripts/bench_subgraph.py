#!/usr/bin/env python3
"""Subgraph-counting bench (BASELINE #7, SAHAD templates u3-1 / u5-1 / u7-1 = paths of 3 /
5 / 7 vertices): seconds per color-coding iteration on a synthetic skewed graph of the
Miami size (2.1M vertices, 51M undirected edges) by default.

python scripts/bench_subgraph.py [--nodes 2.1e6] [--edges 51e6] [--k 5] [--iters 2]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=float, default=2.1e6)
    ap.add_argument("--edges", type=float, default=51e6)
    ap.add_argument("--k", type=int, default=5, help="template u<k>-1: a path of k vertices")
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--strategy", default="allgather", choices=["allgather", "rotation"])
    a = ap.parse_args()
    import torch

    from harp_amd.models.graph import Template, count_subgraphs
    from harp_amd.runtime.launcher import init_distributed, shutdown

    comm = init_distributed()
    n, m = int(a.nodes), int(a.edges)
    g = torch.Generator(device=comm.device).manual_seed(7)
    u = (torch.rand(m, generator=g, device=comm.device) ** 2 * n).long().clamp_max(n - 1)  # skewed degrees
    v = torch.randint(0, n, (m,), generator=g, device=comm.device)
    # drop self loops without a boolean mask (nonzero breaks past 2^31 elements): move them
    v = torch.where(u == v, (v + 1) % n, v)
    src, dst = torch.cat([u, v]), torch.cat([v, u])
    del u, v
    T = Template(a.k, [(i, i + 1) for i in range(a.k - 1)])
    count_subgraphs(comm, T, src, dst, n, iterations=1, seed=1, strategy=a.strategy)  # warmup
    sync = torch.cuda.synchronize if comm.device.type == "cuda" else (lambda: None)
    sync()
    comm.barrier()
    t0 = time.perf_counter()
    res = count_subgraphs(comm, T, src, dst, n, iterations=a.iters, seed=2, strategy=a.strategy)
    sync()
    dt = (time.perf_counter() - t0) / a.iters
    if comm.rank == 0:
        print(json.dumps({"metric": f"subgraph counting s/coloring (u{a.k}-1 path template)", "value": dt,
                          "unit": "s/iter", "n_gpus": comm.world_size, "nodes": n, "edges": m,
                          "k": a.k, "estimate": res["estimate"], "strategy": a.strategy}), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
