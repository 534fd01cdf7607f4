"""PageRank (contrib simplepagerank) and color-coding subgraph counting (FASCIA /
SAHAD): single worker vs closed-form / brute force, P=2/3 gloo runs vs single worker
for both exchange strategies."""
import random

import pytest
import torch

from harp_amd.models import graph as G
from harp_amd.parallel.comm import Communicator
from harp_amd.runtime.launcher import launch


def _random_graph(n=60, m=200, seed=0, dangling=5):
    r = random.Random(seed)
    adj = {v: set() for v in range(n)}
    for _ in range(m):
        a, b = r.randrange(n), r.randrange(n)
        if a != b and a >= dangling:
            adj[a].add(b)
    return [" ".join(str(x) for x in [v] + sorted(adj[v])) for v in range(n)]


def _pr_reference(lines, n, iters, d=0.85):
    pr = torch.full((n,), 1.0 / n, dtype=torch.float64)
    out = {}
    for ln in lines:
        t = [int(x) for x in ln.split()]
        out[t[0]] = t[1:]
    for _ in range(iters):
        new = torch.zeros(n, dtype=torch.float64)
        for s, ts in out.items():
            if ts:
                for t in ts:
                    new[t] += pr[s] / len(ts)
            else:
                new += pr[s] / n
        pr = d * new + (1 - d) / n
    return pr


def test_pagerank_single():
    lines = _random_graph()
    s, d, nodes = G.parse_adjacency(lines)
    pr = G.pagerank(Communicator(), s, d, nodes, 60, iterations=15)
    ref = _pr_reference(lines, 60, 15)
    assert torch.allclose(pr, ref, atol=1e-14)
    assert abs(pr.sum().item() - 1.0) < 1e-12


def _pr_job(comm, lines):
    mine = lines[comm.rank::comm.world_size]
    s, d, nodes = G.parse_adjacency(mine)
    return G.pagerank(comm, s, d, nodes, 60, iterations=15)


def test_pagerank_distributed():
    lines = _random_graph()
    ref = _pr_reference(lines, 60, 15)
    for pr in launch(_pr_job, 3, args=(lines,), timeout=300):
        assert torch.allclose(pr, ref, atol=1e-14)


TEMPLATES = {
    "path3": (3, [(0, 1), (1, 2)]),
    "star4": (4, [(0, 1), (0, 2), (0, 3)]),
    "path5": (5, [(0, 1), (1, 2), (2, 3), (3, 4)]),
    "tree5": (5, [(0, 1), (0, 2), (2, 3), (2, 4)]),
}


def _undirected(n=14, m=30, seed=1):
    r = random.Random(seed)
    E = set()
    while len(E) < m:
        a, b = r.randrange(n), r.randrange(n)
        if a != b:
            E.add((min(a, b), max(a, b)))
    E = sorted(E)
    src = torch.tensor([a for a, b in E] + [b for a, b in E])
    dst = torch.tensor([b for a, b in E] + [a for a, b in E])
    return E, src, dst


@pytest.mark.parametrize("name", sorted(TEMPLATES))
def test_colorful_count_matches_brute_force(name):
    k, te = TEMPLATES[name]
    T = G.Template(k, te)
    E, src, dst = _undirected()
    colors = torch.randint(0, k, (14,), generator=torch.Generator().manual_seed(3))
    dp = G.color_count(Communicator(), T, src, dst, 14, colors)
    bf = G.brute_force_embeddings(T, E, 14, colors.tolist())
    assert dp == bf


def test_estimate_unbiased_on_average():
    k, te = TEMPLATES["path3"]
    T = G.Template(k, te)
    E, src, dst = _undirected()
    exact = G.brute_force_embeddings(T, E, 14) / T.automorphisms()
    est = G.count_subgraphs(Communicator(), T, src, dst, 14, iterations=300, seed=0)["estimate"]
    assert abs(est - exact) / exact < 0.1


def _sc_job(comm, k, te, src, dst, colors, strategy):
    return G.color_count(comm, G.Template(k, te), src, dst, 14, colors, strategy)


@pytest.mark.parametrize("strategy", ["allgather", "rotation"])
def test_color_count_distributed(strategy):
    k, te = TEMPLATES["tree5"]
    E, src, dst = _undirected()
    colors = torch.randint(0, k, (14,), generator=torch.Generator().manual_seed(4))
    ref = G.color_count(Communicator(), G.Template(k, te), src, dst, 14, colors)
    for r in launch(_sc_job, 3, args=(k, te, src, dst, colors, strategy), timeout=300):
        assert r == ref
