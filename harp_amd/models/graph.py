"""Graph applications: PageRank and subgraph counting by color coding (FASCIA / SAHAD).

References:
  * contrib/src/main/java/edu/iu/simplepagerank/PageRankMapper.java:44-190 — adjacency
    lines ``src dst...`` loaded per worker; PR initialised to 1/N and allgathered; per
    iteration every worker adds PR(src)/outdeg to its targets (dangling pages spread
    PR/N to all pages) into a Long2Double KV table, the table is allreduced, and
    ``PR = 0.85 * sum + 0.15 / N``.
  * ml/java/.../subgraph/SCCollectiveMapper.java + colorcount_HJ.java (FASCIA color
    coding: random k-coloring, dynamic programming over a decomposition of the tree
    template into active / passive children, tables of counts per (vertex, color set);
    remote neighbour tables exchanged with regroup / allreduce) and
    ml/java/.../sahad/rotation*/SCCollectiveMapper.java (SAHAD: the passive-child tables
    rotate around the ring instead).

MI355X design:
  * PageRank: edges stay source-partitioned but are grouped by target once into a CSR,
    so a step is one gather SpMV (``csrc/graph.hip`` pagerank_pull_kernel: a power-of-two
    lane group per target row, no fp64 atomics; on one worker it also applies damping,
    the dangling mass and the next step's PR / outdeg in the same pass) into a dense
    length-N vector, then ONE reduce-scatter (each worker
    finalises its slice of pages) and ONE all-gather — half the bytes of the
    reference's allreduce of a KV table, and no hashing.
  * Color coding: count tables are dense [n_vertices, C(k, s)] fp64 matrices (color sets
    in combinatorial-number order); the neighbour sum of a passive table is a sparse x
    dense product, and the active x passive color-set convolution is a gather-multiply
    over a precomputed (C, C1, C \\ C1) index list followed by one scatter-add — all
    vectorised over vertices. Remote passive rows arrive by all-gather ("allgather",
    FASCIA-like) or by rotating row slabs around the ring with async p2p ("rotation",
    SAHAD-like) so the partial SpMM overlaps the next slab's transfer.
"""
from __future__ import annotations

import itertools
import math
import random
import time
from functools import lru_cache
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..parallel.comm import Communicator
from ..ops import graph as GO
from .common import gather_rows


# ---------------------------------------------------------------- input
def parse_adjacency(lines: Sequence[str]) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """``src dst dst ...`` lines -> (src, dst) edge arrays and the list of listed sources."""
    src, dst, nodes = [], [], []
    for ln in lines:
        tok = ln.split()
        if not tok:
            continue
        s = int(tok[0])
        nodes.append(s)
        for t in tok[1:]:
            src.append(s)
            dst.append(int(t))
    return torch.tensor(src, dtype=torch.long), torch.tensor(dst, dtype=torch.long), torch.tensor(nodes, dtype=torch.long)


def load_adjacency_dir(path: str, undirected: bool = True):
    """SAHAD / FASCIA graph files (datasets/daal_subgraph/graphs/*: ``vertex<TAB>n1,n2,...,``
    per line, any number of files) -> (src, dst, n_vertices). ``undirected``: both
    directions of every edge, self loops and duplicates removed (the subgraph counters
    treat the input as a simple undirected graph)."""

    import numpy as np

    from ..utils.datasets import list_files

    srcs, dsts = [], []
    for fn in list_files(path):
        with open(fn) as f:
            for ln in f:
                head, _, rest = ln.partition("\t")
                if not head.strip():
                    continue
                nb = np.array(rest.replace(",", " ").split(), dtype=np.int64)
                srcs.append(np.full(nb.size, int(head), dtype=np.int64))
                dsts.append(nb)
    s = np.concatenate(srcs) if srcs else np.zeros(0, dtype=np.int64)
    t = np.concatenate(dsts) if dsts else np.zeros(0, dtype=np.int64)
    n = int(max(s.max(initial=-1), t.max(initial=-1))) + 1
    if undirected:
        keep = s != t
        a, b = np.minimum(s[keep], t[keep]), np.maximum(s[keep], t[keep])
        key = np.unique(a * n + b)
        a, b = key // n, key % n
        s, t = np.concatenate([a, b]), np.concatenate([b, a])
    return torch.from_numpy(s), torch.from_numpy(t), n


# ---------------------------------------------------------------- PageRank
def pagerank(comm: Communicator, src: torch.Tensor, dst: torch.Tensor, nodes: torch.Tensor, num_urls: int,
             iterations: int = 10, damping: float = 0.85) -> torch.Tensor:
    """``nodes``: pages whose adjacency lists this worker loaded (every page appears in
    exactly one worker's list); (src, dst): their out-edges. Returns the full PR vector
    on every worker."""
    P, me, dev = comm.world_size, comm.rank, comm.device
    N = num_urls
    src, dst, nodes = src.to(dev).long(), dst.to(dev).long(), nodes.to(dev).long()
    chunk = math.ceil(N / P)
    Np = chunk * P
    # a page's out-edges all live on one worker, so the local out-degree is the global one
    outdeg = torch.bincount(src, minlength=N)[:N].to(torch.float64)
    invdeg = torch.where(outdeg > 0, 1.0 / outdeg.clamp_min(1.0), torch.zeros_like(outdeg))
    dvec = torch.zeros(N, dtype=torch.float64, device=dev)
    dvec[nodes[outdeg[nodes] == 0]] = 1.0  # this worker's dangling pages
    # edges grouped by target once: every iteration is a gather (no fp64 atomics)
    csr = GO.build_csr(dst, src, Np)
    pr = torch.full((N,), 1.0 / N, dtype=torch.float64, device=dev)
    x = pr * invdeg
    for _ in range(iterations):
        dm = torch.dot(pr, dvec).reshape(1)  # dangling mass, kept on the device
        if P == 1:
            pr, x = GO.pagerank_pull(csr, x, damping, (1 - damping) / N, damping / N, dm, invdeg, want_xnext=True)
            continue
        contrib, _ = GO.pagerank_pull(csr, x, 1.0, 0.0, 1.0 / N, dm)
        mine = torch.empty(chunk, dtype=torch.float64, device=dev)
        comm.reduce_scatter(mine, contrib)
        mine = damping * mine + (1 - damping) / N
        full = torch.empty(Np, dtype=torch.float64, device=dev)
        comm.all_gather_into(full, mine)
        pr = full[:N]
        x = pr * invdeg
    return pr


# ---------------------------------------------------------------- color coding
class Template:
    """A tree template (k vertices, edge list) rooted at vertex 0, decomposed into
    (vertex, number of children used) sub-templates."""

    def __init__(self, k: int, edges: Sequence[Tuple[int, int]]):
        self.k = k
        adj: Dict[int, List[int]] = {v: [] for v in range(k)}
        for a, b in edges:
            adj[a].append(b)
            adj[b].append(a)
        if len(edges) != k - 1:
            raise ValueError("template must be a tree")
        self.children: Dict[int, List[int]] = {}
        seen = {0}
        order = [0]
        for v in order:
            self.children[v] = [u for u in sorted(adj[v]) if u not in seen]
            seen.update(self.children[v])
            order += self.children[v]
        if len(seen) != k:
            raise ValueError("template must be connected")
        self.adj = adj

    def size(self, v: int, j: Optional[int] = None) -> int:
        ch = self.children[v] if j is None else self.children[v][:j]
        return 1 + sum(self.size(c) for c in ch)

    def automorphisms(self) -> int:
        """|Aut(T)| by brute force over vertex permutations (small templates)."""
        E = {frozenset(e) for e in self._edges()}
        cnt = 0
        for p in itertools.permutations(range(self.k)):
            if all(frozenset((p[a], p[b])) in E for a, b in self._edges()):
                cnt += 1
        return cnt

    def _edges(self):
        return [(v, c) for v in self.children for c in self.children[v]]


@lru_cache(maxsize=None)
def _colorsets(k: int, s: int):
    sets = list(itertools.combinations(range(k), s))
    return sets, {c: i for i, c in enumerate(sets)}


@lru_cache(maxsize=None)
def _split_index(k: int, sa: int, sp: int):
    """Index triples (C, C1, C2) with |C1| = sa, C2 = C \\ C1, |C| = sa + sp."""
    s = sa + sp
    sets, idx = _colorsets(k, s)
    _, ia = _colorsets(k, sa)
    _, ip = _colorsets(k, sp)
    tc, t1, t2 = [], [], []
    for ci, C in enumerate(sets):
        for C1 in itertools.combinations(C, sa):
            C2 = tuple(c for c in C if c not in C1)
            tc.append(ci)
            t1.append(ia[C1])
            t2.append(ip[C2])
    return torch.tensor(tc), torch.tensor(t1), torch.tensor(t2)


def _neighbour_sum(comm: Communicator, adj_src_local: torch.Tensor, adj_dst: torch.Tensor, n_local: int,
                   M_local: torch.Tensor, owner_rows: torch.Tensor, n_total: int, strategy: str) -> torch.Tensor:
    """N[v] = sum_{u in N(v)} M[u] for the local vertices v (local row ids in
    adj_src_local, global neighbour ids in adj_dst)."""
    P = comm.world_size
    out = torch.zeros((n_local, M_local.shape[1]), dtype=M_local.dtype, device=M_local.device)
    if P == 1:
        out.index_add_(0, adj_src_local, M_local[adj_dst])
        return out
    if strategy == "allgather":
        full = gather_rows(comm, M_local)  # rows in rank order: rank r owns vertices r, r+P, ...
        counts = [len(range(r, n_total, P)) for r in range(P)]
        offs = [0]
        for c in counts:
            offs.append(offs[-1] + c)
        owner = adj_dst % P
        row = torch.tensor(offs[:-1], device=adj_dst.device)[owner] + adj_dst // P
        out.index_add_(0, adj_src_local, full[row])
        return out
    # rotation (SAHAD): slabs of equal size travel the ring; each step adds the edges
    # whose neighbour lives in the resident slab
    from ..runtime.dymoro import DeviceRotator

    per = math.ceil(n_total / P)
    slab = torch.zeros((per, M_local.shape[1]), dtype=M_local.dtype, device=M_local.device)
    slab[:n_local] = M_local
    rot = DeviceRotator(comm, [slab], name="sc-rot")
    owner = adj_dst % P
    ring = [(r + 1) % P for r in range(P)]
    for s in range(P):
        cur = rot.get(0)
        src_rank = (comm.rank - s) % P
        m = owner == src_rank
        out.index_add_(0, adj_src_local[m], cur[adj_dst[m] // P])
        if s < P - 1:
            rot.start(0, ring)
    return out


class GraphShard:
    """One worker's share of the graph for the color-coding DP, built once per graph:
    owned vertices v % P == rank, their (local source, global neighbour) edges and, where
    the neighbour table is one contiguous array (P == 1, or the all-gather strategy), a
    CSR over it for the native fp64 SpMM (``ops/graph.py``)."""

    def __init__(self, comm: Communicator, src: torch.Tensor, dst: torch.Tensor, n_vertices: int,
                 strategy: str = "allgather"):
        from ..ops import graph as G

        P, me, dev = comm.world_size, comm.rank, comm.device
        self.own = torch.arange(me, n_vertices, P, device=dev)
        self.n_local = self.own.numel()
        src, dst = src.to(dev), dst.to(dev)
        if P == 1:  # every edge is local (no boolean mask: masks past 2^31 elements break nonzero)
            self.s_loc, self.d_glob = src, dst
        else:
            keep = (src % P) == me
            self.s_loc, self.d_glob = src[keep] // P, dst[keep]
        self.csr = None
        if P == 1 or strategy == "allgather":
            if P == 1:
                row = self.d_glob
            else:  # row of neighbour u in the all-gathered table (rank-major blocks)
                counts = [len(range(r, n_vertices, P)) for r in range(P)]
                offs = torch.tensor([0] + list(itertools.accumulate(counts))[:-1], device=dev)
                row = offs[self.d_glob % P] + self.d_glob // P
            self.csr = G.build_csr(self.s_loc, row, self.n_local)


def color_count(comm: Communicator, template: Template, src: torch.Tensor, dst: torch.Tensor, n_vertices: int,
                colors: torch.Tensor, strategy: str = "allgather", shard: Optional[GraphShard] = None) -> float:
    """Number of colorful embeddings (maps T -> G with all k colors distinct) for the
    given coloring. Each worker owns vertices v with v % P == rank and passes the edges
    (both directions) whose source it owns (or a prebuilt ``shard``)."""
    from ..ops import graph as G

    P, dev = comm.world_size, comm.device
    k = template.k
    if shard is None:
        shard = GraphShard(comm, src, dst, n_vertices, strategy)
    n_local = shard.n_local
    my_col = colors.to(dev)[shard.own]
    base = torch.zeros((n_local, k), dtype=torch.float64, device=dev)
    base[torch.arange(n_local, device=dev), my_col] = 1.0  # size-1 sets are {c} -> index c
    memo: Dict[Tuple[int, int], torch.Tensor] = {}

    def neighbour_sum(Pm: torch.Tensor) -> torch.Tensor:
        if shard.csr is not None:
            full = Pm if P == 1 else gather_rows(comm, Pm)
            return G.spmm(shard.csr, full.contiguous())
        return _neighbour_sum(comm, shard.s_loc, shard.d_glob, n_local, Pm, shard.own, n_vertices, strategy)

    def table(v: int, j: int) -> torch.Tensor:
        key = (v, j)
        if key in memo:
            return memo[key]
        if j == 0:
            memo[key] = base
            return base
        c = template.children[v][j - 1]
        A = table(v, j - 1)
        Pm = table(c, len(template.children[c]))
        sa, sp = template.size(v, j - 1), template.size(c)
        Np = neighbour_sum(Pm)
        tc, t1, t2 = _split_index(k, sa, sp)
        memo[key] = G.combine(A, Np, tc, t1, t2, len(_colorsets(k, sa + sp)[0]))
        return memo[key]

    full = table(0, len(template.children[0]))
    tot = full.sum().reshape(1)
    if P > 1:
        from .common import reduce_partials

        tot = reduce_partials(comm, {"t": tot})["t"]
    return float(tot[0])


def count_subgraphs(comm: Communicator, template: Template, src: torch.Tensor, dst: torch.Tensor, n_vertices: int,
                    iterations: int = 10, seed: int = 0, strategy: str = "allgather") -> Dict[str, float]:
    """Color-coding estimate of the number of (non-induced) copies of ``template``:
    mean colorful count * k^k / k! / |Aut(T)| over ``iterations`` random colorings
    (the same colorings on every worker)."""
    k = template.k
    g = torch.Generator().manual_seed(seed)
    scale = k ** k / math.factorial(k) / template.automorphisms()
    vals = []
    t0 = time.perf_counter()
    shard = GraphShard(comm, src, dst, n_vertices, strategy)
    for _ in range(iterations):
        colors = torch.randint(0, k, (n_vertices,), generator=g)
        vals.append(color_count(comm, template, src, dst, n_vertices, colors, strategy, shard) * scale)
    return {"estimate": sum(vals) / len(vals), "samples": vals, "time_s": time.perf_counter() - t0}


def brute_force_embeddings(template: Template, edges: Sequence[Tuple[int, int]], n: int,
                           colors: Optional[Sequence[int]] = None) -> int:
    """Exact count of (colorful, if colors given) injective homomorphisms T -> G."""
    adj = [set() for _ in range(n)]
    for a, b in edges:
        if a != b:
            adj[a].add(b)
            adj[b].add(a)
    order = [0]
    parent = {0: None}
    for v in order:
        for c in template.children[v]:
            parent[c] = v
            order.append(c)
    cnt = 0

    def rec(i, amap, used):
        nonlocal cnt
        if i == len(order):
            if colors is None or len({colors[x] for x in amap.values()}) == template.k:
                cnt += 1
            return
        t = order[i]
        cand = range(n) if parent[t] is None else adj[amap[parent[t]]]
        for x in cand:
            if x not in used:
                amap[t] = x
                used.add(x)
                rec(i + 1, amap, used)
                used.discard(x)
                del amap[t]

    rec(0, {}, set())
    return cnt
