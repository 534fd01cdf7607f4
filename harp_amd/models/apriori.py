"""Association rules by Apriori (DAAL ``association_rules``, batch).

Reference: ml/daal/.../daal_association (DAAL association_rules Batch with
``minSupport`` / ``minConfidence``; input = (transaction id, item id) pairs; results =
large item sets with their supports and rules ``X => Y`` with confidences).

MI355X design: transactions become a dense 0/1 incidence matrix T [n_trans, n_items]
(bf16 on the GPU: exact for 0/1 products, counts accumulate in fp32). Level-2 supports
for every pair at once are ONE GEMM T^T T on the matrix cores; level k > 2 candidates
(joined + pruned on the host, Apriori property) are counted in chunks as the row-sum of
the product of their gathered columns. A distributed run partitions transactions and
allreduces each level's support vector (one collective per level).
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..parallel.comm import Communicator
from .common import reduce_partials


def incidence(tids: torch.Tensor, items: torch.Tensor, n_items: int, device=None) -> torch.Tensor:
    """(transaction, item) pairs -> dense 0/1 matrix (transactions renumbered densely)."""
    dev = device or tids.device
    ut, t = torch.unique(tids, return_inverse=True)
    T = torch.zeros((ut.numel(), n_items), dtype=torch.float32, device=dev)
    T[t.to(dev), items.to(dev)] = 1.0
    return T


def _allsum(comm, v: torch.Tensor) -> torch.Tensor:
    if comm is None or comm.world_size == 1:
        return v.double()
    return reduce_partials(comm, {"v": v})["v"]


def apriori(T: torch.Tensor, min_support: float = 0.01, min_confidence: float = 0.6,
            comm: Optional[Communicator] = None, max_len: Optional[int] = None,
            chunk: int = 1 << 14) -> Dict[str, object]:
    """Returns large item sets {tuple(items): support fraction} and rules
    [(antecedent, consequent, confidence, support)] sorted like DAAL (by itemset size,
    then lexicographically)."""
    dev = T.device
    n_local = T.shape[0]
    n = float(_allsum(comm, torch.tensor([float(n_local)]))[0])
    need = min_support * n
    mm_dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32
    s1 = _allsum(comm, T.sum(0).double().cpu())
    large: Dict[Tuple[int, ...], float] = {}
    L1 = [i for i in range(T.shape[1]) if s1[i] >= need]
    for i in L1:
        large[(i,)] = float(s1[i])
    prev = [(i,) for i in L1]
    k = 2
    while prev and (max_len is None or k <= max_len):
        if k == 2:
            idx = torch.tensor(L1, device=dev)
            Tc = T[:, idx].to(mm_dtype)
            S = (Tc.t() @ Tc).float() if dev.type == "cuda" else Tc.t() @ Tc
            iu = torch.triu_indices(len(L1), len(L1), 1)
            sup = _allsum(comm, S[iu[0], iu[1]].double().cpu())
            cands = [(L1[a], L1[b]) for a, b in zip(iu[0].tolist(), iu[1].tolist())]
        else:
            prev_set = set(prev)
            cands = []
            for a, b in itertools.combinations(prev, 2):
                if a[:-1] == b[:-1]:
                    c = a + (b[-1],) if a[-1] < b[-1] else b + (a[-1],)
                    if all(sub in prev_set for sub in itertools.combinations(c, k - 1)):
                        cands.append(c)
            cands = sorted(set(cands))
            if not cands:
                break
            C = torch.tensor(cands, device=dev)
            parts = []
            for a in range(0, len(cands), chunk):
                G = T[:, C[a:a + chunk]]  # [n, c, k]
                parts.append(G.prod(2).sum(0).double())
            sup = _allsum(comm, torch.cat(parts).cpu())
        prev = []
        for c, s in zip(cands, sup.tolist()):
            if s >= need:
                large[tuple(c)] = s
                prev.append(tuple(c))
        prev.sort()
        k += 1
    sets = {c: s / n for c, s in sorted(large.items(), key=lambda kv: (len(kv[0]), kv[0]))}
    rules = []
    for c, s in sets.items():
        if len(c) < 2:
            continue
        for r in range(1, len(c)):
            for ante in itertools.combinations(c, r):
                cons = tuple(x for x in c if x not in ante)
                conf = s / sets[ante]
                if conf >= min_confidence:
                    rules.append((ante, cons, conf, s))
    return {"large_itemsets": sets, "rules": rules, "n_transactions": int(n)}
