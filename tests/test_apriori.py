"""Apriori association rules vs a brute-force itemset enumeration, single worker and
2 gloo workers (transactions partitioned, supports allreduced)."""
import itertools
import random

import torch

from harp_amd.models import apriori as AP
from harp_amd.runtime.launcher import launch


def _transactions(n=300, items=12, seed=0):
    r = random.Random(seed)
    tids, its = [], []
    for t in range(n):
        basket = {i for i in range(items) if r.random() < 0.15}
        if r.random() < 0.4:
            basket |= {1, 3, 5}
        if r.random() < 0.3:
            basket |= {2, 7}
        for i in sorted(basket):
            tids.append(t)
            its.append(i)
    return torch.tensor(tids), torch.tensor(its)


def _brute(T, min_sup, min_conf):
    n = T.shape[0]
    rows = [set(torch.nonzero(T[i]).reshape(-1).tolist()) for i in range(n)]
    large = {}
    for k in range(1, T.shape[1] + 1):
        found = False
        for c in itertools.combinations(range(T.shape[1]), k):
            s = sum(1 for r in rows if set(c) <= r) / n
            if s >= min_sup:
                large[c] = s
                found = True
        if not found:
            break
    rules = set()
    for c, s in large.items():
        for r in range(1, len(c)):
            for a in itertools.combinations(c, r):
                if s / large[a] >= min_conf:
                    rules.add((a, tuple(x for x in c if x not in a)))
    return large, rules


def test_apriori_matches_brute_force():
    tids, its = _transactions()
    T = AP.incidence(tids, its, 12)
    out = AP.apriori(T, 0.1, 0.6)
    large, rules = _brute(T, 0.1, 0.6)
    assert set(out["large_itemsets"]) == set(large)
    for c, s in large.items():
        assert abs(out["large_itemsets"][c] - s) < 1e-12
    assert {(a, b) for a, b, _, _ in out["rules"]} == rules
    assert (1, 3, 5) in out["large_itemsets"]


def _job(comm, tids, its):
    m = (tids % comm.world_size) == comm.rank
    T = AP.incidence(tids[m], its[m], 12)
    return AP.apriori(T, 0.1, 0.6, comm=comm)


def test_apriori_distributed():
    tids, its = _transactions()
    single = AP.apriori(AP.incidence(tids, its, 12), 0.1, 0.6)
    for r in launch(_job, 2, args=(tids, its), timeout=300):
        assert r["large_itemsets"].keys() == single["large_itemsets"].keys()
        assert r["n_transactions"] == single["n_transactions"]
        assert [x[:2] for x in r["rules"]] == [x[:2] for x in single["rules"]]
