"""LDA variational Bayes (contrib LDA-CVB): ELBO increases, recovers planted topics,
and the 2-worker allreduce and push/pull runs agree with the single-worker run."""
import torch

from harp_amd.models import lda_vb as V
from harp_amd.parallel.comm import Communicator
from harp_amd.runtime.launcher import launch


def _corpus(n_docs=60, vocab=40, K=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    docs, words, cnts = [], [], []
    for d in range(n_docs):
        t = d % K
        ws = torch.randint(t * 10, t * 10 + 10, (30,), generator=g)
        u, c = torch.unique(ws, return_counts=True)
        docs += [d] * u.numel()
        words += u.tolist()
        cnts += c.tolist()
    return torch.tensor(docs), torch.tensor(words), torch.tensor(cnts, dtype=torch.float64)


def test_lda_vb_single():
    d, w, c = _corpus()
    out = V.train_lda_vb(Communicator(), d, w, c, 60, 40, V.LDAVBConfig(num_topics=4, iterations=15))
    elbo = [h["elbo"] for h in out["history"]]
    assert elbo[-1] > elbo[0]
    # every planted topic's words concentrate in one learned topic
    B = out["log_beta"].exp()
    for t in range(4):
        mass = B[:, t * 10:(t + 1) * 10].sum(1)
        assert mass.max() > 0.9


def _job(comm, d, w, c, strategy):
    P, r = comm.world_size, comm.rank
    m = (d % P) == r
    cfg = V.LDAVBConfig(num_topics=4, iterations=5, strategy=strategy, block=8)
    out = V.train_lda_vb(comm, d[m] // P, w[m], c[m], int(m.sum() and (d[m] // P).max() + 1), 40, cfg)
    return out["gamma"], out["history"][-1]["elbo"]


def test_lda_vb_distributed_strategies_agree():
    d, w, c = _corpus()
    single = V.train_lda_vb(Communicator(), d, w, c, 60, 40, V.LDAVBConfig(num_topics=4, iterations=5, block=8))
    res_ar = launch(_job, 2, args=(d, w, c, "allreduce"), timeout=300)
    res_pp = launch(_job, 2, args=(d, w, c, "push_pull"), timeout=300)
    for r, (ga, ea) in enumerate(res_ar):
        gp, ep = res_pp[r]
        assert torch.allclose(ga, gp, atol=1e-9)
        assert abs(ea - single["history"][-1]["elbo"]) < 1e-6 * abs(ea)
        assert torch.allclose(ga, single["gamma"][r::2], atol=1e-8)
