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


def test_bound_is_the_reference_likelihood_at_the_gamma_fixed_point():
    """The per-iteration bound equals the reference's document likelihood (contrib
    LDAMapper.java:239-344: lnG(sum a) - sum lnG(a) + sum lnG(g) - lnG(sum g) + sum_w n_w
    sum_k phi (log beta - log phi)) once gamma has converged, and is a proper (negative)
    log-likelihood bound."""
    import torch

    g = torch.Generator().manual_seed(2)
    nd, V_, K = 30, 50, 4
    doc = torch.randint(0, nd, (400,), generator=g)
    word = torch.randint(0, V_, (400,), generator=g)
    cnt = torch.randint(1, 4, (400,), generator=g).double()
    beta = torch.rand((K, V_), generator=g, dtype=torch.float64) + 0.5
    log_beta = (beta / beta.sum(1, keepdim=True)).log()
    alpha = torch.full((K,), 0.3, dtype=torch.float64)
    cfg = V.LDAVBConfig(num_topics=K, gamma_iters=2000, gamma_tol=1e-14)
    gamma, phi, logz = V._estep(doc, word, cnt, nd, log_beta, alpha, cfg)
    lg, lw = V._elbo_terms(doc, cnt, gamma, logz, alpha, nd)
    ref = nd * (torch.lgamma(alpha.sum()) - torch.lgamma(alpha).sum())
    ref = ref + torch.lgamma(gamma).sum() - torch.lgamma(gamma.sum(1)).sum()
    ref = ref + (cnt[:, None] * phi * (log_beta[:, word].t() - phi.log())).sum()
    assert abs(float(lg + lw) - float(ref)) < 1e-9 * abs(float(ref))
    assert float(lg + lw) < 0
