"""LDA by variational Bayes (contrib LDA-CVB, "Mr. LDA" style).

Reference: contrib/src/main/java/edu/iu/lda/{LDAMapper.java, LDAMapperDyn.java,
TrainingTask.java}: per document, gamma_k = alpha_k + N_d / K, then iterate
phi_wk ∝ beta_kw exp(digamma(gamma_k)), gamma = alpha + sum_w n_w phi_w until
convergence; the per-word log-phi sufficient statistics are combined across workers
(LDAMapper: allreduce of the whole log-phi table with a log-sum-exp combiner :397;
LDAMapperDyn: push to word owners :380, normaliser allreduce :402, pull of the words a
worker needs :429); alpha is updated by Newton's method from the allreduced alpha
sufficient statistics (:429) and the likelihood is allreduced (:452).

MI355X design: the E-step runs for all local documents at once over the [nnz, K]
token-topic matrix (gather log-beta columns, add digamma(gamma) rows, row softmax,
scatter-add back into gamma) instead of a per-document thread task. Word-topic
statistics are accumulated by one scatter-add; the combine is ONE allreduce of the
dense [K, V] matrix ("allreduce") or a push of word-block partitions to their owners +
a pull of only the blocks this worker's documents touch ("push_pull", parameter-server
style — less traffic when each worker sees a small part of the vocabulary).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from ..core.combiner import ArrCombiner, Operation
from ..core.partition import Partitioner
from ..core.table import Table
from ..parallel import collectives as CL
from ..parallel.comm import Communicator
from .common import reduce_partials


@dataclass
class LDAVBConfig:
    num_topics: int = 10
    iterations: int = 20
    alpha: float = 0.1
    eta: float = 0.01           # symmetric Dirichlet smoothing of beta
    gamma_iters: int = 50
    gamma_tol: float = 1e-4
    update_alpha: bool = True
    strategy: str = "allreduce"  # or "push_pull"
    block: int = 256             # words per push/pull partition
    seed: int = 0
    init: str = "random"         # "uniform": the reference's start (every log beta 0.1, then
                                 # normalised: LDAMapper.java:113-130), which keeps the topics
                                 # symmetric for good


def _estep(doc, word, cnt, n_docs, log_beta, alpha, cfg):
    K = log_beta.shape[0]
    dev = log_beta.device
    Nd = torch.zeros(n_docs, dtype=log_beta.dtype, device=dev).index_add_(0, doc, cnt)
    gamma = alpha[None, :] + (Nd / K)[:, None]
    lb = log_beta[:, word].t()  # [nnz, K]
    # doc-sorted input (the loaders' order): per-doc sums as segment reductions instead of
    # index_add_ atomics that every term of a document sends to one gamma row
    lengths = torch.bincount(doc, minlength=n_docs) if n_docs and bool((doc[1:] >= doc[:-1]).all()) else None
    for _ in range(cfg.gamma_iters):
        lphi = lb + torch.digamma(gamma)[doc]
        phi = torch.softmax(lphi, 1)
        if lengths is not None:
            new = alpha[None, :] + torch.segment_reduce(cnt[:, None] * phi, "sum", lengths=lengths, axis=0, unsafe=True)
        else:
            new = alpha[None, :].expand(n_docs, K).clone()
            new.index_add_(0, doc, cnt[:, None] * phi)
        if cfg.gamma_tol > 0:  # (a fixed pass count needs no host round trip per pass)
            delta = (new - gamma).abs().max() if n_docs else torch.zeros((), device=dev)
            gamma = new
            if float(delta) < cfg.gamma_tol:
                break
        else:
            gamma = new
    lphi = lb + torch.digamma(gamma)[doc]
    logz = torch.logsumexp(lphi, 1)
    phi = torch.exp(lphi - logz[:, None])
    return gamma, phi, logz


def _elbo_terms(doc, cnt, gamma, logz, alpha, n_docs):
    """The variational bound of this worker's documents as (doc part, word part): the doc
    part from gamma, the word part sum_w n_w sum_k phi (log beta + E log theta - log phi) =
    n_w (logz_w - digamma(sum_k gamma_dk)), logz over log beta + digamma(gamma). At the gamma
    fixed point it equals the reference's per-document likelihood (LDAMapper.java:239-344,
    updatePhi :679-717: lnG(sum alpha) - sum lnG(alpha) + sum lnG(gamma) - lnG(sum gamma)
    + sum_w n_w sum_k phi (log beta - log phi))."""
    dsum = torch.digamma(gamma.sum(1, keepdim=True))
    lg = (torch.lgamma(alpha.sum()) - torch.lgamma(alpha).sum()) * n_docs
    lg = lg + ((alpha - gamma) * (torch.digamma(gamma) - dsum)).sum()
    lg = lg + (torch.lgamma(gamma).sum() - torch.lgamma(gamma.sum(1)).sum())
    lw = (cnt * (logz - dsum[:, 0][doc])).sum()
    return lg, lw


def _alpha_newton(alpha, ss, D, iters=20):
    """Newton update of the Dirichlet alpha from sum_d (digamma(gamma_dk) - digamma(sum gamma_d))."""
    a = alpha.clone()
    for _ in range(iters):
        g = D * (torch.digamma(a.sum()) - torch.digamma(a)) + ss
        h = -D * torch.polygamma(1, a)
        z = D * torch.polygamma(1, a.sum())
        c = (g / h).sum() / (1.0 / z + (1.0 / h).sum())
        step = (g - c) / h
        new = a - step
        if bool((new <= 0).any()):
            new = a * 0.5 + 1e-6
        if float((new - a).abs().max()) < 1e-8:
            a = new
            break
        a = new
    return a


def train_lda_vb(comm: Communicator, doc: torch.Tensor, word: torch.Tensor, cnt: torch.Tensor, n_docs_local: int,
                 vocab: int, cfg: LDAVBConfig) -> Dict[str, object]:
    """doc/word/cnt: this worker's sparse doc-term counts (local doc ids 0..n_docs_local-1)."""
    dev = comm.device
    dt = torch.float64
    K = cfg.num_topics
    doc, word, cnt = doc.to(dev), word.to(dev), cnt.to(dev, dt)
    g = torch.Generator().manual_seed(cfg.seed)
    if cfg.init == "uniform":
        beta = torch.ones((K, vocab), dtype=dt)
    else:
        beta = torch.rand((K, vocab), generator=g, dtype=dt) + 1.0
    log_beta = (beta / beta.sum(1, keepdim=True)).log().to(dev)
    alpha = torch.full((K,), cfg.alpha, dtype=dt, device=dev)
    D = float(reduce_partials(comm, {"d": torch.tensor([float(n_docs_local)])})["d"][0])
    hist: List[Dict[str, float]] = []
    blocks_needed = torch.unique(word // cfg.block).tolist()
    nb = math.ceil(vocab / cfg.block)
    for it in range(cfg.iterations):
        t0 = time.perf_counter()
        gamma, phi, logz = _estep(doc, word, cnt, n_docs_local, log_beta, alpha, cfg)
        S = torch.zeros((K, vocab), dtype=dt, device=dev)
        S.index_add_(1, word, (cnt[:, None] * phi).t())
        ss = (torch.digamma(gamma) - torch.digamma(gamma.sum(1, keepdim=True))).sum(0)
        lg, lw = _elbo_terms(doc, cnt, gamma, logz, alpha, n_docs_local)
        if cfg.strategy == "push_pull" and comm.world_size > 1:
            # normaliser = global row sums (allreduce of K values), statistics by push/pull
            red = reduce_partials(comm, {"ss": ss, "ll": (lg + lw).reshape(1), "norm": S.sum(1)})
            S = _push_pull(comm, S, blocks_needed, nb, cfg.block, vocab)
            norm = red["norm"].to(dev)
        else:
            red = reduce_partials(comm, {"S": S, "ss": ss, "ll": (lg + lw).reshape(1)})
            S = red["S"].to(dev)
            norm = S.sum(1)
        log_beta = (S + cfg.eta).log() - (norm + vocab * cfg.eta).log()[:, None]
        if cfg.update_alpha:
            alpha = _alpha_newton(alpha, red["ss"].to(dev), D)
        hist.append({"iter": it + 1, "elbo": float(red["ll"][0]), "time_s": time.perf_counter() - t0})
    return {"log_beta": log_beta, "alpha": alpha, "gamma": gamma, "history": hist}


def _push_pull(comm, S, blocks_needed, nb, blk, vocab):
    """Push local word-block statistics to their owners (combined there), then pull back
    the blocks this worker's documents use. Blocks nobody touches stay zero."""
    K = S.shape[0]
    local = Table(0, ArrCombiner(Operation.SUM))
    for b in blocks_needed:
        local.add(int(b), S[:, b * blk:min(vocab, (b + 1) * blk)].contiguous())
    glob = Table(1, ArrCombiner(Operation.SUM))
    if not CL.push(comm, local, glob, Partitioner(comm.world_size)):
        raise IOError("push failed")
    want = Table(2, ArrCombiner(Operation.SUM))
    for b in blocks_needed:
        want.add(int(b), torch.zeros_like(S[:, b * blk:min(vocab, (b + 1) * blk)]))
    if not CL.pull(comm, want, glob):
        raise IOError("pull failed")
    out = torch.zeros_like(S)
    for b in blocks_needed:
        out[:, b * blk:min(vocab, (b + 1) * blk)] = want[int(b)]
    return out
