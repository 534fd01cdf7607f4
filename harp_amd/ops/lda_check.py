"""Distribution-level checks of the GPU collapsed-Gibbs samplers (``csrc/lda.hip``) against
the collapsed-Gibbs conditional of the reference's sequential sampler
(ml/java/src/main/java/edu/iu/lda/LDAMPTask.java:85-330).

* :func:`run` -- per-token conditional: N independent probe tokens, each alone in its word
  chunk and sharing an identical doc / word state, so the histogram of their new topics
  estimates p(t | rest) (a chi-square per sampler; df ~ merged bins - 1).
* :func:`exact_sweep_check` -- the JOINT distribution of one whole sweep through the
  production instantiation of the dense sampler: packed uint8 doc rows at K = 1000
  (``lda_cgs_kernel<16, unsigned char, 1>``), word rows read from the pull payload and deltas
  written into the push payload of a real :class:`~harp_amd.parallel.sparse_ps.SparseRowPS`
  (sparse slots, sole-chunk count stores and reservation atomics), the longest-first chunk
  descriptors, and word chunks whose consecutive tokens share a document (the prefetched next
  doc row and its same-doc fixup) -- run by one wave walking the descriptors in order
  (``deterministic="lpt"``). R independent replicas of a 7-token micro-corpus give R samples
  of the sweep's final state; its exact distribution is enumerated (4^7 states, the product of
  the sequential conditionals along the kernel's token order), with the two documented model
  choices of the sampler: the topic totals are those of the sweep start (``inv_nk``) and a
  word chunk sees the pulled row plus its own moves (not another chunk's of the same word).

Run as a script for both on the GPU: ``python -m harp_amd.ops.lda_check``.
"""
from __future__ import annotations

import itertools
import json

import numpy as np
import torch

from . import lda as L


# --------------------------------------------------------------------------- probe tokens
def probe_state(K, N, L_doc, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    doc_topics = torch.randint(0, min(K, 40), (L_doc - 1,), generator=g)     # the doc's other tokens
    word_row = torch.zeros(K, dtype=torch.int32)
    word_row.index_add_(0, torch.randint(0, K, (200,), generator=g), torch.ones(200, dtype=torch.int32))
    z0 = int(doc_topics[0])
    nk = torch.randint(10 ** 7, 5 * 10 ** 7, (K,), generator=g).int()
    # tokens: per doc d: probe (word d, topic z0) then L_doc - 1 others (word N + j)
    tdoc = torch.arange(N).repeat_interleave(L_doc).int()
    tword = torch.cat([torch.tensor([0]), torch.arange(1, L_doc)]).repeat(N).int()
    tword[::L_doc] = torch.arange(N).int()
    tword[torch.arange(N * L_doc) % L_doc != 0] += N
    tz = torch.cat([torch.tensor([z0]), doc_topics]).repeat(N).int()
    return tdoc.to(dev), tword.to(dev), tz.to(dev), word_row, nk, z0, doc_topics


def exact(K, word_row, nk, z0, doc_topics, alpha, beta, vbeta):
    nd = torch.bincount(doc_topics, minlength=K).double()   # probe removed
    nw = word_row.double()                                  # probe not in word_row
    p = (nd + alpha) * (nw + beta) / (nk.double() + vbeta)
    return p / p.sum()


def run(K, N, sampler, waves, dev, alpha=0.1, beta=0.01, ndk_dtype=None):
    """Probe-token chi-square for ``sampler`` ("dense" / "sparse"); ``ndk_dtype`` overrides
    the dense sampler's doc-row storage (torch.uint8: the packed rows of the production
    path at K = 1000)."""
    L_doc = 60
    tdoc, tword, tz, word_row, nk_v, z0, doc_topics = probe_state(K, N, L_doc, dev)
    Kp = L.padded_topics(K)
    V = N + L_doc
    vbeta = 1000 * beta
    if ndk_dtype is None:
        ndk_dtype = torch.int16 if dev.type == "cuda" else torch.int32
    ndk = torch.zeros((N, Kp), dtype=ndk_dtype, device=dev)
    nwk = torch.zeros((V, Kp), dtype=torch.int32, device=dev)
    L.count(tdoc, tword, tz, ndk, nwk, None)
    nwk[:N, :K] += word_row.to(dev)[None, :]                 # probe words: row = word_row + probe
    nk = torch.zeros(Kp, dtype=torch.int32, device=dev)
    nk[:K] = nk_v.to(dev)
    probes = torch.arange(N, device=dev) * L_doc
    pd, pw, pz = tdoc[probes].contiguous(), tword[probes].contiguous(), tz[probes].contiguous()
    chunks = L.build_chunks(pw, 64)
    if sampler == "sparse":
        di = L.DocIndex.build(tdoc, tz, N)
        L.SPARSE_WAVES = waves
        L.cgs_sample(pd, pw, pz, chunks, ndk, nwk, nk, K, alpha, beta, vbeta, 77, di, di.tpos[probes].contiguous())
    else:
        L.cgs_sample(pd, pw, pz, chunks, ndk, nwk, nk, K, alpha, beta, vbeta, 77)
    torch.cuda.synchronize() if dev.type == "cuda" else None
    hist = torch.bincount(pz.long().cpu(), minlength=K).double()
    p = exact(K, word_row, nk_v, z0, doc_topics, alpha, beta, vbeta)
    e = p * N
    big = e >= 5
    obs = torch.cat([hist[big], hist[~big].sum()[None]])
    exp = torch.cat([e[big], e[~big].sum()[None]])
    chi2 = float(((obs - exp) ** 2 / exp.clamp_min(1e-9)).sum())
    return {"sampler": sampler, "waves": waves, "K": K, "ndk": str(ndk_dtype).replace("torch.", ""),
            "chi2": round(chi2, 1), "df": int(big.sum()),
            "p_doc_topics": round(float(hist[doc_topics.unique()].sum() / N), 4),
            "exact_p_doc_topics": round(float(p[doc_topics.unique()].sum()), 4)}


# --------------------------------------------------------------------------- one exact sweep
# micro-corpus of one replica (word-sorted tokens): word 0 in docs A, A, B; word 1 in docs
# A, B, B, B. Chunks of at most 3 tokens: word 0 is one (sole) chunk with two consecutive
# doc-A tokens; word 1 splits into [A, B, B] and [B].
ACTIVE = (5, 300, 301, 999)            # lanes 0, 18, 18, 62 of the 16-topics-per-lane rows
DOC_PAT = (0, 0, 1, 0, 1, 1, 1)
WORD_PAT = (0, 0, 0, 1, 1, 1, 1)
Z0_IDX = (0, 1, 3, 2, 0, 1, 3)         # initial topics (indices into ACTIVE)
CHUNK_OF = (0, 0, 0, 1, 1, 1, 2)
WORD_BG = ((3, 0, 7, 1), (0, 4, 1, 2))  # extra word-topic counts of the global table
NK_ACTIVE = (40, 25, 60, 33)           # topic totals (frozen for the sweep)
NK_IDLE = 2_000_000_000                # every other topic: p ~ alpha beta / 2e9, never drawn


def exact_sweep_distribution(order, alpha, beta, vbeta):
    """P(final state) of one sweep of the micro-corpus taking its tokens in ``order`` (local
    indices): the product of the sequential conditionals (each token drawn once, so the final
    state fixes the path). States are 7-digit base-4 numbers, token 0 most significant."""
    T, n = len(ACTIVE), len(DOC_PAT)
    states = np.array(list(itertools.product(range(T), repeat=n)), dtype=np.int64)
    S = states.shape[0]
    z0 = np.array(Z0_IDX)
    cur = np.tile(z0, (S, 1))
    eye = np.eye(T)
    # pulled word rows (sweep start): the word's tokens at their old topics + the background
    snap = np.array(WORD_BG, dtype=np.float64)
    for j in range(n):
        snap[WORD_PAT[j], z0[j]] += 1
    inv = 1.0 / (np.array(NK_ACTIVE, dtype=np.float64) + vbeta)
    logp = np.zeros(S)
    done = []
    for i in order:
        d, w, c = DOC_PAT[i], WORD_PAT[i], CHUNK_OF[i]
        nd = np.zeros((S, T))
        for j in range(n):
            if j != i and DOC_PAT[j] == d:
                nd += eye[cur[:, j]]
        nw = np.tile(snap[w], (S, 1)) - eye[z0[i]]
        for j in done:
            if CHUNK_OF[j] == c:
                nw += eye[cur[:, j]] - eye[z0[j]]
        p = (nd + alpha) * (nw + beta) * inv
        p /= p.sum(1, keepdims=True)
        logp += np.log(p[np.arange(S), states[:, i]])
        cur[:, i] = states[:, i]
        done.append(i)
    return np.exp(logp)


def _chi2(hist, prob):
    N = hist.sum()
    e = prob * N
    big = e >= 5
    obs = np.concatenate([hist[big], [hist[~big].sum()]])
    exp = np.concatenate([e[big], [e[~big].sum()]])
    chi2 = float(((obs - exp) ** 2 / np.maximum(exp, 1e-9)).sum())
    return chi2, int(big.sum())


def exact_sweep_check(dev, R: int = 100_000, seed: int = 1234, alpha: float = 0.3, beta: float = 0.05,
                      vbeta: float = 1.0) -> dict:
    """One sweep of R replicas through the production dense sampler (see the module
    docstring); returns the chi-square of the final states against the exact distribution
    per token order the descriptors produced, plus the exact-count checks."""
    from ..parallel.comm import Communicator
    from ..parallel.sparse_ps import SparseRowPS

    K, n = 1000, len(DOC_PAT)
    Kp = L.padded_topics(K)
    act = torch.tensor(ACTIVE)
    base = torch.arange(R) * 2
    tdoc = (base[:, None] + torch.tensor(DOC_PAT)).reshape(-1).int().to(dev)
    tword = (base[:, None] + torch.tensor(WORD_PAT)).reshape(-1).int().to(dev)
    tz = act[torch.tensor(Z0_IDX)].repeat(R).int().to(dev)
    z_init = tz.clone()
    ndk = torch.zeros((2 * R, Kp), dtype=torch.uint8, device=dev)
    L.count(tdoc, None, tz, ndk)
    glob = torch.zeros((2 * R, Kp), dtype=torch.int32, device=dev)
    L.count(None, tword, tz, None, glob)
    bg = torch.zeros((2, Kp), dtype=torch.int32)
    bg[:, act] = torch.tensor(WORD_BG, dtype=torch.int32)
    bg = bg.to(dev).repeat(R, 1)
    glob += bg
    nk = torch.full((Kp,), NK_IDLE, dtype=torch.int32, device=dev)
    nk[act.to(dev)] = torch.tensor(NK_ACTIVE, dtype=torch.int32, device=dev)
    ids = torch.arange(2 * R, dtype=torch.int64)
    toks = torch.bincount(tword.long().cpu(), minlength=2 * R) + 8  # slot bound: tokens + background
    ps = SparseRowPS(Communicator(None, dev), ids, toks, lambda x: torch.zeros_like(x), lambda x: x, Kp, device=dev)
    pbuf = ps.pull_payload(glob)
    slots = ps.row_slots()
    qbuf = ps.push_payload_buffer()
    chunks = L.build_chunks(tword, 3)
    delta = L.cgs_sample_ps(tdoc, tword, tz, chunks, ndk, nk, K, alpha, beta, vbeta, seed, pbuf, qbuf, slots,
                            ps.overflow, deterministic="lpt")
    desc = L.lpt_desc(chunks, tword, slots)
    ps.push_payload(glob)
    ps.check_overflow()
    torch.cuda.synchronize()
    out = {"replicas": R, "tokens": R * n}
    # exact counts: doc rows, global word rows (pushed deltas), topic delta
    rd = torch.zeros_like(ndk, dtype=torch.int32)
    L.count(tdoc, None, tz, rd)
    rw = torch.zeros_like(glob)
    L.count(None, tword, tz, None, rw)
    moved = torch.zeros(Kp, dtype=torch.int64, device=dev)
    moved.index_add_(0, tz.long(), torch.ones_like(tz, dtype=torch.int64))
    moved.index_add_(0, z_init.long(), -torch.ones_like(tz, dtype=torch.int64))
    out["counts_exact"] = bool(torch.equal(ndk.int(), rd) and torch.equal(glob, rw + bg)
                               and torch.equal(delta.long(), moved))
    out["moved_fraction"] = round(float((tz != z_init).float().mean()), 4)
    # token order per replica from the descriptor order (chunk starts 7 r, 7 r + 3, 7 r + 6)
    pos = torch.empty(desc.shape[0], dtype=torch.int64, device=dev)
    rank_of_start = torch.full((R * n,), -1, dtype=torch.int64, device=dev)
    rank_of_start[desc[:, 0]] = torch.arange(desc.shape[0], device=dev)
    r0 = torch.arange(R, device=dev) * n
    p0, p1, p2 = rank_of_start[r0], rank_of_start[r0 + 3], rank_of_start[r0 + 6]
    assert bool((p0 >= 0).all() and (p1 >= 0).all() and (p2 > torch.maximum(p0, p1)).all())
    w0_first = (p0 < p1).cpu().numpy()
    del pos
    # final states
    zf = tz.view(R, n).cpu()
    lut = torch.full((K + 64,), -1, dtype=torch.int64)
    lut[act] = torch.arange(len(ACTIVE))
    idx = lut[zf.long()]
    stray = int((idx < 0).any(1).sum())
    ok = (idx >= 0).all(1)
    code = (idx.clamp_min(0) * (4 ** torch.arange(n - 1, -1, -1))).sum(1).numpy()
    out["stray_draws"] = stray
    groups = []
    chi2_sum, df_sum = 0.0, 0
    for first, order in ((True, (0, 1, 2, 3, 4, 5, 6)), (False, (3, 4, 5, 0, 1, 2, 6))):
        m = (w0_first == first) & ok.numpy()
        if m.sum() == 0:
            continue
        prob = exact_sweep_distribution(order, alpha, beta, vbeta)
        hist = np.bincount(code[m], minlength=prob.size).astype(np.float64)
        c2, df = _chi2(hist, prob)
        chi2_sum += c2
        df_sum += df
        # per-token marginals too (|observed - exact| in standard errors, the worst token)
        states = np.array(list(itertools.product(range(4), repeat=n)))
        worst = 0.0
        for i in range(n):
            pm = np.bincount(states[:, i], weights=prob, minlength=4)
            om = np.bincount(idx[torch.from_numpy(m)][:, i].numpy(), minlength=4) / m.sum()
            se = np.sqrt(pm * (1 - pm) / m.sum())
            worst = max(worst, float(np.max(np.abs(om - pm) / np.maximum(se, 1e-12))))
        groups.append({"w0_chunk_first": first, "samples": int(m.sum()), "chi2": round(c2, 1), "df": df,
                       "worst_marginal_z": round(worst, 2)})
    out["groups"] = groups
    out["chi2"] = round(chi2_sum, 1)
    out["df"] = df_sum
    return out


if __name__ == "__main__":
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if dev.type == "cuda":
        print(json.dumps(exact_sweep_check(dev)), flush=True)
    N = 200000
    for K in (300, 1000, 2000):
        if K <= 1024:
            print(json.dumps(run(K, N, "dense", 0, dev)), flush=True)
            if dev.type == "cuda" and K > 512:
                print(json.dumps(run(K, N, "dense", 0, dev, ndk_dtype=torch.uint8)), flush=True)
        for w in (1, 8):
            print(json.dumps(run(K, N, "sparse", w, dev)), flush=True)


# --------------------------------------------------------------------------- likelihood spread
def loglik_spread(dev, K: int, seeds=(0, 1, 2, 3), iterations: int = 20) -> dict:
    """Per-token log-likelihood after ``iterations`` sweeps of the GPU sampler and of the
    exact sequential CPU sampler on the test corpus of tests/test_lda_gpu.py, for several
    sampler seeds: the run-to-run spread of each, and the GPU - CPU gap of the means, in
    nats per token (what the GPU-vs-CPU quality test bounds)."""
    from ..models.lda import LDAConfig, run_lda, synthetic_corpus
    from ..parallel.comm import Communicator

    toks = synthetic_corpus(2000, 3000, 20, 60, seed=4)
    n = toks[0].numel()
    out = {"K": K, "tokens": n}
    for name, d in (("gpu", dev), ("cpu", torch.device("cpu"))):
        vals = []
        for s in seeds:
            cfg = LDAConfig(num_topics=K, alpha=50.0 / K, beta=0.01, iterations=iterations,
                            print_interval=iterations, seed=s)
            vals.append(run_lda(Communicator(None, d), cfg, 2000, 3000, toks)["loglik"][-1][1] / n)
        out[name] = [round(v, 5) for v in vals]
        out[name + "_spread"] = round(max(vals) - min(vals), 5)
    out["gap_of_means"] = round(abs(sum(out["gpu"]) / len(seeds) - sum(out["cpu"]) / len(seeds)), 5)
    return out
