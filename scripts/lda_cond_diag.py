"""Per-token conditional distribution of the LDA samplers vs the exact collapsed-Gibbs
conditional: N independent probe tokens, each alone in its word chunk and sharing an
identical doc / word state, so the histogram of their new topics estimates p(t | rest).
Prints a chi-square statistic per sampler (df ~ number of merged bins - 1)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from harp_amd.ops import lda as L


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


def run(K, N, sampler, waves, dev, alpha=0.1, beta=0.01):
    L_doc = 60
    tdoc, tword, tz, word_row, nk_v, z0, doc_topics = probe_state(K, N, L_doc, dev)
    Kp = L.padded_topics(K)
    V = N + L_doc
    vbeta = 1000 * beta
    ndk = torch.zeros((N, Kp), dtype=torch.int16 if dev.type == "cuda" else torch.int32, device=dev)
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
    return {"sampler": sampler, "waves": waves, "K": K, "chi2": round(chi2, 1), "df": int(big.sum()),
            "p_doc_topics": round(float(hist[doc_topics.unique()].sum() / N), 4),
            "exact_p_doc_topics": round(float(p[doc_topics.unique()].sum()), 4)}


if __name__ == "__main__":
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    N = 200000
    for K in (300, 2000):
        if K <= 1024:
            print(json.dumps(run(K, N, "dense", 0, dev)), flush=True)
        for w in (1, 8):
            print(json.dumps(run(K, N, "sparse", w, dev)), flush=True)
