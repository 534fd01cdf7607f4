"""Fixed-layout sparse push / pull (parallel.sparse_ps + ops.rowcodec) on gloo ranks:
pulled rows equal the owners' rows, delta pushes add exactly the local changes, and LDA
push-pull over sparse rows leaves bit-identical counts to the dense block path."""
import pytest
import torch

from harp_amd.ops import rowcodec as RC
from harp_amd.runtime.launcher import launch

K = 64


def test_codec_roundtrip_cpu():
    g = torch.Generator().manual_seed(0)
    src = torch.zeros((50, K + 4), dtype=torch.int32)
    for r in range(50):
        nz = torch.randperm(K, generator=g)[: r % 50]
        src[r, nz] = torch.randint(-9, 9, (nz.numel(),), generator=g, dtype=torch.int32)
    bound = torch.tensor([r % 50 for r in range(50)])
    caps = RC.slot_caps(bound, K)
    assert (caps < 0).any() and (caps >= 0).any()  # both slot kinds exercised
    rows = torch.randperm(50, generator=g).to(torch.int32)
    off, nb = RC.layout(caps[rows.long()], K)
    buf = torch.zeros(nb, dtype=torch.uint8)
    ov = torch.zeros(1, dtype=torch.int32)
    RC.encode(src, K, rows, off, caps[rows.long()].to(torch.int32), buf, ov)
    assert int(ov) == 0
    dst = torch.full((50, K), 7, dtype=torch.int32)
    RC.decode(dst, K, rows, off, caps[rows.long()].to(torch.int32), buf)
    assert torch.equal(dst, src[:, :K])
    # delta against the decoded payload, then add back
    cur = src.clone()
    cur[3, :5] += 2
    cur[10, 7] -= 1
    dcaps = RC.slot_caps(torch.full((50,), 6), K)[rows.long()].to(torch.int32)
    doff, dnb = RC.layout(dcaps.long(), K)
    dbuf = torch.zeros(dnb, dtype=torch.uint8)
    RC.encode(cur, K, rows, doff, dcaps, dbuf, ov, buf, off, caps[rows.long()].to(torch.int32))
    acc = src[:, :K].clone()
    RC.decode(acc, K, rows, doff, dcaps, dbuf, add=True)
    assert torch.equal(acc, cur[:, :K]) and int(ov) == 0
    # overflow: a bound that is too small is flagged
    small = torch.zeros(50, dtype=torch.int32)
    soff, snb = RC.layout(small.long(), K)
    RC.encode(src, K, rows, soff, small, torch.zeros(max(snb, 16), dtype=torch.uint8), ov)
    assert int(ov) == 1


def _ps_worker(comm, owner_slots=False):
    from harp_amd.parallel.sparse_ps import SparseRowPS

    P, me = comm.world_size, comm.rank
    V, B = 300, 16
    g = torch.Generator().manual_seed(100 + me)
    want = torch.unique(torch.randint(0, V, (120,), generator=g))
    toks = torch.randint(1, 6, (want.numel(),), generator=g)
    nblocks = (V + B - 1) // B
    owned = list(range(me, nblocks, P))
    glob = torch.zeros((len(owned) * B, K), dtype=torch.int32)
    ps = SparseRowPS(comm, want, toks, lambda i: (i // B) % P, lambda i: (i // B) // P * B + i % B, K,
                     torch.device("cpu"))
    # initial push of random counts (bounded by the tokens), then pull back
    local = torch.zeros((want.numel(), K), dtype=torch.int32)
    for i in range(want.numel()):
        t = torch.randint(0, K, (int(toks[i]),), generator=g)
        local[i].index_add_(0, t, torch.ones_like(t, dtype=torch.int32))
    if owner_slots:
        ps.use_owner_slots()
        ps.push_initial(local)
    else:
        ps.push(local, glob, delta=False)
    pulled = torch.zeros_like(local)
    ps.pull(glob, pulled)
    # a "sweep": move some tokens between topics, push the delta
    cur = pulled.clone()
    for i in range(0, want.numel(), 3):
        nzt = torch.nonzero(local[i]).flatten()
        if nzt.numel():
            a = int(nzt[0])
            b = int(torch.randint(0, K, (1,), generator=g))
            cur[i, a] -= 1
            cur[i, b] += 1
    ps.push(cur, glob, delta=True)
    ps.check_overflow()
    if owner_slots:
        assert not glob.any()  # the owner table lives in the slots until asked for
        ps.owner_to_dense(glob)
    return {"want": want, "local": local, "pulled": pulled, "delta": cur - pulled, "glob": glob, "owned": owned,
            "bytes": ps.bytes_per_call(), "dedup": ps._dedup is not None}


@pytest.mark.parametrize("owner_slots", [False, True])
@pytest.mark.parametrize("P", [1, 2, 3])
def test_sparse_ps_push_pull(P, owner_slots):
    """Owner slots (the table held as canonical slots, pushes merged) give the same rows."""
    res = launch(_ps_worker, P, args=(owner_slots,), timeout=300)
    V, B = 300, 16
    tot0 = torch.zeros((V, K), dtype=torch.int32)
    dtot = torch.zeros((V, K), dtype=torch.int32)
    for r in res:
        tot0.index_add_(0, r["want"], r["local"])
        dtot.index_add_(0, r["want"], r["delta"])
    for r in res:
        assert torch.equal(r["pulled"], tot0[r["want"]])  # pull = the owners' summed rows
        assert r["dedup"] == (P > 1)  # rows wanted by several ranks: encoded once, slots copied
    final = tot0 + dtot
    for r in res:  # owners hold exactly the sum of initial counts and every delta
        for j, b in enumerate(r["owned"]):
            lo, hi = b * B, min(b * B + B, V)
            assert torch.equal(r["glob"][j * B:j * B + hi - lo], final[lo:hi])


def _lda_pp(comm, mode):
    from harp_amd.models.lda import LDAConfig, LDAPushPullMapper, synthetic_corpus
    from harp_amd.runtime.mapper import KeyValReader

    doc, word = synthetic_corpus(400, 700, 8, 30, seed=4)
    cfg = LDAConfig(num_topics=24, alpha=0.1, beta=0.01, iterations=3, print_interval=3, block_words=64,
                    sparse_comm=mode, local_server=False)
    m = LDAPushPullMapper(comm, cfg, 400, 700, (doc, word))
    m.run(KeyValReader([]))
    ids = m.glob.sorted_ids()
    return {"mode": m.comm_mode, "glob": torch.stack([m.glob[b] for b in ids]).cpu() if ids else None, "ids": ids,
            "nk": m.nk.cpu(), "tz": m.tz.cpu(), "loglik": m.result["loglik"]}


@pytest.mark.parametrize("P", [2, 3])
def test_lda_sparse_rows_bit_identical_to_dense(P):
    dense = launch(_lda_pp, P, args=("off",), timeout=600)
    sparse = launch(_lda_pp, P, args=("on",), timeout=600)
    for d, s in zip(dense, sparse):
        assert d["mode"] == "dense" and s["mode"] == "sparse"
        assert d["ids"] == s["ids"]
        assert torch.equal(d["tz"], s["tz"])
        assert torch.equal(d["nk"], s["nk"])
        if d["glob"] is not None:
            assert torch.equal(d["glob"], s["glob"])
        assert d["loglik"] == s["loglik"]


def test_merge_oracle_cpu():
    """rowcodec.merge (CPU oracle): canonical slot + several delta slots (repeated topics,
    sparse and dense) -> ascending topics without zeros; overflow and negative flags."""
    g = torch.Generator().manual_seed(3)
    n = 6
    base = torch.zeros((n, K), dtype=torch.int32)
    for r in range(n):
        t = torch.randint(0, K, (5 + 4 * r,), generator=g)
        base[r].index_add_(0, t, torch.ones_like(t, dtype=torch.int32))
    caps = RC.slot_caps(base.sum(1) + 8, K).to(torch.int32)
    off, nb = RC.layout(caps.long(), K)
    canon = torch.zeros(nb, dtype=torch.uint8)
    ov = torch.zeros(1, dtype=torch.int32)
    RC.encode(base, K, torch.arange(n, dtype=torch.int32), off, caps, canon, ov)
    # deltas: rows 0, 2, 2, 5 (row 2 twice), moves of counts between topics
    owners = [0, 2, 2, 5]
    delta = torch.zeros((len(owners), K), dtype=torch.int32)
    for j, r in enumerate(owners):
        src = int(torch.nonzero(base[r]).flatten()[j])  # distinct topics for the two row-2 deltas
        delta[j, src] -= 1
        delta[j, (src + 7 + j) % K] += 1
    dcap = RC.slot_caps(torch.full((len(owners),), 4), K).to(torch.int32)
    doff, dnb = RC.layout(dcap.long(), K)
    dbuf = torch.zeros(dnb, dtype=torch.uint8)
    RC.encode(delta, K, torch.arange(len(owners), dtype=torch.int32), doff, dcap, dbuf, ov)
    ptr = torch.tensor([0, 1, 1, 3, 3, 3, 4], dtype=torch.int32)
    idx = torch.tensor([0, 1, 2, 3], dtype=torch.int32)
    RC.merge(canon, off, caps, ptr, idx, dbuf, doff, dcap, K, ov)
    want = base.clone()
    want.index_add_(0, torch.tensor(owners), delta)
    got = torch.zeros_like(want)
    RC.decode(got, K, torch.arange(n, dtype=torch.int32), off, caps, canon)
    assert torch.equal(got, want) and int(ov) == 0
    neg = torch.zeros_like(delta[:1])
    neg[0, int(torch.nonzero(base[1] == 0)[0])] = -1
    RC.encode(neg, K, torch.zeros(1, dtype=torch.int32), doff[:1], dcap[:1], dbuf, ov)
    RC.merge(canon, off, caps, torch.tensor([0, 0, 1, 1, 1, 1, 1], dtype=torch.int32),
             torch.zeros(1, dtype=torch.int32), dbuf, doff, dcap, K, ov)
    assert int(ov) & 2


def test_reset_slots_cpu():
    """reset_slots empties every slot (nnz 0, dense rows zero) and leaves entry bytes alone."""
    caps = torch.tensor([3, -1, 0, 5], dtype=torch.int32)
    off, nb = RC.layout(caps.long(), K)
    buf = torch.full((nb,), 7, dtype=torch.uint8)
    RC.reset_slots(buf, off, caps, K)
    w32 = buf.view(torch.int32)
    for o, c in zip(off.tolist(), caps.tolist()):
        if c < 0:
            assert not w32[o // 4:o // 4 + K].any()
        else:
            assert int(w32[o // 4]) == 0 and (c == 0 or int(buf[o + 4]) == 7)
