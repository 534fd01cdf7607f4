"""LDA push-pull over sparse rows with TWO ranks on one GPU (gloo ranks stage their
all-to-alls through the host, parallel/comm.py): the fused-rows mode (the sampler reads
the pull payload and writes the push payload) against the decode / re-encode mode, in the
deterministic one-wave sampler: identical token topics on every rank, and the exact
count-rebuild invariant across ranks."""
import pytest
import torch

from harp_amd.runtime.launcher import launch

pytestmark = pytest.mark.gpu


def _worker(comm, fused, K=64):
    from harp_amd.models.lda import LDAConfig, LDAPushPullMapper, synthetic_corpus
    from harp_amd.parallel.comm import Communicator
    from harp_amd.runtime.mapper import KeyValReader

    dev = torch.device("cuda", 0)
    gcomm = Communicator(None, dev)
    toks = synthetic_corpus(2000, 3000, 20, 40, seed=5)
    cfg = LDAConfig(num_topics=K, alpha=0.1, beta=0.01, iterations=6, print_interval=3, block_words=256,
                    sparse_comm="on", local_server=False, seed=1, deterministic=True, fused_rows=fused)
    m = LDAPushPullMapper(gcomm, cfg, 2000, 3000, toks)
    m.run(KeyValReader([]))
    ok = m.check_counts()
    dense = int((m.slots[1] < 0).sum().item()) if m.result["fused_rows"] else 0
    return {"tz": m.tz.cpu(), "ok": ok, "fused": m.result["fused_rows"], "ll": [v for _, v in m.result["loglik"]],
            "dense_slots": dense}


# K = 50: K % 4 != 0, the padded row's tail topics must come from the dense pull slots too;
# K = 2000: the sparse doc-span sampler (K > 1024) with fused rows (sparse and dense slots)
@pytest.mark.parametrize("K", [64, 50, 2000])
def test_fused_rows_two_ranks_match_unfused(cuda, K):
    a = launch(_worker, 2, args=(True, K), timeout=300)
    b = launch(_worker, 2, args=(False, K), timeout=300)
    assert K > 1024 or any(r["dense_slots"] > 0 for r in a), "no dense pull slot exercised"
    for ra, rb in zip(a, b):
        assert ra["fused"] and not rb["fused"]
        assert ra["ok"] and rb["ok"]
        assert torch.equal(ra["tz"], rb["tz"])
        assert ra["ll"] == rb["ll"]
