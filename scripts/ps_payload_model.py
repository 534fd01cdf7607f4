#!/usr/bin/env python3
"""Payload bytes of LDA push-pull at a P-rank shape, computed on the CPU without launching
ranks: the same slot layout as parallel.sparse_ps (pull caps min(K, global tokens of the
word), push caps min(K, 2 x rank tokens), dense slot when not smaller, 16-B alignment)
against the dense word-block path (every touched 4096-word block, both directions).

python scripts/ps_payload_model.py [--docs 1e6] [--vocab 1e6] [--topics 1000] [--ranks 8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=float, default=1e6)
    ap.add_argument("--vocab", type=float, default=1e6)
    ap.add_argument("--topics", type=int, default=1000)
    ap.add_argument("--len", type=int, default=100)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--block-words", type=int, default=4096)
    a = ap.parse_args()
    import torch

    from harp_amd.models.lda import synthetic_corpus
    from harp_amd.ops import lda as L
    from harp_amd.ops import rowcodec as RC

    nd, V, P, B = int(a.docs), int(a.vocab), a.ranks, a.block_words
    Kp = L.padded_topics(a.topics)
    doc, word = synthetic_corpus(nd, V, 1000, a.len, seed=3)
    glob_cnt = torch.bincount(word, minlength=V)
    recs = []
    for r in range(P):
        w = word[doc % P == r]
        ids, cnt = torch.unique(w, return_counts=True)
        own = (ids // B) % P
        remote = own != r
        pull = RC.slot_sizes(RC.slot_caps(glob_cnt[ids], Kp), Kp)
        push = RC.slot_sizes(RC.slot_caps(2 * cnt, Kp), Kp)
        blocks = torch.unique(ids // B)
        rblocks = int(((blocks % P) != r).sum())
        recs.append({"rank": r, "tokens": int(w.numel()), "touched_words": int(ids.numel()),
                     "sparse_remote_bytes": int(pull[remote].sum() + push[remote].sum()),
                     "dense_remote_bytes": 2 * rblocks * B * Kp * 4})
    sp = max(x["sparse_remote_bytes"] for x in recs)
    de = max(x["dense_remote_bytes"] for x in recs)
    print(json.dumps({"ranks": P, "docs": nd, "vocab": V, "topics": a.topics, "K_pad": Kp,
                      "max_rank_sparse_bytes_per_iter": sp, "max_rank_dense_bytes_per_iter": de,
                      "sparse_over_dense": round(sp / de, 4), "per_rank": recs}))


if __name__ == "__main__":
    main()
