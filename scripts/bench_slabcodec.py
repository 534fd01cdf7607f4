#!/usr/bin/env python3
"""Slab codec cost and payload size at the LDA bench's per-rank slab shape: a 1M-word x
1000-topic model of 1e8 Zipf-distributed tokens split into P*S = 16 slices (P = 8 ranks, 2
slices each): 62,500 words x 1024 padded topics per slab.
python scripts/bench_slabcodec.py [--words 1e6] [--tokens 1e8] [--topics 1000] [--slices 16]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--words", type=float, default=1e6)
    ap.add_argument("--tokens", type=float, default=1e8)
    ap.add_argument("--topics", type=int, default=1000)
    ap.add_argument("--slices", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch

    from harp_amd.ops import lda as L
    from harp_amd.ops.slabcodec import SlabCodec, capacity

    dev = torch.device("cuda")
    V, T, K = int(a.words), int(a.tokens), a.topics
    Kp = L.padded_topics(K)
    # Zipf word frequencies over a random word permutation (slices get a mix of ranks)
    g = torch.Generator(device=dev).manual_seed(0)
    p = 1.0 / torch.arange(1, V + 1, device=dev, dtype=torch.float64)
    p = p[torch.randperm(V, generator=g, device=dev)]
    vps = (V + a.slices - 1) // a.slices
    w = torch.multinomial(p[:vps].float() / p.sum().float(), T // a.slices, replacement=True, generator=g)
    z = torch.randint(0, K, (w.numel(),), generator=g, device=dev)
    slab = torch.zeros(vps * Kp, dtype=torch.int32, device=dev)
    slab.index_add_(0, w * Kp + z, torch.ones_like(w, dtype=torch.int32))
    slab = slab.view(vps, Kp)
    cap = capacity(slab.sum(1, dtype=torch.int64), Kp)
    c = SlabCodec(vps, Kp, cap, dev)
    buf, out = c.empty_payload(), torch.empty_like(slab)
    c.encode(slab, buf)
    c.decode(buf, out)
    torch.cuda.synchronize()
    assert torch.equal(out, slab)
    t = {}
    for name, fn in (("encode", lambda: c.encode(slab, buf)), ("decode", lambda: c.decode(buf, out))):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        e.synchronize()
        t[name] = s.elapsed_time(e) / a.reps
    nnz = int((slab != 0).sum())
    print(json.dumps({"rows": vps, "cols": Kp, "tokens_in_slab": int(w.numel()), "nnz": nnz, "cap": cap,
                      "dense_MB": c.dense_nbytes() / 1e6, "payload_MB": c.nbytes / 1e6,
                      "ratio": c.dense_nbytes() / c.nbytes, "encode_ms": round(t["encode"], 4),
                      "decode_ms": round(t["decode"], 4),
                      "xgmi_ms_dense_at_50GBps": c.dense_nbytes() / 50e9 * 1e3,
                      "xgmi_ms_payload_at_50GBps": c.nbytes / 50e9 * 1e3}), flush=True)


if __name__ == "__main__":
    main()
