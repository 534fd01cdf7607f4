#!/usr/bin/env python3
"""LDA-CGS bench (BASELINE config #5: 1M docs x 1M vocab x 1000 topics): sampled
tokens/sec and seconds per iteration with word-slice model rotation. Strong scaling.

python scripts/bench_lda.py [--docs 1e6] [--vocab 1e6] [--topics 1000] [--len 100] [--iters 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=float, default=1e6)
    ap.add_argument("--vocab", type=float, default=1e6)
    ap.add_argument("--topics", type=int, default=1000)
    ap.add_argument("--len", type=int, default=100)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--max-chunk", type=int, default=0, help="tokens per word chunk (0: LDAConfig default)")
    ap.add_argument("--strategy", default="rotation", choices=["rotation", "push_pull"])
    ap.add_argument("--sparse-comm", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--fused-rows", default="on", choices=["on", "off"],
                    help="push_pull with sparse rows: the sampler reads pull slots / writes push slots")
    ap.add_argument("--slices", type=int, default=0, help="rotation: word slices per worker (0: LDAConfig default)")
    ap.add_argument("--local-server", default="on", choices=["on", "off"],
                    help="push_pull at P=1: off runs the pull / push collectives even on one rank")
    ap.add_argument("--owner-slots", default="on", choices=["on", "off"],
                    help="push_pull, fused rows: owner table held as canonical slots (merge on push)")
    a = ap.parse_args()
    import torch

    from harp_amd.models.lda import LDACollectiveMapper, LDAConfig, LDAPushPullMapper, synthetic_corpus
    from harp_amd.ops import lda as L
    from harp_amd.runtime.launcher import init_distributed, shutdown
    from harp_amd.runtime.mapper import KeyValReader

    comm = init_distributed()
    nd, V = int(a.docs), int(a.vocab)
    t0 = time.perf_counter()
    toks = synthetic_corpus(nd, V, 1000, a.len, seed=3, device=comm.device)
    gen = time.perf_counter() - t0
    cfg = LDAConfig(num_topics=a.topics, alpha=50.0 / a.topics, beta=0.01, iterations=a.warmup + a.iters,
                    sparse_comm=a.sparse_comm, local_server=a.local_server == "on", fused_rows=a.fused_rows == "on",
                    owner_slots=a.owner_slots == "on")
    if a.max_chunk:
        cfg.max_chunk = a.max_chunk
    if a.slices:
        cfg.num_slices = a.slices
    cls = LDAPushPullMapper if a.strategy == "push_pull" else LDACollectiveMapper
    m = cls(comm, cfg, nd, V, toks)
    del toks
    t0 = time.perf_counter()
    m.init_model(KeyValReader([]))
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    ll0 = m.log_likelihood(-1)
    for it in range(a.warmup):
        m.iterate(it)
    if hasattr(m, "rot"):
        m.rot.wait_all()
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    n = 0
    for it in range(a.warmup, a.warmup + a.iters):
        n += m.iterate(it)
    if hasattr(m, "rot"):
        m.rot.wait_all()
    torch.cuda.synchronize()
    comm.barrier()
    dt = time.perf_counter() - t0
    ll = m.log_likelihood(a.warmup + a.iters)
    extra = {"comm_mode": getattr(m, "comm_mode", "rotation"), "fused_rows": bool(getattr(m, "fused", False))}
    if getattr(m, "ps", None) is not None:  # sparse push/pull: codec + exchange time per call
        ps = m.ps
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        reps = 10
        fused = getattr(m, "fused", False)
        ev[0].record()
        for _ in range(reps):
            if fused:
                ps.pull_payload(m._glob_rows())
            else:
                ps.pull(m._glob_rows(), m.pull_buf)
        ev[1].record()
        for _ in range(reps):
            if fused:
                ps.push_payload_buffer()
                ps.push_payload(m._glob_rows())  # empty deltas
            else:
                ps.push(m.pull_buf, m._glob_rows())  # zero deltas: same payload work as a real push
        ev[2].record()
        ev[2].synchronize()
        pb, qb = ps.bytes_per_call(remote_only=False)
        extra.update({"pull_ms": ev[0].elapsed_time(ev[1]) / reps, "push_ms": ev[1].elapsed_time(ev[2]) / reps,
                      "pull_payload_bytes": pb, "push_payload_bytes": qb, "rows": ps.n_rows,
                      "dense_rows_bytes": ps.n_rows * m.Kp * 4})
        ps.check_overflow()
    tot = torch.tensor([float(n)], dtype=torch.float64, device=comm.device)
    if comm.world_size > 1:
        comm.all_reduce(tot)
    if comm.rank == 0:
        print(json.dumps({"peak_hbm_gb": torch.cuda.max_memory_allocated() / 2**30, "dense_doc_topic": m.ndk is not None,
                          "metric": f"LDA-CGS sampled tokens/sec ({a.strategy})", "value": float(tot.item()) / dt,
                          "unit": "tokens/s", "s_per_iter": dt / a.iters, "n_gpus": comm.world_size,
                          "docs": nd, "vocab": V, "topics": a.topics, "tokens": int(tot.item()) // a.iters,
                          "sampler": "sparse" if m.doc_index is not None else "dense",
                          "sparse_waves": L.SPARSE_WAVES, "max_chunk": L.max_chunk(cfg.max_chunk, m.sparse),
                          "chunk_order": os.environ.get("HARP_LDA_ORDER", "lpt"), "loglik_init": ll0, "loglik_end": ll, "init_s": init_s, "gen_s": gen, **extra}), flush=True)
    shutdown()


if __name__ == "__main__":
    main()
