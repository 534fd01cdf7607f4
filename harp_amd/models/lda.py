"""LDA collapsed Gibbs sampling with model rotation (Harp LDA-CGS).

Reference: ml/java/.../lda/LDAMPCollectiveMapper.java:183-378 — the word-topic model is
regrouped by word id into 2 slices per worker (LDAUtil.java:159-213), doc-topic counts
stay local, topic sums are allreduced per iteration (:424-461), the word slices rotate
(dymoro Rotator, ring order) while the SparseLDA sampler (LDAMPTask.java:85-330) runs on
the resident slice; log-likelihood every ``printInterval`` via allreduce (:699-745,
CalcLikelihoodTask.java:60-78 mallet Dirichlet terms).

MI355X design: tokens are bucketed once by word slice and word-sorted into chunks; each
resident-slice pass is one ``lda_cgs`` kernel (K <= 1024: wave per word chunk, register
word row, wave-scan sampler; larger K: the sparse-doc sampler, workgroup per word chunk
with the word row in LDS and the doc bucket read from a doc-order topic list); slices rotate on private RCCL channels (DeviceRotator) overlapping
the next slice's sampling; topic-sum deltas are allreduced once per iteration.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from ..ops import lda as L
from ..ops import rowcodec as RC
from ..runtime.dymoro import BudgetTuner, DeviceRotator, RotationSchedule, StepBudget, ring_strides
from ..runtime.mapper import CollectiveMapper, Context, KeyValReader
from ..ops.sorting import SORT_CHUNK, argsort_small_keys
from .common import reduce_partials


@dataclass
class LDAConfig:
    num_topics: int = 100
    alpha: float = 0.01
    beta: float = 0.01
    iterations: int = 10
    num_slices: int = 0       # word slices per worker; 0 = 1 on one worker (rotation: 37.4 -> 29.4 ms per
                              # full-size sweep, profiles/r5_lda_slices), else 2 (transfers overlap compute)
    print_interval: int = 5
    seed: int = 0
    max_chunk: int = 0        # tokens per word chunk; 0 = ops.lda.max_chunk's default (dense sampler:
                              # n_tokens / 3072 within [2048, 32768]; sparse sampler: 65536)
    block_words: int = 4096   # push/pull strategy: words per model partition
    sparse_comm: str = "auto"  # push/pull: "on" = fixed-layout sparse rows (parallel.sparse_ps, HIP codec),
                               # "off" = dense word blocks, "auto" = whichever the link/HBM model says is faster
    local_server: bool = True  # push-pull, one worker owning every touched block: sample in the table
    rotate_codec: str = "auto"  # rotation: "on" sends word-topic slabs as sparse payloads (ops/slabcodec),
                                # "auto" when that payload is at most half the dense slab, "off" dense
    checkpoint_dir: str = ""  # .hpt checkpoints (token topics, doc-topic, resident word slices)
    checkpoint_every: int = 0  # iterations between checkpoints (0: never)
    model_dir: str = ""       # word-model dumps every print_interval*10 iterations + at the end
    time_budget_ms: float = 0.0  # >0: time-bounded rotation steps (LDAMPCollectiveMapper timer); 0: full sweeps
    budget_pieces: int = 8    # launches a step's word chunks are cut into
    min_bound: int = 0        # with a budget: retune it every iteration so the trained percentage lands
    max_bound: int = 0        # in [min_bound, max_bound] (dymoro.BudgetTuner); 0 / 0: the budget stays fixed
    deterministic: bool = False  # GPU: one wave samples in order (bit-reproducible; tests / debugging only)
    owner_slots: bool = True  # fused rows: the owner holds its table as the canonical pull slots (merge on push)
    fused_rows: bool = True   # push-pull over sparse rows, GPU dense sampler: sample straight from the pull
                              # payload into the push payload (no dense local table, no decode / re-encode)


def synthetic_corpus(n_docs: int, vocab: int, true_topics: int, mean_len: int, seed: int = 0, device="cpu"):
    """Token arrays (doc, word) from a structured LDA-like generator: each true topic owns
    a random vocabulary subset with Zipf weights; docs mix 1-3 topics."""
    g = torch.Generator(device=device).manual_seed(seed)
    lens = torch.poisson(torch.full((n_docs,), float(mean_len), device=device), generator=g).long().clamp_min(1)
    doc = torch.repeat_interleave(torch.arange(n_docs, device=device), lens)
    n = doc.numel()
    dtop = torch.randint(0, true_topics, (n_docs, 3), generator=g, device=device)
    pick = torch.randint(0, 3, (n,), generator=g, device=device)
    topic = dtop[doc, pick]
    del pick  # (in-place steps below: a clueweb1-share corpus has 3.7e9 tokens)
    per = max(vocab // true_topics, 1)
    u = torch.rand(n, generator=g, device=device)
    idx = u.pow_(3).mul_(per).long().clamp_max_(per - 1)  # Zipf-like rank within the topic's words
    del u
    idx += topic.mul_(per)
    del topic
    idx.remainder_(vocab)
    perm = torch.randperm(vocab, generator=g, device=device)
    word = perm[idx]
    return doc, word


def _max_doc_len(doc: torch.Tensor, K: int, n_tokens: int) -> Optional[int]:
    """The corpus's longest document (global doc ids: the same on every worker), when it
    decides the sampler (ops.lda.use_sparse: K <= 1024 on a big corpus); else None."""
    if K > 1024 or n_tokens < L.SPARSE_MIN_TOKENS or doc.numel() == 0:
        return None
    return int(torch.bincount(doc).max())


class LDACollectiveMapper(CollectiveMapper):
    budget = None  # StepBudget when cfg.time_budget_ms > 0
    tuner = None   # BudgetTuner when a [min_bound, max_bound] band is set

    def __init__(self, comm=None, config: Optional[LDAConfig] = None, n_docs: int = 0, vocab: int = 0,
                 tokens=None, metrics=None):
        super().__init__(comm, metrics)
        self.cfg = config or LDAConfig()
        if self.cfg.num_slices <= 0:  # auto: one slice on one worker (nothing rotates to overlap), else two
            from dataclasses import replace

            self.cfg = replace(self.cfg, num_slices=1 if self.get_num_workers() == 1 else 2)
        self.n_docs, self.vocab = n_docs, vocab
        self._tokens = tokens
        self.loglik: List[Tuple[int, float]] = []
        self.iter_times: List[float] = []

    def init_model(self, reader: KeyValReader) -> None:
        cfg = self.cfg
        P, me, dev = self.get_num_workers(), self.get_self_id(), self.device
        S = cfg.num_slices
        ns = P * S
        K = cfg.num_topics
        self.Kp = L.padded_topics(K)
        doc, word = self._tokens
        # same choice on every worker, by the tokens ONE worker samples (the sparse sampler's
        # per-word setup does not pay at a few tokens per word: 8-GPU share, 12.5M tokens over
        # 1M words, dense 10.0 vs sparse 14.0 ms per sweep, profiles/r4_lda_share)
        self.sparse = L.use_sparse(K, doc.numel() // P, _max_doc_len(doc, K, doc.numel() // P))
        self._tokens = None  # the mapper keeps only its own token arrays (int32, word-sorted)
        if P > 1:
            mine = (doc % P) == me
            doc, word = doc[mine].to(dev), word[mine].to(dev)
            del mine
        else:
            doc, word = doc.to(dev), word.to(dev)
        self.ndoc_local = (self.n_docs - me + P - 1) // P
        ldoc = (doc // P).to(torch.int32)
        del doc
        # word -> (slice, row in slice): seeded permutation, equal slice sizes
        gperm = torch.Generator().manual_seed(cfg.seed + 99)
        perm = torch.randperm(self.vocab, generator=gperm)
        self.vps = math.ceil(self.vocab / ns)
        pos = torch.empty(self.vocab, dtype=torch.int32)
        pos[perm] = torch.arange(self.vocab, dtype=torch.int32)
        key = pos.to(dev)[word]  # = slice * vps + row in slice
        del word
        if key.numel() <= SORT_CHUNK:
            order = torch.argsort(key.long())
        else:  # an 8-GPU share of clueweb1 (3.7e9 tokens) is past torch's per-call sort limit
            order = argsort_small_keys(key, ns * self.vps)
        self.tdoc = ldoc[order].contiguous()
        del ldoc
        counts = torch.bincount(key // self.vps, minlength=ns).cpu()
        self.tword = (key[order] % self.vps).contiguous()
        del key, order
        self.offsets = [0] + torch.cumsum(counts, 0).tolist()
        self.chunks = []
        for s in range(ns):
            a, b = self.offsets[s], self.offsets[s + 1]
            self.chunks.append(L.build_chunks(self.tword[a:b], L.max_chunk(cfg.max_chunk, self.sparse, b - a)))
        gz = torch.Generator(device=dev if dev.type == "cuda" else "cpu").manual_seed(cfg.seed * 7 + me)
        self.tz = torch.randint(0, K, (self.tdoc.numel(),), generator=gz, device=dev, dtype=torch.int32)
        self.doc_index = L.DocIndex.build(self.tdoc, self.tz, self.ndoc_local) if self.sparse else None
        self.orders = [L.chunk_order(c) for c in self.chunks] if self.doc_index is not None else [None] * ns
        # counts: doc-topic local; word-topic global (allreduced once), then each worker keeps
        # the slices of its initial placement
        self.ndk = self._doc_topic_table()
        nwk_full = torch.zeros((ns * self.vps, self.Kp), dtype=torch.int32, device=dev)
        nk = torch.zeros(self.Kp, dtype=torch.int32, device=dev)
        for s in range(ns):
            a, b = self.offsets[s], self.offsets[s + 1]
            rows = (self.tword[a:b].long() + s * self.vps).to(torch.int32)
            L.count(self.tdoc[a:b], rows, self.tz[a:b], self.ndk, nwk_full, nk)
        red = reduce_partials(self.comm, {"nwk": nwk_full, "nk": nk}, dtype=torch.float64) if P > 1 else None
        if red is not None:
            nwk_full = red["nwk"].round().to(torch.int32)
            nk = red["nk"].round().to(torch.int32)
        self.nk = nk
        # slice k rotates on its own ring stride: the slices' transfers use different xGMI
        # links (dymoro.ring_strides); every schedule places block `me` here at step 0
        self.schedules = [RotationSchedule(P, None, stride=st) for st in ring_strides(P, S)]
        self.schedule = self.schedules[0]
        block = self.schedule.block_at(me, 0, 0)
        # (one worker: the slabs ARE the table, no copy -- 41 GB at clueweb1's K = 10,000)
        slabs = [nwk_full[(block * S + k) * self.vps:(block * S + k + 1) * self.vps] for k in range(S)]
        if P > 1:
            slabs = [t.clone() for t in slabs]
        self.codec = self._rotation_codec(nwk_full, ns) if P > 1 else None
        del nwk_full
        self.rot = DeviceRotator(self.comm, slabs, name="lda-w", metrics=self.metrics, codec=self.codec)
        self.vbeta = self.vocab * cfg.beta
        self.word_perm = perm  # slice s holds words perm[s*vps:(s+1)*vps]
        self._init_budget()

    def _doc_topic_table(self) -> Optional[torch.Tensor]:
        """Dense doc-topic counts, or None for the sparse sampler on the GPU: it samples from
        the doc-order topic lists (DocIndex) alone, and a dense table would cost ndocs x K_pad
        counts (20 KB per document at K = 10,000; the reference's SparseLDA keeps doc rows
        sparse too)."""
        if self.sparse and self.tz.device.type == "cuda" and L._lib.use_native(self.tz):
            return None
        maxlen = int(torch.bincount(self.tdoc, minlength=1).max()) if self.tdoc.numel() else 0
        return torch.zeros((self.ndoc_local, self.Kp), dtype=L.doc_topic_dtype(self.device, maxlen),
                           device=self.device)

    def _doc_loglik(self) -> torch.Tensor:
        K = self.cfg.num_topics
        if self.ndk is None:
            return L.doc_loglik_terms(self.doc_index, self.cfg.alpha, K)
        return L.loglik_terms(self.ndk, self.cfg.alpha, K)

    def _init_budget(self) -> None:
        cfg = self.cfg
        self.budget = StepBudget(cfg.time_budget_ms / 1e3, self.device) if cfg.time_budget_ms > 0 else None
        self._chunk_cursor, self._chunks_host = {}, {}
        self.tuner = BudgetTuner(cfg.min_bound, cfg.max_bound) if (
            self.budget is not None and (cfg.min_bound > 0 or cfg.max_bound > 0)) else None
        self.budget_history: List[float] = [self.budget.budget_s] if self.budget is not None else []
        if self.tuner is not None:  # the tuner's denominator: every worker's tokens
            t = torch.tensor([float(self.tdoc.numel())], dtype=torch.float64, device=self.device)
            if self.get_num_workers() > 1:
                self.comm.all_reduce(t)
            self.total_tokens = int(t.item())

    def _rotation_codec(self, nwk_full: torch.Tensor, ns: int):
        """Sparse slab payloads for the rotation when they pay. A word's token total (its
        row sum) never changes during sampling, so the payload bound computed here from
        the allreduced counts is the same on every worker and holds for the whole run."""
        from ..ops.slabcodec import SlabCodec, capacity

        mode = self.cfg.rotate_codec
        if mode == "off" or self.Kp > 65536:
            return None
        tokens = nwk_full.sum(1, dtype=torch.int64)
        cap = max(capacity(tokens[s * self.vps:(s + 1) * self.vps], self.Kp) for s in range(ns))
        codec = SlabCodec(self.vps, self.Kp, cap, self.device)
        if mode == "auto" and 2 * codec.nbytes > codec.dense_nbytes():
            return None
        return codec

    def iterate(self, it: int) -> int:
        cfg = self.cfg
        P, me, S = self.get_num_workers(), self.get_self_id(), cfg.num_slices
        delta_total = torch.zeros(self.Kp, dtype=torch.int32, device=self.device)
        n = 0
        c0 = self.budget.compute_s if self.budget is not None else 0.0
        for s in range(P):
            nk_view = self.nk + delta_total  # own updates are visible immediately
            for k in range(S):
                slab = self.rot.get(k)
                gs = self.schedules[k].block_at(me, it, s) * S + k
                a, b = self.offsets[gs], self.offsets[gs + 1]
                if b > a and cfg.time_budget_ms > 0:
                    m, delta_total = self._budget_step(gs, slab, delta_total, it, s, k)
                    nk_view = self.nk + delta_total
                    n += m
                elif b > a:
                    d = L.cgs_sample(self.tdoc[a:b], self.tword[a:b], self.tz[a:b], self.chunks[gs], self.ndk, slab,
                                     nk_view, cfg.num_topics, cfg.alpha, cfg.beta, self.vbeta,
                                     (cfg.seed << 40) ^ (it << 20) ^ (s << 8) ^ k, self.doc_index,
                                     self.doc_index.tpos[a:b] if self.doc_index is not None else None,
                                     self.orders[gs], deterministic=cfg.deterministic)
                    delta_total += d
                    nk_view = self.nk + delta_total
                    n += b - a
                self.rot.start(k, self.schedules[k].rotation_map(it, s))
        # topic sums: allreduce the iteration's deltas (LDAMPCollectiveMapper.java:439-461)
        if P > 1:
            with self.metrics.time_collective("allreduce", "lda", "topic-delta", self.Kp * 8, self.device):
                dt = reduce_partials(self.comm, {"d": delta_total}, dtype=torch.float64)["d"].round().to(torch.int32)
        else:
            dt = delta_total
        self.nk += dt
        if self.tuner is not None:  # LDAMPCollectiveMapper.java:295-314
            self.budget.budget_s = self.tuner(self, self.budget.budget_s, self.budget.compute_s - c0, n,
                                              self.total_tokens, P * S, it, "lda")
            self.budget_history.append(self.budget.budget_s)
        return n

    def _budget_step(self, gs: int, slab, delta_total, it: int, s: int, k: int):
        """Sample slice ``gs`` for at most the step budget, in pieces of consecutive word
        chunks; a per-slice chunk cursor makes the next visit continue where the budget
        cut this one (tokens not reached keep their topic for this iteration)."""
        cfg = self.cfg
        ch = self.chunks[gs]
        chh = self._chunks_host.get(gs)
        if chh is None:
            chh = self._chunks_host[gs] = ch.cpu().tolist()
        nch = len(chh) - 1
        NP = max(1, cfg.budget_pieces)
        a = self.offsets[gs]
        state = {"delta": delta_total, "j": 0}

        def piece():
            # piece q = chunks [q*nch/NP, (q+1)*nch/NP): an exact partition of the slice;
            # the next piece index persists per slice
            q = self._chunk_cursor.get(gs, 0)
            self._chunk_cursor[gs] = (q + 1) % NP
            c0, c1 = (q * nch) // NP, ((q + 1) * nch) // NP
            if c1 == c0:
                return 0
            t0, t1 = a + chh[c0], a + chh[c1]
            sub = ch[c0:c1 + 1] - chh[c0]
            tpos = self.doc_index.tpos[t0:t1] if self.doc_index is not None else None
            d = L.cgs_sample(self.tdoc[t0:t1], self.tword[t0:t1], self.tz[t0:t1], sub, self.ndk, slab,
                             self.nk + state["delta"], cfg.num_topics, cfg.alpha, cfg.beta, self.vbeta,
                             (cfg.seed << 40) ^ (it << 20) ^ (s << 8) ^ (k << 4) ^ state["j"], self.doc_index, tpos, deterministic=cfg.deterministic)
            state["delta"] = state["delta"] + d
            state["j"] += 1
            return t1 - t0

        n, _ = self.budget.run(piece for _ in range(max(1, cfg.budget_pieces)) if nch)
        return n, state["delta"]

    def log_likelihood(self, it: int) -> float:
        """Full joint log-likelihood (word + doc parts), each slice counted once: at step
        0 of the next iteration every slice is resident on exactly one worker."""
        cfg = self.cfg
        K = cfg.num_topics
        self.rot.wait_all()
        wp = torch.zeros(2, dtype=torch.float64, device=self.device)
        for k in range(cfg.num_slices):
            wp += L.loglik_terms(self.rot.slabs[k], cfg.beta, K)
        dp = self._doc_loglik()
        tot = reduce_partials(self.comm, {"w": wp[:1], "d": dp})
        nk = self.nk[:K].double()
        topic = (torch.lgamma(torch.tensor(self.vbeta, dtype=torch.float64)) - torch.lgamma(nk + self.vbeta)).sum()
        return float(tot["w"][0] + topic.cpu() + tot["d"].sum())

    def map_collective(self, reader: KeyValReader, context: Context) -> None:
        self.init_model(reader)
        start = self.start_iteration = self.resume()
        for it in range(start, self.cfg.iterations):
            self.metrics.begin_iteration()
            t0 = time.perf_counter()
            n = self.iterate(it)
            self.rot.wait_all()
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            self.iter_times.append(time.perf_counter() - t0)
            self.metrics.end_iteration("lda", it, tokens=n, iter_s=self.iter_times[-1], strategy="rotation")
            if self.cfg.print_interval and ((it + 1) % self.cfg.print_interval == 0 or it + 1 == self.cfg.iterations):
                self.loglik.append((it + 1, self.log_likelihood(it)))
            self._after_iteration(it)
        codec = getattr(self, "codec", None)
        self.result = {"loglik": self.loglik, "iter_s": self.iter_times, "start_iteration": start,
                       "rotate_payload_bytes": codec.nbytes if codec is not None else 0}

    # -- checkpoint / resume / model output --------------------------------------------------
    def _ckpt(self):
        from ..utils.checkpoint import Checkpointer

        return Checkpointer(self.cfg.checkpoint_dir, self.comm, self.cfg.checkpoint_every)

    def _after_iteration(self, it: int) -> None:
        cfg = self.cfg
        if getattr(self, "codec", None) is not None:
            self.codec.check_overflow()
        self.inject_fault(it)
        if self._ckpt().due(it):
            self.checkpoint(it)
        if cfg.model_dir and cfg.print_interval and ((it + 1) % (cfg.print_interval * 10) == 0
                                                     or it + 1 == cfg.iterations):
            self.print_word_model(f"{cfg.model_dir}/tmp_word_model/{it + 1}", it + 1)
            if it + 1 == cfg.iterations and self.is_master() and self.loglik:
                from ..utils.model_io import write_scalar

                write_scalar(f"{cfg.model_dir}/evaluation", self.loglik[-1][1])

    def _resident_words(self, it: int):
        """(k, real word ids) of the word slices resident on this rank when ``it`` starts."""
        S = self.cfg.num_slices
        block = self.schedule.block_at(self.get_self_id(), it, 0)
        out = []
        for k in range(S):
            lo = (block * S + k) * self.vps
            hi = min(lo + self.vps, self.vocab)
            out.append((k, self.word_perm[lo:hi] if hi > lo else self.word_perm[:0]))
        return out

    def _state_tables(self, it: int) -> dict:
        from ..utils.checkpoint import blob_table, tensor_table

        self.rot.wait_all()
        tabs = {"tz": blob_table(self.tz), "nk": blob_table(self.nk)}
        if self.ndk is not None:
            tabs["ndk"] = blob_table(self.ndk)
        for k, words in self._resident_words(it + 1):
            tabs[f"W{k}"] = tensor_table(self.rot.slabs[k][: words.numel()], words)
        return tabs

    def checkpoint(self, it: int) -> str:
        """After iteration ``it``: this rank's token topics z, doc-topic counts, topic sums
        and its resident word-topic slices (global word ids). Token order is a function of
        the input split, so resume needs the same world size."""
        return self._ckpt().save(it, self._state_tables(it), extra={"loglik": [list(x) for x in self.loglik]})

    def _restore_common(self, man, tabs) -> int:
        if man["world"] != self.get_num_workers():
            raise ValueError(f"LDA resume needs the checkpoint's world size {man['world']} "
                             f"(token topics are per-rank state), got {self.get_num_workers()}")
        self.tz.copy_(tabs["tz"][0].to(self.device))
        if self.ndk is not None:
            if "ndk" in tabs:
                self.ndk.copy_(tabs["ndk"][0].to(self.device))
            else:  # written by a run without the dense table: recount from the topics
                self.ndk.zero_()
                L.count(self.tdoc, None, self.tz, self.ndk)
        self.nk.copy_(tabs["nk"][0].to(self.device))
        if self.doc_index is not None:
            self.doc_index = L.DocIndex.build(self.tdoc, self.tz, self.ndoc_local)
        self.loglik = [tuple(x) for x in man["extra"].get("loglik", [])]
        return int(man["iteration"]) + 1

    def resume(self) -> int:
        got = self._ckpt().load_latest(device=self.device, rng=True)
        if got is None:
            return 0
        man, tabs = got
        it = self._restore_common(man, tabs)
        for k, words in self._resident_words(it):
            t = tabs[f"W{k}"]
            assert t.ids == words.tolist(), "resident word slice does not match the checkpoint"
            slab = self.rot.slabs[k]
            slab.zero_()
            slab[: words.numel()] = t.buffer.to(self.device)
        return it

    def print_word_model(self, folder: str, next_it: int) -> str:
        """Reference printWordTableMap: ``<folder>/<worker>`` with one line per word
        resident here when iteration ``next_it`` starts: ``wordID topic:count ...``."""
        from ..utils.model_io import write_topic_counts

        self.rot.wait_all()
        ids, rows = [], []
        for k, words in self._resident_words(next_it):
            ids.append(words)
            rows.append(self.rot.slabs[k][: words.numel()])
        return write_topic_counts(f"{folder}/{self.get_self_id()}", torch.cat(ids), torch.cat(rows),
                                  self.cfg.num_topics)


def run_lda(comm, cfg: LDAConfig, n_docs: int, vocab: int, tokens) -> dict:
    m = LDACollectiveMapper(comm, cfg, n_docs, vocab, tokens)
    m.run(KeyValReader([]))
    return m.result


class LDAPushPullMapper(LDACollectiveMapper):
    """LDA-CGS with the word-topic model as a parameter-server table (BASELINE config #5:
    "push-pull parameter server collective"; the pattern of contrib LDAMapperDyn.java:
    push :380 / pull :429, applied to the collapsed Gibbs sampler).

    The model is a distributed global packed table of word blocks (``block_words`` rows
    x K_pad int32 counts; owner = block id % P, the default Partitioner). Per iteration a
    worker pulls the blocks its tokens touch into one contiguous device slab, runs the
    ``lda_cgs`` kernel over all of its tokens against that snapshot (bulk-synchronous
    staleness, like the reference's stale topic sums), and pushes the count deltas back
    to the owners, where the SUM combiner merges them; topic-sum deltas are allreduced."""

    def init_model(self, reader: KeyValReader) -> None:
        from ..core.combiner import ArrCombiner, Operation
        from ..core.table import PackedTable

        cfg = self.cfg
        P, me, dev = self.get_num_workers(), self.get_self_id(), self.device
        K = cfg.num_topics
        self.Kp = L.padded_topics(K)
        B = self.B = int(getattr(cfg, "block_words", 0) or 4096)
        doc, word = self._tokens
        self._tokens = None
        # same choice on every worker, by the tokens ONE worker samples (the sparse sampler's
        # per-word setup does not pay at a few tokens per word: 8-GPU share, 12.5M tokens over
        # 1M words, dense 10.0 vs sparse 14.0 ms per sweep, profiles/r4_lda_share)
        self.sparse = L.use_sparse(K, doc.numel() // P, _max_doc_len(doc, K, doc.numel() // P))
        # narrow (uint16) owner table when no word has 65536 tokens (global counts: the same
        # decision on every worker): half the bytes of every pull encode
        self.narrow = (dev.type == "cuda" and cfg.sparse_comm != "off" and os.environ.get("HARP_LDA_NARROW", "1") != "0"
                       and word.numel() > 0 and RC.narrow_ok(int(torch.bincount(word).max())))
        mine = (doc % P) == me
        doc, word = doc[mine].to(dev), word[mine].to(dev)
        del mine
        self.ndoc_local = (self.n_docs - me + P - 1) // P
        ldoc = (doc // P).to(torch.int32)
        del doc
        blocks = torch.unique(word // B)
        self.need = blocks.cpu().tolist()
        nblocks = math.ceil(self.vocab / B)
        owned = list(range(me, nblocks, P))
        self.sum = ArrCombiner(Operation.SUM)
        # a single worker that owns every block its tokens touch, in the same order: its
        # server table IS the sampled slab, so pull (a copy), the before-snapshot, the delta
        # and push (an add back) are four full-model passes that leave the same counts;
        # the table aliases the slab and they are skipped (cfg.local_server=False keeps them)
        self.local_server = P == 1 and cfg.local_server and self.need == owned
        self.ps = None
        if not self.local_server:
            self.ps = self._sparse_plan(word)  # None: the dense block path is cheaper / unsupported
        if self.ps is not None:
            # sparse rows: the local table holds exactly the touched words, in id order
            lrow = torch.searchsorted(self.touched, word)
        else:
            lrow = torch.searchsorted(blocks, word // B) * B + word % B
        order = torch.argsort(lrow, stable=True)  # token order by word id in either layout
        self.tdoc = ldoc[order].contiguous()
        self.tword = lrow[order].to(torch.int32).contiguous()
        self.chunk_idx = L.build_chunks(self.tword, L.max_chunk(cfg.max_chunk, self.sparse, self.tword.numel()))
        gz = torch.Generator(device=dev if dev.type == "cuda" else "cpu").manual_seed(cfg.seed * 7 + me)
        self.tz = torch.randint(0, K, (self.tdoc.numel(),), generator=gz, device=dev, dtype=torch.int32)
        self.doc_index = L.DocIndex.build(self.tdoc, self.tz, self.ndoc_local) if self.sparse else None
        self.ndk = self._doc_topic_table()
        nrows = self.touched.numel() if self.ps is not None else len(self.need) * B
        slab = torch.zeros((nrows, self.Kp), dtype=torch.int32, device=dev)
        nk = torch.zeros(self.Kp, dtype=torch.int32, device=dev)
        L.count(self.tdoc, self.tword, self.tz, self.ndk, slab, nk)
        if P > 1:
            nk = reduce_partials(self.comm, {"nk": nk}, dtype=torch.float64)["nk"].round().to(torch.int32)
        self.nk = nk
        # distributed global table: owned word blocks, one packed [n_owned, B, K_pad] slab
        nneed = len(self.need)
        if self.ps is not None:
            self.pull_buf = slab
            gdt = torch.int16 if self.narrow and self.Kp % 8 == 0 else torch.int32
            gbuf = torch.zeros((len(owned), B, self.Kp), dtype=gdt, device=dev)
            self.glob = PackedTable(owned, gbuf, table_id=1, combiner=self.sum)
            self.glob.static_layout = True
            self.before = self.want_pt = None
            # fused rows: the dense sampler reads the pull payload and writes the push payload
            # itself, so the dense local table is only the initial-count source
            # (the sparse doc-span sampler too: the doc-order lists replace the doc table)
            self.fused = (cfg.fused_rows and dev.type == "cuda" and L._lib.use_native(self.tz)
                          and ((not self.sparse and K <= 1024)
                               or (self.sparse and self.ndk is None and L.SPAN and K <= L.MAX_TOPICS)))
            # fused rows + owner slots: the owner's table is held as the canonical slots the
            # pull sends, so a sweep has no pull encode and the push is a slot merge (the dense
            # table is filled only for the likelihood / checkpoints, _sync_glob)
            if self.fused and cfg.owner_slots:
                self.ps.use_owner_slots()
                self.ps.push_initial(self.pull_buf)
                self._glob_stale = True
            else:
                self.ps.push(self.pull_buf, self._glob_rows(), delta=False)  # initial counts into an empty model
            if self.fused:
                self.slots = self.ps.row_slots()
                self.pull_buf = None
        else:
            # one persistent buffer of the blocks this worker's tokens touch: pulled into,
            # sampled on in place, turned into the count delta and pushed back (cached plans)
            self.pull_buf = slab.view(nneed, B, self.Kp) if nneed else torch.zeros((0, B, self.Kp), dtype=torch.int32,
                                                                                  device=dev)
            gbuf = self.pull_buf if self.local_server else torch.zeros((len(owned), B, self.Kp), dtype=torch.int32,
                                                                       device=dev)
            self.glob = PackedTable(owned, gbuf, table_id=1, combiner=self.sum)
            self.before = None if self.local_server else torch.empty_like(self.pull_buf)
            self.want_pt = PackedTable(self.need, self.pull_buf, table_id=3, combiner=self.sum)
            for t in (self.glob, self.want_pt):
                t.static_layout = True
            if not self.local_server:
                self._push_delta()  # initial counts = a delta against an all-zero model
        self.vbeta = self.vocab * cfg.beta

    # link / HBM model for the auto choice: all-to-all bytes spread over min(P-1, 7) xGMI
    # links at a practical ~100 GB/s each; HBM passes at ~4 TB/s (read + write streams)
    A2A_LINK_BPS = 100e9
    HBM_BPS = 4e12

    def _sparse_plan(self, word: torch.Tensor):
        """Build the fixed-layout sparse push/pull plan (``parallel.sparse_ps``) unless
        ``sparse_comm`` is "off", K exceeds the codec's row limit, or (``auto``) the
        modelled time of the dense block path is lower. Collective; every rank decides
        from allreduced estimates, so all take the same path."""
        from ..ops.rowcodec import MAX_K
        from ..parallel.sparse_ps import SparseRowPS

        cfg = self.cfg
        mode = cfg.sparse_comm
        if mode not in ("on", "off", "auto"):
            raise ValueError(f"sparse_comm={mode!r}: expected on, off or auto")
        P, B, Kp = self.get_num_workers(), self.B, self.Kp
        if mode == "off" or Kp > MAX_K or Kp % 4:
            return None
        self.touched, tok = torch.unique(word, return_counts=True)
        ps = SparseRowPS(self.comm, self.touched, tok, lambda i: (i // B) % P, lambda i: (i // B) // P * B + i % B,
                         Kp, self.device)
        if mode == "on":
            return ps
        pull_b, push_b = ps.bytes_per_call(remote_only=True)
        row_b = Kp * 4
        nblk = len(self.need)
        dense_remote = 2 * nblk * B * row_b * (P - 1) / P
        links = max(1, min(P - 1, 7))
        t_dense = dense_remote / (self.A2A_LINK_BPS * links) + 7 * nblk * B * row_b / self.HBM_BPS
        t_sparse = (pull_b + push_b) / (self.A2A_LINK_BPS * links) + 3 * self.touched.numel() * row_b / self.HBM_BPS
        est = torch.tensor([t_dense - t_sparse], dtype=torch.float64, device=self.device)
        if P > 1:
            self.comm.all_reduce(est)
        self.comm_model = {"t_dense_s": t_dense, "t_sparse_s": t_sparse, "sparse_bytes": pull_b + push_b,
                           "dense_bytes": int(dense_remote)}
        return ps if float(est.item()) > 0 else None

    def _glob_rows(self) -> torch.Tensor:
        return self.glob.buffer.view(-1, self.Kp)

    def _sync_glob(self) -> None:
        """Dense owner table from the owner slots (owner-slot mode keeps it stale while sampling)."""
        if self.ps is not None and self.ps.owner_slots and getattr(self, "_glob_stale", False):
            self.ps.owner_to_dense(self._glob_rows())
            self._glob_stale = False

    @property
    def comm_mode(self) -> str:
        return "local" if self.local_server else ("sparse" if self.ps is not None else "dense")

    def _push_delta(self) -> None:
        if not self.push("lda", "push-model", self.want_pt, self.glob, None):
            raise IOError("push failed")

    def _pull(self) -> torch.Tensor:
        # every needed block has an owner, so the overwrite pull rewrites all of them
        if not self.pull("lda", "pull-model", self.want_pt, self.glob, True, overwrite=True):
            raise IOError("pull failed")
        return self.pull_buf.view(-1, self.Kp)

    def _timed_ps(self, kind: str, fn, nbytes: int) -> None:
        with self.metrics.time_collective(kind, "lda", f"{kind}-model", nbytes if self.get_num_workers() > 1 else 0,
                                          self.device):
            fn()

    def iterate(self, it: int) -> int:
        cfg = self.cfg
        seed = (cfg.seed << 40) ^ (it << 20) ^ 0x5A
        if self.local_server:
            n = self.tz.numel()
            if n:
                d = L.cgs_sample(self.tdoc, self.tword, self.tz, self.chunk_idx, self.ndk, self.pull_buf.view(-1, self.Kp),
                                 self.nk, cfg.num_topics, cfg.alpha, cfg.beta, self.vbeta, seed, self.doc_index, deterministic=cfg.deterministic)
                self.nk += d
            return n
        if self.ps is not None and getattr(self, "fused", False):
            pull_b, push_b = self.ps.bytes_per_call(remote_only=True)
            self._timed_ps("pull", lambda: self.ps.pull_payload(self._glob_rows()), pull_b)
            pbuf, qbuf = self.ps.pull_recv.buf, self.ps.push_payload_buffer()
            n = self.tz.numel()
            d = (L.cgs_sample_ps(self.tdoc, self.tword, self.tz, self.chunk_idx, self.ndk, self.nk, cfg.num_topics,
                                 cfg.alpha, cfg.beta, self.vbeta, seed, pbuf, qbuf, self.slots, self.ps.overflow,
                                 deterministic=cfg.deterministic, doc_index=self.doc_index)
                 if n else torch.zeros(self.Kp, dtype=torch.int32, device=self.device))
            self._timed_ps("push", lambda: self.ps.push_payload(self._glob_rows()), push_b)
            self._glob_stale = True
            if self.get_num_workers() > 1:
                with self.metrics.time_collective("allreduce", "lda", "topic-delta", self.Kp * 8, self.device):
                    d = reduce_partials(self.comm, {"d": d}, dtype=torch.float64)["d"].round().to(torch.int32)
            self.nk += d
            return n
        if self.ps is not None:
            pull_b, push_b = self.ps.bytes_per_call(remote_only=True)
            self._timed_ps("pull", lambda: self.ps.pull(self._glob_rows(), self.pull_buf), pull_b)
            slab = self.pull_buf
        else:
            slab = self._pull()
            self.before.copy_(self.pull_buf)
        n = self.tz.numel()
        if n:
            d = L.cgs_sample(self.tdoc, self.tword, self.tz, self.chunk_idx, self.ndk, slab, self.nk,
                             cfg.num_topics, cfg.alpha, cfg.beta, self.vbeta, seed, self.doc_index, deterministic=cfg.deterministic)
        else:
            d = torch.zeros(self.Kp, dtype=torch.int32, device=self.device)
        if self.ps is not None:
            self._timed_ps("push", lambda: self.ps.push(self.pull_buf, self._glob_rows()), push_b)
        else:
            slab -= self.before.view(-1, self.Kp)
            self._push_delta()
        if self.get_num_workers() > 1:
            with self.metrics.time_collective("allreduce", "lda", "topic-delta", self.Kp * 8, self.device):
                d = reduce_partials(self.comm, {"d": d}, dtype=torch.float64)["d"].round().to(torch.int32)
        self.nk += d
        return n

    def _after_iteration(self, it: int) -> None:
        if self.ps is not None:
            self.ps.check_overflow()
        super()._after_iteration(it)

    def token_words(self) -> torch.Tensor:
        """Global word id of each (sorted) local token, from its row in the local layout."""
        if self.ps is not None:
            return self.touched.to(self.device)[self.tword.long()]
        need = torch.tensor(self.need, dtype=torch.int64, device=self.device)
        r = self.tword.long()
        return need[r // self.B] * self.B + r % self.B

    def check_counts(self) -> bool:
        """Exact invariant (test / debug; dense [vocab, K_pad] scratch): the word-topic
        counts rebuilt from every worker's (word, z) equal the server table at each owner,
        and the topic sums equal their column sums. Collective; same answer on all ranks."""
        self._sync_glob()
        Kp, B, P = self.Kp, self.B, self.get_num_workers()
        nblocks = math.ceil(self.vocab / B)
        flat = self.token_words() * Kp + self.tz.long()
        rebuilt = torch.bincount(flat, minlength=nblocks * B * Kp).view(nblocks, B, Kp).to(torch.float64)
        if P > 1:
            self.comm.all_reduce(rebuilt)
        ok = bool(torch.equal(rebuilt.sum((0, 1)).round().to(torch.int32), self.nk))
        for b in self.glob.sorted_ids():
            ok = ok and bool(torch.equal(rebuilt[b].round().to(torch.int32), RC.widen(self.glob[b])))
        flag = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=self.device)
        if P > 1:
            self.comm.all_reduce(flag)
        return float(flag.item()) == 0.0

    def log_likelihood(self, it: int) -> float:
        cfg = self.cfg
        K = cfg.num_topics
        wp = torch.zeros(2, dtype=torch.float64, device=self.device)
        self._sync_glob()
        for p in self.glob.get_partitions():  # each block counted once, at its owner
            wp += L.loglik_terms(RC.widen(p.get()), cfg.beta, K)
        dp = self._doc_loglik()
        tot = reduce_partials(self.comm, {"w": wp[:1], "d": dp})
        nk = self.nk[:K].double()
        topic = (torch.lgamma(torch.tensor(self.vbeta, dtype=torch.float64)) - torch.lgamma(nk + self.vbeta)).sum()
        return float(tot["w"][0] + topic.cpu() + tot["d"].sum())

    def map_collective(self, reader: KeyValReader, context: Context) -> None:
        self.init_model(reader)
        start = self.start_iteration = self.resume()
        for it in range(start, self.cfg.iterations):
            self.metrics.begin_iteration()
            t0 = time.perf_counter()
            n = self.iterate(it)
            if self.device.type == "cuda":
                torch.cuda.synchronize()
            self.iter_times.append(time.perf_counter() - t0)
            self.metrics.end_iteration("lda", it, tokens=n, iter_s=self.iter_times[-1], strategy="push_pull")
            if self.cfg.print_interval and ((it + 1) % self.cfg.print_interval == 0 or it + 1 == self.cfg.iterations):
                self.loglik.append((it + 1, self.log_likelihood(it)))
            self._after_iteration(it)
        self.result = {"loglik": self.loglik, "iter_s": self.iter_times, "start_iteration": start,
                       "local_server": self.local_server, "comm_mode": self.comm_mode,
                       "fused_rows": bool(getattr(self, "fused", False))}

    def _state_tables(self, it: int) -> dict:
        from ..utils.checkpoint import blob_table, tensor_table

        tabs = {"tz": blob_table(self.tz), "nk": blob_table(self.nk)}
        if self.ndk is not None:
            tabs["ndk"] = blob_table(self.ndk)
        self._sync_glob()
        ids = self.glob.sorted_ids()
        if ids:
            tabs["glob"] = tensor_table(torch.stack([RC.widen(self.glob[b]) for b in ids]), ids)
        return tabs

    def resume(self) -> int:
        got = self._ckpt().load_latest(device=self.device, rng=True)
        if got is None:
            return 0
        man, tabs = got
        it = self._restore_common(man, tabs)
        if "glob" in tabs:
            g = tabs["glob"]
            for j, b in enumerate(g.ids):
                self.glob[b].copy_(g.buffer[j].to(self.device))  # (into a narrow table: uint16 bit patterns)
            if self.ps is not None and self.ps.owner_slots:
                self.ps.owner_from_dense(self._glob_rows())
                self._glob_stale = False
        return it

    def print_word_model(self, folder: str, next_it: int = 0) -> str:
        """Word rows of the global-table blocks this rank owns (``wordID topic:count ...``)."""
        from ..utils.model_io import write_topic_counts

        self._sync_glob()
        ids, rows = [], []
        for b in self.glob.sorted_ids():
            lo = b * self.B
            n = max(0, min(self.B, self.vocab - lo))
            ids.append(torch.arange(lo, lo + n))
            rows.append(RC.widen(self.glob[b][:n]))
        if not ids:
            ids, rows = [torch.zeros(0, dtype=torch.long)], [torch.zeros((0, self.Kp), dtype=torch.int32)]
        return write_topic_counts(f"{folder}/{self.get_self_id()}", torch.cat(ids), torch.cat(rows).cpu(),
                                  self.cfg.num_topics)


def run_lda_push_pull(comm, cfg: LDAConfig, n_docs: int, vocab: int, tokens) -> dict:
    m = LDAPushPullMapper(comm, cfg, n_docs, vocab, tokens)
    m.run(KeyValReader([]))
    return m.result
