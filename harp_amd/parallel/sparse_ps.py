"""Sparse parameter-server push / pull of count-table rows over fixed-size payloads.

The reference's parameter-server path moves sparse rows: ``push`` / ``pull`` of
``TopicCountList`` partitions (contrib/src/main/java/edu/iu/lda/LDAMapperDyn.java:380 push,
:429 pull; the packed (count << 32) + topic longs of ml/java/src/main/java/edu/iu/lda/
LDAUtil.java:159-213), routed per call by partition-set exchanges
(core/harp-collective/.../LocalGlobalSyncCollective.java:456-698).

MI355X design (:class:`SparseRowPS`): the routing and every payload size are fixed ONCE.
Each worker names the global rows (word ids) its tokens touch and its token count per
row; the owners learn every requester's rows and counts in one all-to-all and derive the
slot capacities both ends agree on:

* pull  (owner -> requester): min(K, global tokens of the word) nonzeros per row;
* push  (requester -> owner): min(K, 2 x the requester's tokens of the word) -- a
  resampled token moves one count between two topics.

A call is then: one HIP encode pass over the rows (``ops.rowcodec``), ONE fixed-split
``all_to_all_single`` of uint8 payloads, one decode pass. No size exchange, no host sync,
no per-partition objects. The push encodes the count DELTA against the pulled snapshot
by reading the pull payload itself (no dense snapshot copy of the model).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch

from ..ops import rowcodec as RC
from .comm import Communicator


def _a2a_ints(comm: Communicator, per_dest: List[torch.Tensor]) -> List[torch.Tensor]:
    """All-to-all-v of int64 vectors (plan build only)."""
    if comm.world_size == 1:
        return [per_dest[0].clone()]
    msgs = [x.contiguous().to(torch.int64).view(torch.uint8).to(comm.device) for x in per_dest]
    got = comm.all_to_all_bytes(msgs)
    return [g.cpu().view(torch.int64) if g.numel() else torch.zeros(0, dtype=torch.int64) for g in got]


class _Side:
    """Row list + slot layout of one direction at one end (rows grouped by peer)."""

    def __init__(self, rows: List[torch.Tensor], caps: List[torch.Tensor], K: int, device):
        offs, splits, base = [], [], 0
        for c in caps:
            off, nb = RC.layout(c, K, base)
            offs.append(off)
            splits.append(nb)
            base += nb
        cat = lambda xs, dt: (torch.cat(xs) if xs else torch.zeros(0, dtype=torch.int64)).to(dt)  # noqa: E731
        self.rows = cat(rows, torch.int32).contiguous().to(device)
        self.off = cat(offs, torch.int64).contiguous().to(device)
        self.cap = cat(caps, torch.int32).contiguous().to(device)
        self.splits = splits
        self.nbytes = base
        self.buf = torch.empty(max(base, RC.ALIGN), dtype=torch.uint8, device=device)


class SparseRowPS:
    """Fixed-layout sparse push / pull between requesters' local row tables and the
    owners' global table (int32 count rows of width K, SUM combine).

    ``want_ids`` (sorted, unique int64): global row ids this worker uses; its local table
    holds id ``want_ids[i]`` at row i. ``want_tokens``: this worker's token count per
    wanted id (the slot bounds). ``owner_of(ids) -> ranks`` and ``owner_row(ids) -> row in
    the owner's table`` describe the global table. Build is collective."""

    def __init__(self, comm: Communicator, want_ids: torch.Tensor, want_tokens: torch.Tensor,
                 owner_of: Callable[[torch.Tensor], torch.Tensor], owner_row: Callable[[torch.Tensor], torch.Tensor],
                 K: int, device: Optional[torch.device] = None):
        self.comm = comm
        self.K = int(K)
        P = comm.world_size
        dev = torch.device(device) if device is not None else comm.device
        self.device = dev
        ids = want_ids.cpu().to(torch.int64)
        toks = want_tokens.cpu().to(torch.int64)
        own = owner_of(ids).cpu().to(torch.int64)
        lrow = torch.arange(ids.numel(), dtype=torch.int64)
        per_ids, per_toks, per_lrow = [], [], []
        for o in range(P):
            m = own == o
            per_ids.append(ids[m])
            per_toks.append(toks[m])
            per_lrow.append(lrow[m])
        # owners learn each requester's rows and token counts
        got_ids = _a2a_ints(comm, per_ids)
        got_toks = _a2a_ints(comm, per_toks)
        allids = torch.cat(got_ids) if got_ids else torch.zeros(0, dtype=torch.int64)
        if allids.numel():
            uniq, inv = torch.unique(allids, return_inverse=True)
            glob_tok = torch.zeros(uniq.numel(), dtype=torch.int64).index_add_(0, inv, torch.cat(got_toks))
        pull_caps_out, o = [], 0  # owner side: pull caps per requester
        for g in got_ids:
            n = g.numel()
            gt = glob_tok[inv[o:o + n]] if n else torch.zeros(0, dtype=torch.int64)
            pull_caps_out.append(RC.slot_caps(gt, self.K))
            o += n
        # requesters learn the pull caps of their rows (same order as they asked)
        pull_caps_in = _a2a_ints(comm, pull_caps_out)
        push_caps_out = [RC.slot_caps(2 * t, self.K) for t in per_toks]
        push_caps_in = [RC.slot_caps(2 * t, self.K) for t in got_toks]
        orows = [owner_row(g).cpu().to(torch.int64) if g.numel() else torch.zeros(0, dtype=torch.int64)
                 for g in got_ids]
        self.pull_send = _Side(orows, pull_caps_out, self.K, dev)       # owner: glob rows -> requesters
        self.pull_recv = _Side(per_lrow, pull_caps_in, self.K, dev)     # requester: -> local rows
        self.push_send = _Side(per_lrow, push_caps_out, self.K, dev)    # requester: deltas of local rows
        self.push_recv = _Side(orows, push_caps_in, self.K, dev)        # owner: += into glob rows
        if P == 1:
            # one rank: both ends derive the same layout from the same caps, so the receive
            # side reads the send payload in place (no loopback copy)
            assert self.pull_recv.nbytes == self.pull_send.nbytes and self.push_recv.nbytes == self.push_send.nbytes
            self.pull_recv.buf = self.pull_send.buf
            self.push_recv.buf = self.push_send.buf
        # owner side: a row wanted by several requesters is encoded ONCE into a canonical
        # slot (its pull cap is the same for every requester: global tokens) and copied into
        # each requester's slot -- the row read once, not once per requester
        self._dedup = None
        srows = self.pull_send.rows.cpu().long()
        if P > 1 and srows.numel():
            uq, inv = torch.unique(srows, return_inverse=True)
            if uq.numel() < srows.numel():
                first = torch.full((uq.numel(),), srows.numel(), dtype=torch.int64).scatter_reduce_(
                    0, inv, torch.arange(srows.numel()), reduce="amin")
                ucap = self.pull_send.cap.cpu()[first].to(torch.int64)
                coff, cnb = RC.layout(ucap, self.K)
                self._dedup = (uq.to(torch.int32).to(dev), coff.to(dev), ucap.to(torch.int32).to(dev),
                               torch.empty(max(cnb, RC.ALIGN), dtype=torch.uint8, device=dev),
                               coff[inv].contiguous().to(dev))
        self.overflow = torch.zeros(1, dtype=torch.int32, device=dev)
        self.n_rows = int(ids.numel())
        self._pulled = False
        self._owner = None  # owner table held as canonical slots (use_owner_slots)

    def _encode_pull(self, glob_rows: torch.Tensor) -> None:
        s = self.pull_send
        if self._owner is not None:  # owner slots: the canonical slots are the rows
            if not self._owner["alias"]:
                urows, coff, ucap, cbuf, src_off = self._dedup
                RC.copy_slots(cbuf, src_off, s.buf, s.off, s.cap, self.K)
            return
        if self._dedup is None:
            RC.encode(glob_rows, self.K, s.rows, s.off, s.cap, s.buf, self.overflow)
            return
        urows, coff, ucap, cbuf, src_off = self._dedup
        RC.encode(glob_rows, self.K, urows, coff, ucap, cbuf, self.overflow)
        RC.copy_slots(cbuf, src_off, s.buf, s.off, s.cap, self.K)

    # -- traffic accounting ---------------------------------------------------------------
    def bytes_per_call(self, remote_only: bool = True) -> Tuple[int, int]:
        """(pull, push) bytes this rank sends per call (to other ranks when ``remote_only``)."""
        me = self.comm.rank
        f = lambda s: sum(b for r, b in enumerate(s.splits) if not (remote_only and r == me))  # noqa: E731
        return f(self.pull_send), f(self.push_send)

    # -- collectives ---------------------------------------------------------------------
    def _exchange(self, send: _Side, recv: _Side) -> None:
        if self.comm.world_size == 1:
            if send.nbytes and recv.buf.data_ptr() != send.buf.data_ptr():
                recv.buf[:send.nbytes].copy_(send.buf[:send.nbytes])
            return
        self.comm.all_to_all_single(recv.buf[:recv.nbytes], send.buf[:send.nbytes], recv.splits, send.splits)

    def pull(self, glob_rows: torch.Tensor, local: torch.Tensor) -> None:
        """``local[i] := glob row of want_ids[i]`` for every wanted row (owners encode from
        ``glob_rows`` [rows, >=K])."""
        s, r = self.pull_send, self.pull_recv
        self._encode_pull(glob_rows)
        self._exchange(s, r)
        RC.decode(local, self.K, r.rows, r.off, r.cap, r.buf)
        self._pulled = True

    def push(self, local: torch.Tensor, glob_rows: torch.Tensor, delta: bool = True) -> None:
        """Owners add each requester's rows into ``glob_rows``. ``delta``: the rows minus
        the snapshot of the last :meth:`pull` (read from its payload); otherwise the rows
        themselves (e.g. initial counts against an empty model)."""
        s, r, pr = self.push_send, self.push_recv, self.pull_recv
        if delta:
            if not self._pulled:
                raise RuntimeError("delta push needs a preceding pull (its payload is the snapshot)")
            RC.encode(local, self.K, s.rows, s.off, s.cap, s.buf, self.overflow, pr.buf, pr.off, pr.cap)
        else:
            RC.encode(local, self.K, s.rows, s.off, s.cap, s.buf, self.overflow)
        self._exchange(s, r)
        if self._owner is not None:
            self._merge_pushed()
        else:
            RC.decode(glob_rows, self.K, r.rows, r.off, r.cap, r.buf, add=True)

    # -- fused rows (the sampler reads pull slots and writes push slots itself) -----------
    def row_slots(self):
        """Per LOCAL row: (pull slot offset, pull cap, push slot offset, push cap) device
        arrays, for kernels that read rows straight from the pull payload and write their
        deltas straight into the push payload (csrc/lda.hip ``harp_lda_cgs_ps``). Every
        local row has one owner, so it has exactly one slot per direction."""
        if getattr(self, "_row_slots", None) is None:
            n, dev = self.n_rows, self.device

            def inv(side):
                off = torch.zeros(max(n, 1), dtype=torch.int64, device=dev)
                cap = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
                if side.rows.numel():
                    r = side.rows.long()
                    off[r] = side.off
                    cap[r] = side.cap
                return off, cap

            self._row_slots = inv(self.pull_recv) + inv(self.push_send)
        return self._row_slots

    def pull_payload(self, glob_rows: torch.Tensor) -> torch.Tensor:
        """The pull without its decode: owners encode, one all-to-all; returns the received
        payload (slots per :meth:`row_slots`)."""
        s, r = self.pull_send, self.pull_recv
        self._encode_pull(glob_rows)
        self._exchange(s, r)
        self._pulled = True
        return r.buf

    def push_payload_buffer(self) -> torch.Tensor:
        """The push payload with every slot emptied (nnz 0, dense slots zero) for a kernel to fill."""
        s = self.push_send
        RC.reset_slots(s.buf, s.off, s.cap, self.K)
        return s.buf

    def push_payload(self, glob_rows: torch.Tensor) -> None:
        """The push of a payload a kernel filled (:meth:`push_payload_buffer`): one
        all-to-all, owners add the slots (repeated topics in a slot add up)."""
        s, r = self.push_send, self.push_recv
        self._exchange(s, r)
        if self._owner is not None:
            self._merge_pushed()
        else:
            RC.decode(glob_rows, self.K, r.rows, r.off, r.cap, r.buf, add=True)

    # -- owner table held as slots ---------------------------------------------------------
    def use_owner_slots(self) -> None:
        """Hold the owner's share of the table as CANONICAL SLOTS instead of dense rows: one
        slot per owned row that any requester uses (capacity min(K, the word's global tokens),
        so it always fits), ascending topics without zeros. The pull then needs no encode (one
        rank: the slots ARE the pull payload; otherwise a slot copy per requester, or none
        when every row has one requester) and the push is a per-row merge of the canonical
        slot with the pushed delta slots (``ops.rowcodec.merge``) instead of scattered atomic
        adds into a dense table. Dense rows for the likelihood / checkpoints come from
        :meth:`owner_to_dense`. Call before the first push; the slots start empty."""
        s, r = self.pull_send, self.push_recv
        if self._dedup is None:  # every owned row has one slot in the pull payload: alias it
            crow, coff, ccap, cbuf = s.rows, s.off, s.cap, s.buf
            alias = True
        else:
            crow, coff, ccap, cbuf, _ = self._dedup
            alias = False
        cbuf.zero_()
        n = crow.numel()
        # CSR: received push slots grouped by their canonical row
        if r.rows.numel() and n:
            srt, perm = torch.sort(crow.long())
            pos = torch.searchsorted(srt, r.rows.long())
            if bool((pos >= n).any()) or not bool(torch.equal(srt[pos.clamp(max=n - 1)], r.rows.long())):
                raise RuntimeError("sparse push/pull: a pushed row has no canonical slot")
            ci = perm[pos]
            order = torch.argsort(ci, stable=True)
            cnt = torch.bincount(ci, minlength=n)
        else:
            order = torch.zeros(0, dtype=torch.int64, device=self.device)
            cnt = torch.zeros(n, dtype=torch.int64, device=self.device)
        ptr = torch.zeros(n + 1, dtype=torch.int64, device=self.device)
        ptr[1:] = torch.cumsum(cnt, 0)
        self._owner = {"rows": crow, "off": coff, "cap": ccap, "buf": cbuf, "alias": alias,
                       "src_ptr": ptr.to(torch.int32).contiguous(), "src_idx": order.to(torch.int32).contiguous()}
        self._owner["plan"] = RC.merge_plan(coff, ccap, self._owner["src_ptr"], self._owner["src_idx"], r.off,
                                            r.cap, self.K)

    @property
    def owner_slots(self) -> bool:
        return self._owner is not None

    def _merge_pushed(self) -> None:
        o, r = self._owner, self.push_recv
        RC.merge(o["buf"], o["off"], o["cap"], o["src_ptr"], o["src_idx"], r.buf, r.off, r.cap, self.K,
                 self.overflow, o["plan"])

    def push_initial(self, local: torch.Tensor) -> None:
        """Initial counts (the rows themselves, not a delta) into the empty owner slots."""
        s, r = self.push_send, self.push_recv
        RC.encode(local, self.K, s.rows, s.off, s.cap, s.buf, self.overflow)
        self._exchange(s, r)
        self._merge_pushed()

    def owner_to_dense(self, glob_rows: torch.Tensor) -> torch.Tensor:
        """Dense owner rows from the canonical slots (rows nobody uses are zero)."""
        o = self._owner
        glob_rows.zero_()
        RC.decode(glob_rows, self.K, o["rows"], o["off"], o["cap"], o["buf"], add=True)
        return glob_rows

    def owner_from_dense(self, glob_rows: torch.Tensor) -> None:
        """Canonical slots from dense owner rows (checkpoint restore)."""
        o = self._owner
        RC.encode(glob_rows, self.K, o["rows"], o["off"], o["cap"], o["buf"], self.overflow)

    def check_overflow(self) -> None:
        if int(self.overflow.item()):
            raise RuntimeError("sparse push/pull overflow: a row held more nonzeros than its token bound")
