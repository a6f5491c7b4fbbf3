"""Row-sharded item table for the multi-GPU step (SURVEY.md §8e ii).

The reference trains one dense ``nn.Embedding(T, d)`` (``etpgt/model/base.py:36``) with a
dense AdamW (``scripts/train/train_baseline.py:252-256``); it has no multi-GPU path.  In
the data-parallel step of ``etpgt.train.distributed`` every rank keeps the whole table
and its moments and receives every rank's touched rows.  Here the table, ``exp_avg``,
``exp_avg_sq`` and the lazy-table stamps are row-sharded instead: global row ``r`` lives
on rank ``r % P`` as local row ``r // P`` (cyclic: Zipf-hot items spread over every
owner).  Per step (``include/gtr.h``, ``gtr_shard_*``):

    begin     sorted contribution list of the rank's own batch (global row ids)
    route     unique rows per owner -> send_ids[P][cap]; the batch's ids -> compact rows
    A2A ids   RCCL all-to-all
    serve     owners bring the requested rows to step t-1 (bitwise the dense zero-gradient
              AdamW) -> send_rows[P][cap][D]
    A2A rows  == the layer-0 halo fetch of source embeddings
    forward / loss / backward / weight gradients on the compact rows (unchanged kernels)
    pack      summed gradient row per requested row -> send_grads; small-parameter
              gradient + loss -> small_pack
    A2A grads + all-gather of the small packs
    update    owners: rank-ordered sum / P + AdamW (the arithmetic of gtr_dp_tail), stamps;
              every rank: the small parameters from the gathered packs

Per rank and step the table traffic is the rows its batch touches plus the rows it owns
that any rank touched, instead of every rank's touched rows (all-gather) or the whole
table (dense sweep).  Results are bit-identical to the replicated data-parallel step
with the lazy table (same per-rank sums, same rank-ordered averaging, same catch-up).
"""

from __future__ import annotations

import contextlib
import ctypes as C
import math
import os

import torch

from etpgt.backend import _lib as L
from etpgt.train.distributed import all_gather_packs, all_to_all, world_info


def shard_capacity(m_cap: int, num_items: int, world: int, slack: float | None = None) -> int:
    """Slots per peer block (count slot included).  A requester asks one owner for at
    most min(m_cap, rows the owner holds) distinct rows; under cyclic ownership the
    distinct ids of a batch split evenly, so the block is sized at ``slack`` x the even
    share (the all-to-alls move whole blocks) unless the exact bound is smaller.  A batch
    that overflows a block is flagged (``status``) and raises on the host."""
    if slack is None:
        slack = float(os.environ.get("GTR_SHARD_SLACK", "1.5"))
    exact = min(m_cap, (num_items + world - 1) // world)
    even = max(64, int(math.ceil(slack * m_cap / world)) + 64)
    return 1 + min(exact, even)


def block_rows(batches, world: int, split: bool) -> tuple[int, int]:
    """The most distinct rows one rank asks one owner for in one step, over ``batches``
    (host SessionBatch objects): (class 0, class 1) with two row classes -- class 0 the
    rows a node of the batch reads, class 1 the rows only the scoring readout reads
    (targets / negatives) -- or (all rows, 0) with one.  Owner of row r: r % world."""
    import numpy as np

    def arr(t):
        return np.asarray(t.detach().cpu() if hasattr(t, "detach") else t, dtype=np.int64).reshape(-1)

    def most(rows):
        return int(np.bincount(rows % world, minlength=world).max()) if rows.size else 0

    m0 = m1 = 0
    for b in batches:
        nodes = np.unique(arr(b.x))
        score = np.unique(np.concatenate([arr(b.target_item), arr(b.negative_items)]))
        if split:
            m0 = max(m0, most(nodes))
            m1 = max(m1, most(np.setdiff1d(score, nodes, assume_unique=True)))
        else:
            m0 = max(m0, most(np.union1d(nodes, score)))
    return m0, m1


class ShardState:
    """This rank's rows of the item table and their AdamW / lazy-table state."""

    def __init__(self, step, group=None):
        self.step = step
        self.group = group
        self.rank, self.world = world_info(group)
        if self.world > 16:
            raise ValueError("the row-sharded table supports at most 16 ranks")
        eng = step.eng
        T, D, P, p = eng.T, eng.D, self.world, self.rank
        dev = step.dev
        self.T, self.D = T, D
        self.local_rows = (T - p + P - 1) // P
        self.rows_max = (T + P - 1) // P
        w = eng.model.item_embedding.weight.data
        self.table = w[p::P].contiguous().clone()  # [local_rows, D]
        self.m = torch.zeros_like(self.table)
        self.v = torch.zeros_like(self.table)
        self.stamp = torch.zeros(self.local_rows, dtype=torch.int32, device=dev)
        self.status = torch.zeros(4, dtype=torch.int32, device=dev)
        self._checks = 0
        self._check_every = max(1, int(os.environ.get("GTR_SHARD_CHECK_EVERY", "64")))
        self.consts = None
        self.stale = False  # the model's item_embedding.weight lags the shards
        self.s = L.GtrShard()
        self._alloc_consts(1 << 12)
        # rows a node of the batch reads, stamped with the step (two-class exchange)
        self.node_mark = torch.zeros(T, dtype=torch.int32, device=dev)
        self.s.node_mark = self.node_mark.data_ptr()
        # collectives that overlap compute need a device transport (RCCL): gloo stages
        # through the host in line with the step
        import torch.distributed as dist

        self.device_collectives = dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "nccl"

    def _alloc_consts(self, cap: int):
        c = torch.zeros(cap, 2, dtype=torch.float32, device=self.step.dev)
        if self.consts is not None:
            k = min(cap, self.consts.shape[0])
            c[:k].copy_(self.consts[:k])
        self.consts = c
        self._fill()

    def _fill(self):
        s = self.s
        s.num_items, s.world, s.rank, s.local_rows, s.dim = self.T, self.world, self.rank, self.local_rows, self.D
        s.table, s.m, s.v, s.stamp = (self.table.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                                      self.stamp.data_ptr())
        s.consts, s.consts_cap = self.consts.data_ptr(), self.consts.shape[0]
        s.status = self.status.data_ptr()
        s.opt = self.step.adam

    def ensure_steps(self, steps: int) -> bool:
        """Grow the per-step scalar table before step ``steps``; True if pointers moved."""
        if steps + 2 < self.consts.shape[0]:
            return False
        cap = 2 * self.consts.shape[0]
        while steps + 2 >= cap:
            cap *= 2
        self._alloc_consts(cap)
        return True

    def check_status(self, block: bool = False, steps: int = 1):
        """Raise if any step since the last check overflowed an exchange block.  Called
        before every launch with the number of steps that launch runs (1, or n for a
        multi-step graph); every rank counts the same steps, so every rank checks at the
        same host step -- once GTR_SHARD_CHECK_EVERY (64) steps have been launched since the
        last check, and at ``block=True`` (sync_table / export) -- after its queue has
        drained.  A check drains the queue up to the steps launched BEFORE it, so an
        overflow is raised at most check_every + n steps after the flagged step (n: the
        steps per launch).  The overflow flag reaches every rank inside the flagged step
        (k_shard_update folds the ranks' flags into the sticky status[1]), so all ranks
        raise together instead of one rank leaving the others blocked in the next
        collective.  A flagged step trains as a zero-gradient step on the rows it could
        not fetch."""
        self._checks += int(steps)
        if not block and self._checks < self._check_every:
            return
        self._checks = 0
        torch.cuda.current_stream(self.step.dev).synchronize()
        if int(self.status[1].item()) != 0:
            raise RuntimeError("row-sharded table: a batch requested more rows from one owner than the "
                               "exchange capacity holds (raise GTR_SHARD_SLACK)")

    # ---------------------------------------------------------------- the full table
    def flush(self):
        """Bring every local row to the current step (lazy zero-gradient updates)."""
        st = self.step
        lz = L.GtrLazy()
        lz.consts, lz.cap = self.consts.data_ptr(), self.consts.shape[0]
        lz.table, lz.m, lz.v, lz.opt = self.table.data_ptr(), self.m.data_ptr(), self.v.data_ptr(), st.adam
        L.check(L.lib().gtr_lazy_flush(self.local_rows, self.D, self.stamp.data_ptr(), st.step_dev.data_ptr(),
                                       C.byref(lz), torch.cuda.current_stream(st.dev).cuda_stream), "lazy_flush")

    def _gather(self, local: torch.Tensor) -> torch.Tensor:
        P, D = self.world, self.D
        pad = torch.zeros(self.rows_max, D, dtype=local.dtype, device=local.device)
        pad[: self.local_rows].copy_(local)
        allr = torch.zeros(P, self.rows_max * D, dtype=local.dtype, device=local.device)
        all_gather_packs(allr, pad.view(-1), self.group)
        return allr.view(P, self.rows_max, D).transpose(0, 1).reshape(self.rows_max * P, D)[: self.T]

    def gather_table(self):
        """Collective: the full [T, D] table (and its moments) on every rank."""
        self.flush()
        return self._gather(self.table), self._gather(self.m), self._gather(self.v)

    def sync_model(self):
        """Collective: write the full table into the model's item_embedding.weight."""
        tab, _, _ = self.gather_table()
        with torch.no_grad():
            self.step.eng.model.item_embedding.weight.data.copy_(tab)
        self.stale = False


class ShardExchange:
    """Per-capacity exchange buffers and launches of the sharded step."""

    def __init__(self, step, state: ShardState, rows: tuple[int, int] | None = None):
        """``rows``: (class 0, class 1) distinct rows per owner and step to size the blocks
        for (``block_rows`` over the batches to run, agreed across the ranks --
        ``FusedTrainStep.fit_shard_blocks``); None: the static bound ``shard_capacity``."""
        self.step, self.state = step, state
        eng, caps, dev = step.eng, step.caps, step.dev
        P, D = state.world, eng.D
        self.m_cap = caps.n_cap + caps.b_cap * (1 + caps.n_neg)
        # two row classes (include/gtr.h gtr_shard): class 0 = rows a node reads (layer 0
        # needs them), class 1 = rows only the scoring readout reads, which travel during
        # the forward; default at P > 1 (GTR_SHARD_SPLIT=0 / 1 overrides)
        e = os.environ.get("GTR_SHARD_SPLIT")
        self.split = (e == "1") if e is not None else P > 1
        if self.split:
            self.cap = shard_capacity(caps.n_cap, eng.T, P)
            self.cap_s = shard_capacity(self.m_cap, eng.T, P)
        else:
            self.cap = shard_capacity(self.m_cap, eng.T, P)
            self.cap_s = 0
        if rows is not None:  # blocks sized to the batches (never above the static bound)
            self.cap = max(2, min(self.cap, 1 + int(rows[0])))
            if self.split:
                self.cap_s = max(2, min(self.cap_s, 1 + int(rows[1])))
        self.blk = self.cap + self.cap_s
        state.s.cap, state.s.cap_s = self.cap, self.cap_s
        state.s.grad_stride, state.s.small_stride, state.s.pack_parts = 0, 0, 0
        slots = P * self.blk
        rows = P * self.cap + P * self.cap_s
        i32 = dict(dtype=torch.int32, device=dev)
        f32 = dict(dtype=torch.float32, device=dev)
        # one rank: nothing crosses a link, so every receive buffer IS its send buffer and
        # the exchanges are no-ops (no 2 x slots x D copies per step; the kernels never read
        # and write the same buffer of a pair in one launch); GTR_SHARD_NOALIAS=1 keeps the
        # copies (a one-rank rehearsal of the collectives and their overlap)
        self.alias = P == 1 and os.environ.get("GTR_SHARD_NOALIAS") != "1"
        self.send_ids = torch.zeros(slots, **i32)
        self.recv_ids = self.send_ids if self.alias else torch.zeros(slots, **i32)
        self.send_rows = torch.zeros(rows, D, **f32)
        self.recv_rows = self.send_rows if self.alias else torch.zeros(rows, D, **f32)  # the compact "table"
        self.send_grads = torch.zeros(slots, D, **f32)
        self.recv_grads = self.send_grads if self.alias else torch.zeros(slots, D, **f32)
        # overlap: a compute stream forked from the step's stream beside a collective; the
        # collective itself stays on the step's stream (RCCL captured on a forked stream
        # does not survive hipGraph capture on this stack -- scripts/dbg/capture_probe.py)
        self.can_overlap = not self.alias and state.device_collectives
        self.cs = torch.cuda.Stream(dev) if self.can_overlap else None
        self.forked = False
        self.ckeys = torch.zeros(self.m_cap, **i32)
        self.node_item_c = torch.zeros(caps.n_cap, **i32)
        self.target_c = torch.zeros(caps.b_cap, **i32)
        self.negatives_c = torch.zeros(max(1, caps.b_cap * caps.n_neg), **i32)
        self.node_pe_c = torch.zeros(caps.n_cap, eng.K, **f32) if eng.K > 0 else None
        nb = C.c_size_t(0)
        L.check(L.lib().gtr_shard_route_scratch(self.m_cap, P, C.byref(nb)), "shard_route_scratch")
        self.scratch = torch.zeros(max(int(nb.value), 16), dtype=torch.uint8, device=dev)
        F = eng.flat.layout.total
        self.small_words = (F + 2 + 3) & ~3  # flat gradient | loss | overflow flag
        self.small_all = torch.zeros(P, self.small_words, **f32)
        self.small_pack = self.small_all[0] if self.alias else torch.zeros(self.small_words, **f32)
        self.bs_c = self._compact(step.bs)
        self.bs_c_pe = self._compact(step.bs_pe) if step.bs_pe is not None else None

    def fork(self):
        """Compute launched under ``side()`` from here on runs on the compute stream, after
        the work queued so far; collectives queued next on the step's stream run beside it."""
        self.cs.wait_stream(torch.cuda.current_stream(self.step.dev))
        self.forked = True

    def side(self):
        return torch.cuda.stream(self.cs) if self.forked else contextlib.nullcontext()

    def join(self):
        """The step's stream waits for the compute forked since ``fork``."""
        if self.forked:
            torch.cuda.current_stream(self.step.dev).wait_stream(self.cs)
            self.forked = False

    def _compact(self, bs):
        """The batch struct the layer kernels read: ids -> compact rows; PE per node."""
        c = L.GtrBatch()
        C.memmove(C.byref(c), C.byref(bs), C.sizeof(bs))
        c.node_item, c.target, c.negatives = (self.node_item_c.data_ptr(), self.target_c.data_ptr(),
                                              self.negatives_c.data_ptr())
        if bs.node_pe is None and self.node_pe_c is not None:
            c.node_pe = self.node_pe_c.data_ptr()
        return c

    def table_ptr(self) -> int:
        return self.recv_rows.data_ptr()

    def compact(self, with_pe: bool):
        return self.bs_c_pe if with_pe else self.bs_c

    # ---------------------------------------------------------------- launches
    def route(self, bs, stream):
        st, eng = self.step, self.step.eng
        pe_tab, node_pe = None, None
        if self.node_pe_c is not None and bs.node_pe is None:
            pe = eng.model.laplacian_pe._cached_pe
            if pe is None:
                raise RuntimeError("Laplacian PE not precomputed. Call precompute() first.")
            pe_tab, node_pe = pe.data_ptr(), self.node_pe_c.data_ptr()
        L.check(L.lib().gtr_shard_route(C.byref(bs), st.skeys.data_ptr(), st.svals.data_ptr(), C.byref(self.state.s),
                                        self.send_ids.data_ptr(), self.ckeys.data_ptr(), self.node_item_c.data_ptr(),
                                        self.target_c.data_ptr(), self.negatives_c.data_ptr(), pe_tab, eng.K, node_pe,
                                        self.scratch.data_ptr(), self.scratch.numel(), stream), "shard_route")

    def exchange_ids(self):
        if not self.alias:
            all_to_all(self.recv_ids, self.send_ids, self.state.group)

    def serve(self, stream):
        L.check(L.lib().gtr_shard_serve(C.byref(self.state.s), self.recv_ids.data_ptr(), self.send_rows.data_ptr(),
                                        stream), "shard_serve")

    def exchange_rows(self, overlap: bool = False):
        """The rows layer 0 needs (class 0), then the class-1 rows -- beside the forward
        when ``overlap`` (the forward forked onto the compute stream, joined before the
        readout).  One class: all rows at once."""
        if self.alias:
            return
        n = self.state.world * self.cap
        all_to_all(self.recv_rows[:n], self.send_rows[:n], self.state.group)
        if self.cap_s:
            if overlap and self.can_overlap:
                self.fork()
            all_to_all(self.recv_rows[n:], self.send_rows[n:], self.state.group)

    def pack(self, bs, stream, parts: int = 0):
        """parts: 1 the gradient rows, 2 the small-parameter pack (after the weight
        gradients), 0 both."""
        st = self.step
        self.state.s.pack_parts = parts
        try:
            L.check(L.lib().gtr_shard_pack(C.byref(bs), C.byref(self.state.s), C.byref(st.tail), self.ckeys.data_ptr(),
                                           st.segs, st.nseg, self.send_grads.data_ptr(), self.small_pack.data_ptr(),
                                           stream), "shard_pack")
        finally:
            self.state.s.pack_parts = 0

    def exchange_grads(self):
        """The gradient rows' all-to-all (beside the forked weight gradients + small pack
        when overlapping), the join, then the all-gather of the small packs."""
        if not self.alias:
            all_to_all(self.recv_grads, self.send_grads, self.state.group)
        self.join()
        if not self.alias:
            all_gather_packs(self.small_all, self.small_pack, self.state.group)

    def update(self, stream):
        st = self.step
        L.check(L.lib().gtr_shard_update(C.byref(self.state.s), C.byref(st.tail), self.recv_ids.data_ptr(),
                                         self.recv_grads.data_ptr(), self.small_all.data_ptr(), self.small_words,
                                         stream), "shard_update")
        self.state.stale = True

    def volume(self) -> dict:
        """Bytes each rank sends per step over the collectives (fixed-size blocks)."""
        P, D = self.state.world, self.step.eng.D
        return {"ids": 4 * P * self.blk, "rows_layer0": 4 * P * self.cap * D, "rows_scoring": 4 * P * self.cap_s * D,
                "grads": 4 * P * self.blk * D, "small": 4 * self.small_words * P, "cap": self.cap,
                "cap_scoring": self.cap_s, "overlap_capable": self.can_overlap}
