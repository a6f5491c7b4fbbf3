"""Fused training step: forward + loss + backward + (Adam|AdamW) in HIP kernels,
captured once into a hipGraph and replayed per batch.

One step of ``Trainer.train_epoch`` (trainer.py:80-133) with
``torch.optim.AdamW(lr, weight_decay)`` (train_baseline.py:252-256), as nine
launches on one stream (the blob copy, then):

  step_begin -> conv_fwd(0..L-1) -> readout_loss(FWD|LOSS|BWD) -> conv_bwd(L-1..0)
  -> wgrad(all layers) -> step_tail

step_begin advances the step / dropout counters, stamps the touched table rows and
builds the sorted table-gradient contribution list; step_tail applies AdamW to the
touched rows (segment sums of the contributions), to the untouched rows (g = 0: the
same arithmetic as the dense reference update, 24 B/element instead of 32) and to
every small parameter, and sums the loss.  The item table never gets a dense
gradient.  Optimizer state (exp_avg, exp_avg_sq, step) lives in this object;
``export_optimizer_state`` writes it into a ``torch.optim.AdamW`` state layout.
"""

from __future__ import annotations

import ctypes as C
import os

import torch

from etpgt.backend import _lib as L
from etpgt.backend.engine import Engine, readout_grid
from etpgt.data.batch import Caps, SessionBatch


class FusedTrainStep:
    def __init__(self, model, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-5, decoupled: bool = True, loss: str = "bpr",
                 temperature: float = 1.0, alpha: float = 0.7, caps: Caps | None = None,
                 use_graph: bool = True, data_parallel: bool | None = None, process_group=None,
                 lazy: bool = False, sync_bn: bool = False, lagged: bool = False, shard_table: bool = False):
        if loss not in ("bpr", "listwise", "dual", "sampled_softmax"):
            raise ValueError(f"Unknown loss type: {loss}")
        if getattr(model, "use_ffn", False):
            # the FFN variant trains data parallel (replicated or row-sharded table), with or
            # without SyncBN; SyncBN folds the gathered rows in the FFN's first GEMM (dim 64 / 128,
            # expansion 4)
            if os.environ.get("GTR_TAILW") == "1":
                raise NotImplementedError("the FFN variant (use_ffn=True) has no GTR_TAILW step")
            if sync_bn and not (model.embedding_dim in (64, 128) and getattr(model, "ffn_expansion", 4) == 4):
                raise NotImplementedError("SyncBN with the FFN variant covers dim 64 / 128 at ffn_expansion 4")
        self.model = model
        self.eng: Engine = model.hip_engine()
        self.dev = self.eng.device
        self.loss_kind = L.GTR_LOSS[loss]
        self.temperature = float(temperature)
        self.alpha = float(alpha)
        self.use_graph = use_graph
        # data parallel (one process per GPU): gradients averaged over the ranks by one
        # all-gather per step (etpgt.train.distributed); default: on when the default
        # process group spans more than one rank
        from etpgt.train.distributed import world_info

        self.group = process_group
        self.rank, self.world = world_info(process_group)
        # row-sharded item table (etpgt.train.sharded, SURVEY.md §8e ii): rank p owns the rows
        # r % P == p and their AdamW state; rows travel by all-to-all
        self.shard_table = bool(shard_table)
        if self.shard_table and (lazy or lagged):
            raise ValueError("the row-sharded table keeps its own lazy stamps (no lazy/lagged option)")
        self.data_parallel = (self.world > 1) if data_parallel is None else bool(data_parallel)
        self.data_parallel = self.data_parallel or self.shard_table

        # SyncBN: BatchNorm statistics over every rank's batch (all-gathered partials per
        # BatchNorm), so N ranks train exactly like one GPU on the concatenated batch
        self.sync_bn = bool(sync_bn)
        if self.sync_bn and not self.data_parallel:
            raise ValueError("sync_bn needs the data-parallel step")
        self.dp = None
        self.sync_alias = False
        self.graph_b = None
        self._coll_capture_refused = False  # set once if the transport refuses stream capture
        eng = self.eng
        T, D = eng.T, eng.D
        self.adam = L.GtrAdam()
        self.adam.lr, self.adam.beta1, self.adam.beta2 = float(lr), float(betas[0]), float(betas[1])
        self.adam.eps, self.adam.weight_decay, self.adam.decoupled = float(eps), float(weight_decay), int(decoupled)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=self.dev)
        # device-side running sum of the steps' losses (gtr_tail.loss_acc): the Trainer reads
        # it once per epoch instead of one loss per step (steps chained in one graph)
        self.loss_acc = torch.zeros(1, dtype=torch.float64, device=self.dev)
        self.adam.step_dev = self.step_dev.data_ptr()
        self.adam.step_offset = 0  # kernels after gtr_step_begin see the current step
        tab_rows = 1 if self.shard_table else T  # sharded: the moments live in the shards
        self.m_tab = torch.zeros(tab_rows, D, dtype=torch.float32, device=self.dev)
        self.v_tab = torch.zeros(tab_rows, D, dtype=torch.float32, device=self.dev)
        self.m_flat = torch.zeros_like(eng.flat.flat)
        self.v_flat = torch.zeros_like(eng.flat.flat)
        self.stamp = torch.zeros(tab_rows, dtype=torch.int32, device=self.dev)
        # deferred zero-gradient AdamW of untouched table rows (gtr_lazy in gtr.h):
        # bitwise-identical to the dense update, applied when a row is next read or on flush()
        # lagged: lazy-table stamps, and the chain's launches sweep the PREVIOUS step's
        # untouched rows (gtr_sweep.lag), so the sweep needs no knowledge of this step's
        # touched rows -- in data parallel those are the ranks' union, known only after
        # the exchange; rows the step reads are one step behind at most
        self.lagged = bool(lagged) and not bool(lazy)
        self.lazy = bool(lazy) or self.lagged
        self._host_steps = 0
        self._dirty = False
        self._gen = 0  # bumped whenever a buffer a captured graph points at may have moved
        self.lz = None
        if self.lazy:
            self._lazy_alloc(1 << 16)
            model.__dict__["_lazy_sync"] = self.flush  # forward / predict / state_dict bring rows up to date
        self.shard_state = None
        self.shard = None
        if self.shard_table:
            from etpgt.train.sharded import ShardState

            self.shard_state = ShardState(self, process_group)
            model.__dict__["_lazy_sync"] = self._shard_guard
        self._force_split = None  # the halo step (etpgt.train.halo) runs the split layer path
        self._loss_batch = 0.0    # gtr_config.loss_batch (halo cuts: global B / P)
        self.caps = None
        self.graph = None
        self.builder = None
        self._builder_B = None  # sessions of the device-built batch (None: the builder's B)
        if caps is not None:
            self._bind(caps)

    # ------------------------------------------------------------------ lazy table
    def _lazy_alloc(self, cap: int):
        consts = torch.zeros(cap, 2, dtype=torch.float32, device=self.dev)
        old = getattr(self, "lazy_consts", None)
        if old is not None:
            keep = min(cap, old.shape[0])
            consts[:keep].copy_(old[:keep])
        self.lazy_consts = consts
        if getattr(self, "lazy_cnt", None) is None:
            self.lazy_cnt = torch.zeros(4, dtype=torch.int32, device=self.dev)
        lz = L.GtrLazy()
        lz.consts, lz.cap, lz.cnt = consts.data_ptr(), cap, self.lazy_cnt.data_ptr()
        lz.table = self.eng.model.item_embedding.weight.data_ptr()
        lz.m, lz.v = self.m_tab.data_ptr(), self.v_tab.data_ptr()
        lz.opt = self.adam
        self.lz = lz
        if getattr(self, "tail", None) is not None:
            self.tail.lazy_consts = consts.data_ptr()
        if getattr(self, "sweep", None) is not None and self.sweep.lag:
            self.sweep.consts = consts.data_ptr()
        self.graph = self.graph_pe = self.graph_b = None  # captured pointers changed
        self.resident_graphs = None
        self._gen += 1

    def flush(self):
        """Bring every table row up to the current step (lazy mode; no-op otherwise)."""
        if not self.lazy or not self._dirty:
            return
        L.check(L.lib().gtr_lazy_flush(self.eng.T, self.eng.D, self.stamp.data_ptr(), self.step_dev.data_ptr(),
                                       C.byref(self.lz), torch.cuda.current_stream(self.dev).cuda_stream),
                "lazy_flush")
        self._dirty = False

    # ------------------------------------------------------------------ buffers
    def _agree(self, caps: Caps) -> Caps:
        """DP: every rank binds the same capacities (the packs are all-gathered)."""
        if not (self.data_parallel and self.world > 1):
            return caps
        import torch.distributed as dist

        dev = self.dev if dist.get_backend(self.group) != "gloo" else "cpu"
        t = torch.tensor([caps.n_cap, caps.b_cap, caps.e_cap], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        n, b, e = (int(v) for v in t.tolist())
        return Caps(n, b, e, caps.n_neg)

    def fit_shard_blocks(self, batches, headroom: float = 1.1):
        """Row-sharded table: size the exchange blocks to the most distinct rows any rank
        asks one owner for over ``batches`` (each rank passes its own; the ranks agree on
        the maximum -- a collective) times ``headroom``, instead of the static bound of
        ``shard_capacity`` (the all-to-alls move whole blocks, so smaller blocks
        are less xGMI traffic per step).  A later batch that needs more rows overflows its
        block: the step is flagged and applied as a zero-gradient step, and the host raises
        at the next check.  Without headroom the maximum over the bench's 64 staged batches
        per rank is exceeded by 0.9 % of later rank-batches (6.8 % of 8-rank steps) on the C4
        data; 5 % headroom already leaves none of 2,048 (scripts/block_overflow.py,
        profiles/r06/block_overflow_c4_n8_b1024.json), so the default takes 10 %.  Rebuilds
        the exchange buffers: captured graphs go stale."""
        if self.shard is None:
            raise RuntimeError("fit_shard_blocks needs the row-sharded table (shard_table=True)")
        import math

        from etpgt.train.sharded import ShardExchange, block_rows

        r = tuple(int(math.ceil(v * float(headroom))) for v in block_rows(batches, self.world, self.shard.split))
        if self.world > 1:
            import torch.distributed as dist

            dev = self.dev if dist.get_backend(self.group) != "gloo" else "cpu"
            t = torch.tensor(list(r), dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            r = tuple(int(v) for v in t.tolist())
        self.shard = ShardExchange(self, self.shard_state, rows=r)
        self.graph = self.graph_pe = self.graph_b = None
        self.resident_graphs = None
        self._gen += 1
        return self.shard.cap, self.shard.cap_s

    def _bind(self, caps: Caps):
        eng = self.eng
        caps = self._agree(caps)
        self.caps = caps
        self._gen += 1  # every buffer below is reallocated: multi-step handles go stale
        self.ws = eng.workspace(caps, split=self._force_split, sync=self.sync_bn and self.world > 1)
        from etpgt.data.batch import blob_layout

        self.blob = torch.zeros(blob_layout(caps)["_total"], dtype=torch.int32, device=self.dev)
        self.node_pe = None
        if eng.K > 0:
            self.node_pe_buf = torch.zeros(caps.n_cap, eng.K, dtype=torch.float32, device=self.dev)
        self.bs = eng.batch_struct(caps, self.blob, None)
        self.bs_pe = eng.batch_struct(caps, self.blob, self.node_pe_buf) if eng.K > 0 else None
        m_cap = caps.n_cap + caps.b_cap * (1 + caps.n_neg)
        self.m_cap = m_cap
        self.keys = torch.zeros(m_cap, dtype=torch.int32, device=self.dev)
        self.vals = torch.zeros(m_cap, dtype=torch.int32, device=self.dev)
        self.skeys = torch.zeros(m_cap, dtype=torch.int32, device=self.dev)
        self.svals = torch.zeros(m_cap, dtype=torch.int32, device=self.dev)
        nb = C.c_size_t(0)
        L.check(L.lib().gtr_contrib_sort_bytes(m_cap, eng.T, C.byref(nb)), "sort_bytes")
        self.sort_tmp = torch.zeros(max(int(nb.value), 16), dtype=torch.uint8, device=self.dev)
        # opt-in (GTR_WFOLD=1): weight gradients folded into the fused backward (each row
        # group writes its split-K partial; no gtr_wgrad launch for the layers) -- the fused
        # layer path at D <= 64, not with GTR_TAILW=1.  Measured neutral at C2 (0.0794 ms both
        # ways): the gtr_wgrad launch (7.9 us) goes, but each gtr_conv_bwd grows by 4 us
        # (1.5 us of MFMA phase, the rest draining its 64 KB of partials at the kernel's end)
        self.wfold = (not bool(self.ws.split) and eng.D <= 64 and os.environ.get("GTR_TAILW", "0") != "1"
                      and os.environ.get("GTR_WFOLD", "0") == "1")
        wstride = self.ws.enable_wfold(eng) if self.wfold else 0
        if not self.wfold:
            for l in range(eng.L):
                self.ws.structs[l].wfold = None
        self.segs, self.nseg = eng.segments(self.ws, wfold=self.wfold)
        self.cfg = eng.config(self.ws, True)
        self.cfg.loss_batch = float(self._loss_batch)
        self.cfg.wfold_stride = wstride
        # large batches: every layer as projection GEMM + attention launches (Engine.layer_fwd /
        # layer_bwd); under SyncBN one merged BatchNorm row per rank and layer is gathered
        # (gtr_config.split_sync) instead of every row group's partials
        self.split = bool(self.ws.split)
        ws = self.ws
        t = L.GtrTail()
        t.skeys, t.svals = self.skeys.data_ptr(), self.svals.data_ptr()
        t.dx0, t.se = ws.dx0.data_ptr(), ws.se.data_ptr()
        t.coef_tgt, t.coef_neg = ws.coef_tgt.data_ptr(), ws.coef_neg.data_ptr()
        t.table = eng.model.item_embedding.weight.data_ptr()
        t.table_m, t.table_v, t.stamp = self.m_tab.data_ptr(), self.v_tab.data_ptr(), self.stamp.data_ptr()
        t.flat, t.flat_m, t.flat_v = eng.flat.flat.data_ptr(), self.m_flat.data_ptr(), self.v_flat.data_ptr()
        t.flat_total = eng.flat.layout.total
        # with consumer-side reduction the readout leaves its loss partials to the tail
        t.loss_part = ws.loss_part.data_ptr() if self.cfg.consumer_reduce else None
        t.loss_out = ws.loss_out.data_ptr()
        t.loss_acc = self.loss_acc.data_ptr()
        t.loss_nparts = readout_grid(caps.b_cap)
        # untouched-row AdamW spread over the layer kernels' idle CUs (single GPU, small
        # grids): the chain's 2L launches each sweep a slice of the table (gtr_sweep)
        self.sweep = None
        t.sweep_from = 0
        chain = os.environ.get("GTR_CHAIN_SWEEP", "1") != "0" and (not self.lazy or self.lagged)
        # slots: conv_fwd(l) -> l, readout -> L, conv_bwd(l) -> 2L - l; weighted by the
        # launches' measured slack (the readout is shorter than a layer kernel)
        wts = [1.0] * eng.L + [0.75] + [1.0] * eng.L
        if eng.D <= 64:  # round 6 A/B at C2 (scripts/gpu/sweep_wts.sh): forward slices 0.75, the
            # last layer's backward 1.25 -- 0.0745 -> 0.0741 ms per step (twice, alternating runs)
            wts = [0.75] * eng.L + [0.75] + [1.25] + [1.0] * (eng.L - 1)
        if os.environ.get("GTR_SWEEP_WTS"):  # experiments: comma-separated slot weights
            wts = [float(x) for x in os.environ["GTR_SWEEP_WTS"].split(",")]
        # single-GPU small batches: gtr_step_begin's work runs as extra workgroups of
        # conv_fwd(0) (gtr_begin) -- one launch less; that launch stamps the touched rows,
        # so it carries no sweep slice
        self.begin_fused = (not self.data_parallel and not self.lazy and m_cap <= 8192 and eng.T < (1 << 19)
                            and not self.split and os.environ.get("GTR_BEGIN_FUSED", "1") != "0")
        if self.begin_fused:
            wts[0] = 0.0
        # data parallel: the union of the ranks' touched rows is known once the sorted keys
        # are all-gathered (early, overlapped with the forward), so only the launches after
        # the union stamp (readout, conv_bwd) can sweep
        # (never with the row-sharded table: its moments / stamps live in the shards, and the
        # model's table copy is stale -- no chain sweep may touch them)
        self.early_union = (self.data_parallel and chain and not self.sync_bn and not self.lagged
                            and not self.shard_table and os.environ.get("GTR_DP_EARLY", "0") == "1")
        if self.early_union:
            wts = [0.0] * eng.L + wts[eng.L:]
        slots = len(wts)
        if chain and not self.shard_table and not self.split \
                and (not self.data_parallel or self.early_union or self.lagged) \
                and self.ws.g_cap <= 128 and slots <= L.SWEEP_SLOTS:
            sw = L.GtrSweep()
            sw.table = eng.model.item_embedding.weight.data_ptr()
            sw.m, sw.v, sw.stamp = self.m_tab.data_ptr(), self.v_tab.data_ptr(), self.stamp.data_ptr()
            sw.opt = self.adam  # copied by value (step_dev: device counter)
            tot, acc = sum(wts), 0.0
            if self.early_union:
                self.keys_all = torch.zeros(self.world, m_cap, dtype=torch.int32, device=self.dev)
            for i in range(L.SWEEP_SLOTS + 1):
                sw.bounds[i] = eng.T if i >= slots else int(eng.T * acc / tot)
                if i < slots:
                    acc += wts[i]
            sw.dim = eng.D
            # extra workgroups per launch: 0 = fill the CUs the launch's row groups leave
            # (C2: 224-232 per launch, 352k sessions/s against 342k at a fixed 128; every
            # workgroup on a CU of its own, the row groups packable onto one XCD); at D = 128
            # a fixed 128 measured 2 % faster (C3 193k against 189k)
            sw.blocks = int(os.environ.get("GTR_SWEEP_BLOCKS", 0 if eng.D <= 64 else 128))
            sw.lag = 1 if self.lagged else 0
            sw.consts = self.lazy_consts.data_ptr() if self.lagged else None
            self.sweep = sw
            self.cfg.sweep = C.addressof(sw)
            t.sweep_from = eng.T
        t.lazy_consts = self.lazy_consts.data_ptr() if self.lazy else None
        nc = int(L.lib().gtr_tail_carry_floats(m_cap, eng.D))
        self.carry = torch.zeros(max(nc, 4), dtype=torch.float32, device=self.dev) if nc > 0 else None
        t.carry = self.carry.data_ptr() if self.carry is not None else None
        self.cfg.begin, self.cfg.ctr_add, t.rng_inc = None, 0, None
        if self.begin_fused:
            bg = L.GtrBegin()
            bg.skeys, bg.svals, bg.stamp = self.skeys.data_ptr(), self.svals.data_ptr(), self.stamp.data_ptr()
            bg.step_dev, bg.num_items = self.step_dev.data_ptr(), eng.T
            self.begin_st = bg
            self.cfg.begin = C.addressof(bg)
            self.cfg.ctr_add = 1  # the tail advances the dropout counter at the end of the step
            t.rng_inc = eng.rng_ctr.data_ptr()
        self.tail = t
        if self.shard_table:
            from etpgt.train.sharded import ShardExchange

            self.dp = None
            self.shard = ShardExchange(self, self.shard_state)
        elif self.data_parallel:
            from etpgt.train.distributed import DpExchange

            self.dp = DpExchange(self, self.group)
        if self.sync_bn:
            self._sync_alloc()
        # opt-in (GTR_TAILW=1): weight gradients and optimizer tail in one launch
        # (gtr_step_tail_wgrad: split-K tiles, each tile's last arriving chunk applies AdamW);
        # bitwise the two launches but slower (C2 0.083 -> 0.102 ms: one workgroup per tile
        # walks its 4k elements' partials serially); needs the sweep in the chain or a lazy table
        self.tail_wgrad = (self.dp is None and self.shard is None and m_cap <= 8192
                           and (self.lazy or t.sweep_from >= eng.T) and os.environ.get("GTR_TAILW", "0") == "1")
        if self.tail_wgrad:
            self.tile_cnt = torch.zeros(4096, dtype=torch.int32, device=self.dev)
            lay = eng.flat.layout
            gb = [i for i in range(self.nseg)
                  if any(self.segs[i].begin == lay.seg(f"{l}.{n}").begin for l in range(eng.L) for n in ("gamma", "beta"))]
            self.segs_gb = (L.GtrSegment * max(1, len(gb)))()
            for j, i in enumerate(gb):
                self.segs_gb[j] = self.segs[i]
            self.nseg_gb = len(gb)
            self.layer_flat = (C.c_int64 * (3 * eng.L))(*[lay.seg(f"{l}.{n}").begin for l in range(eng.L)
                                                          for n in ("w_all", "b_all", "w_beta")])
            self.pe_flat = (C.c_int64 * 2)(lay.seg("pe.w").begin, lay.seg("pe.b").begin) if eng.K > 0 else None
        self.graph = None
        self.graph_pe = None
        self.graph_b = None
        self.resident = None  # bind_resident: batch images bound to this workspace
        self.resident_graphs = None

    def workspace_ranges(self) -> list[tuple[str, int, int]]:
        """(name, first byte, end byte) of every device buffer the step's kernels write:
        the contribution keys / values and their sorted copies, the sort scratch, the batch
        image, the carry scratch and the workspace's activations (the round-3
        Onesweep fault: check that no carved buffer overlaps another)."""
        out = []

        def add(name, t):
            if isinstance(t, torch.Tensor) and t.is_cuda and t.numel() > 0:
                out.append((name, t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()))

        for name in ("keys", "vals", "skeys", "svals", "sort_tmp", "blob", "carry", "m_tab", "v_tab", "stamp",
                     "m_flat", "v_flat"):
            add(name, getattr(self, name, None))
        for name, t in vars(self.ws).items():
            add(f"ws.{name}", t)
        for l, lay in enumerate(getattr(self.ws, "layers", [])):
            for name, t in lay.items():
                add(f"ws.layers[{l}].{name}", t)
        return out

    def check_workspace_overlap(self) -> None:
        """Raise if two of the step's device buffers overlap (views of one allocation that
        share bytes are reported by name)."""
        rs = sorted(self.workspace_ranges(), key=lambda r: r[1])
        for (n0, a0, b0), (n1, a1, b1) in zip(rs, rs[1:]):
            if a1 < b0 and not (a0 == a1 and b0 == b1):
                raise RuntimeError(f"workspace overlap: {n0} [{a0:#x}, {b0:#x}) and {n1} [{a1:#x}, {b1:#x})")

    def ensure_caps(self, batch: SessionBatch):
        N, B, E, n = batch.sizes()
        if self.data_parallel and self.world > 1:  # collective: the ranks grow together
            import torch.distributed as dist

            dev = self.dev if dist.get_backend(self.group) != "gloo" else "cpu"
            t = torch.tensor([N, B, E], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            N, B, E = (int(v) for v in t.tolist())
        if self.caps is None:
            self._bind(Caps.bucket(2 * N, B, 2 * E, n))
        elif not self.caps.fits(N, B, E, n):
            if n != self.caps.n_neg:
                raise ValueError("the number of negatives per session must stay fixed")
            self._bind(self.caps.grow(N, B, E, n))

    def load(self, batch: SessionBatch) -> bool:
        """Copy a batch into the fixed device blob (one H2D/D2D copy). Returns
        whether the batch carries precomputed PE rows."""
        self.ensure_caps(batch)
        batch.check_ids(self.eng.T)
        _, host = batch.packed(self.caps)
        src = torch.from_numpy(host)
        self.blob.copy_(src.to(self.dev, non_blocking=True) if self.blob.device != src.device else src)
        if self.eng.K > 0 and batch.laplacian_pe is not None:
            pe = batch.laplacian_pe
            self.node_pe_buf[: pe.shape[0]].copy_(pe.to(self.dev, torch.float32))
            return True
        return False

    def load_blob(self, blob: torch.Tensor):
        """D2D copy of a pre-staged packed blob of the same capacities."""
        self.blob.copy_(blob, non_blocking=True)

    def attach_builder(self, builder, num_batches: int | None = None, extra=()):
        """Build every batch on the device inside the step (etpgt.data.gpu_batch): each
        ``run()`` first writes the builder's next batch into the batch image, and the
        build is captured in the step's hipGraph with the rest.  Capacities cover the
        builder's next ``num_batches`` batches (default: one epoch of its order) and the
        ``(position, sessions)`` windows of ``extra``."""
        caps = self._planned_caps(builder, num_batches, extra)
        if self.caps is None or not self.caps.fits(caps.n_cap, caps.b_cap, caps.e_cap, caps.n_neg):
            self._bind(caps if self.caps is None else self.caps.grow(caps.n_cap, caps.b_cap, caps.e_cap, caps.n_neg))
        self.builder = builder
        self.graph = self.graph_pe = self.graph_b = None
        self.resident_graphs = None
        self._gen += 1

    def _planned_caps(self, builder, num_batches: int | None, extra=()) -> Caps:
        """Capacities of the builder's next batches; data parallel: agreed over the ranks
        FIRST, so that every rank takes the same rebind decision (a rank-local one would
        leave the others waiting in _bind's collective)."""
        caps = builder.plan_caps(num_batches, int(builder.cursor.item()), extra)
        if caps.n_neg != (self.caps.n_neg if self.caps is not None else caps.n_neg):
            raise ValueError("the number of negatives per session must stay fixed")
        return self._agree(caps)

    def refresh_builder_caps(self, num_batches: int | None = None, extra=()):
        """Grow the capacities if the attached builder's next ``num_batches`` batches need it
        (collective in data parallel); the captured graphs survive when nothing grows."""
        if self.builder is None:
            raise RuntimeError("no device batch builder attached")
        caps = self._planned_caps(self.builder, num_batches, extra)
        if not self.caps.fits(caps.n_cap, caps.b_cap, caps.e_cap, caps.n_neg):
            self.attach_builder(self.builder, num_batches, extra)

    def detach_builder(self):
        self.builder = None
        self.graph = self.graph_pe = self.graph_b = None
        self.resident_graphs = None
        self._gen += 1

    # ------------------------------------------------------------------ launches
    def _sync_alloc(self):
        """Gather buffers of the SyncBN partials: per layer, every rank's forward
        (count, mean, M2) rows and backward (sum dy, sum dy*xhat) rows."""
        eng, ws, W = self.eng, self.ws, self.world
        D, Lc = eng.D, eng.L
        g = ws.g_cap
        rg = readout_grid(self.caps.b_cap)
        self.sync_bufs = []
        # one rank: the "gathered" partials ARE the producer's own rows, so the consumers read
        # them in place and no gather (a copy per BatchNorm, four per step at L = 2) runs;
        # GTR_SYNC_NOALIAS=1 keeps the copies (a one-rank rehearsal of the gathers)
        self.sync_alias = W == 1 and os.environ.get("GTR_SYNC_NOALIAS") != "1"
        for l in range(Lc):
            # fused kernels: every row group's partial rows; split path: ONE merged forward row
            # (count, mean, M2) and the finalized backward sums per rank (gtr_config.split_sync)
            rows_f = 1 if self.split else g
            rows_b = 1 if self.split else (rg if l == Lc - 1 else g)
            st = ws.structs[l]
            if self.sync_alias:
                pa = ws.layers[l]["bn_part"]
                ga = ws.layers[l]["bn_gsum" if self.split else "bn_gpart"]
            else:
                pa = torch.zeros(W, rows_f * (1 + 2 * D), dtype=torch.float32, device=self.dev)
                ga = torch.zeros(W, rows_b * 2 * D, dtype=torch.float32, device=self.dev)
            st.bn_part_all, st.bn_gpart_all = pa.data_ptr(), ga.data_ptr()
            st.nparts_fwd, st.nparts_bwd = W * rows_f, W * rows_b
            self.sync_bufs.append((pa, ga, rows_f * (1 + 2 * D), rows_b * 2 * D))
        self.cfg.consumer_reduce = 1
        self.cfg.sync_bn = 1
        self.cfg.split_sync = 1 if self.split else 0

    def _gather_fwd(self, l):
        from etpgt.train.distributed import all_gather_packs

        if self.sync_alias:
            return
        pa, _, n, _ = self.sync_bufs[l]
        all_gather_packs(pa, self.ws.layers[l]["bn_part"].view(-1)[:n], self.group)

    def _gather_bwd(self, l):
        from etpgt.train.distributed import all_gather_packs

        if self.sync_alias:
            return
        _, ga, _, n = self.sync_bufs[l]
        src = self.ws.layers[l]["bn_gsum" if self.split else "bn_gpart"]
        all_gather_packs(ga, src.view(-1)[:n], self.group)

    def _begin(self, bs, st):
        eng = self.eng
        lib = L.lib()
        if self.builder is not None:
            self.builder.launch(bs, self.caps, st, self._builder_B)
        if self.begin_fused:  # runs inside conv_fwd(0)
            return
        if self.lazy:
            L.check(lib.gtr_step_begin_lazy(C.byref(bs), eng.T, eng.D, self.keys.data_ptr(), self.vals.data_ptr(),
                                            self.skeys.data_ptr(), self.svals.data_ptr(), self.stamp.data_ptr(),
                                            self.step_dev.data_ptr(), eng.rng_ctr.data_ptr(),
                                            self.sort_tmp.data_ptr(), self.sort_tmp.numel(), C.byref(self.lz), st),
                    "step_begin_lazy")
        else:
            L.check(lib.gtr_step_begin(C.byref(bs), eng.T, self.keys.data_ptr(), self.vals.data_ptr(),
                                       self.skeys.data_ptr(), self.svals.data_ptr(), self.stamp.data_ptr(),
                                       self.step_dev.data_ptr(), eng.rng_ctr.data_ptr(), self.sort_tmp.data_ptr(),
                                       self.sort_tmp.numel(), st), "step_begin")

    def _launch_a(self, with_pe: bool):
        """[device batch build] -> step_begin -> forward + loss -> backward (+ the DP pack)."""
        eng = self.eng
        ws, cfg = self.ws, self.cfg
        bs = self.bs_pe if with_pe else self.bs
        st = torch.cuda.current_stream(self.dev).cuda_stream
        self._begin(bs, st)
        eng.run_forward(ws, cfg, bs, L.RO_FWD | L.RO_LOSS | L.RO_BWD, self.loss_kind, self.temperature, self.alpha,
                        split=self.split)
        eng.run_backward(ws, cfg, bs, wgrad=not self.tail_wgrad, split=self.split)
        if self.dp is not None:
            self.dp.launch_pack(bs, st)

    def _launch_b(self, with_pe: bool):
        """Optimizer tail: local (step_tail) or rank-averaged (dp_tail)."""
        eng = self.eng
        bs = self.bs_pe if with_pe else self.bs
        st = torch.cuda.current_stream(self.dev).cuda_stream
        if self.dp is not None:
            self.dp.launch_tail(bs, st)
        elif self.tail_wgrad:
            pe = self.model.laplacian_pe._cached_pe if eng.K > 0 else None
            ws = self.ws
            L.check(L.lib().gtr_step_tail_wgrad(C.byref(self.cfg), C.byref(bs), ws.structs,
                                                None if pe is None else pe.data_ptr(), ws.slab_ptrs,
                                                None if ws.pe_slab is None else ws.pe_slab.data_ptr(), ws.P,
                                                eng.flat.layout.slab_stride, self.layer_flat, self.pe_flat, eng.T,
                                                C.byref(self.tail), self.segs_gb, self.nseg_gb, C.byref(self.adam),
                                                self.tile_cnt.data_ptr(), self.tile_cnt.numel(), st),
                    "step_tail_wgrad")
        else:
            L.check(L.lib().gtr_step_tail(C.byref(bs), eng.T, eng.D, C.byref(self.tail), self.segs, self.nseg,
                                          C.byref(self.adam), st), "step_tail")

    def _pieces(self, with_pe: bool):
        """The step as (launches, collective-after) pieces: one piece single-GPU; the
        halves around the gradient all-gather in DP mode; with SyncBN also a cut after
        every producer of BatchNorm partials (all-gather of the partials)."""
        if self.shard is not None:
            # a launch or capture that raised between fork() and join() (e.g. a refused RCCL
            # capture retried piece by piece) must not leave later launches on the forked stream
            self.shard.forked = False
            return self._shard_pieces(with_pe)
        if self.dp is None:
            def whole():
                self._launch_a(with_pe)
                self._launch_b(with_pe)
            return [(whole, None)]
        if not self.sync_bn and not (self.early_union and self.sweep is not None):
            return [(lambda: self._launch_a(with_pe), self.dp.exchange), (lambda: self._launch_b(with_pe), None)]
        if not self.sync_bn:
            return self._early_pieces(with_pe)
        eng, ws, cfg = self.eng, self.ws, self.cfg
        bs = self.bs_pe if with_pe else self.bs
        lib = L.lib()
        Lc = eng.L

        def st():
            return torch.cuda.current_stream(self.dev).cuda_stream

        ffn = ws.ffns is not None  # a layer's BatchNorm is then folded by its FFN's first GEMM

        def fwd(l):
            def f():
                if l == 0:
                    self._begin(bs, st())
                if ffn and l > 0:
                    eng.ffn_fwd(ws, cfg, bs, l - 1, st())
                eng.layer_fwd(ws, cfg, bs, l, eng.fill_embed(), st(), self.split)
            return f

        def head():
            if ffn:
                eng.ffn_fwd(ws, cfg, bs, Lc - 1, st())
            eng.run_head(ws, cfg, bs, L.RO_FWD | L.RO_LOSS | L.RO_BWD, self.loss_kind, self.temperature, self.alpha)
            if ffn:  # layer Lc-1's dy and BatchNorm sums come from its FFN's backward
                eng.ffn_bwd(ws, cfg, bs, Lc - 1, st())

        def bwd(l):
            def f():
                eng.layer_bwd(ws, cfg, bs, l, st(), self.split)
                if ffn and l > 0:
                    eng.ffn_bwd(ws, cfg, bs, l - 1, st())
                if l == 0:
                    eng._wgrad(ws, cfg, bs, 0, Lc, st())
                    self.dp.launch_pack(bs, st())
            return f

        pieces = [(fwd(l), (lambda l=l: self._gather_fwd(l))) for l in range(Lc)]
        pieces.append((head, lambda: self._gather_bwd(Lc - 1)))
        for l in range(Lc - 1, 0, -1):
            pieces.append((bwd(l), (lambda l=l: self._gather_bwd(l - 1))))
        pieces.append((bwd(0), self.dp.exchange))
        pieces.append((lambda: self._launch_b(with_pe), None))
        return pieces

    def _shard_pieces(self, with_pe: bool):
        """Row-sharded table: begin + route | A2A ids | serve | A2A rows | forward, loss,
        backward (SyncBN: cut after every BatchNorm partial producer) + pack | A2A grads +
        all-gather of the small packs | owner update (etpgt.train.sharded)."""
        eng, ws, cfg, sh = self.eng, self.ws, self.cfg, self.shard
        bs = self.bs_pe if with_pe else self.bs
        bc = sh.compact(with_pe)
        lib = L.lib()
        Lc = eng.L
        tab = sh.table_ptr()

        def st():
            return torch.cuda.current_stream(self.dev).cuda_stream

        def begin_route():
            if self.builder is not None:
                self.builder.launch(bs, self.caps, st(), self._builder_B)
            L.check(lib.gtr_step_begin(C.byref(bs), eng.T, self.keys.data_ptr(), self.vals.data_ptr(),
                                       self.skeys.data_ptr(), self.svals.data_ptr(), None, self.step_dev.data_ptr(),
                                       eng.rng_ctr.data_ptr(), self.sort_tmp.data_ptr(), self.sort_tmp.numel(), st()),
                    "step_begin")
            sh.route(bs, st())

        ffn = ws.ffns is not None  # FFN blocks: placed as in _pieces (a layer's BatchNorm folded by its FFN)

        def fwd(l):
            with sh.side():  # beside the class-1 (scoring) rows' exchange when forked
                if ffn and l > 0:
                    eng.ffn_fwd(ws, cfg, bc, l - 1, st())
                eng.layer_fwd(ws, cfg, bc, l, eng.fill_embed(tab), st(), self.split)

        def head():
            sh.join()
            if ffn:
                eng.ffn_fwd(ws, cfg, bc, Lc - 1, st())
            eng.run_head(ws, cfg, bc, L.RO_FWD | L.RO_LOSS | L.RO_BWD, self.loss_kind, self.temperature, self.alpha,
                         table=tab)
            if ffn:  # layer Lc-1's dy and BatchNorm sums come from its FFN's backward
                eng.ffn_bwd(ws, cfg, bc, Lc - 1, st())

        # the scoring rows beside the forward and the gradient rows beside the weight
        # gradients: RCCL, the step captured whole (or eager) -- never across the
        # boundaries of separately captured pieces
        overlap = sh.can_overlap and (not self.use_graph or self._graph_collectives())

        def bwd(l):
            eng.layer_bwd(ws, cfg, bc, l, st(), self.split)
            if ffn and l > 0:
                eng.ffn_bwd(ws, cfg, bc, l - 1, st())
            if l == 0:
                if overlap:  # gradient rows packed first; they travel beside the weight gradients
                    sh.pack(bs, st(), parts=1)
                    sh.fork()
                    with sh.side():
                        eng._wgrad(ws, cfg, bc, 0, Lc, st())
                        sh.pack(bs, st(), parts=2)
                else:
                    eng._wgrad(ws, cfg, bc, 0, Lc, st())
                    sh.pack(bs, st())

        last = sh.exchange_grads
        pieces = [(begin_route, sh.exchange_ids), (lambda: sh.serve(st()), lambda: sh.exchange_rows(overlap))]
        if not self.sync_bn:
            def middle():
                for l in range(Lc):
                    fwd(l)
                head()
                for l in range(Lc - 1, -1, -1):
                    bwd(l)
            pieces.append((middle, last))
        else:
            for l in range(Lc):
                pieces.append(((lambda l=l: fwd(l)), (lambda l=l: (sh.join(), self._gather_fwd(l)))))
            pieces.append((head, lambda: self._gather_bwd(Lc - 1)))
            for l in range(Lc - 1, 0, -1):
                pieces.append(((lambda l=l: bwd(l)), (lambda l=l: self._gather_bwd(l - 1))))
            pieces.append(((lambda: bwd(0)), last))
        pieces.append((lambda: sh.update(st()), None))
        return pieces

    def _shard_guard(self):
        """Model hook (forward / predict / state_dict): the item table of a sharded step
        lives in the ranks' shards; reading the model's copy needs sync_table() first."""
        if self.shard_state is not None and self.shard_state.stale:
            raise RuntimeError("the item table is row-sharded across the ranks: call "
                               "FusedTrainStep.sync_table() on every rank before reading the model")

    def sync_table(self):
        """Collective (every rank): bring the shards to the current step and write the full
        table into the model's item_embedding.weight (and the moments into m_tab / v_tab)."""
        if self.shard_state is None:
            self.flush()
            return
        self.shard_state.check_status(block=True)
        tab, m, v = self.shard_state.gather_table()
        with torch.no_grad():
            self.model.item_embedding.weight.data.copy_(tab)
        self.m_tab, self.v_tab = m, v
        self.shard_state.stale = False

    def _early_pieces(self, with_pe: bool):
        """DP with the early union: begin | all-gather the sorted keys (async, overlapped
        with the forward) | forward | wait + union stamp + readout + backward (carrying the
        sweep slices) + pack | all-gather the packs | dp tail (touched rows only)."""
        from etpgt.train.distributed import start_all_gather

        eng, ws, cfg = self.eng, self.ws, self.cfg
        bs = self.bs_pe if with_pe else self.bs
        lib = L.lib()

        def st():
            return torch.cuda.current_stream(self.dev).cuda_stream

        pending = {}

        def begin():
            self._begin(bs, st())

        def keys_start():
            pending["w"] = start_all_gather(self.keys_all, self.skeys, self.group)

        def fwd():
            emb = eng.fill_embed()
            for l in range(eng.L):
                eng.layer_fwd(ws, cfg, bs, l, emb, st(), self.split)

        def keys_wait():
            pending.pop("w").wait()

        def rest():
            L.check(lib.gtr_dp_union_stamp(self.keys_all.data_ptr(), self.keys_all.numel(), eng.T,
                                           self.stamp.data_ptr(), self.step_dev.data_ptr(), st()), "dp_union_stamp")
            eng.run_head(ws, cfg, bs, L.RO_FWD | L.RO_LOSS | L.RO_BWD, self.loss_kind, self.temperature, self.alpha)
            eng.run_backward(ws, cfg, bs, split=self.split)
            self.dp.launch_pack(bs, st())

        return [(begin, keys_start), (fwd, keys_wait), (rest, self.dp.exchange),
                (lambda: self._launch_b(with_pe), None)]

    def _graph_collectives(self) -> bool:
        """RCCL collectives captured inside the step's hipGraph (one graph per step instead
        of one per piece).  Only for the nccl (RCCL) backend -- gloo round-trips through
        host memory -- and off with GTR_GRAPH_COLL=0."""
        if (self.dp is None and self.shard is None) or self.world <= 1 and os.environ.get("GTR_GRAPH_COLL") != "1":
            return False
        if os.environ.get("GTR_GRAPH_COLL", "1") == "0" or self._coll_capture_refused:
            return False
        import torch.distributed as dist

        return dist.is_available() and dist.is_initialized() and dist.get_backend(self.group) == "nccl"

    def _collective_free(self) -> bool:
        """True when no piece of the step runs a real collective: one rank with aliased
        exchange buffers (DpExchange.alias / ShardExchange.alias), no SyncBN gathers, no
        early union -- the pieces then run as ONE graph, with no host launch between them."""
        if (self.sync_bn and not self.sync_alias) or self.early_union:
            return False
        if self.shard is not None:
            return self.shard.alias
        if self.dp is not None:
            return self.dp.alias
        return True

    def _one_graph(self) -> bool:
        """The whole step captured as one graph (collective-free, or RCCL collectives
        captured inside it)."""
        return self._collective_free() or self._graph_collectives()

    def _graph_pieces(self, with_pe: bool):
        pieces = self._pieces(with_pe)
        if len(pieces) == 1 or not self._one_graph():
            return pieces

        def whole():
            for launch, coll in pieces:
                launch()
                if coll is not None:
                    coll()
        return [(whole, None)]

    def _launch(self, with_pe: bool):
        for launch, coll in self._pieces(with_pe):
            launch()
            if coll is not None:
                coll()

    def _capture(self, fn):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.graph(g, stream=s):
            fn()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        return g

    def bind_resident(self, blobs):
        """Zero-copy steps over packed batch images already resident in HBM (the same
        capacities as the step's own blob): each image gets its own batch struct and, on
        first use, its own captured graph, so ``run_resident(i)`` launches straight on
        image i instead of copying it into the step's blob first."""
        if self.caps is None:
            raise RuntimeError("bind the step's capacities first (load one batch)")
        if self.shard is not None:
            raise NotImplementedError("resident batch images are not supported with the row-sharded table")
        n = self.blob.numel()
        for b in blobs:
            if b.numel() != n or b.dtype != self.blob.dtype or b.device != self.blob.device:
                raise ValueError("resident images must match the step's blob (size, dtype, device)")
        self.resident = [(b, self.eng.batch_struct(self.caps, b, None)) for b in blobs]
        self.resident_graphs = None
        self._gen += 1

    def _with_bs(self, bs, fn):
        saved = self.bs
        self.bs = bs
        try:
            return fn()
        finally:
            self.bs = saved

    def prepare_resident(self):
        """Capture every resident image's graph now (after at least one eager step), so
        that no capture falls into a timed region."""
        if self.resident is None:
            raise RuntimeError("bind_resident first")
        if self.resident_graphs is None:
            self.resident_graphs = [None] * len(self.resident)
        for i, (_, bs) in enumerate(self.resident):
            if self.resident_graphs[i] is None:
                self.resident_graphs[i] = self._with_bs(bs, lambda: self._capture_pieces(False))

    def run_resident(self, i: int):
        """One training step over resident image i (see bind_resident)."""
        if self.resident is None:
            raise RuntimeError("bind_resident first")
        self.eng.check_intact()
        if not self.model.training:
            raise RuntimeError("FusedTrainStep requires model.train()")
        if self.lazy:
            if self._host_steps + 2 >= self.lz.cap:
                self._lazy_alloc(2 * self.lz.cap)
            self._host_steps += 1
            self._dirty = True
        bs = self.resident[i][1]
        if not self.use_graph:
            self._with_bs(bs, lambda: self._launch(False))
            return self.ws.loss_out[0]
        if self.resident_graphs is None:
            self.resident_graphs = [None] * len(self.resident)
        graphs = self.resident_graphs[i]
        if graphs is None:
            self._with_bs(bs, lambda: self._launch(False))  # eager step (first touch), then capture
            torch.cuda.synchronize(self.dev)
            self.resident_graphs[i] = self._with_bs(bs, lambda: self._capture_pieces(False))
            return self.ws.loss_out[0]
        for g, coll in graphs:
            g.replay()
            if coll is not None:
                coll()
        return self.ws.loss_out[0]

    def capture_steps(self, start: int, n: int) -> dict:
        """``n`` consecutive training steps over the resident images start, start + 1, ...
        (mod their count) captured as ONE hipGraph: the steps' launches follow each other
        inside the graph, so the queue runs step after step without a graph launch -- and
        its host round trip -- between them.  Single GPU only (the data-parallel and
        sharded steps keep their collectives between graph pieces).  Every step is the
        full step (``run_resident`` of the same images n times, launch for launch); the
        handle is for ``run_steps``."""
        if self.resident is None:
            raise RuntimeError("bind_resident first")
        if not self.use_graph:
            raise RuntimeError("capture_steps needs use_graph=True")
        if self.dp is not None or self.shard_state is not None or self.world > 1:
            raise NotImplementedError("multi-step graphs are single-GPU: collectives stay between graph pieces")
        if n <= 0:
            raise ValueError("capture_steps needs n >= 1")
        nimg = len(self.resident)

        def fn():
            for k in range(n):
                bs = self.resident[(start + k) % nimg][1]
                self._with_bs(bs, lambda: self._launch(False))

        return {"graph": self._capture(fn), "n": int(n), "lz_cap": self.lz.cap if self.lazy else None,
                "gen": self._gen}

    def capture_steps_copied(self, images, start: int, n: int, reserve: int = 0) -> dict | None:
        """``n`` consecutive data-parallel steps, each copying pre-staged image
        (start + k) mod len(images) into the step's blob (the D2D copy ``load_blob`` makes)
        and running the step with its RCCL collectives, captured as ONE hipGraph.  Only
        where the collectives are captured in the step's graph anyway (RCCL, N > 1 or
        GTR_GRAPH_COLL=1), or where the step has none (one rank, aliased exchange buffers).  Every rank captures, then the ranks agree (all-reduce outside
        any capture): if any rank's capture was refused, every rank returns None and keeps
        the per-step path.  The per-step constants (row-sharded table, lazy table) are
        grown first for ``reserve`` more steps (their pointers are captured)."""
        if not self.use_graph or not self._one_graph():
            return None
        if n <= 0:
            raise ValueError("capture_steps_copied needs n >= 1")
        nimg = len(images)
        for img in images:
            if img.numel() != self.blob.numel() or img.dtype != self.blob.dtype or img.device != self.blob.device:
                raise ValueError("images must match the step's blob (size, dtype, device)")

        def fn():
            for k in range(n):
                self.blob.copy_(images[(start + k) % nimg], non_blocking=True)
                self._launch(False)

        return self._capture_multi(fn, n, reserve, collective=not self._collective_free())

    def capture_steps_built(self, n: int, reserve: int = 0) -> dict | None:
        """``n`` consecutive steps over the attached device batch builder's next batches
        (``attach_builder``: each step's captured build writes the next batch into the
        blob and advances the device cursor by the global batch) as ONE hipGraph -- the
        drop-in ``Trainer``'s epoch loop (trainer.py:80-133) runs its full batches in such
        chunks.  Single GPU, or data parallel with RCCL collectives captured in the step;
        None where the step cannot be captured whole (gloo: collectives between graph
        pieces), and then on every rank.  Replay with ``run_steps``; every step is the full
        step of ``run()``."""
        if self.builder is None:
            raise RuntimeError("capture_steps_built needs a device batch builder (attach_builder)")
        if n <= 0:
            raise ValueError("capture_steps_built needs n >= 1")
        multi = self.dp is not None or self.shard is not None
        if not self.use_graph or (multi and not self._one_graph()):
            return None

        def fn():
            for _ in range(n):
                self._launch(False)

        return self._capture_multi(fn, n, reserve, collective=multi and not self._collective_free())

    def _capture_multi(self, fn, n: int, reserve: int, collective: bool) -> dict | None:
        """Capture ``fn`` (n steps) as one graph after growing the per-step constants for
        ``reserve`` more steps; with collectives, every rank agrees on refusal."""
        need = self._host_steps + max(reserve, n) + 2
        if self.lazy and need >= self.lz.cap:
            cap = self.lz.cap
            while need >= cap:
                cap *= 2
            self._lazy_alloc(cap)
        if self.shard_state is not None and self.shard_state.ensure_steps(need):
            self.graph = self.graph_pe = self.graph_b = None  # consts moved: the per-step graphs recapture
            self.resident_graphs = None
            self._gen += 1
        g, err = None, None
        if not collective:
            g = self._capture(fn)
        else:
            try:
                g = self._capture(fn)
            except RuntimeError as e:
                if "captur" not in str(e).lower():
                    raise
                err = e
                torch.cuda.synchronize(self.dev)
            if self._ranks_agree_refused(err is not None):
                return None
        return {"graph": g, "n": int(n), "lz_cap": self.lz.cap if self.lazy else None,
                "consts": self.shard_state.consts.data_ptr() if self.shard_state is not None else None,
                "gen": self._gen}

    def stale_reason(self, h: dict) -> str | None:
        """Why a multi-step handle can no longer be replayed (None: it can): its captured
        buffers were rebound (``_gen``), or the per-step constants it points at were -- or
        for its ``h["n"]`` more steps would have to be -- reallocated."""
        n = h["n"]
        if h.get("gen") != self._gen:
            return "the step's buffers were rebound since this multi-step graph was captured: capture the steps again"
        if self.shard_state is not None:
            ss = self.shard_state
            if h.get("consts") != ss.consts.data_ptr() or self._host_steps + n + 2 >= ss.consts.shape[0]:
                return ("the row-sharded table's step constants were (or would have to be) reallocated: "
                        "capture the steps again")
        if self.lazy and (h["lz_cap"] != self.lz.cap or self._host_steps + n + 2 >= self.lz.cap):
            return "the lazy table's step constants were (or would have to be) reallocated: capture the steps again"
        return None

    def run_steps(self, h: dict):
        """Replay a ``capture_steps`` / ``capture_steps_copied`` graph: ``h["n"]`` training
        steps in one launch.  Every check runs before any state changes: a handle whose
        captured buffers were rebound since (``_gen``), or whose per-step constants would
        have to grow, raises and leaves the step untouched."""
        self.eng.check_intact()
        if not self.model.training:
            raise RuntimeError("FusedTrainStep requires model.train()")
        n = h["n"]
        why = self.stale_reason(h)
        if why is not None:
            raise RuntimeError(why)
        self._host_steps += n
        if self.lazy:
            self._dirty = True
        if self.shard_state is not None:
            self.shard_state.check_status(steps=n)
        h["graph"].replay()
        return self.ws.loss_out[0]

    def _capture_pieces(self, with_pe: bool):
        if not self._graph_collectives():
            return [(self._capture(launch), coll) for launch, coll in self._graph_pieces(with_pe)]
        graphs, err = None, None
        try:
            graphs = [(self._capture(launch), coll) for launch, coll in self._graph_pieces(with_pe)]
        except RuntimeError as e:
            if "captur" not in str(e).lower():
                raise
            err = e
            torch.cuda.synchronize(self.dev)
        # a transport that refuses stream capture: keep the collectives between graph pieces,
        # for this step object only -- and on every rank, so the ranks agree first (every
        # rank reaches this all-reduce whether its own capture succeeded or not)
        if self._ranks_agree_refused(err is not None):
            import warnings

            self._coll_capture_refused = True
            warnings.warn(f"capturing the collectives failed ({err or 'on another rank'}); "
                          "falling back to one graph per piece")
            graphs = [(self._capture(launch), coll) for launch, coll in self._graph_pieces(with_pe)]
        return graphs

    def _ranks_agree_refused(self, refused: bool) -> bool:
        """True if any rank's capture of the collectives was refused (MAX all-reduce,
        outside any capture)."""
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()) or self.world <= 1:
            return refused
        dev = self.dev if dist.get_backend(self.group) != "gloo" else "cpu"
        t = torch.tensor([int(refused)], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return bool(t.item())

    def capture(self, with_pe: bool = False):
        """Capture the step's pieces into hipGraphs (after one eager warm-up step): the
        whole step single-GPU; the pieces between collectives in DP mode."""
        graphs = self._capture_pieces(with_pe)
        if with_pe:
            self.graph_pe = graphs
        else:
            self.graph = graphs
        return graphs

    def run_partial(self, B: int):
        """One step whose device-built batch holds ``B`` sessions instead of the builder's
        batch size (the last, partial batch of an epoch, as a DataLoader with
        drop_last=False yields it): launched eagerly, the captured graph keeps the full
        batch size."""
        if self.builder is None:
            raise RuntimeError("run_partial needs a device batch builder (attach_builder)")
        self._builder_B = int(B)
        try:
            return self.run(eager=True)
        finally:
            self._builder_B = None

    def run(self, with_pe: bool = False, eager: bool = False):
        """One training step over the batch currently in the device blob."""
        self.eng.check_intact()
        if not self.model.training:
            raise RuntimeError("FusedTrainStep requires model.train()")
        if self.shard_state is not None:
            self._host_steps += 1
            if self.shard_state.ensure_steps(self._host_steps):
                self.graph = self.graph_pe = self.graph_b = None  # consts moved: recapture
                self.resident_graphs = None
                self._gen += 1
            self.shard_state.check_status(steps=1)
        if self.lazy:
            if self._host_steps + 2 >= self.lz.cap:
                self._lazy_alloc(2 * self.lz.cap)
            self._host_steps += 1
            self._dirty = True
        if self.use_graph and not eager:
            graphs = self.graph_pe if with_pe else self.graph
            if graphs is None:
                self._launch(with_pe)  # eager warm-up (first touch of every code path)
                torch.cuda.synchronize(self.dev)
                self.capture(with_pe)
                return self.ws.loss_out[0]
            for g, coll in graphs:
                g.replay()
                if coll is not None:
                    coll()
        else:
            self._launch(with_pe)
        return self.ws.loss_out[0]

    def __call__(self, batch: SessionBatch):
        if self.eng.K > 0 and batch.laplacian_pe is None and self.model.laplacian_pe._cached_pe is None:
            raise RuntimeError("Laplacian PE not precomputed. Call precompute() first.")
        N = batch.sizes()[0]
        if N <= 1:
            raise ValueError("Expected more than 1 value per channel when training (BatchNorm1d)")
        with_pe = self.load(batch)
        return self.run(with_pe)

    def close(self):
        """Drop every captured graph of this step (per-step, per-image and, by bumping the
        binding generation, the multi-step handles callers hold -- those must be dropped by
        their holders too) and drain the device.  A graph that captured an RCCL collective
        pins its communicator: ``dist.destroy_process_group()`` does not return while such
        a graph is alive (scripts/dbg/teardown_probe.py), so multi-rank drivers call this
        first.  The step stays usable: the next ``run`` captures again."""
        import gc

        self.graph = self.graph_pe = self.graph_b = None
        self.resident_graphs = None
        self._gen += 1
        gc.collect()
        torch.cuda.synchronize(self.dev)

    # ------------------------------------------------------------------ state
    @property
    def steps(self) -> int:
        return int(self.step_dev.item())

    def export_optimizer_state(self, optimizer: torch.optim.Optimizer):
        """Write exp_avg / exp_avg_sq / step into a torch Adam(W) optimizer's state
        (row-sharded table: collective, gathers the shards first)."""
        if self.shard_state is not None:
            self.sync_table()
        self.flush()
        t = torch.tensor(float(self.steps))
        tab = self.model.item_embedding.weight
        views_m = self.eng.flat.grad_views(self.m_flat)
        views_v = self.eng.flat.grad_views(self.v_flat)
        pm = {id(p): (m, v) for p, m, v in zip(self.eng.flat.params(), views_m, views_v)}
        pm[id(tab)] = (self.m_tab, self.v_tab)
        for group in optimizer.param_groups:
            for p in group["params"]:
                if id(p) in pm:
                    m, v = pm[id(p)]
                    optimizer.state[p] = {"step": t.clone(), "exp_avg": m.clone(), "exp_avg_sq": v.clone()}
