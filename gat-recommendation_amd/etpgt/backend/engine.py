"""Device-side engine of the GraphTransformer hot path.

Owns (per model):
  * the flat dense-parameter buffer: every parameter except the item table is a
    view into one fp32 buffer laid out in 256-aligned segments
    [w_all (query,key,value,skip) | b_all | w_beta | bn_gamma | bn_beta] per layer
    and [wpe | bpe] for the LapPE projection, so one kernel updates them all;
  * per-capacity workspaces (saved activations, gradient slabs, arrival counters);
  * the ctypes argument structs, built once per workspace so a launch costs one
    foreign call.

Kernel order of one training step:
  conv_fwd(0..L-1) -> readout_loss(FWD|LOSS|BWD) -> conv_bwd(L-1..0) -> wgrad
  -> adamw_rows + adamw_small (-> step_end); contrib_prep -> adamw_sweep and
  contrib_sort run on side streams, overlapped with the chain.
"""

from __future__ import annotations

import ctypes as C
import os
import math
from dataclasses import dataclass

import torch

from etpgt.backend import _lib as L
from etpgt.data.batch import Caps, SessionBatch, blob_layout

ALIGN = 256


def _al(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass
class Seg:
    name: str
    begin: int
    numel: int
    shape: tuple


class ParamLayout:
    """Flat layout of the dense (non-table) parameters of a GraphTransformer."""

    def __init__(self, D: int, L_: int, pe_k: int, ffn: bool = False, ffn_expansion: int = 4):
        self.D, self.L, self.K, self.ffn = D, L_, pe_k, ffn
        F = ffn_expansion * D
        self.F = F if ffn else 0
        self.segs: dict[str, Seg] = {}
        off = 0

        def add(name, shape):
            nonlocal off
            n = int(math.prod(shape))
            self.segs[name] = Seg(name, off, n, tuple(shape))
            off += _al(n)

        for l in range(L_):
            add(f"{l}.w_all", (4 * D, D))
            add(f"{l}.b_all", (4 * D,))
            add(f"{l}.w_beta", (1, 3 * D))
            add(f"{l}.gamma", (D,))
            add(f"{l}.beta", (D,))
            if ffn:  # ffns.{l}.0 / ffns.{l}.3 (graph_transformer.py:88-100), F = ffn_expansion * D
                add(f"{l}.ffn_w1", (F, D))
                add(f"{l}.ffn_b1", (F,))
                add(f"{l}.ffn_w2", (D, F))
                add(f"{l}.ffn_b2", (D,))
        if pe_k > 0:
            add("pe.w", (D, pe_k))
            add("pe.b", (D,))
        self.total = off
        self.layer_block = 4 * D * D + 4 * D + 3 * D   # slab layout of one layer
        self.pe_block = D * pe_k + D if pe_k > 0 else 0
        self.slab_stride = _al(max(self.layer_block, self.pe_block))
        # gtr_ffn_wgrad slab of one layer: [dW1 F*D | db1 F | dW2 D*F | db2 D]
        self.ffn_block = 2 * F * D + F + D if ffn else 0
        self.ffn_stride = _al(self.ffn_block) if ffn else 0

    def seg(self, name: str) -> Seg:
        return self.segs[name]


def model_param_map(model) -> list[tuple[str, torch.nn.Parameter, int]]:
    """(flat segment, parameter, row offset) for every dense parameter of the model."""
    D = model.hidden_dim
    out = []
    for l, (conv, bn) in enumerate(zip(model.convs, model.batch_norms)):
        out += [
            (f"{l}.w_all", conv.lin_query.weight, 0), (f"{l}.w_all", conv.lin_key.weight, D),
            (f"{l}.w_all", conv.lin_value.weight, 2 * D), (f"{l}.w_all", conv.lin_skip.weight, 3 * D),
            (f"{l}.b_all", conv.lin_query.bias, 0), (f"{l}.b_all", conv.lin_key.bias, D),
            (f"{l}.b_all", conv.lin_value.bias, 2 * D), (f"{l}.b_all", conv.lin_skip.bias, 3 * D),
            (f"{l}.w_beta", conv.lin_beta.weight, 0),
            (f"{l}.gamma", bn.weight, 0), (f"{l}.beta", bn.bias, 0),
        ]
        if getattr(model, "use_ffn", False):
            ffn = model.ffns[l]
            out += [(f"{l}.ffn_w1", ffn[0].weight, 0), (f"{l}.ffn_b1", ffn[0].bias, 0),
                    (f"{l}.ffn_w2", ffn[3].weight, 0), (f"{l}.ffn_b2", ffn[3].bias, 0)]
    if model.use_laplacian_pe:
        out += [("pe.w", model.laplacian_pe.projection.weight, 0), ("pe.b", model.laplacian_pe.projection.bias, 0)]
    return out


class FlatParams:
    """Re-points the model's dense parameters at views of one flat device buffer."""

    def __init__(self, model, device):
        self.model = model
        self.layout = ParamLayout(model.hidden_dim, model.num_layers, model.laplacian_k if model.use_laplacian_pe else 0,
                                  bool(getattr(model, "use_ffn", False)), int(getattr(model, "ffn_expansion", 4)))
        self.device = device
        self.flat = torch.zeros(self.layout.total, dtype=torch.float32, device=device)
        self.map = model_param_map(model)
        D = model.hidden_dim
        with torch.no_grad():
            for name, p, row in self.map:
                view = self._view(name, p, row, D)
                view.copy_(p.data.to(device=device, dtype=torch.float32))
                p.data = view
        self._ptrs = self._snapshot()

    def _view(self, name, p, row, D):
        s = self.layout.seg(name)
        n = p.numel()
        start = s.begin + row * (D if name.endswith("w_all") else 1)
        return self.flat[start : start + n].view(p.shape)

    def _snapshot(self):
        return tuple(p.data_ptr() for _, p, _ in self.map)

    def intact(self) -> bool:
        return self._snapshot() == self._ptrs

    def params(self) -> list[torch.nn.Parameter]:
        return [p for _, p, _ in self.map]

    def grad_views(self, flat_grad: torch.Tensor) -> list[torch.Tensor]:
        D = self.model.hidden_dim
        out = []
        for name, p, row in self.map:
            s = self.layout.seg(name)
            start = s.begin + row * (D if name.endswith("w_all") else 1)
            out.append(flat_grad[start : start + p.numel()].view(p.shape))
        return out

    def seg_ptr(self, name: str) -> int:
        return self.flat.data_ptr() + 4 * self.layout.seg(name).begin


def _i32(n, device):
    return torch.zeros(max(int(n), 1), dtype=torch.int32, device=device)


def _f32(*shape, device):
    return torch.zeros(*[max(int(s), 1) for s in shape], dtype=torch.float32, device=device)


def readout_grid(b_cap: int) -> int:
    """Workgroups of gtr_readout_loss (= its loss / BN-sum partial count)."""
    return int(L.lib().gtr_readout_grid(int(b_cap)))


def split_default(D: int, g_cap: int, sync: bool = False) -> bool:
    """The split (GEMM + attention) layer path: GTR_SPLIT=1 / 0 forces it on / off (tests,
    A/B); by default at D in {64, 128} from 513 row groups on (measured, scripts/dbg/kbench.py
    full steps: the fused row-group kernels win up to B = 2048 -- C3 B = 1024 315 vs 363 us,
    B = 2048 414 vs 433; C2 B = 1024 187 vs 248, B = 2048 231 vs 264 -- and the split path
    from B = 3072 / 4096 on).  Under SyncBN across ranks (``sync``) from 129 groups on: the
    split path gathers ONE merged BatchNorm row per rank where the fused kernels gather
    every row group's partials and each consumer workgroup reduces all of them."""
    if D not in (64, 128):
        return False
    e = os.environ.get("GTR_SPLIT")
    if e is not None:
        return e == "1"
    return g_cap > (128 if sync else 512)


class Workspace:
    """Capacity-sized activations + gradient buffers for one in-flight batch."""

    def __init__(self, eng: "Engine", caps: Caps, R: int, P: int, split: bool | None = None, sync: bool = False):
        dev = eng.device
        D, H, Lc = eng.D, eng.H, eng.L
        self.caps, self.R, self.P = caps, R, P
        n, b, e, k = caps.n_cap, caps.b_cap, caps.e_cap, max(caps.n_neg, 1)
        g = (n + R - 1) // R
        self.g_cap = g
        # BatchNorm partial rows: one per row group, or per 8 rows on the split path's
        # row-parallel attention (gtr_attn_fwd); arrival counters: two per bucket of 32
        parts = max(g, (n + 7) // 8)
        self.layers = []
        self.structs = (L.GtrLayer * Lc)()
        for l in range(Lc):
            t = dict(
                xin=_f32(n, D, device=dev), qkvs=_f32(n, 4 * D, device=dev), alpha=_f32(e, H, device=dev),
                agg=_f32(n, D, device=dev), gate=_f32(n, device=dev), out=_f32(n, D, device=dev),
                bn_stats=_f32(2 * D, device=dev), bn_part=_f32(parts, 1 + 2 * D, device=dev),
                bn_gsum=_f32(2 * D, device=dev), bn_gpart=_f32(max(g, 256), 2 * D, device=dev),
                # arrival counters: [0..3] + two per bucket of 32 partial rows -- the row groups
                # or the <= 256 workgroups of the split path's dX GEMM (gtr_qkvs_bwd)
                cnt=_i32(8 + 2 * max((parts + 31) // 32, 8), dev), dy=_f32(n, D, device=dev),
                dqkvs=_f32(n, 4 * D, device=dev),
                du=_f32(n, device=dev), dlogit=_f32(e, H, device=dev), dagg=_f32(n, D, device=dev),
            )
            self.layers.append(t)
        # large batches: each layer as GEMM + attention launches (gtr_qkvs_* / gtr_attn_*)
        # instead of one fused launch -- from more row groups than the chip has CUs / 2
        # (the fused kernels re-fetch W_all per 16-row group), D in {64, 128}
        self.split = split_default(D, g, sync) if split is None else (bool(split) and D in (64, 128))
        if eng.ffn:  # the feed-forward blocks run on the split layer path only
            self.split = True
        self.dx0 = _f32(n, D, device=dev)
        self.se = _f32(b, D, device=dev)
        self.dse_in = _f32(b, D, device=dev)
        self.dse_out = _f32(b, D, device=dev)
        self.coef_tgt = _f32(b, device=dev)
        self.coef_neg = _f32(b * k, device=dev)
        self.loss_part = _f32(512, device=dev)
        self.loss_out = _f32(1, device=dev)
        self.head_cnt = _i32(4, dev)
        lay = eng.flat.layout
        self.slabs = _f32(Lc, P, lay.slab_stride, device=dev)
        self.pe_slab = _f32(P, lay.slab_stride, device=dev) if eng.K > 0 else None
        self.slab_ptrs = (C.c_void_p * Lc)(*[self.slabs[l].data_ptr() for l in range(Lc)])
        self.wfold = None  # [Lc, g_cap, slab_stride]: per-row-group weight-gradient partials
        self.head = L.GtrHead()
        self.ffns = None
        if eng.ffn:
            self._alloc_ffn(eng, n, parts, g)
        self._fill_layer_structs(eng)

    def _alloc_ffn(self, eng, n, parts, g):
        """Feed-forward blocks (gtr_ffn per layer), their weight-gradient slabs, and the
        readout's view of the last layer: an identity BatchNorm layer over ffn.z (statistics
        0 / 1, gamma 1, beta 0, zero residual; run with dropout 0 and eps 0), so the mean
        readout reads z as it is and writes d/dz into ffn.dz."""
        dev = eng.device
        D, Lc = eng.D, eng.L
        F = eng.flat.layout.F
        self.ffns = []
        self.ffn_structs = []
        for l in range(Lc):
            t = dict(y=_f32(n, D, device=dev), a=_f32(n, F, device=dev), z=_f32(n, D, device=dev),
                     dz=_f32(n, D, device=dev), g2=_f32(n, D, device=dev), da=_f32(n, F, device=dev))
            self.ffns.append(t)
            fs = L.GtrFfn()
            for f in ("y", "a", "z", "dz", "g2", "da"):
                setattr(fs, f, t[f].data_ptr())
            fs.expansion = F // D
            self.ffn_structs.append(fs)
        self.ffn_slabs = _f32(Lc, self.P, eng.flat.layout.ffn_stride, device=dev)
        last = self.ffns[Lc - 1]
        self.ro_ident = dict(
            xin=_f32(n, D, device=dev),
            stats=torch.cat([torch.zeros(D), torch.ones(D)]).to(dev),
            gamma=torch.ones(D, device=dev), beta=torch.zeros(D, device=dev),
            rmean=torch.zeros(D, device=dev), rvar=torch.ones(D, device=dev),
            nbt=torch.zeros(1, dtype=torch.int64, device=dev),
            part=_f32(parts, 1 + 2 * D, device=dev), gsum=_f32(2 * D, device=dev),
            gpart=_f32(max(g, 512), 2 * D, device=dev),
            cnt=_i32(8 + 2 * max((parts + 31) // 32, 8), dev),
        )
        r = self.ro_ident
        self.ro_structs = (L.GtrLayer * Lc)()
        s = self.ro_structs[Lc - 1]
        s.out, s.xin, s.bn_stats = last["z"].data_ptr(), r["xin"].data_ptr(), r["stats"].data_ptr()
        s.bn_gamma, s.bn_beta = r["gamma"].data_ptr(), r["beta"].data_ptr()
        s.bn_rmean, s.bn_rvar, s.bn_nbt = r["rmean"].data_ptr(), r["rvar"].data_ptr(), r["nbt"].data_ptr()
        s.bn_part, s.bn_gsum, s.bn_gpart, s.cnt = (r["part"].data_ptr(), r["gsum"].data_ptr(),
                                                   r["gpart"].data_ptr(), r["cnt"].data_ptr())
        s.dy = last["dz"].data_ptr()

    def readout_args(self, cfg):
        """(config, layer structs) of the readout: with FFN blocks the identity view of the
        last block's output (dropout 0, eps 0, fixed statistics: no SyncBN fold -- the last
        layer's BatchNorm was folded by its FFN's first GEMM)."""
        if self.ffns is None:
            return cfg, self.structs
        c = type(cfg).from_buffer_copy(cfg)
        c.dropout = 0.0
        c.bn_eps = 0.0
        c.sync_bn = 0
        c.consumer_reduce = 0
        c.split_sync = 0
        return c, self.ro_structs

    def enable_wfold(self, eng) -> int:
        """Per-row-group weight-gradient partials for the fused backward (gtr_layer.wfold);
        returns the slab stride for gtr_config.wfold_stride."""
        lay = eng.flat.layout
        if self.wfold is None:
            self.wfold = _f32(eng.L, self.g_cap, lay.slab_stride, device=eng.device)
        for l in range(eng.L):
            self.structs[l].wfold = self.wfold[l].data_ptr()
        return lay.slab_stride

    def _fill_layer_structs(self, eng):
        for l, t in enumerate(self.layers):
            s = self.structs[l]
            for f in ("xin", "qkvs", "alpha", "agg", "gate", "out", "bn_stats", "bn_part", "bn_gsum",
                      "bn_gpart", "cnt", "dy", "dqkvs", "du", "dlogit", "dagg"):
                setattr(s, f, t[f].data_ptr())
        self.refresh_params(eng)

    def refresh_params(self, eng):
        for l in range(eng.L):
            s = self.structs[l]
            bn = eng.model.batch_norms[l]
            s.w_all = eng.flat.seg_ptr(f"{l}.w_all")
            s.b_all = eng.flat.seg_ptr(f"{l}.b_all")
            s.w_beta = eng.flat.seg_ptr(f"{l}.w_beta")
            s.bn_gamma = eng.flat.seg_ptr(f"{l}.gamma")
            s.bn_beta = eng.flat.seg_ptr(f"{l}.beta")
            s.bn_rmean = bn.running_mean.data_ptr()
            s.bn_rvar = bn.running_var.data_ptr()
            s.bn_nbt = bn.num_batches_tracked.data_ptr()
            if self.ffns is not None:
                fs = self.ffn_structs[l]
                fs.w1, fs.b1 = eng.flat.seg_ptr(f"{l}.ffn_w1"), eng.flat.seg_ptr(f"{l}.ffn_b1")
                fs.w2, fs.b2 = eng.flat.seg_ptr(f"{l}.ffn_w2"), eng.flat.seg_ptr(f"{l}.ffn_b2")
                s.ffn = C.addressof(fs)


class Engine:
    """Binds a GraphTransformer (reference layout) to libgtr_hip on one device."""

    def __init__(self, model, device: torch.device):
        if device.type != "cuda":
            raise RuntimeError("the GraphTransformer hot path runs on an MI355X (gfx950) GPU only")
        lib = L.lib()
        L.check(lib.gtr_device_check(device.index if device.index is not None else torch.cuda.current_device()),
                "device check")
        self.model = model
        self.device = device
        self.D = model.hidden_dim
        self.H = model.num_heads
        self.L = model.num_layers
        self.K = model.laplacian_k if model.use_laplacian_pe else 0
        self.T = model.num_items
        self.ffn = bool(getattr(model, "use_ffn", False))
        self.flat = FlatParams(model, device)
        self.rng_ctr = torch.zeros(1, dtype=torch.int32, device=device)
        self.seed = int(torch.randint(0, 2**31 - 1, (1,), generator=torch.Generator().manual_seed(0x5EED)).item())
        self.embed = L.GtrEmbed()
        self._ws_cache: dict[Caps, Workspace] = {}
        self._ws_free: dict[Caps, list] = {}  # (workspace, release event) whose backward has run

    # ------------------------------------------------------------------ helpers
    def check_intact(self):
        if not self.flat.intact():
            raise RuntimeError("model parameters were re-allocated after binding the HIP engine "
                               "(e.g. model.to()); re-create the engine")

    def choose_R(self, caps: Caps) -> int:
        return caps.R

    def choose_P(self, caps: Caps) -> int:
        # split-K of the weight gradients: <= 32 node rows per workgroup up to 2048 rows, <= 64
        # slabs (one chunk over ~110 rows made k_wgrad 2x slower at C2: measured 0.105 ->
        # 0.119 ms/step); past 2048 rows chunks of >= 128 rows, where the QKVS tiles run on
        # MFMA (GTR_WGRAD_MFMA_ROWS) -- C5 at B = 1024 (3.5k rows) had 64 VALU chunks of 55
        rows = int(os.environ.get("GTR_WGRAD_ROWS", "0"))  # diagnostics / tuning
        if rows <= 0 and caps.n_cap > 2048:
            return max(1, min(64, caps.n_cap // 128))  # (floor: every chunk >= 128 rows)
        rows = rows if rows > 0 else 32
        return max(1, min(64, (caps.n_cap + rows - 1) // rows))

    def workspace(self, caps: Caps, fresh: bool = False, split: bool | None = None, sync: bool = False) -> Workspace:
        """Workspace of these capacities; ``split`` forces the split (GEMM + attention) layer
        path on or off (None: split_default; ``sync``: SyncBN across ranks)."""
        if fresh:
            return Workspace(self, caps, self.choose_R(caps), self.choose_P(caps), split, sync)
        key = (caps, split, bool(sync))
        ws = self._ws_cache.pop(key, None)
        if ws is None:
            ws = Workspace(self, caps, self.choose_R(caps), self.choose_P(caps), split, sync)
        self._ws_cache[key] = ws  # most recently used last
        while len(self._ws_cache) > 8:
            self._ws_cache.pop(next(iter(self._ws_cache)))
        return ws

    def acquire_workspace(self, caps: Caps) -> Workspace:
        """A workspace owned by one autograd forward until its backward has run: reused
        from the free list (release_workspace) instead of allocating ~40 buffers per step.
        The release recorded an event on the stream of the backward that last used the
        workspace; the acquiring stream waits on it, so a forward on another stream (or
        under another ``torch.cuda.stream`` context) cannot overwrite buffers a queued
        backward still reads."""
        free = self._ws_free.get(caps)
        if not free:
            return self.workspace(caps, fresh=True)
        ws, ev = free.pop()
        torch.cuda.current_stream(self.device).wait_event(ev)
        return ws

    def release_workspace(self, ws: Workspace) -> None:
        free = self._ws_free.setdefault(ws.caps, [])
        if len(free) < 2:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            free.append((ws, ev))

    def config(self, ws: Workspace, training: bool) -> L.GtrConfig:
        m = self.model
        cfg = L.GtrConfig()
        cfg.num_items = self.T
        cfg.dim = self.D
        cfg.heads = self.H
        cfg.pe_k = self.K
        cfg.num_layers = self.L
        cfg.row_group = ws.R
        cfg.training = 1 if training else 0
        cfg.dropout = float(m.dropout)
        bn = m.batch_norms[0]
        cfg.bn_eps = float(bn.eps)
        cfg.bn_momentum = float(bn.momentum if bn.momentum is not None else 0.1)
        cfg.seed = self.seed
        cfg.rng_ctr = self.rng_ctr.data_ptr()
        # consumer-side reduction of BatchNorm partials pays while a consumer block can
        # fold every group's partial in its prologue; large grids use the last arriver
        cred = os.environ.get("GTR_CONSUMER_REDUCE")
        cfg.consumer_reduce = int(cred) if cred is not None else (1 if ws.g_cap <= 64 else 0)
        if ws.split:  # the split path's producers finalize their BatchNorm statistics
            cfg.consumer_reduce = 0
        return cfg

    def fill_embed(self, table: int | None = None):
        """Layer-0 inputs; ``table``: another row buffer standing in for the item table
        (the fetched rows of the row-sharded step, indexed by the batch's compact ids)."""
        m = self.model
        e = self.embed
        e.table = m.item_embedding.weight.data_ptr() if table is None else table
        if self.K > 0:
            pe = m.laplacian_pe._cached_pe
            e.pe_tab = None if pe is None else pe.data_ptr()
            e.wpe = self.flat.seg_ptr("pe.w")
            e.bpe = self.flat.seg_ptr("pe.b")
        else:
            e.pe_tab = e.wpe = e.bpe = None
        return e

    @staticmethod
    def batch_struct(caps: Caps, blob: torch.Tensor, node_pe: torch.Tensor | None = None) -> L.GtrBatch:
        lay = blob_layout(caps)
        base = blob.data_ptr()
        bs = L.GtrBatch()
        for name in ("hdr", "node_item", "node_ptr", "in_ptr", "in_src", "out_ptr", "out_edge", "out_dst",
                     "target", "negatives", "grp_row", "grp_edge"):
            setattr(bs, name, base + 4 * lay[name][0])
        bs.node_pe = None if node_pe is None else node_pe.data_ptr()
        bs.n_cap, bs.b_cap, bs.e_cap, bs.n_neg = caps.n_cap, caps.b_cap, caps.e_cap, caps.n_neg
        return bs

    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    # ------------------------------------------------------------------ launches
    def layer_fwd(self, ws: Workspace, cfg: L.GtrConfig, bs: L.GtrBatch, l: int, emb, st: int,
                  split: bool | None = None):
        """Forward of layer l: one fused launch, or (split) the projection GEMM + attention."""
        lib = L.lib()
        if ws.split if split is None else split:
            L.check(lib.gtr_qkvs_fwd(C.byref(cfg), C.byref(bs), C.byref(emb), ws.structs, l, st), "qkvs_fwd")
            L.check(lib.gtr_attn_fwd(C.byref(cfg), C.byref(bs), ws.structs, l, st), "attn_fwd")
        else:
            L.check(lib.gtr_conv_fwd(C.byref(cfg), C.byref(bs), C.byref(emb), ws.structs, l, st), "conv_fwd")

    def layer_bwd(self, ws: Workspace, cfg: L.GtrConfig, bs: L.GtrBatch, l: int, st: int,
                  split: bool | None = None):
        """Backward of layer l: one fused launch, or (split) the attention backward + dX GEMM."""
        lib = L.lib()
        if ws.split if split is None else split:
            L.check(lib.gtr_attn_bwd(C.byref(cfg), C.byref(bs), ws.structs, l, st), "attn_bwd")
            L.check(lib.gtr_qkvs_bwd(C.byref(cfg), C.byref(bs), ws.structs, l, ws.dx0.data_ptr(), st), "qkvs_bwd")
        else:
            L.check(lib.gtr_conv_bwd(C.byref(cfg), C.byref(bs), ws.structs, l, ws.dx0.data_ptr(), st), "conv_bwd")

    def ffn_fwd(self, ws: Workspace, cfg: L.GtrConfig, bs: L.GtrBatch, l: int, st: int):
        """Layer l's feed-forward block (use_ffn=True): y, a, z (gtr_ffn_fwd)."""
        L.check(L.lib().gtr_ffn_fwd(C.byref(cfg), C.byref(bs), ws.structs, l, st), "ffn_fwd")

    def ffn_bwd(self, ws: Workspace, cfg: L.GtrConfig, bs: L.GtrBatch, l: int, st: int, wgrad: bool = True):
        """Layer l's feed-forward backward (-> layers[l].dy + its BatchNorm sums) and, with
        ``wgrad``, its weight-gradient slabs."""
        lib = L.lib()
        L.check(lib.gtr_ffn_bwd(C.byref(cfg), C.byref(bs), ws.structs, l, st), "ffn_bwd")
        if wgrad:
            L.check(lib.gtr_ffn_wgrad(C.byref(cfg), C.byref(bs), ws.structs, l, ws.ffn_slabs[l].data_ptr(),
                                      ws.P, self.flat.layout.ffn_stride, st), "ffn_wgrad")

    def run_forward(self, ws: Workspace, cfg: L.GtrConfig, bs: L.GtrBatch, flags: int,
                    loss_kind: int = 0, temperature: float = 1.0, alpha: float = 0.7, split: bool | None = None):
        st = self.stream()
        emb = self.fill_embed()
        for l in range(self.L):
            self.layer_fwd(ws, cfg, bs, l, emb, st, split)
            if ws.ffns is not None:
                self.ffn_fwd(ws, cfg, bs, l, st)
        self.run_head(ws, cfg, bs, flags, loss_kind, temperature, alpha)

    def run_head(self, ws, cfg, bs, flags, loss_kind=0, temperature=1.0, alpha=0.7, dse_out=False, table=None):
        h, tab = self.fill_head(ws, flags, loss_kind, temperature, alpha, dse_out, table)
        rcfg, structs = ws.readout_args(cfg)
        L.check(L.lib().gtr_readout_loss(C.byref(rcfg), C.byref(bs), tab, structs, C.byref(h), self.stream()),
                "readout_loss")

    def fill_head(self, ws, flags, loss_kind=0, temperature=1.0, alpha=0.7, dse_out=False, table=None):
        """The readout's gtr_head (workspace pointers + loss settings) and table pointer."""
        h = ws.head
        h.flags = flags
        h.loss_kind = loss_kind
        h.temperature = float(temperature)
        h.dual_alpha = float(alpha)
        h.se = ws.se.data_ptr()
        h.dse_in = ws.dse_in.data_ptr()
        h.dse_out = ws.dse_out.data_ptr() if dse_out else None
        h.coef_tgt = ws.coef_tgt.data_ptr()
        h.coef_neg = ws.coef_neg.data_ptr()
        h.loss_part = ws.loss_part.data_ptr()
        h.loss_out = ws.loss_out.data_ptr()
        h.cnt = ws.head_cnt.data_ptr()
        tab = self.model.item_embedding.weight.data_ptr() if table is None else table
        return h, tab

    def _wgrad(self, ws, cfg, bs, l0, l1, st):
        if cfg.wfold_stride > 0:  # the layer jobs ran in gtr_conv_bwd (wfold): the PE job only
            l1 = l0
        pe_tab = None
        if self.K > 0 and self.model.laplacian_pe._cached_pe is not None:
            pe_tab = self.model.laplacian_pe._cached_pe.data_ptr()
        L.check(L.lib().gtr_wgrad(C.byref(cfg), C.byref(bs), ws.structs, ws.dx0.data_ptr(), pe_tab, ws.slab_ptrs,
                                  None if ws.pe_slab is None else ws.pe_slab.data_ptr(), ws.P,
                                  self.flat.layout.slab_stride, l0, l1, st), "wgrad")

    def run_backward(self, ws: Workspace, cfg: L.GtrConfig, bs: L.GtrBatch, side: torch.cuda.Stream | None = None,
                     wgrad: bool = True, split: bool | None = None):
        """conv_bwd(L-1..0) + weight-gradient slabs; expects layers[L-1].dy / bn_gsum.
        With ``side``, layer l >= 1 weight gradients run on that stream concurrently
        with conv_bwd(l-1..0); the caller must join ``side`` before reading slabs.
        ``wgrad=False``: the weight gradients are left to the fused tail."""
        lib = L.lib()
        main = torch.cuda.current_stream(self.device)
        st = main.cuda_stream
        if ws.ffns is not None:
            side = None  # FFN blocks: every gradient kernel on the main stream
        for l in range(self.L - 1, -1, -1):
            if ws.ffns is not None:
                self.ffn_bwd(ws, cfg, bs, l, st, wgrad)
            self.layer_bwd(ws, cfg, bs, l, st, split)
            if wgrad and side is not None and l >= 1:
                side.wait_stream(main)
                self._wgrad(ws, cfg, bs, l, l + 1, side.cuda_stream)
        if not wgrad:
            return
        if side is not None:
            self._wgrad(ws, cfg, bs, 0, 1, st)
        else:
            self._wgrad(ws, cfg, bs, 0, self.L, st)

    def segments(self, ws: Workspace, wfold: bool = False):
        """Segment table mapping each flat parameter segment to its gradient source;
        ``wfold``: the layer weights' partials are the fused backward's per-row-group slabs
        (Workspace.enable_wfold), summed over the batch's live groups."""
        lay = self.flat.layout
        segs = []
        D, K = self.D, self.K
        stride = lay.slab_stride
        for l in range(self.L):
            base = ws.wfold[l].data_ptr() if wfold else ws.slabs[l].data_ptr()
            n, live = (ws.g_cap, 1) if wfold else (ws.P, 0)
            g = ws.layers[l]["bn_gsum"].data_ptr()
            for name, src, np_, lv in ((f"{l}.w_all", base, n, live), (f"{l}.b_all", base + 4 * (4 * D * D), n, live),
                                       (f"{l}.w_beta", base + 4 * (4 * D * D + 4 * D), n, live),
                                       (f"{l}.gamma", g + 4 * D, 1, 0), (f"{l}.beta", g, 1, 0)):
                s = lay.seg(name)
                segs.append((s.begin, s.numel, src, stride, np_, lv))
            if ws.ffns is not None:
                fb, F = ws.ffn_slabs[l].data_ptr(), lay.F
                for name, off in ((f"{l}.ffn_w1", 0), (f"{l}.ffn_b1", F * D), (f"{l}.ffn_w2", F * D + F),
                                  (f"{l}.ffn_b2", 2 * F * D + F)):
                    s = lay.seg(name)
                    segs.append((s.begin, s.numel, fb + 4 * off, lay.ffn_stride, ws.P, 0))
        if K > 0:
            base = ws.pe_slab.data_ptr()
            for name, src in (("pe.w", base), ("pe.b", base + 4 * D * K)):
                s = lay.seg(name)
                segs.append((s.begin, s.numel, src, stride, ws.P, 0))
        arr = (L.GtrSegment * len(segs))()
        for i, (b, n, src, ps, npart, lv) in enumerate(segs):
            arr[i].begin, arr[i].len, arr[i].src, arr[i].pstride, arr[i].nparts = b, n, src, ps, npart
            arr[i].live_groups = lv
        return arr, len(segs)

    def reduce_small_grads(self, ws: Workspace, flat_grad: torch.Tensor):
        segs, n = self.segments(ws)
        L.check(L.lib().gtr_adamw_small(None, None, None, flat_grad.data_ptr(), self.flat.layout.total, segs, n,
                                        None, self.stream()), "adamw_small(reduce)")

    # ------------------------------------------------------------------ batches
    def prepare(self, batch) -> tuple[Caps, torch.Tensor, torch.Tensor | None]:
        from etpgt.data.gpu_batch import DeviceBatch

        if isinstance(batch, DeviceBatch):  # built on the device: ids checked by the builder
            if batch.blob.device != self.device:
                raise ValueError("device-built batch lives on another device than the model")
            return batch.caps, batch.blob, None
        if not isinstance(batch, SessionBatch):
            batch = SessionBatch(batch.x, batch.edge_index, getattr(batch, "batch", None),
                                 getattr(batch, "target_item", None), getattr(batch, "negative_items", None),
                                 getattr(batch, "laplacian_pe", None), getattr(batch, "ptr", None))
        batch.check_ids(self.T)
        caps, blob = batch.device_blob(self.device)
        pe = batch.laplacian_pe
        node_pe = None
        if self.K > 0 and pe is not None:
            node_pe = torch.zeros(caps.n_cap, self.K, dtype=torch.float32, device=self.device)
            node_pe[: pe.shape[0]].copy_(pe.to(self.device, torch.float32))
        return caps, blob, node_pe
