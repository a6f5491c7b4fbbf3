"""Autograd entry points over libgtr_hip (the eager / torch.autograd path).

* ``score_loss``: BPR / listwise / dual sampled scoring loss (base.py:80-113,
  losses.py:8-201) — forward and backward in one kernel launch, the backward
  applied with the saved coefficients (dense table gradient by ``gtr_scatter_rows``).
* ``GraphTransformerFn``: the whole GraphTransformer forward (all layers + mean
  readout) as one autograd node; its backward runs readout-bwd, conv_bwd per
  layer, the weight-gradient kernel and the slab reduction.

The fused training step (etpgt.train.fused) drives the same kernels without
autograd and with the optimizer fused in.
"""

from __future__ import annotations

import ctypes as C

import torch

from etpgt.backend import _lib as L


def _dev_i32(t: torch.Tensor, device) -> torch.Tensor:
    return t.to(device=device, dtype=torch.int32).contiguous()


_HDR: dict = {}


def _score_hdr(B: int, n: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    """Batch header + zero session pointers of a scoring-only launch, cached per shape: a
    fresh torch.tensor(..., device=cuda) every step is a host-to-device copy that waits
    for the stream (the host would stall behind every queued kernel)."""
    key = (str(device), int(B), int(n))
    t = _HDR.get(key)
    if t is None:
        if len(_HDR) > 64:
            _HDR.clear()
        hdr = torch.tensor([0, B, 0, n, 0, 0, 0, 0], dtype=torch.int32).to(device)
        t = _HDR[key] = (hdr, torch.zeros(B + 1, dtype=torch.int32, device=device))
    return t


# ---- torch.library registrations (the kernels are visible to FX /
# torch.compile / fake-tensor tracing as ops of the ``etpgt`` namespace, with fake
# implementations for shape inference and registered autograd formulas).
def _score_loss_launch(se: torch.Tensor, table: torch.Tensor, target: torch.Tensor, negatives: torch.Tensor,
                       kind: int, temperature: float, alpha: float):
    lib = L.lib()
    dev = se.device
    B, D = se.shape
    n = negatives.numel() // max(B, 1)
    if D not in (32, 64, 128, 256):
        raise ValueError(f"embedding dim {D} unsupported by the HIP scoring kernel")
    if table.shape[1] != D:
        raise ValueError("session embedding and item table dims differ")
    se_c = se.detach().float().contiguous()
    tgt = _dev_i32(target.reshape(-1), dev)
    neg = _dev_i32(negatives.reshape(-1), dev)
    hdr, node_ptr = _score_hdr(B, n, dev)
    bs = L.GtrBatch()
    bs.hdr, bs.node_ptr, bs.target, bs.negatives = hdr.data_ptr(), node_ptr.data_ptr(), tgt.data_ptr(), neg.data_ptr()
    bs.n_cap, bs.b_cap, bs.e_cap, bs.n_neg = 1, B, 1, n
    cfg = L.GtrConfig()
    cfg.num_items, cfg.dim, cfg.heads, cfg.num_layers, cfg.row_group = table.shape[0], D, 1, 1, 16
    cfg.training, cfg.bn_eps, cfg.bn_momentum = 0, 1e-5, 0.1
    layer = (L.GtrLayer * 1)()
    dse = torch.empty(B, D, dtype=torch.float32, device=dev)
    coef_t = torch.empty(B, dtype=torch.float32, device=dev)
    coef_n = torch.empty(B * n, dtype=torch.float32, device=dev)
    part = torch.empty(512, dtype=torch.float32, device=dev)
    loss = torch.empty(1, dtype=torch.float32, device=dev)
    cnt = torch.zeros(4, dtype=torch.int32, device=dev)
    h = L.GtrHead()
    h.flags, h.loss_kind, h.temperature, h.dual_alpha = L.RO_LOSS, int(kind), float(temperature), float(alpha)
    h.se, h.dse_out, h.coef_tgt, h.coef_neg = se_c.data_ptr(), dse.data_ptr(), coef_t.data_ptr(), coef_n.data_ptr()
    h.loss_part, h.loss_out, h.cnt = part.data_ptr(), loss.data_ptr(), cnt.data_ptr()
    tab = table.detach().contiguous()
    st = torch.cuda.current_stream(dev).cuda_stream
    L.check(lib.gtr_readout_loss(C.byref(cfg), C.byref(bs), tab.data_ptr(), layer, C.byref(h), st), "score_loss")
    return loss.reshape(()), dse, coef_t, coef_n


@torch.library.custom_op("etpgt::score_loss", mutates_args=())
def _score_loss_op(se: torch.Tensor, table: torch.Tensor, target: torch.Tensor, negatives: torch.Tensor,
                   kind: int, temperature: float, alpha: float
                   ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """BPR / listwise / dual sampled scoring loss (base.py:80-113, losses.py:8-164) on
    gtr_readout_loss: (loss, d loss / d se, d loss / d score of each target, of each
    negative)."""
    return _score_loss_launch(se, table, target, negatives, kind, temperature, alpha)


@_score_loss_op.register_fake
def _(se, table, target, negatives, kind, temperature, alpha):
    B, D = se.shape
    n = negatives.numel() // max(B, 1)
    return (se.new_empty(()), se.new_empty(B, D), se.new_empty(B), se.new_empty(B * n))


@torch.library.custom_op("etpgt::score_rows_grad", mutates_args=())
def _score_rows_grad_op(se: torch.Tensor, coef_t: torch.Tensor, coef_n: torch.Tensor, target: torch.Tensor,
                        negatives: torch.Tensor, num_items: int) -> torch.Tensor:
    """The item-table gradient of the scoring loss: dense [T, D], every target / negative
    row's coef * se (gtr_scatter_rows: sorted-segment sums, deterministic)."""
    B, D = se.shape
    n = negatives.numel() // max(B, 1)
    dev = se.device
    dtab = torch.zeros(num_items, D, dtype=torch.float32, device=dev)
    tgt = _dev_i32(target.reshape(-1), dev)
    neg = _dev_i32(negatives.reshape(-1), dev)
    hdr, node_ptr = _score_hdr(B, n, dev)
    bs = L.GtrBatch()
    bs.hdr, bs.node_ptr, bs.target, bs.negatives = hdr.data_ptr(), node_ptr.data_ptr(), tgt.data_ptr(), neg.data_ptr()
    bs.n_cap, bs.b_cap, bs.e_cap, bs.n_neg = 1, B, 1, n
    st = torch.cuda.current_stream(dev).cuda_stream
    se_c = se.detach().float().contiguous()
    L.check(L.lib().gtr_scatter_rows(C.byref(bs), D, 1, se_c.data_ptr(), coef_t.contiguous().data_ptr(),
                                     coef_n.contiguous().data_ptr(), dtab.data_ptr(), st), "scatter_rows")
    return dtab


@_score_rows_grad_op.register_fake
def _(se, coef_t, coef_n, target, negatives, num_items):
    return se.new_empty(num_items, se.shape[1])


def _score_loss_setup(ctx, inputs, output):
    se, table, target, negatives = inputs[:4]
    _, dse, coef_t, coef_n = output
    ctx.save_for_backward(se, dse, coef_t, coef_n, target, negatives)
    ctx.num_items = table.shape[0]


def _score_loss_backward(ctx, g_loss, g_dse, g_ct, g_cn):
    se, dse, coef_t, coef_n, target, negatives = ctx.saved_tensors
    dse_g = dse * g_loss if ctx.needs_input_grad[0] else None
    dtab = None
    if ctx.needs_input_grad[1]:
        dtab = torch.ops.etpgt.score_rows_grad(se, coef_t, coef_n, target, negatives, ctx.num_items) * g_loss
    return dse_g, dtab, None, None, None, None, None


torch.library.register_autograd("etpgt::score_loss", _score_loss_backward, setup_context=_score_loss_setup)


def score_loss(se, target, negatives, table, kind="bpr", temperature=1.0, alpha=0.7):
    """Sampled scoring loss on the HIP kernel.  ``table`` is the item-table weight
    (or an nn.Embedding)."""
    if isinstance(table, torch.nn.Embedding):
        table = table.weight
    if se.device.type != "cuda":
        raise RuntimeError("score_loss runs on the MI355X HIP path only (tensors are on CPU)")
    if kind not in L.GTR_LOSS or kind == "none":
        raise ValueError(f"Unknown loss type: {kind}")
    B = se.shape[0]
    if negatives.dim() == 1:
        negatives = negatives.view(B, -1)
    return torch.ops.etpgt.score_loss(se, table, target, negatives, L.GTR_LOSS[kind], float(temperature),
                                      float(alpha))[0]


# Engines reachable from the ``etpgt::graph_transformer_eval`` op by an integer handle
# (ops take tensors and scalars only); weak, so a dropped model frees its engine.
import weakref  # noqa: E402

_ENGINES: "weakref.WeakValueDictionary[int, object]" = weakref.WeakValueDictionary()


def engine_handle(eng) -> int:
    h = id(eng)
    _ENGINES[h] = eng
    return h


@torch.library.custom_op("etpgt::graph_transformer_eval", mutates_args=())
def _graph_transformer_eval_op(blob: torch.Tensor, node_pe: torch.Tensor | None, table: torch.Tensor,
                               params: list[torch.Tensor], engine: int, n_cap: int, b_cap: int, e_cap: int,
                               n_neg: int, num_graphs: int) -> torch.Tensor:
    """Inference forward of the whole GraphTransformer (eval mode: running BatchNorm
    statistics, no dropout; graph_transformer.py:126-182): session embeddings [B, d] from a
    packed batch image.  Pure -- no buffer is written -- so FX / torch.compile graphs of
    serving code see it as one op."""
    from etpgt.data.batch import Caps

    eng = _ENGINES.get(int(engine))
    if eng is None:
        raise RuntimeError("etpgt::graph_transformer_eval: the engine handle is gone (model freed)")
    eng.check_intact()
    caps = Caps(n_cap, b_cap, e_cap, n_neg)
    ws = eng.workspace(caps)
    cfg = eng.config(ws, False)
    bs = eng.batch_struct(caps, blob, node_pe)
    eng.run_forward(ws, cfg, bs, L.RO_FWD)
    return ws.se[:num_graphs].clone()


@_graph_transformer_eval_op.register_fake
def _(blob, node_pe, table, params, engine, n_cap, b_cap, e_cap, n_neg, num_graphs):
    return table.new_empty(num_graphs, table.shape[1])


class GraphTransformerFn(torch.autograd.Function):
    """Whole-model forward as one autograd node (inputs: table + dense params)."""

    @staticmethod
    def forward(ctx, eng, caps, blob, node_pe, B, training, need_grad, table, *params):
        eng.check_intact()
        need_grad = bool(need_grad) and training
        ws = eng.acquire_workspace(caps) if need_grad else eng.workspace(caps)
        rng = torch.empty(1, dtype=torch.int32, device=eng.device)
        rng.copy_(eng.rng_ctr)
        if training:
            eng.rng_ctr.add_(1)
        cfg = eng.config(ws, training)
        cfg.rng_ctr = rng.data_ptr()
        bs = eng.batch_struct(caps, blob, node_pe)
        eng.run_forward(ws, cfg, bs, L.RO_FWD)
        se = ws.se[:B].clone()
        ctx.eng = None
        ctx.done = False
        if need_grad:
            ctx.eng, ctx.ws, ctx.cfg, ctx.bs, ctx.B = eng, ws, cfg, bs, B
            ctx.keep = (blob, node_pe, rng)
        return se

    @staticmethod
    def backward(ctx, dse):
        if ctx.done:
            raise RuntimeError("the GraphTransformer's saved activations were released after the first backward "
                               "(backward twice / retain_graph is not supported on the HIP path)")
        if ctx.eng is None:
            raise RuntimeError("backward through the GraphTransformer requires train() mode "
                               "(BatchNorm batch statistics) and grad mode at forward time")
        eng, ws, cfg, bs, B = ctx.eng, ctx.ws, ctx.cfg, ctx.bs, ctx.B
        ws.dse_in[:B].copy_(dse)
        eng.run_head(ws, cfg, bs, L.RO_BWD)
        eng.run_backward(ws, cfg, bs)
        flat_grad = torch.empty(eng.flat.layout.total, dtype=torch.float32, device=eng.device)
        eng.reduce_small_grads(ws, flat_grad)
        table = eng.model.item_embedding.weight
        dtab = torch.zeros_like(table)
        L.check(L.lib().gtr_scatter_rows(C.byref(bs), eng.D, 0, ws.dx0.data_ptr(), None, None, dtab.data_ptr(),
                                         eng.stream()), "scatter_rows")
        grads = eng.flat.grad_views(flat_grad)
        ctx.done = True
        eng.release_workspace(ws)  # the gradients above are fresh tensors; ws may serve the next forward
        return (None, None, None, None, None, None, None, dtab, *grads)


_TOPK_WS: dict = {}


@torch.library.custom_op("etpgt::score_topk", mutates_args=())
def _score_topk_op(se: torch.Tensor, table: torch.Tensor, k: int, exclude_ptr: torch.Tensor | None,
                   exclude_ids: torch.Tensor | None) -> tuple[torch.Tensor, torch.Tensor]:
    """Full-catalog scores se @ table.T and their top-k (gtr_score_topk / _masked)."""
    B, D = se.shape
    T = table.shape[0]
    dev = se.device
    idx = torch.empty(B, k, dtype=torch.int64, device=dev)
    sc = torch.empty(B, k, dtype=torch.float32, device=dev)
    if B == 0:
        return idx, sc
    lib = L.lib()
    nb = C.c_size_t(0)
    L.check(lib.gtr_topk_workspace_bytes(B, T, k, C.byref(nb)), "topk_workspace_bytes")
    key = (str(dev), int(nb.value))
    ws = _TOPK_WS.get(key)
    if ws is None:
        _TOPK_WS.clear()
        ws = torch.empty(int(nb.value), dtype=torch.uint8, device=dev)
        _TOPK_WS[key] = ws
    s = se.detach().float().contiguous()
    t = table.detach().float().contiguous()
    st = torch.cuda.current_stream(dev).cuda_stream
    if exclude_ptr is None:
        L.check(lib.gtr_score_topk(s.data_ptr(), B, D, t.data_ptr(), T, int(k), idx.data_ptr(), sc.data_ptr(),
                                   ws.data_ptr(), ws.numel(), st), "score_topk")
    else:
        L.check(lib.gtr_score_topk_masked(s.data_ptr(), B, D, t.data_ptr(), T, int(k), exclude_ptr.data_ptr(),
                                          exclude_ids.data_ptr(), idx.data_ptr(), sc.data_ptr(), ws.data_ptr(),
                                          ws.numel(), st), "score_topk_masked")
    return idx, sc


@_score_topk_op.register_fake
def _(se, table, k, exclude_ptr, exclude_ids):
    B = se.shape[0]
    return se.new_empty(B, k, dtype=torch.int64), se.new_empty(B, k)


def score_topk(se: torch.Tensor, table: torch.Tensor, k: int, exclude: list | None = None
               ) -> tuple[torch.Tensor, torch.Tensor]:
    """Full-catalog scores ``se @ table.T`` and their top-k (base.py:59-78) on the HIP
    kernel (gtr_score_topk, op ``etpgt::score_topk``): returns (item ids [B, k] int64,
    scores [B, k] fp32), best first; ties resolve to the lower item id.  No [B, T] score
    matrix is materialised.  ``exclude``: per-session iterables of item ids that may not
    be returned (serving's seen-item / padding mask); missing results come back as id -1,
    score -inf."""
    if isinstance(table, torch.nn.Embedding):
        table = table.weight
    if se.device.type != "cuda":
        raise RuntimeError("predict runs on the MI355X HIP path only (tensors are on CPU)")
    if se.dim() != 2 or table.dim() != 2 or se.shape[1] != table.shape[1]:
        raise ValueError(f"session embeddings {tuple(se.shape)} do not match the item table {tuple(table.shape)}")
    B = se.shape[0]
    T = table.shape[0]
    if k > T:
        raise RuntimeError(f"selected index k out of range (k={k} > {T} items)")
    if exclude is None:
        return torch.ops.etpgt.score_topk(se, table, int(k), None, None)
    if len(exclude) != B:
        raise ValueError("exclude needs one id list per session")
    lists = [sorted(set(int(v) for v in e)) for e in exclude]
    ptr = [0]
    for e in lists:
        ptr.append(ptr[-1] + len(e))
    ids = [v for e in lists for v in e] or [0]
    ptr_d = torch.tensor(ptr, dtype=torch.int32, device=se.device)
    ids_d = torch.tensor(ids, dtype=torch.int32, device=se.device)
    return torch.ops.etpgt.score_topk(se, table, int(k), ptr_d, ids_d)
