"""Per-layer halo exchange for destination-range cuts that split sessions.

The default multi-GPU step cuts the global batch on SESSION boundaries (the reference's
loader keeps a session's subgraph whole, ``etpgt/train/dataloader.py:157-202``), so no
attention edge crosses a rank and the only exchange is the layer-0 row fetch of the
item table.  This module is the general mechanism behind a flag: the batch graph is cut
into contiguous DESTINATION-node ranges (``cuts``; default: equal node counts), wherever
those fall, and

* every rank computes Q / K / V / S (``gtr_qkvs_fwd``) for its own destination rows;
* per layer, the K / V rows of the sources of its edges that live on other ranks (its
  ghost rows) arrive by one all-to-all (``kv_fwd``: the north star's "all-gather of halo
  source embeddings each layer", restricted to the rows each rank needs) into rows
  ``[N, N + G)`` of its qkvs buffer -- the attention kernels read them like local rows;
* backward, ``gtr_attn_bwd`` also writes dK / dV of the ghost rows (``hdr[6]``: the source
  rows, gtr.h); they travel back to their owners, which add them to their own rows in
  rank order before the dX GEMM (``kv_bwd``);
* a session that straddles a cut is read out by the rank holding its first node: the
  straddling tail's last-layer rows (pre-BatchNorm output and layer input) arrive as the
  first ghost rows, right after the local rows, so the session stays one contiguous row
  range (``ro_fwd``); the readout's gradient rows go back to the owners (``ro_bwd``);
* BatchNorm statistics are over the global batch (SyncBN, one merged row per rank), the
  loss means divide by global B / P (``gtr_config.loss_batch``: ranks own unequal session
  counts), and the gradients are averaged by the data-parallel exchange
  (``etpgt.train.distributed``) -- so P ranks train like ONE GPU on the global batch, up to
  the order of the cross-rank sums.

The exchanges are torch collectives between the step's launches (all-to-all over RCCL, or
gloo through host memory for the shared-device tests); the blocks are sized by the
largest ghost count of any rank pair.  Every rank plans every rank's part from the same
global batch, so no index metadata is exchanged.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from etpgt.data.batch import Caps, SessionBatch, _np, blob_layout
from etpgt.train.distributed import all_to_all
from etpgt.train.fused import FusedTrainStep


@dataclass
class HaloPart:
    """One rank's share of a global batch cut at destination-node ranges."""

    rank: int
    lo: int                # global rows [lo, hi) are this rank's destination rows
    hi: int
    ghosts: np.ndarray     # global node ids of the ghost rows, in slot order
    n_readout: int         # the first n_readout ghosts: the tail of the straddling session
    node_ptr: np.ndarray   # owned sessions' row ranges (local row index, ghosts past N)
    x: np.ndarray          # item ids of the local + ghost rows
    in_ptr: np.ndarray
    in_src: np.ndarray
    out_ptr: np.ndarray
    out_edge: np.ndarray
    out_dst: np.ndarray
    target: np.ndarray
    negatives: np.ndarray

    @property
    def n_local(self) -> int:
        return self.hi - self.lo

    @property
    def n_ext(self) -> int:
        return self.n_local + int(self.ghosts.size)

    @property
    def num_sessions(self) -> int:
        return int(self.node_ptr.size) - 1

    @property
    def num_edges(self) -> int:
        return int(self.in_src.size)


def default_cuts(num_nodes: int, world: int) -> np.ndarray:
    """Equal destination-node ranges (cut wherever they fall, sessions included)."""
    return np.array([(r * num_nodes) // world for r in range(world + 1)], np.int64)


def plan_halo(sb: SessionBatch, world: int, cuts=None) -> list[HaloPart]:
    """Cut ``sb`` into ``world`` destination-node ranges and plan every rank's part."""
    N, B, E, n_neg = sb.sizes()
    cuts = default_cuts(N, world) if cuts is None else np.asarray(cuts, np.int64)
    if cuts.shape != (world + 1,) or cuts[0] != 0 or cuts[-1] != N or np.any(np.diff(cuts) <= 0):
        raise ValueError("cuts must be increasing from 0 to num_nodes with one range per rank")
    x = _np(sb.x).astype(np.int64)
    ei = _np(sb.edge_index).astype(np.int64).reshape(2, -1)
    src, dst = ei[0], ei[1]
    ptr = _np(sb.ptr).astype(np.int64)
    tgt = _np(sb.target_item).astype(np.int64).reshape(-1)
    neg = _np(sb.negative_items).astype(np.int64).reshape(B, -1) if n_neg else np.zeros((B, 0), np.int64)
    starts = ptr[:-1]
    parts = []
    for r in range(world):
        lo, hi = int(cuts[r]), int(cuts[r + 1])
        own = np.nonzero((starts >= lo) & (starts < hi))[0]
        if own.size == 0:
            raise ValueError(f"rank {r} owns no session (its node range lies inside one session): "
                             "use fewer ranks or other cuts")
        p_end = int(ptr[own[-1] + 1])
        ro = np.arange(hi, max(hi, p_end), dtype=np.int64)  # the straddling session's tail
        sel = (dst >= lo) & (dst < hi)
        s_g, d_g = src[sel], dst[sel]
        outside = (s_g < lo) | (s_g >= max(hi, p_end))
        kv = np.unique(s_g[outside])
        ghosts = np.concatenate([ro, kv])
        n_loc = hi - lo
        # extended row index of a global node: local rows, then the readout tail (contiguous
        # with the local rows), then the other ghosts
        s_ext = np.where(outside, n_loc + ro.size + np.searchsorted(kv, s_g), s_g - lo)
        d_loc = d_g - lo
        order = np.argsort(d_loc, kind="stable")  # CSR by destination, edge order kept per row
        in_src = s_ext[order]
        in_ptr = np.zeros(n_loc + 1, np.int64)
        np.cumsum(np.bincount(d_loc, minlength=n_loc), out=in_ptr[1:])
        n_ext = n_loc + ghosts.size
        out_edge = np.argsort(in_src, kind="stable")  # CSR by source over local + ghost rows
        out_dst = d_loc[order][out_edge]
        out_ptr = np.zeros(n_ext + 1, np.int64)
        np.cumsum(np.bincount(in_src, minlength=n_ext), out=out_ptr[1:])
        parts.append(HaloPart(
            rank=r, lo=lo, hi=hi, ghosts=ghosts, n_readout=int(ro.size),
            node_ptr=np.append(starts[own], p_end) - lo, x=np.concatenate([x[lo:hi], x[ghosts]]),
            in_ptr=in_ptr, in_src=in_src, out_ptr=out_ptr, out_edge=out_edge, out_dst=out_dst,
            target=tgt[own], negatives=neg[own].reshape(-1)))
    return parts


def halo_caps(parts: list[HaloPart], n_neg: int) -> Caps:
    """Capacities covering every rank's part (local + ghost rows)."""
    n = max(p.n_ext for p in parts)
    b = max(p.num_sessions for p in parts)
    e = max(p.num_edges for p in parts)
    return Caps.bucket(n, b, max(e, 1), n_neg)


def pack_halo(part: HaloPart, caps: Caps) -> np.ndarray:
    """The int32 batch image of one rank's part (data/batch.py blob_layout) with
    hdr[6] = local + ghost rows."""
    N, G, B, E = part.n_local, part.ghosts.size, part.num_sessions, part.num_edges
    if not caps.fits(N + G, B, E, caps.n_neg):
        raise ValueError(f"halo part (rows {N}+{G}, B={B}, E={E}) exceeds capacity {caps}")
    lay = blob_layout(caps)
    blob = np.zeros(lay["_total"], np.int32)

    def put(name, arr, fill=None):
        o, sz = lay[name]
        a = np.asarray(arr, np.int64)
        blob[o: o + a.shape[0]] = a
        if fill is not None and a.shape[0] < sz:
            blob[o + a.shape[0]: o + sz] = fill

    R = caps.R
    ng = (N + R - 1) // R
    st = part.node_ptr[:-1]
    sog = np.searchsorted(st, np.arange(ng + 1) * R, side="left")
    grp_row = np.minimum(np.append(part.node_ptr, N)[np.minimum(sog, B)], N)
    grp_row[-1] = N
    grp_edge = part.in_ptr[grp_row]
    put("hdr", [N, B, E, caps.n_neg, ng, R, N + G, 0])
    put("grp_row", grp_row, fill=N)
    put("grp_edge", grp_edge, fill=E)
    put("node_item", part.x)
    put("node_ptr", part.node_ptr, fill=int(part.node_ptr[-1]))
    put("in_ptr", part.in_ptr, fill=E)
    put("in_src", part.in_src)
    put("out_ptr", part.out_ptr, fill=E)
    put("out_edge", part.out_edge)
    put("out_dst", part.out_dst)
    put("target", part.target)
    if caps.n_neg:
        put("negatives", part.negatives)
    return blob


class HaloExchange:
    """Device index plans of one rank for the four halo exchanges."""

    def __init__(self, parts: list[HaloPart], rank: int, dev, group=None):
        P = len(parts)
        self.P, self.rank, self.group, self.dev = P, rank, group, dev
        me = parts[rank]
        cuts = np.array([p.lo for p in parts] + [parts[-1].hi], np.int64)

        def owner(g):
            return np.searchsorted(cuts, g, side="right") - 1

        def plans(readout_only: bool):
            recv_slots, send_rows, cap = [], [], 1
            for q in range(P):
                gh = me.ghosts[: me.n_readout] if readout_only else me.ghosts
                sl = np.nonzero(owner(gh) == q)[0] if q != rank else np.zeros(0, np.int64)
                recv_slots.append(torch.as_tensor(me.n_local + sl, dtype=torch.long, device=dev))
                pq = parts[q]
                gq = pq.ghosts[: pq.n_readout] if readout_only else pq.ghosts
                rows = gq[owner(gq) == rank] - me.lo if q != rank else np.zeros(0, np.int64)
                send_rows.append(torch.as_tensor(rows, dtype=torch.long, device=dev))
            for r in range(P):  # the block: the largest count of any ordered rank pair
                pr = parts[r]
                for gh in (pr.ghosts[: pr.n_readout] if readout_only else pr.ghosts,):
                    if gh.size:
                        cap = max(cap, int(np.bincount(owner(gh), minlength=P).max()))
            return recv_slots, send_rows, cap

        self.kv = plans(False)
        self.ro = plans(True)
        self.ghost_rows = int(me.ghosts.size)

    def _a2a(self, send: torch.Tensor) -> torch.Tensor:
        recv = torch.empty_like(send)
        all_to_all(recv, send, self.group)
        return recv

    def fetch(self, buf: torch.Tensor, c0: int, c1: int, readout_only: bool = False) -> None:
        """buf[ghost slots, c0:c1] <- the owners' buf[rows, c0:c1]."""
        recv_slots, send_rows, cap = self.ro if readout_only else self.kv
        send = torch.zeros(self.P, cap, c1 - c0, dtype=buf.dtype, device=buf.device)
        for q in range(self.P):
            if send_rows[q].numel():
                send[q, : send_rows[q].numel()] = buf[send_rows[q], c0:c1]
        recv = self._a2a(send)
        for q in range(self.P):
            if recv_slots[q].numel():
                buf[recv_slots[q], c0:c1] = recv[q, : recv_slots[q].numel()]

    def give_back(self, buf: torch.Tensor, c0: int, c1: int, readout_only: bool = False) -> None:
        """The owners' buf[rows, c0:c1] += (readout: =) this rank's buf[ghost slots, c0:c1],
        peers in rank order (deterministic)."""
        recv_slots, send_rows, cap = self.ro if readout_only else self.kv
        send = torch.zeros(self.P, cap, c1 - c0, dtype=buf.dtype, device=buf.device)
        for q in range(self.P):
            if recv_slots[q].numel():
                send[q, : recv_slots[q].numel()] = buf[recv_slots[q], c0:c1]
        recv = self._a2a(send)
        for q in range(self.P):
            n = send_rows[q].numel()
            if n:
                if readout_only:  # a row belongs to one session: exactly one rank reads it out
                    buf[send_rows[q], c0:c1] = recv[q, :n]
                else:
                    buf[send_rows[q], c0:c1] = buf[send_rows[q], c0:c1] + recv[q, :n]


class HaloTrainStep(FusedTrainStep):
    """Data-parallel training step over a global batch cut at destination-node ranges
    (``cuts``: world + 1 increasing node offsets, default equal ranges), with the per-layer
    halo exchange above.  Every rank calls it with the SAME global batch; SyncBN; the split
    layer path (projection GEMM + row-parallel attention); eager launches."""

    def __init__(self, model, cuts=None, **kw):
        for k in ("lazy", "lagged", "shard_table"):
            if kw.get(k):
                raise ValueError(f"the halo step does not combine with {k}")
        kw.update(data_parallel=True, sync_bn=True, use_graph=False)
        super().__init__(model, **kw)
        if self.eng.D not in (64, 128):
            raise NotImplementedError("the halo step runs the split layer path (D in {64, 128})")
        import os

        if os.environ.get("GTR_ATTN", "").startswith("g"):
            raise ValueError("the halo step needs the row-parallel attention (unset GTR_ATTN=group)")
        self._force_split = True
        self.cuts = cuts
        self.halo = None
        self.parts = None

    def _bind(self, caps: Caps):
        super()._bind(caps)
        if not self.split:
            raise RuntimeError("the halo step needs the split layer path")

    def __call__(self, batch: SessionBatch):
        if self.eng.K > 0 and self.model.laplacian_pe._cached_pe is None:
            raise RuntimeError("Laplacian PE not precomputed. Call precompute() first.")
        N, B, E, n_neg = batch.sizes()
        if N <= 1:
            raise ValueError("Expected more than 1 value per channel when training (BatchNorm1d)")
        batch.check_ids(self.eng.T)
        parts = plan_halo(batch, self.world, self.cuts)
        caps = halo_caps(parts, n_neg)
        self._loss_batch = B / self.world
        if self.caps is None or not self.caps.fits(caps.n_cap, caps.b_cap, caps.e_cap, caps.n_neg):
            self._bind(caps if self.caps is None else self.caps.grow(caps.n_cap, caps.b_cap, caps.e_cap, n_neg))
        self.cfg.loss_batch = float(self._loss_batch)
        self.parts = parts
        self.halo = HaloExchange(parts, self.rank, self.dev, self.group)
        blob = torch.from_numpy(pack_halo(parts[self.rank], self.caps))
        self.blob.copy_(blob.to(self.dev))
        return self.run()

    def _pieces(self, with_pe: bool):
        import ctypes as C

        from etpgt.backend import _lib as L

        eng, ws, cfg, hx = self.eng, self.ws, self.cfg, self.halo
        bs = self.bs
        lib = L.lib()
        Lc, D = eng.L, eng.D

        def st():
            return torch.cuda.current_stream(self.dev).cuda_stream

        def proj(l):
            def f():
                if l == 0:
                    self._begin(bs, st())
                L.check(lib.gtr_qkvs_fwd(C.byref(cfg), C.byref(bs), C.byref(eng.fill_embed()), ws.structs, l, st()),
                        "qkvs_fwd")
            return f

        def attn(l):
            return lambda: L.check(lib.gtr_attn_fwd(C.byref(cfg), C.byref(bs), ws.structs, l, st()), "attn_fwd")

        def after_attn(l):
            def f():
                self._gather_fwd(l)
                if l == Lc - 1:  # the straddling sessions' last-layer rows for the readout
                    hx.fetch(ws.layers[l]["out"], 0, D, readout_only=True)
                    hx.fetch(ws.layers[l]["xin"], 0, D, readout_only=True)
            return f

        def head():
            eng.run_head(ws, cfg, bs, L.RO_FWD | L.RO_LOSS | L.RO_BWD, self.loss_kind, self.temperature, self.alpha)

        def after_head():
            hx.give_back(ws.layers[Lc - 1]["dy"], 0, D, readout_only=True)
            self._gather_bwd(Lc - 1)

        def attn_bwd(l):
            return lambda: L.check(lib.gtr_attn_bwd(C.byref(cfg), C.byref(bs), ws.structs, l, st()), "attn_bwd")

        def dx(l):
            def f():
                L.check(lib.gtr_qkvs_bwd(C.byref(cfg), C.byref(bs), ws.structs, l, ws.dx0.data_ptr(), st()),
                        "qkvs_bwd")
                if l == 0:
                    eng._wgrad(ws, cfg, bs, 0, Lc, st())
                    self.dp.launch_pack(bs, st())
            return f

        pieces = []
        for l in range(Lc):  # K / V of the ghost rows: columns [D, 3D) of qkvs
            pieces.append((proj(l), (lambda l=l: hx.fetch(ws.layers[l]["qkvs"], D, 3 * D))))
            pieces.append((attn(l), after_attn(l)))
        pieces.append((head, after_head))
        for l in range(Lc - 1, -1, -1):
            pieces.append((attn_bwd(l), (lambda l=l: hx.give_back(ws.layers[l]["dqkvs"], D, 3 * D))))
            pieces.append((dx(l), (lambda l=l: self._gather_bwd(l - 1)) if l > 0 else self.dp.exchange))
        pieces.append((lambda: self._launch_b(with_pe), None))
        return pieces
