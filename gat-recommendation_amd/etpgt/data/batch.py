"""Session batch layout (PyG ``Batch`` duck type) and its packed HBM image.

The reference hands the model a PyG ``Batch`` (dataloader.py:157-202): ``x`` [N]
global item ids, ``edge_index`` [2, E] offset by the cumulative node count,
``batch`` [N] sorted session ids, ``target_item`` [B], ``negative_items`` [B*n]
and optionally ``laplacian_pe`` [N, k].  ``SessionBatch`` keeps exactly those
fields (so reference-style code reads it unchanged) and adds the derived index
structures the HIP kernels consume: session offsets (PyG ``ptr``), CSR by
destination (attention softmax / aggregation) and CSR by source (dK / dV
gathered without atomics).

``pack_batch`` writes all int32 index arrays into ONE contiguous blob with a
fixed-capacity layout, so a batch moves to the device with a single copy and a
captured hipGraph can be replayed over batches of any shape within capacity.
"""

from __future__ import annotations

import os

from dataclasses import dataclass

import numpy as np
import torch


def _np(t) -> np.ndarray:
    if isinstance(t, torch.Tensor):
        return t.detach().cpu().numpy()
    return np.asarray(t)


@dataclass(frozen=True)
class Caps:
    """Capacities of a packed batch (node, session, edge, negatives per session)."""

    n_cap: int
    b_cap: int
    e_cap: int
    n_neg: int

    @property
    def R(self) -> int:
        """Row-group width of the layer kernels: a workgroup owns every session whose
        first node lies in [g*R, (g+1)*R)."""
        # a group's rows are R plus the tail of its last session, and the LDS fast path of
        # the layer kernels takes <= 32 rows at D = 128 (RMAX): R = 32 sent nearly every
        # group of a large batch down the global-memory path
        # small batches (<= 32 groups of 8): a group of ~8 rows fills ONE 16-row MFMA tile in
        # the QKVS projection and dX instead of two, and its attention phases are half as
        # long; the groups are still few enough to share one XCD (measured C2 0.0903 ->
        # 0.0866 ms, C3 0.150 -> 0.142 ms per step; R = 8 at B = 8192 took 1.25 -> 1.70 ms)
        r = os.environ.get("GTR_ROW_GROUP")  # experiments: a fixed width
        if r:
            return int(r)
        if self.n_cap <= 256:
            return 8
        return 16 if self.n_cap <= 65536 else 32

    @property
    def g_cap(self) -> int:
        return (self.n_cap + self.R - 1) // self.R

    def fits(self, n: int, b: int, e: int, n_neg: int) -> bool:
        return n <= self.n_cap and b <= self.b_cap and e <= self.e_cap and n_neg == self.n_neg

    @staticmethod
    def bucket(n: int, b: int, e: int, n_neg: int) -> "Caps":
        """Round capacities up on a geometric grid (4 steps per doubling) so that
        batches of varying shape share a few workspaces / captured graphs."""
        def up(x):
            x = max(int(x), 1)
            p = 16
            while p < x:
                p = p * 2
            for q in (p // 2 + p // 8, p // 2 + p // 4, p // 2 + 3 * p // 8, p):
                if q >= x and q >= 16:
                    return q
            return p
        return Caps(up(n), up(b), up(e), n_neg)

    def grow(self, n: int, b: int, e: int, n_neg: int) -> "Caps":
        def up(x, have):
            return have if x <= have else max(int(x * 1.25) + 16, 16)
        return Caps(up(n, self.n_cap), up(b, self.b_cap), up(e, self.e_cap), n_neg)


def _align4(x: int) -> int:
    return (x + 3) & ~3


def blob_layout(caps: Caps) -> dict:
    """int32 offsets of each array inside the packed blob (16-byte aligned regions)."""
    n, b, e, k = caps.n_cap, caps.b_cap, caps.e_cap, max(caps.n_neg, 1)
    g = caps.g_cap
    sizes = [
        ("hdr", 8), ("node_item", n), ("node_ptr", b + 1), ("in_ptr", n + 1), ("in_src", e),
        ("out_ptr", n + 1), ("out_edge", e), ("out_dst", e), ("target", b), ("negatives", b * k),
        ("grp_row", g + 1), ("grp_edge", g + 1),
    ]
    off, lay = 0, {}
    for name, sz in sizes:
        lay[name] = (off, sz)
        off += _align4(max(sz, 1))
    lay["_total"] = off
    return lay


class SessionBatch:
    """PyG-Batch-compatible session batch (x, edge_index, batch, ptr, target_item,
    negative_items, laplacian_pe) with lazily built CSR structures."""

    def __init__(self, x, edge_index, batch=None, target_item=None, negative_items=None,
                 laplacian_pe=None, ptr=None, num_graphs=None):
        self.x = x
        self.edge_index = edge_index
        if batch is None and ptr is not None:
            p = _np(ptr).astype(np.int64)
            batch = torch.from_numpy(np.repeat(np.arange(len(p) - 1), np.diff(p)))
        self.batch = batch
        self.target_item = target_item
        self.negative_items = negative_items
        self.laplacian_pe = laplacian_pe
        self._ptr = ptr
        self._num_graphs = num_graphs
        self._packed = None  # (caps, host int32 blob)
        self._device_blob = {}  # (device, caps) -> device tensor

    # --- PyG Batch surface ------------------------------------------------------------
    @property
    def num_graphs(self) -> int:
        if self._num_graphs is not None:
            return int(self._num_graphs)
        if self.target_item is not None:
            return int(self.target_item.shape[0])
        b = _np(self.batch)
        return int(b.max()) + 1 if b.size else 0

    @property
    def num_nodes(self) -> int:
        return int(self.x.shape[0])

    @property
    def num_edges(self) -> int:
        return int(self.edge_index.shape[1])

    @property
    def ptr(self) -> torch.Tensor:
        if self._ptr is None:
            b = _np(self.batch).astype(np.int64)
            counts = np.bincount(b, minlength=self.num_graphs) if b.size else np.zeros(self.num_graphs, np.int64)
            p = np.zeros(len(counts) + 1, np.int64)
            np.cumsum(counts, out=p[1:])
            self._ptr = torch.from_numpy(p)
        return self._ptr

    def to(self, device, non_blocking: bool = False) -> "SessionBatch":
        """Move tensors (like PyG ``Batch.to``) and stage the packed index blob on
        ``device`` with one copy, so the model's kernels find it ready."""
        def mv(t):
            return None if t is None else t.to(device, non_blocking=non_blocking)

        out = SessionBatch(
            mv(self.x), mv(self.edge_index), mv(self.batch), mv(self.target_item), mv(self.negative_items),
            mv(self.laplacian_pe), self.ptr, self._num_graphs,
        )
        out._packed = self._packed
        out._device_blob = self._device_blob
        if torch.device(device).type == "cuda":
            out.device_blob(torch.device(device))
        return out

    # --- packed image -------------------------------------------------------------------
    def check_ids(self, num_items: int) -> None:
        """Every item id (nodes, targets, negatives) must index the item table."""
        for name in ("x", "target_item", "negative_items"):
            t = getattr(self, name)
            if t is None or t.numel() == 0:
                continue
            a = _np(t)
            if a.min() < 0 or a.max() >= num_items:
                raise IndexError(f"{name} holds item ids outside [0, {num_items})")

    def sizes(self) -> tuple[int, int, int, int]:
        B = self.num_graphs
        n_neg = 0
        if self.negative_items is not None and B > 0:
            n_neg = int(self.negative_items.numel()) // B
        return self.num_nodes, B, self.num_edges, n_neg

    def packed(self, caps: Caps | None = None) -> tuple[Caps, np.ndarray]:
        if self._packed is not None and (caps is None or self._packed[0] == caps):
            return self._packed
        N, B, E, n_neg = self.sizes()
        if caps is None:
            caps = Caps.bucket(N, B, E, n_neg)
        self._packed = (caps, pack_batch(self, caps))
        return self._packed

    def device_blob(self, device: torch.device, caps: Caps | None = None) -> tuple[Caps, torch.Tensor]:
        caps, host = self.packed(caps)
        key = (str(device), caps)
        t = self._device_blob.get(key)
        if t is None:
            t = torch.from_numpy(host).to(device, non_blocking=False)
            self._device_blob[key] = t
        return caps, t


def build_csr(src: np.ndarray, dst: np.ndarray, n: int):
    """CSR by destination (stable: keeps the original edge order inside a row) and
    CSR by source over the destination-ordered edge positions."""
    E = src.shape[0]
    order = np.argsort(dst, kind="stable")
    in_src = src[order]
    dst_sorted = dst[order]
    in_ptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(dst, minlength=n), out=in_ptr[1:])
    order2 = np.argsort(in_src, kind="stable")  # positions in dst order, grouped by source
    out_edge = order2
    out_dst = dst_sorted[order2]
    out_ptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(src, minlength=n), out=out_ptr[1:])
    assert out_edge.shape[0] == E
    return in_ptr, in_src, out_ptr, out_edge, out_dst, order


def pack_batch(sb: SessionBatch, caps: Caps) -> np.ndarray:
    """Validate a batch and write its int32 HBM image (see ``blob_layout``)."""
    N, B, E, n_neg = sb.sizes()
    if not caps.fits(N, B, E, n_neg):
        raise ValueError(f"batch (N={N}, B={B}, E={E}, n={n_neg}) exceeds capacity {caps}")
    x = _np(sb.x).astype(np.int64)
    ei = _np(sb.edge_index).astype(np.int64).reshape(2, -1)
    if sb.batch is not None and N:
        bv = _np(sb.batch).astype(np.int64)
        if bv.shape[0] != N or np.any(np.diff(bv) < 0) or bv[0] < 0:
            raise ValueError("batch vector must be sorted with contiguous sessions (PyG layout)")
    ptr = _np(sb.ptr).astype(np.int64)
    if ptr.shape[0] != B + 1 or ptr[0] != 0 or ptr[-1] != N or np.any(np.diff(ptr) < 0):
        raise ValueError("batch vector must be sorted with contiguous sessions (PyG layout)")
    if N and np.any(np.diff(ptr) == 0):
        raise ValueError("every session needs at least one node")
    src, dst = ei[0], ei[1]
    if E and (src.min() < 0 or dst.min() < 0 or src.max() >= N or dst.max() >= N):
        raise ValueError("edge_index out of range")
    if E:
        sess = np.repeat(np.arange(B), np.diff(ptr))
        if np.any(sess[src] != sess[dst]):
            raise ValueError("edges must stay inside one session (block-diagonal batch)")
    in_ptr, in_src, out_ptr, out_edge, out_dst, _ = build_csr(src, dst, N)
    lay = blob_layout(caps)
    blob = np.zeros(lay["_total"], np.int32)

    def put(name, arr, fill=None):
        o, sz = lay[name]
        a = np.asarray(arr, np.int64)
        blob[o : o + a.shape[0]] = a
        if fill is not None and a.shape[0] < sz:
            blob[o + a.shape[0] : o + sz] = fill

    # row groups: group g = sessions whose first node lies in [g*R, (g+1)*R)
    R = caps.R
    G = (N + R - 1) // R
    starts = ptr[:-1]
    sess_of_group = np.searchsorted(starts, np.arange(G + 1) * R, side="left")
    grp_row = np.append(ptr, N)[np.minimum(sess_of_group, B)]
    grp_row[-1] = N
    grp_edge = in_ptr[grp_row]
    put("hdr", [N, B, E, n_neg, G, R, 0, 0])
    put("grp_row", grp_row, fill=N)
    put("grp_edge", grp_edge, fill=E)
    put("node_item", x)
    put("node_ptr", ptr, fill=N)
    put("in_ptr", in_ptr, fill=E)
    put("in_src", in_src)
    put("out_ptr", out_ptr, fill=E)
    put("out_edge", out_edge)
    put("out_dst", out_dst)
    if sb.target_item is not None:
        put("target", _np(sb.target_item).reshape(-1))
    if sb.negative_items is not None and n_neg:
        put("negatives", _np(sb.negative_items).reshape(-1))
    return blob


def collate_sessions(items: list[dict]) -> SessionBatch:
    """Batch per-session dicts {x [n] global ids, edge_index [2,e] local, target_item,
    negative_items [n_neg]} the way ``Batch.from_data_list`` does."""
    xs, eis, bs, tg, ng = [], [], [], [], []
    off = 0
    for b, it in enumerate(items):
        x = _np(it["x"]).astype(np.int64)
        ei = _np(it["edge_index"]).astype(np.int64).reshape(2, -1)
        xs.append(x)
        eis.append(ei + off)
        bs.append(np.full(x.shape[0], b, np.int64))
        off += x.shape[0]
        if it.get("target_item") is not None:
            tg.append(int(_np(it["target_item"]).reshape(())))
        if it.get("negative_items") is not None:
            ng.append(_np(it["negative_items"]).astype(np.int64).reshape(-1))
    cat = lambda l, shape: np.concatenate(l) if l else np.zeros(shape, np.int64)  # noqa: E731
    return SessionBatch(
        torch.from_numpy(cat(xs, (0,))),
        torch.from_numpy(np.concatenate(eis, axis=1) if eis else np.zeros((2, 0), np.int64)),
        torch.from_numpy(cat(bs, (0,))),
        torch.tensor(tg, dtype=torch.long) if tg else None,
        torch.from_numpy(np.concatenate(ng)) if ng else None,
        num_graphs=len(items),
    )


class Data:
    """PyG ``torch_geometric.data.Data`` duck type for the graph-level call sites that
    need one (``LaplacianPECached.precompute(Data(edge_index=..., num_nodes=...))``,
    reference train_baseline.py:236-243): keyword attributes, ``num_nodes`` inferred
    from ``x`` or ``edge_index`` when not given."""

    def __init__(self, x=None, edge_index=None, num_nodes: int | None = None, **kwargs):
        self.x = x
        self.edge_index = edge_index
        self._num_nodes = num_nodes
        for k, v in kwargs.items():
            setattr(self, k, v)

    @property
    def num_nodes(self) -> int:
        if self._num_nodes is not None:
            return int(self._num_nodes)
        if self.x is not None:
            return int(self.x.shape[0])
        if self.edge_index is not None and self.edge_index.numel():
            return int(self.edge_index.max()) + 1
        return 0
