"""GPU batch constructor: SessionDataset.__getitem__ + collate_fn
(etpgt/train/dataloader.py:64-202) as HIP kernels (libgtr_hip ``gtr_build_batch``).

``GpuSessionStore`` keeps a dataset resident in HBM: the click sequences (CSR by
session), an open-addressing hash of the co-occurrence edge keys item_i * T + item_j
(graph_edges.csv, item_i <= item_j) and every session's node / edge counts.
``GpuBatchBuilder`` walks an epoch order of session ids with a device cursor and writes
each batch straight into a fused step's packed batch image — the training step then
runs without any host work per batch, and the build is captured in the step's hipGraph
(``FusedTrainStep.attach_builder``).

Semantics per session: the last ``max_session_length`` clicks, target = the last,
nodes = sorted unique context ids, edges = graph edges with both endpoints in the
context (directed item_i -> item_j, (src, dst) order), ``num_negatives`` negatives
uniform in [1, T) rejecting the session's clicks.  The reference draws negatives with
``torch.randint`` on the host; here they come from a counter-based hash of (seed, batch
position, draw) — the same distribution, reproducible on the device
(oracle/batch_ref.py restates the stream for the parity tests).
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from etpgt.backend import _lib as L
from etpgt.data.batch import Caps, blob_layout


class GpuSessionStore:
    def __init__(self, session_ptr, session_items, edge_keys, num_items: int, device, max_session_length: int = 50):
        ptr = np.asarray(session_ptr, np.int64)
        items = np.asarray(session_items, np.int64)
        if ptr.ndim != 1 or ptr.size < 2 or ptr[0] != 0 or np.any(np.diff(ptr) < 0) or ptr[-1] != items.size:
            raise ValueError("session_ptr must be a CSR offset array over session_items")
        if np.any(np.diff(ptr) < 2):
            raise ValueError("every session needs at least 2 clicks (a context and a target)")
        if not 2 <= max_session_length <= 64:
            raise ValueError("max_session_length must be in [2, 64] on the GPU batch constructor")
        if items.size and (items.min() < 0 or items.max() >= num_items):
            raise IndexError(f"session items outside [0, {num_items})")
        if items.size >= 2**31:
            raise ValueError("more than 2^31 clicks")
        self.device = torch.device(device)
        self.T = int(num_items)
        self.S = int(ptr.size - 1)
        self.max_len = int(max_session_length)
        dev = self.device
        self.ptr_d = torch.from_numpy(ptr.astype(np.int32)).to(dev)
        self.items_d = torch.from_numpy(items.astype(np.int32)).to(dev)
        keys = np.asarray(edge_keys, np.int64)
        lib = L.lib()
        ns = C.c_int64(0)
        L.check(lib.gtr_edge_hash_slots(int(keys.size), C.byref(ns)), "edge_hash_slots")
        self.num_slots = int(ns.value)
        self.slots = torch.empty(self.num_slots, dtype=torch.int64, device=dev)
        keys_d = torch.from_numpy(keys).to(dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        L.check(lib.gtr_edge_hash_build(keys_d.data_ptr(), int(keys.size), self.slots.data_ptr(), self.num_slots, st),
                "edge_hash_build")
        self.nodes_d = torch.zeros(self.S, dtype=torch.int32, device=dev)
        self.edges_d = torch.zeros(self.S, dtype=torch.int32, device=dev)
        self.ss = L.GtrSessions()
        self.ss.sess_ptr, self.ss.sess_items = self.ptr_d.data_ptr(), self.items_d.data_ptr()
        self.ss.sess_nodes, self.ss.sess_edges = self.nodes_d.data_ptr(), self.edges_d.data_ptr()
        self.ss.num_sessions, self.ss.num_items = self.S, self.T
        L.check(lib.gtr_session_counts(C.byref(self.ss), self.slots.data_ptr(), self.num_slots, self.max_len,
                                       self.nodes_d.data_ptr(), self.edges_d.data_ptr(), st), "session_counts")
        self.nodes = self.nodes_d.cpu().numpy().astype(np.int64)
        self.edges = self.edges_d.cpu().numpy().astype(np.int64)

    @classmethod
    def from_synthetic(cls, data, device, max_session_length: int = 50) -> "GpuSessionStore":
        return cls(data.session_ptr, data.session_items, data.edge_keys, data.table_rows, device, max_session_length)

    @classmethod
    def from_dataset(cls, ds, device) -> "GpuSessionStore":
        """From an etpgt.train.SessionDataset (sessions in session-id order)."""
        ei = ds.edge_index.numpy()
        keys = np.unique(ei[0].astype(np.int64) * ds.num_items + ei[1].astype(np.int64))
        return cls(ds._ptr, ds._items, keys, ds.num_items, device, ds.max_session_length)


class GpuBatchBuilder:
    """Batches of ``batch_size`` sessions in epoch order, built on the device."""

    def __init__(self, store: GpuSessionStore, batch_size: int, num_negatives: int, seed: int = 0,
                 stride: int | None = None):
        """``stride``: positions the cursor advances per batch (default ``batch_size``); a
        data-parallel rank r of P builds its share of each global batch with
        ``stride = P * batch_size`` from a cursor started at ``r * batch_size``
        (gtr_build_batch_strided)."""
        if batch_size <= 0 or batch_size > 16384:
            raise ValueError("batch_size must be in [1, 16384] on the GPU batch constructor")
        if num_negatives <= 0:
            raise ValueError("num_negatives must be positive")
        if stride is not None and stride < batch_size:
            raise ValueError("stride must be >= batch_size")
        self.store = store
        self.B = int(batch_size)
        self.stride = int(batch_size if stride is None else stride)
        self.n_neg = int(num_negatives)
        self.seed = int(seed) & 0x7FFFFFFF
        dev = store.device
        self.cursor = torch.zeros(1, dtype=torch.int64, device=dev)
        self.start = torch.zeros(1, dtype=torch.int64, device=dev)
        # [this batch's code, sticky OR since the last check_status()] (gtr_build_batch)
        self.status = torch.zeros(2, dtype=torch.int32, device=dev)
        self.pos = 0  # host mirror of the device cursor
        self.scratch = None
        self.order_h = np.arange(store.S, dtype=np.int64)
        self.order_d = torch.from_numpy(self.order_h.astype(np.int32)).to(dev)

    def set_epoch_order(self, order, position: int = 0) -> None:
        """Session ids in visiting order (e.g. a permutation); batches wrap around."""
        o = np.asarray(order, np.int64)
        if o.ndim != 1 or o.size == 0 or o.min() < 0 or o.max() >= self.store.S:
            raise ValueError("order must list session ids in [0, S)")
        self.order_h = o
        new = torch.from_numpy(o.astype(np.int32))
        prev = getattr(self, "order_d", None)
        if prev is not None and prev.numel() == new.numel():
            # in place: a step graph captured with this builder holds the buffer's address
            # (a fresh tensor would leave the graph reading the previous epoch's freed order)
            prev.copy_(new)
        else:
            self.order_d = new.to(self.store.device)
        self.seek(position)

    def seek(self, position: int) -> None:
        """Put the cursor at ``position`` (the next batch's first session)."""
        self.cursor.fill_(int(position))
        self.pos = int(position)

    def batch_sizes(self, num_batches: int, position: int = 0) -> tuple[np.ndarray, np.ndarray]:
        """(N, E) of the next ``num_batches`` batches from ``position`` (host, from the counts)."""
        idx = (position + self.stride * np.arange(num_batches)[:, None] + np.arange(self.B)[None, :]) \
            % self.order_h.size
        sess = self.order_h[idx]
        return self.store.nodes[sess].sum(1), self.store.edges[sess].sum(1)

    def plan_caps(self, num_batches: int | None = None, position: int = 0, extra=()) -> Caps:
        """Capacities covering the next ``num_batches`` batches (default: one epoch) and
        every ``(position, sessions)`` window in ``extra`` (e.g. a data-parallel rank's
        last, partial batch, which starts at ``i*P*B + rank*b`` rather than on the
        stride grid)."""
        if num_batches is None:
            num_batches = max(1, -(-self.order_h.size // self.stride))
        N, E = self.batch_sizes(num_batches, position)
        n_max, e_max = int(N.max()), int(E.max())
        for pos, b in extra:
            n, e = self._sizes_at(int(pos), int(b))
            n_max, e_max = max(n_max, n), max(e_max, e)
        return Caps.bucket(n_max, self.B, max(e_max, 1), self.n_neg)

    def launch(self, bs: L.GtrBatch, caps: Caps, stream: int, B: int | None = None) -> None:
        """Build the next batch (``B`` sessions, default the builder's batch size) into the
        batch image ``bs`` (capacities ``caps``)."""
        B = self.B if B is None else int(B)
        if not 0 < B <= caps.b_cap:
            raise ValueError(f"batch of {B} sessions does not fit b_cap {caps.b_cap}")
        if self.scratch is None or self.scratch.numel() < 2 * caps.b_cap + 2:
            # + 2: the one-launch build's arrival ticket (gtr_build_batch, zero between builds)
            self.scratch = torch.zeros(2 * caps.b_cap + 2, dtype=torch.int32, device=self.store.device)
            self._ticket_at = 2 * caps.b_cap
        elif getattr(self, "_ticket_at", None) != 2 * caps.b_cap:
            # rebound to other capacities: the ticket words may hold a node / edge offset the
            # multi-workgroup scan (B > 256) wrote there -- the last-arriver test would then
            # never fire and the cursor would stop advancing
            self.scratch[2 * caps.b_cap: 2 * caps.b_cap + 2].zero_()
            self._ticket_at = 2 * caps.b_cap
        st = self.store
        stride = max(self.stride, B)
        L.check(L.lib().gtr_build_batch_strided(C.byref(st.ss), st.slots.data_ptr(), st.num_slots, st.max_len,
                                                self.order_d.data_ptr(), self.cursor.data_ptr(), B, stride, caps.R,
                                                self.seed, C.byref(bs), self.scratch.data_ptr(),
                                                self.start.data_ptr(), self.status.data_ptr(), stream),
                "build_batch")
        self.pos += stride

    def check_status(self, group=None) -> None:
        """Raise if any batch built since the last check failed (host sync).  Under a
        process group of more than one rank the sticky code is MAX-all-reduced first, so
        every rank raises at the same point (a rank-local raise would leave the others
        blocked in the step's next collective)."""
        code = int(self.status[1].item())
        self.status.zero_()
        import torch.distributed as dist

        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dev = self.store.device if dist.get_backend(group) != "gloo" else "cpu"
            t = torch.tensor([code], dtype=torch.int32, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            code = int(t.item())
        if code & 2:
            raise RuntimeError("negative sampling: a session holds (nearly) every catalog item, so no "
                               "negative outside it exists (the reference would loop forever)")
        if code & 1:
            raise RuntimeError("GPU batch exceeded its capacities")

    def build(self, caps: Caps | None = None, B: int | None = None) -> tuple[Caps, torch.Tensor]:
        """Build the next batch into a fresh blob (eager; tests and tools)."""
        from etpgt.backend.engine import Engine

        B = self.B if B is None else int(B)
        if caps is None:
            N, E = self._sizes_at(self.pos, B)
            caps = Caps.bucket(N, B, max(E, 1), self.n_neg)
        blob = torch.zeros(blob_layout(caps)["_total"], dtype=torch.int32, device=self.store.device)
        bs = Engine.batch_struct(caps, blob)
        self.launch(bs, caps, torch.cuda.current_stream(self.store.device).cuda_stream, B)
        self.check_status()
        return caps, blob

    def _sizes_at(self, position: int, B: int) -> tuple[int, int]:
        sess = self.order_h[(position + np.arange(B)) % self.order_h.size]
        return int(self.store.nodes[sess].sum()), int(self.store.edges[sess].sum())

    def build_device_batch(self, B: int | None = None) -> "DeviceBatch":
        """The next batch as a PyG-Batch-like object whose index arrays live in HBM."""
        B = self.B if B is None else int(B)
        N, _ = self._sizes_at(self.pos, B)
        caps, blob = self.build(None, B)
        return DeviceBatch(caps, blob, N, B, self.n_neg)


class DeviceBatch:
    """A batch built on the device (``GpuBatchBuilder``): the packed image plus the PyG
    ``Batch`` fields the model / Trainer read (``x``, ``target_item``,
    ``negative_items``, ``num_graphs``), as views into the image (int32 -> int64)."""

    laplacian_pe = None

    def __init__(self, caps: Caps, blob: torch.Tensor, num_nodes: int, num_graphs: int, n_neg: int):
        self.caps, self.blob = caps, blob
        self._N, self._B, self._n = int(num_nodes), int(num_graphs), int(n_neg)
        self._lay = blob_layout(caps)

    def _view(self, name: str, count: int) -> torch.Tensor:
        o, _ = self._lay[name]
        return self.blob[o: o + count].long()

    @property
    def num_graphs(self) -> int:
        return self._B

    @property
    def num_nodes(self) -> int:
        return self._N

    @property
    def x(self) -> torch.Tensor:
        return self._view("node_item", self._N)

    @property
    def target_item(self) -> torch.Tensor:
        return self._view("target", self._B)

    @property
    def negative_items(self) -> torch.Tensor:
        return self._view("negatives", self._B * self._n)

    @property
    def ptr(self) -> torch.Tensor:
        return self._view("node_ptr", self._B + 1)

    @property
    def batch(self) -> torch.Tensor:
        p = self.ptr
        return torch.repeat_interleave(torch.arange(self._B, device=p.device), p[1:] - p[:-1])

    def to(self, device, non_blocking: bool = False) -> "DeviceBatch":
        d = torch.device(device)
        if d.type != self.blob.device.type or (d.index is not None and d.index != self.blob.device.index):
            raise ValueError("a device-built batch stays on the device it was built on")
        return self
