"""Session dataset / collate — API of etpgt/train/dataloader.py (reference).

Same constructor, item semantics and batch layout as the reference
(dataloader.py:22-241): sessions sorted by timestamp, truncated to the last
``max_session_length`` events, target = last event, context = the rest,
negatives drawn with ``torch.randint(1, num_items)`` rejecting session items,
induced subgraph = graph edges with both endpoints in the context in the stored
``(item_i, item_j)`` direction.  Differences are in HOW, not WHAT: the induced
subgraph is found by binary search over sorted edge keys instead of a pandas
``isin`` over all 737k edges per session (≈24 ms -> tens of µs), and
``collate_fn`` returns an ``etpgt.data.SessionBatch`` (PyG ``Batch`` duck type
with the packed CSR image the HIP kernels consume).
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import pandas as pd
import torch
from torch.utils.data import Dataset

from etpgt.data.batch import SessionBatch


class SessionDataset(Dataset):
    def __init__(self, sessions_path: Path | str, graph_edges_path: Path | str, num_negatives: int = 5,
                 max_session_length: int = 50):
        self.sessions_path = Path(sessions_path)
        self.graph_edges_path = Path(graph_edges_path)
        self.num_negatives = num_negatives
        self.max_session_length = max_session_length
        self.sessions_df = pd.read_csv(sessions_path)
        df = self.sessions_df.sort_values(["session_id", "timestamp"], kind="stable")
        sid = df["session_id"].to_numpy()
        self._items = df["itemid"].to_numpy().astype(np.int64)
        bounds = np.nonzero(np.r_[True, sid[1:] != sid[:-1], True])[0]
        self._ptr = bounds
        self.session_ids = list(sid[bounds[:-1]])
        g = pd.read_csv(graph_edges_path, usecols=["item_i", "item_j"])
        ii = g["item_i"].to_numpy().astype(np.int64)
        jj = g["item_j"].to_numpy().astype(np.int64)
        self.edge_index = torch.from_numpy(np.stack([ii, jj]))
        self.num_items = int(max(self._items.max(initial=0), ii.max(initial=0), jj.max(initial=0)) + 1)
        self._T = self.num_items
        keys = ii * self._T + jj
        order = np.argsort(keys, kind="stable")
        self._ekeys = keys[order]
        self._eorder = order

    def __len__(self) -> int:
        return len(self.session_ids)

    def __getitem__(self, idx: int) -> dict:
        items = self._items[self._ptr[idx] : self._ptr[idx + 1]]
        if len(items) > self.max_session_length:
            items = items[-self.max_session_length :]
        target = items[-1]
        context = items[:-1]
        return {
            "session_items": torch.tensor(context, dtype=torch.long),
            "target_item": torch.tensor(target, dtype=torch.long),
            "negative_items": torch.tensor(self._sample_negatives(items), dtype=torch.long),
            "edge_index": self._build_session_subgraph(context),
        }

    def _sample_negatives(self, session_items: np.ndarray) -> list:
        s = set(int(v) for v in session_items)
        out = []
        while len(out) < self.num_negatives:
            v = torch.randint(1, self.num_items, (1,)).item()
            if v not in s:
                out.append(v)
        return out

    def _build_session_subgraph(self, context_items: np.ndarray) -> torch.Tensor:
        u = np.unique(context_items)
        if u.size == 0:
            return torch.zeros((2, 0), dtype=torch.long)
        a, b = np.meshgrid(u, u, indexing="ij")
        k = (a * self._T + b).reshape(-1)
        lo = np.searchsorted(self._ekeys, k, side="left")
        hi = np.searchsorted(self._ekeys, k, side="right")
        sel = np.concatenate([self._eorder[l:h] for l, h in zip(lo, hi) if h > l]) if np.any(hi > lo) else np.zeros(0, np.int64)
        if sel.size == 0:
            return torch.zeros((2, 0), dtype=torch.long)
        sel.sort()  # reference keeps graph-file order
        return self.edge_index[:, torch.from_numpy(sel)]


def collate_fn(batch: list[dict]) -> SessionBatch:
    """Global -> local remap per session + PyG-style concatenation (dataloader.py:157-202)."""
    xs, eis, bv, tg, ng = [], [], [], [], []
    off = 0
    for b, item in enumerate(batch):
        uniq = torch.unique(item["session_items"])
        ei = item["edge_index"]
        if ei.numel() > 0:
            u = uniq.numpy()
            src = np.searchsorted(u, ei[0].numpy())
            dst = np.searchsorted(u, ei[1].numpy())
            ok = (src < u.size) & (dst < u.size)
            ok &= (u[np.minimum(src, u.size - 1)] == ei[0].numpy()) & (u[np.minimum(dst, u.size - 1)] == ei[1].numpy())
            local = torch.from_numpy(np.stack([src[ok], dst[ok]]).astype(np.int64))
        else:
            local = torch.zeros((2, 0), dtype=torch.long)
        xs.append(uniq)
        eis.append(local + off)
        bv.append(torch.full((uniq.numel(),), b, dtype=torch.long))
        off += uniq.numel()
        tg.append(item["target_item"].reshape(()))
        ng.append(item["negative_items"].reshape(-1))
    return SessionBatch(torch.cat(xs), torch.cat(eis, dim=1), torch.cat(bv), torch.stack(tg), torch.cat(ng),
                        num_graphs=len(batch))


def create_dataloader(sessions_path: Path | str, graph_edges_path: Path | str, batch_size: int = 32,
                      num_negatives: int = 5, max_session_length: int = 50, shuffle: bool = True,
                      num_workers: int = 0, device_builder: bool = False, device: str = "cuda",
                      seed: int = 0, rank: int = 0, world: int = 1):
    """dataloader.py:205-241.  ``device_builder=True`` returns a ``DeviceSessionLoader``:
    the same epochs (order, batch sizes, last partial batch) built on the GPU
    (etpgt.data.gpu_batch) instead of host workers; ``Trainer`` then captures the build
    inside the fused step.  ``rank`` / ``world`` (device builder only): this rank's share
    of each global batch of ``world * batch_size`` sessions (data parallel)."""
    ds = SessionDataset(sessions_path, graph_edges_path, num_negatives, max_session_length)
    if device_builder:
        return DeviceSessionLoader(ds, batch_size, num_negatives, shuffle=shuffle, device=device, seed=seed,
                                   rank=rank, world=world)
    if world > 1:
        raise NotImplementedError("data-parallel training builds its batches on the GPU (device_builder=True)")
    return torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers,
                                       collate_fn=collate_fn)


class DeviceSessionLoader:
    """The epochs of ``DataLoader(SessionDataset, batch_size, shuffle, collate_fn)`` with
    every batch built on the GPU.

    * Order: every epoch consumes the global torch RNG exactly as iterating a
      ``DataLoader(shuffle=...)`` does: one int64 draw for the iterator's ``_base_seed``
      (``_BaseDataLoaderIter.__init__``), then -- ``shuffle=True`` -- the
      ``RandomSampler``'s seed draw and ``torch.randperm`` under it; ``shuffle=False``
      walks session-id order.  A run seeded like the reference therefore visits its first
      epoch in the reference's order (pinned against a real DataLoader in
      tests/test_host.py), and every later epoch too when nothing else draws from the
      global CPU generator between epochs -- true for the reference's CUDA runs with
      ``num_workers > 0`` (its default 4: the per-sample ``torch.randint`` negatives of
      dataloader.py:107-124 draw inside the workers).  With ``num_workers=0`` those draws
      consume the main process's generator, so later epochs' orders differ.
    * Batches: ``len(loader)`` = ceil(S / batch_size), the last one partial
      (``drop_last=False``).
    * Per session: the reference's example (last ``max_session_length`` clicks, target,
      sorted unique context, induced directed edges) bit for bit; negatives uniform in
      [1, T) rejecting the session's clicks, from the device's counter-based stream keyed
      by (seed, epoch * S + position) instead of ``torch.randint`` (same distribution,
      fresh every epoch).
    Iterating yields ``DeviceBatch`` objects (PyG-Batch-like views of HBM images) for any
    consumer; ``Trainer``'s fused step instead attaches ``builder`` and builds inside its
    captured graph.

    Data parallel (``world`` > 1, one process per GPU): every rank draws the same epoch
    order (same seed, same global-RNG draws) and rank r builds sessions
    [i*P*B + r*B, +B) of it for global batch i -- with the position-keyed negatives a
    single GPU draws for that global batch of P*B sessions (gtr_build_batch_strided).  The
    epoch is the full global batches, then -- when the remaining R sessions give every rank
    at least one -- a last global batch of P*floor(R/P) sessions split evenly; the
    R mod P sessions left over are dropped (DistributedSampler's drop_last rule, so that
    every rank's loss mean weighs equally)."""

    def __init__(self, dataset: SessionDataset, batch_size: int, num_negatives: int, shuffle: bool = True,
                 device: str = "cuda", seed: int = 0, rank: int = 0, world: int = 1):
        from etpgt.data.gpu_batch import GpuSessionStore

        self.dataset = dataset
        self._setup(GpuSessionStore.from_dataset(dataset, device), len(dataset), batch_size, num_negatives, shuffle,
                    seed, rank, world)

    @classmethod
    def from_store(cls, store, batch_size: int, num_negatives: int, shuffle: bool = True, seed: int = 0,
                   rank: int = 0, world: int = 1) -> "DeviceSessionLoader":
        """The same loader over a session store already resident on the device
        (``GpuSessionStore.from_synthetic``: the bench's RetailRocket-shaped sessions)."""
        self = cls.__new__(cls)
        self.dataset = None
        self._setup(store, int(store.S), batch_size, num_negatives, shuffle, seed, rank, world)
        return self

    def _setup(self, store, num_sessions, batch_size, num_negatives, shuffle, seed, rank, world):
        from etpgt.data.gpu_batch import GpuBatchBuilder

        if not 0 <= rank < world:
            raise ValueError("rank must lie in [0, world)")
        self.num_sessions = int(num_sessions)
        self.batch_size = int(batch_size)
        self.shuffle = bool(shuffle)
        self.rank, self.world = int(rank), int(world)
        self.store = store
        self.builder = GpuBatchBuilder(self.store, self.batch_size, num_negatives, seed=seed,
                                       stride=self.batch_size * self.world)
        self.epoch = -1
        self.order = None

    def __len__(self) -> int:
        return len(self.batch_sizes())

    def batch_sizes(self) -> list[int]:
        """Sessions of this rank's batches in an epoch."""
        S, B, P = self.num_sessions, self.batch_size, self.world
        full, rem = divmod(S, B * P)
        last = rem // P
        return [B] * full + ([last] if last > 0 else [])

    def batch_start(self, i: int) -> int:
        """Cursor position (epoch order, plus epoch * S) of this rank's batch i."""
        S, B, P = self.num_sessions, self.batch_size, self.world
        b = self.batch_sizes()[i]
        return self.epoch * S + i * B * P + self.rank * b

    def _epoch_order(self) -> np.ndarray:
        n = self.num_sessions
        torch.empty((), dtype=torch.int64).random_()  # _BaseDataLoaderIter.__init__: _base_seed
        if not self.shuffle:
            return np.arange(n, dtype=np.int64)
        seed = int(torch.empty((), dtype=torch.int64).random_().item())  # RandomSampler.__iter__
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(n, generator=g).numpy().astype(np.int64)

    def start_epoch(self) -> None:
        """Draw the next epoch's order and put the builder at its start."""
        self.epoch += 1
        self.order = self._epoch_order()
        self.builder.set_epoch_order(self.order, position=self.epoch * self.num_sessions + self.rank * self.batch_size)

    def __iter__(self):
        self.start_epoch()
        for i, b in enumerate(self.batch_sizes()):
            self.builder.seek(self.batch_start(i))
            yield self.builder.build_device_batch(b)
