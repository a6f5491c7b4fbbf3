"""Batch-construction oracle — TEST INFRASTRUCTURE ONLY (imported by tests/ only).

Parity pinning: the reference dataloader imports torch_geometric (absent here), so it
cannot run; this restatement is pinned by reading dataloader.py:64-202 only (parity
unpinned against executed reference output) and cross-checked against the host
SessionDataset / collate_fn mirror in tests/test_host.py.

CPU restatement of the reference's per-session example + collate semantics
(etpgt/train/dataloader.py:64-202) used to check the GPU batch constructor
(libgtr_hip gtr_build_batch, etpgt.data.gpu_batch):

* ``__getitem__`` (dataloader.py:64-104): the last ``max_session_length`` clicks
  (:84-85), target = the last click (:88), context = the rest (:91);
* ``_build_session_subgraph`` (:126-155): graph edges (item_i, item_j) with both ends in
  the context, in graph-file order (the edge keys are sorted, so (item_i, item_j)
  ascending), directed item_i -> item_j;
* ``collate_fn`` (:157-202): nodes = sorted unique context ids (``unique()``), edges
  remapped to local indices, PyG concatenation;
* ``_sample_negatives`` (:106-124): uniform in [1, T) rejecting session clicks, with
  replacement across draws.  The reference's ``torch.randint`` host stream is replaced
  by the device's counter-based stream (hash of seed, batch position, draw index; 64
  draws per round, accepted in draw order), restated here bit for bit.
"""

from __future__ import annotations

import numpy as np


def _u32(x):
    return np.asarray(x, dtype=np.uint64) & np.uint64(0xFFFFFFFF)


def mix3(a, b, c):
    """gtr_common.cuh mix3 in uint32 arithmetic (vectorised over c)."""
    M = np.uint64(0xFFFFFFFF)
    a, b, c = _u32(a), _u32(b), _u32(c)
    h = (a * np.uint64(0x9E3779B1)) & M
    h ^= (b + np.uint64(0x7F4A7C15) + ((h << np.uint64(6)) & M) + (h >> np.uint64(2))) & M
    h = (h * np.uint64(0x85EBCA77)) & M
    h ^= (c * np.uint64(0xC2B2AE3D)) & M
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x7FEB352D)) & M
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x846CA68B)) & M
    h ^= h >> np.uint64(16)
    return h


def negatives(seed: int, pos: int, clicks: np.ndarray, n: int, T: int) -> np.ndarray:
    seen = set(int(v) for v in clicks)
    out = []
    rnd = 0
    if len(seen & set(range(1, T))) == T - 1:  # nothing to find: the device builder gives up
        raise RuntimeError("negative sampling: the session covers the whole catalog")
    while len(out) < n:  # rejection until n are found (dataloader.py:107-124)
        if rnd == 1 << 20:
            raise RuntimeError("negative sampling: the session covers (nearly) the whole catalog")
        h = mix3(seed, pos, rnd * 64 + np.arange(64, dtype=np.uint64))
        cand = 1 + (h % np.uint64(T - 1)).astype(np.int64)
        for c in cand:
            if int(c) not in seen:
                out.append(int(c))
                if len(out) == n:
                    break
        rnd += 1
    return np.array(out, np.int64)


def session_example(ptr, items, edge_keys, T: int, s: int, max_len: int, n_neg: int, seed: int, pos: int) -> dict:
    clicks = np.asarray(items[ptr[s]:ptr[s + 1]], np.int64)[-max_len:]
    target = int(clicks[-1])
    ctx = clicks[:-1]
    uniq = np.unique(ctx)
    ia, ib = np.triu_indices(uniq.size)
    keys = uniq[ia] * T + uniq[ib]
    hit = np.isin(keys, edge_keys)
    return {"x": uniq, "edge_index": np.stack([ia[hit], ib[hit]]).astype(np.int64), "target_item": target,
            "negative_items": negatives(seed, pos, clicks, n_neg, T)}


def build_batch(ptr, items, edge_keys, T: int, order, start: int, B: int, max_len: int, n_neg: int,
                seed: int) -> list[dict]:
    """The per-session examples of the batch order[(start + b) % S], b < B."""
    S = len(ptr) - 1
    return [session_example(ptr, items, edge_keys, T, int(order[(start + b) % S]), max_len, n_neg, seed, start + b)
            for b in range(B)]
