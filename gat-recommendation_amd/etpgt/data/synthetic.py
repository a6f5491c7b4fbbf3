"""Synthetic RetailRocket-shaped workload — no dataset download.

Shape targets (docs/DATA_PIPELINE.md:127-137,200-206,287-295 of the reference):
82,173 items (table T = 82,174 with padding row 0), 737,716 canonical graph edges
(item_i <= item_j, self loops kept), 120,436 training sessions of length
3 + Geometric(mean 2.55) truncated to 50, Zipf item popularity with 30 % revisits
(scripts/data/00_generate_synthetic_data.py:24-139 semantics).  The co-occurrence
graph is built from the sessions with the +-5 window of scripts/data/04_build_graph.py
and padded with popularity-weighted random pairs to the target edge count.
Per-session batches follow etpgt/train/dataloader.py:64-202: context = all clicks
but the last, nodes = sorted unique context ids, edges = graph edges with both
endpoints in the context, directed smaller -> larger id (plus self loops),
negatives uniform in [1, T) excluding the session's items.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from etpgt.data.batch import SessionBatch

RETAILROCKET = dict(num_items=82_173, num_sessions=120_436, num_edges=737_716)
YOOCHOOSE_SCALE = dict(num_items=1_000_000, num_sessions=500_000, num_edges=9_000_000)


@dataclass
class SyntheticData:
    num_items: int          # T - 1 real items, ids 1..num_items
    session_ptr: np.ndarray  # [S+1]
    session_items: np.ndarray  # [sum len] item ids in click order
    edge_keys: np.ndarray    # sorted int64 keys a*T + b (a <= b)
    seed: int

    @property
    def table_rows(self) -> int:
        return self.num_items + 1

    @property
    def num_sessions(self) -> int:
        return self.session_ptr.shape[0] - 1

    def edge_index(self) -> np.ndarray:
        T = self.table_rows
        return np.stack([self.edge_keys // T, self.edge_keys % T])

    def session(self, s: int) -> np.ndarray:
        return self.session_items[self.session_ptr[s] : self.session_ptr[s + 1]]


def _zipf_sampler(rng, n_items: int, s: float):
    pop = 1.0 / np.arange(1, n_items + 1, dtype=np.float64) ** s
    cdf = np.cumsum(pop)
    cdf /= cdf[-1]
    perm = rng.permutation(n_items).astype(np.int64) + 1  # popularity rank -> item id

    def draw(k):
        r = np.searchsorted(cdf, rng.random(k), side="right")
        return perm[np.minimum(r, n_items - 1)]

    return draw


def make_sessions_and_graph(num_items: int = RETAILROCKET["num_items"],
                            num_sessions: int = RETAILROCKET["num_sessions"],
                            num_edges: int = RETAILROCKET["num_edges"],
                            zipf_s: float = 1.0, revisit: float = 0.3, max_len: int = 50,
                            window: int = 5, seed: int = 42) -> SyntheticData:
    rng = np.random.default_rng(seed)
    draw = _zipf_sampler(rng, num_items, zipf_s)
    lens = np.minimum(3 + rng.geometric(1.0 / 3.55, size=num_sessions) - 1, max_len).astype(np.int64)
    ptr = np.zeros(num_sessions + 1, np.int64)
    np.cumsum(lens, out=ptr[1:])
    total = int(ptr[-1])
    items = draw(total)
    pos = np.arange(total, dtype=np.int64) - np.repeat(ptr[:-1], lens)
    rev = (pos > 0) & (rng.random(total) < revisit)
    for p in range(1, max_len):
        idx = np.nonzero(rev & (pos == p))[0]
        if idx.size == 0:
            continue
        j = (rng.random(idx.size) * p).astype(np.int64)
        items[idx] = items[idx - p + j]
    T = num_items + 1
    sess_len = np.repeat(lens, lens)
    keys = []
    for off in range(1, window + 1):
        i = np.nonzero(pos + off < sess_len)[0]
        a, b = items[i], items[i + off]
        keys.append(np.minimum(a, b) * T + np.maximum(a, b))
    ek = np.unique(np.concatenate(keys))
    if ek.size < num_edges:
        need = num_edges - ek.size
        extra = []
        while need > 0:
            a, b = draw(need * 2), draw(need * 2)
            k = np.unique(np.minimum(a, b) * T + np.maximum(a, b))
            k = k[~np.isin(k, ek, assume_unique=False)]
            if extra:
                k = k[~np.isin(k, np.concatenate(extra))]
            k = rng.permutation(k)[:need]
            extra.append(k)
            need -= k.size
        ek = np.unique(np.concatenate([ek] + extra))
    return SyntheticData(num_items, ptr, items, ek, seed)


def session_example(data: SyntheticData, s: int, num_neg: int, rng: np.random.Generator) -> dict:
    """One session in the training layout (dataloader.py:64-124,157-202)."""
    T = data.table_rows
    seq = data.session(s)
    ctx = seq[:-1]
    uniq = np.unique(ctx)
    u = uniq.shape[0]
    ia, ib = np.triu_indices(u)  # a <= b (uniq sorted) incl. self pairs
    k = uniq[ia] * T + uniq[ib]
    pos = np.searchsorted(data.edge_keys, k)
    pos = np.minimum(pos, data.edge_keys.shape[0] - 1)
    hit = data.edge_keys[pos] == k
    ei = np.stack([ia[hit], ib[hit]]).astype(np.int64)
    seen = np.unique(seq)
    negs = np.empty(num_neg, np.int64)
    filled = 0
    while filled < num_neg:  # the first candidates outside the session, in draw order
        cand = rng.integers(1, T, size=num_neg * 2)
        ok = cand[~np.isin(cand, seen)][: num_neg - filled]
        negs[filled: filled + ok.size] = ok
        filled += ok.size
    return {"x": uniq.astype(np.int64), "edge_index": ei, "target_item": int(seq[-1]), "negative_items": negs}


def make_batches(data: SyntheticData, batch_size: int, num_batches: int, num_neg: int, seed: int = 42,
                 start: int = 0) -> list[SessionBatch]:
    """``num_batches`` consecutive batches of a seeded shuffle of the sessions."""
    from etpgt.data.batch import collate_sessions

    rng = np.random.default_rng(seed + 1)
    order = np.random.default_rng(seed).permutation(data.num_sessions)
    out = []
    for bi in range(num_batches):
        idx = order[(start + bi * batch_size + np.arange(batch_size)) % data.num_sessions]
        out.append(collate_sessions([session_example(data, int(s), num_neg, rng) for s in idx]))
    return out


def random_pe_table(num_rows: int, k: int, seed: int = 42) -> torch.Tensor:
    """|N(0, 1/sqrt(T))| stand-in for the [T, k] LapPE table (values do not affect timing)."""
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(num_rows, k, generator=g) / float(np.sqrt(num_rows))).abs()


def batch_stats(batches) -> dict:
    n = np.array([b.num_nodes for b in batches], np.float64)
    e = np.array([b.num_edges for b in batches], np.float64)
    B = np.array([b.num_graphs for b in batches], np.float64)
    return {"nodes_per_session": float(n.sum() / B.sum()), "edges_per_session": float(e.sum() / B.sum()),
            "max_nodes": int(n.max()), "max_edges": int(e.max())}
