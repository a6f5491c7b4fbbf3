"""Config C1 plumbing: the reference's run_full_pipeline.py quick path on the HIP model.

BASELINE.json configs[0] — "graph_transformer_optimized on 1k-node synthetic graph,
CPU reference path, 100 sessions, 3 epochs (run_full_pipeline.py plumbing)":

* ``generate_synthetic_events``   scripts/data/00_generate_synthetic_data.py:24-139,
  reproduced bit for bit: the same draws, in the same order, from the streams the
  reference seeds with ``set_seed`` (Python ``random`` and numpy's legacy global
  generator; here private instances seeded the same way, so the caller's global state is
  untouched): Zipf(1.5) item popularity, session length U[3, 20], 70 % new item /
  30 % re-view of a viewed item, exponential 5-minute gaps capped at 30 minutes,
  view / addtocart / transaction mix, then the timestamp sort.
* ``sessionize_events``           scripts/data/02_sessionize.py:25-81 (30-minute
  inactivity gap per visitor, sessions of >= 3 events, ``sess_<n>`` ids).
* ``build_co_event_graph``        scripts/data/04_build_graph.py:23-127 (pairs within
  +-5 steps of a session, canonical item_i <= item_j, count / last_ts, most frequent
  first; the event-pair histogram column is not kept: nothing on the hot path reads it).
* ``create_test_subset``          run_full_pipeline.py:34-82 (first ``num_sessions``
  sessions, graph edges among their items).
* ``create_batch_from_sessions``  run_full_pipeline.py:85-179 (first ``batch_size``
  sessions, timestamp order, context = all but the last event, sorted unique context
  items as nodes, induced co-event edges in BOTH directions, self loops when a session
  has none, the first ``num_negatives`` catalogue items outside the session as
  negatives; item ids remapped to 0..num_items-1 so id 0 is a real item that the
  embedding's padding_idx=0 silences, as in the reference).
* ``test_model_with_real_data``   run_full_pipeline.py:182-270 (Adam(lr=1e-3), the
  listwise loss on ``model.item_embedding``, ``num_epochs`` steps on the one batch).

Pandas sorts use the reference's calls (default, non-stable quicksort), so ties come
out in the same order.  tests/golden/c1_data.npz holds the reference scripts' own
output for seed 42 (oracle/gen_golden.py), which these functions reproduce exactly
(tests/test_host.py).  The model runs on the HIP path (libgtr_hip): there is no CPU
fallback here.
"""

from __future__ import annotations

import random
import time
from datetime import datetime

import numpy as np
import pandas as pd
import torch

from etpgt.data.batch import SessionBatch, collate_sessions
from etpgt.train.losses import create_loss_function

SESSION_GAP_MS = 30 * 60 * 1000  # 02_sessionize.py:20-22
MIN_SESSION_LENGTH = 3
CO_EVENT_WINDOW = 5  # 04_build_graph.py:21
_EVENT_PROBS = (  # (in cart, viewed before, new item)
    {"view": 0.3, "addtocart": 0.2, "transaction": 0.5},
    {"view": 0.6, "addtocart": 0.35, "transaction": 0.05},
    {"view": 0.85, "addtocart": 0.13, "transaction": 0.02},
)


def generate_synthetic_events(num_sessions: int = 10000, num_items: int = 5000, min_session_length: int = 3,
                              max_session_length: int = 20, start_date: str = "2024-01-01",
                              duration_days: int = 90, seed: int = 42) -> pd.DataFrame:
    """Synthetic RetailRocket-like events (timestamp, visitorid, event, itemid,
    transactionid), sorted by timestamp; one visitor per generated session."""
    py = random.Random(seed)              # == random.seed(seed)
    npr = np.random.RandomState(seed)     # == np.random.seed(seed)
    pop = npr.zipf(1.5, num_items)
    pop = pop / pop.sum()
    start_ts = int(datetime.strptime(start_date, "%Y-%m-%d").timestamp() * 1000)
    end_ts = start_ts + duration_days * 24 * 60 * 60 * 1000
    rows = []
    for s in range(num_sessions):
        length = py.randint(min_session_length, max_session_length)
        ts = py.randint(start_ts, end_ts - 3600000)
        viewed, cart = set(), set()
        for e in range(length):
            if e > 0:
                ts += min(int(npr.exponential(300)), 1800) * 1000
            if e == 0 or py.random() < 0.7:
                item = int(npr.choice(num_items, p=pop))
            elif viewed:
                item = int(py.choice(list(viewed)))
            else:
                item = int(npr.choice(num_items, p=pop))
            probs = _EVENT_PROBS[0] if item in cart else _EVENT_PROBS[1] if item in viewed else _EVENT_PROBS[2]
            ev = py.choices(list(probs.keys()), weights=list(probs.values()))[0]
            viewed.add(item)
            if ev == "addtocart":
                cart.add(item)
            rows.append({"timestamp": ts, "visitorid": f"visitor_{s}", "event": ev, "itemid": item,
                         "transactionid": f"txn_{s}_{e}" if ev == "transaction" else None})
    return pd.DataFrame(rows).sort_values("timestamp").reset_index(drop=True)


def sessionize_events(events_df: pd.DataFrame, gap_ms: int = SESSION_GAP_MS,
                      min_length: int = MIN_SESSION_LENGTH) -> pd.DataFrame:
    """Sessions by visitor and inactivity gap, with a ``session_id`` column."""
    df = events_df.sort_values(["visitorid", "timestamp"]).reset_index(drop=True)
    gap = df.groupby("visitorid")["timestamp"].diff()
    df["session_id"] = "sess_" + (gap.isna() | (gap > gap_ms)).cumsum().astype(str)
    size = df.groupby("session_id").size()
    return df[df["session_id"].isin(size[size >= min_length].index)].copy()


def build_co_event_graph(sessions_df: pd.DataFrame, window: int = CO_EVENT_WINDOW) -> pd.DataFrame:
    """Co-event edges (item_i <= item_j, count, last_ts), most frequent first."""
    edges: dict[tuple[int, int], list[int]] = {}
    for _, g in sessions_df.groupby("session_id"):
        ev = g.sort_values("timestamp").reset_index(drop=True)
        items = ev["itemid"].tolist()
        tss = ev["timestamp"].tolist()
        for i in range(len(items)):
            for j in range(i + 1, min(i + window + 1, len(items))):
                a, b, ts = items[i], items[j], tss[i]
                if a > b:
                    a, b, ts = b, a, tss[j]
                rec = edges.setdefault((a, b), [0, 0])
                rec[0] += 1
                rec[1] = max(rec[1], ts)
    df = pd.DataFrame([{"item_i": a, "item_j": b, "count": c, "last_ts": t} for (a, b), (c, t) in edges.items()],
                      columns=["item_i", "item_j", "count", "last_ts"])
    return df.sort_values("count", ascending=False).reset_index(drop=True)


def create_test_subset(sessions_df: pd.DataFrame, graph_df: pd.DataFrame,
                       num_sessions: int = 100) -> tuple[pd.DataFrame, pd.DataFrame]:
    """The first ``num_sessions`` sessions (file order) and the graph edges among their
    items (run_full_pipeline.py:34-82, in memory)."""
    keep = sessions_df["session_id"].unique()[:num_sessions]
    sub = sessions_df[sessions_df["session_id"].isin(keep)]
    items = set(sub["itemid"].unique())
    return sub, graph_df[graph_df["item_i"].isin(items) & graph_df["item_j"].isin(items)]


def create_batch_from_sessions(sessions_df: pd.DataFrame, graph_df: pd.DataFrame, batch_size: int = 8,
                               num_negatives: int = 5) -> tuple[SessionBatch, int]:
    """The reference's quick-path batch (run_full_pipeline.py:85-179) as a SessionBatch."""
    session_ids = sessions_df["session_id"].unique()[:batch_size]
    all_items = sorted(sessions_df["itemid"].unique())
    item_to_idx = {item: idx for idx, item in enumerate(all_items)}
    num_items = len(all_items)
    gi = graph_df["item_i"].to_numpy()
    gj = graph_df["item_j"].to_numpy()
    examples = []
    for sid in session_ids:
        sd = sessions_df[sessions_df["session_id"] == sid].sort_values("timestamp")
        items = sd["itemid"].to_numpy()
        if len(items) < 2:
            continue
        context, target = items[:-1], items[-1]
        local_items = sorted({item_to_idx[i] for i in context})
        local = {v: k for k, v in enumerate(local_items)}
        cset = set(context.tolist())
        mask = np.fromiter((a in cset and b in cset for a, b in zip(gi, gj)), dtype=bool, count=len(gi))
        if mask.any():
            src = [local[item_to_idx[i]] for i in gi[mask]]
            dst = [local[item_to_idx[j]] for j in gj[mask]]
            ei = np.array([src + dst, dst + src], dtype=np.int64)
        else:
            n = len(local_items)
            ei = np.array([list(range(n)), list(range(n))], dtype=np.int64)
        seen = {item_to_idx[i] for i in items}
        avail = [i for i in range(num_items) if i not in seen]
        negs = np.array(avail[:num_negatives], dtype=np.int64)
        if len(negs) < num_negatives:
            negs = torch.randint(0, num_items, (num_negatives,)).numpy()
        examples.append({"x": np.array(local_items, np.int64), "edge_index": ei,
                         "target_item": item_to_idx[target], "negative_items": negs})
    if not examples:
        raise ValueError("No valid sessions found")
    batch = collate_sessions(examples)
    batch.negative_items = batch.negative_items.view(len(examples), num_negatives)
    return batch, num_items


def test_model_with_real_data(model_name: str, create_fn, config: dict, batch, num_epochs: int = 3,
                              device: str = "cuda", loss: str = "listwise") -> dict:
    """Adam(lr=1e-3) + listwise loss for ``num_epochs`` steps on one batch
    (run_full_pipeline.py:182-270); returns the reference's result dict."""
    start = time.time()
    try:
        model = create_fn(**config).to(device)
        batch = batch.to(device)
        optimizer = torch.optim.Adam(model.parameters(), lr=0.001)
        loss_fn = create_loss_function(loss)
        losses = []
        for _ in range(num_epochs):
            model.train()
            optimizer.zero_grad()
            se = model(batch)
            out = loss_fn(se, batch.target_item, batch.negative_items, model.item_embedding)
            lval = out[0] if isinstance(out, tuple) else out
            lval.backward()
            optimizer.step()
            losses.append(float(lval.item()))
        duration = time.time() - start
        if any(np.isnan(v) for v in losses):
            return {"model": model_name, "status": "FAIL", "error": "NaN loss detected", "duration": duration,
                    "losses": losses}
        pc = sum(p.numel() for p in model.parameters())
        return {"model": model_name, "status": "PASS", "duration": duration, "losses": losses,
                "final_loss": losses[-1], "param_count": pc, "param_count_millions": pc / 1e6, "model_obj": model}
    except (RuntimeError, ValueError, NotImplementedError) as e:
        return {"model": model_name, "status": "FAIL", "error": str(e), "duration": time.time() - start}
