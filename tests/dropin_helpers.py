"""Tiny reference-format CSVs for the train_baseline.py drop-in tests: sessions
(timestamp, visitorid, event, itemid, transactionid, session_id; tests/test_contracts.py:33
of the reference) and graph_edges.csv (item_i <= item_j, count; 04_build_graph.py:85-100)."""

from __future__ import annotations

import numpy as np
import pandas as pd

from etpgt.data.synthetic import make_sessions_and_graph


def write_csvs(tmp_path, num_items=120, num_train=150, num_val=40, seed=5):
    data = make_sessions_and_graph(num_items=num_items, num_sessions=num_train + num_val, num_edges=600, seed=seed)
    rows = []
    for s in range(data.num_sessions):
        for k, it in enumerate(data.session(s).tolist()):
            rows.append((1000 * s + k, f"v{s}", "view", int(it), None, s))
    df = pd.DataFrame(rows, columns=["timestamp", "visitorid", "event", "itemid", "transactionid", "session_id"])
    train = df[df.session_id < num_train]
    val = df[df.session_id >= num_train]
    d = tmp_path / "processed"
    d.mkdir(parents=True, exist_ok=True)
    train.to_csv(d / "train.csv", index=False)
    val.to_csv(d / "val.csv", index=False)
    ei = data.edge_index()
    pd.DataFrame({"item_i": ei[0], "item_j": ei[1], "count": np.ones(ei.shape[1], np.int64)}).to_csv(
        d / "graph_edges.csv", index=False)
    return d


# reference scripts/train/train_baseline.py:13-22 import list, plus etpgt.utils (:3)
REFERENCE_IMPORTS = {
    "etpgt.model": ["create_gat", "create_graph_transformer", "create_graph_transformer_optimized",
                    "create_graphsage", "GAT", "GraphSAGE", "GraphTransformer", "BaseRecommendationModel",
                    "SessionReadout"],
    "etpgt.train.dataloader": ["create_dataloader", "SessionDataset", "collate_fn"],
    "etpgt.train.trainer": ["Trainer"],
    "etpgt.utils.logging": ["get_logger"],
    "etpgt.utils.seed": ["set_seed"],
    "etpgt.utils": ["load_config", "save_json", "load_json", "compute_recall_at_k", "compute_ndcg_at_k",
                    "set_seed", "get_logger"],
    "etpgt.utils.io": ["load_config", "save_json", "load_json"],
}


def c1_inputs():
    """Config C1's data chain: the reference's scripts/data 00 -> 02 -> 04 as restated by
    etpgt.pipeline (pinned to their own output by tests/golden/c1_data.npz), then
    run_full_pipeline.py's 100-session subset: (events, sessions, graph, (subset, graph))."""
    from etpgt.pipeline import build_co_event_graph, create_test_subset, generate_synthetic_events, sessionize_events

    ev = generate_synthetic_events(num_sessions=100, num_items=1000, seed=42)
    sd = sessionize_events(ev)
    g = build_co_event_graph(sd)
    return ev, sd, g, create_test_subset(sd, g, num_sessions=100)
