"""Recall@K / NDCG@K (reference: etpgt/utils/metrics.py:6-110)."""

import torch


def compute_recall_at_k(predictions: torch.Tensor, targets: torch.Tensor, k: int) -> float:
    hits = (predictions[:, :k] == targets.unsqueeze(1)).any(dim=1).float()
    return hits.mean().item()


def compute_ndcg_at_k(predictions: torch.Tensor, targets: torch.Tensor, k: int) -> float:
    matches = (predictions[:, :k] == targets.unsqueeze(1)).float()
    positions = torch.argmax(matches, dim=1)
    has = matches.sum(dim=1) > 0
    dcg = torch.where(has, 1.0 / torch.log2(positions.float() + 2.0), torch.zeros_like(positions, dtype=torch.float32))
    return dcg.mean().item()


def compute_stratified_metrics(predictions, targets, strata, k_values=None) -> dict:
    k_values = k_values or [10, 20]
    out = {}
    for s in torch.unique(strata):
        m = strata == s
        r = {"count": int(m.sum().item())}
        for k in k_values:
            r[f"recall@{k}"] = compute_recall_at_k(predictions[m], targets[m], k)
            r[f"ndcg@{k}"] = compute_ndcg_at_k(predictions[m], targets[m], k)
        out[f"stratum_{s.item()}"] = r
    return out
