"""Utilities (reference: etpgt/utils/__init__.py)."""

from etpgt.utils.metrics import compute_ndcg_at_k, compute_recall_at_k, compute_stratified_metrics
from etpgt.utils.seed import set_seed

__all__ = ["compute_recall_at_k", "compute_ndcg_at_k", "compute_stratified_metrics", "set_seed"]
