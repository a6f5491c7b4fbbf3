"""Utilities (reference: etpgt/utils/__init__.py)."""

from etpgt.utils.io import load_config, load_json, save_json
from etpgt.utils.logging import get_logger
from etpgt.utils.metrics import compute_ndcg_at_k, compute_recall_at_k, compute_stratified_metrics
from etpgt.utils.seed import set_seed

__all__ = [
    "load_config",
    "save_json",
    "load_json",
    "compute_recall_at_k",
    "compute_ndcg_at_k",
    "compute_stratified_metrics",
    "set_seed",
    "get_logger",
]
