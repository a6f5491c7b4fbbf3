"""GAT baseline — API of etpgt/model/gat.py (reference).

Outside the hot-path scope (not the north-star model): the
names exist so that ``scripts/train/train_baseline.py``'s imports
(reference train_baseline.py:13-18) resolve, but building the model raises.
"""

from __future__ import annotations

import torch.nn as nn

_OUT_OF_SCOPE = ("the GAT baseline is outside the MI355X hot path (SURVEY.md §2 row 7); "
                 "use --model graph_transformer_optimized")


class GAT(nn.Module):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError(_OUT_OF_SCOPE)


def create_gat(num_items: int, embedding_dim: int = 256, hidden_dim: int = 256, num_layers: int = 3,
               num_heads: int = 4, dropout: float = 0.1, readout_type: str = "mean") -> GAT:
    return GAT(num_items, embedding_dim, hidden_dim, num_layers, num_heads, dropout, readout_type)
