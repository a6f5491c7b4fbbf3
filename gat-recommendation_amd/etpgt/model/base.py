"""Base model, session readout and BPR loss — API of etpgt/model/base.py (reference).

``BaseRecommendationModel`` keeps the reference's item table (base.py:35-37:
``nn.Embedding(num_items, d, padding_idx=0)`` + xavier on rows 1..), ``predict``
(base.py:59-78) and ``compute_loss`` (BPR, base.py:80-113).  ``compute_loss`` runs
the fused scoring kernel (libgtr_hip ``gtr_readout_loss`` in LOSS mode).
"""

from __future__ import annotations

from abc import ABC, abstractmethod

import torch
import torch.nn as nn

from etpgt.backend.ops import score_loss, score_topk


class BaseRecommendationModel(nn.Module, ABC):
    def __init__(self, num_items: int, embedding_dim: int = 256, hidden_dim: int = 256,
                 num_layers: int = 3, dropout: float = 0.1):
        super().__init__()
        self.num_items = num_items
        self.embedding_dim = embedding_dim
        self.hidden_dim = hidden_dim
        self.num_layers = num_layers
        self.dropout = dropout
        self.item_embedding = nn.Embedding(num_items, embedding_dim, padding_idx=0)
        nn.init.xavier_uniform_(self.item_embedding.weight[1:])

    @abstractmethod
    def forward(self, batch):
        ...

    def _sync_lazy(self) -> None:
        """A fused step in lazy mode defers untouched rows' zero-gradient AdamW updates;
        bring the table up to date before anything outside the step reads it."""
        cb = self.__dict__.get("_lazy_sync")
        if cb is not None:
            cb()

    def state_dict(self, *args, **kwargs):
        self._sync_lazy()
        return super().state_dict(*args, **kwargs)

    def get_item_embeddings(self) -> torch.Tensor:
        self._sync_lazy()
        return self.item_embedding.weight

    def predict(self, session_embeddings: torch.Tensor, k: int = 20) -> torch.Tensor:
        """Top-k item ids by dot product over the full catalog (base.py:59-78; no
        masking of seen items or row 0, as in the reference), fused scoring + top-k
        on the HIP kernel (gtr_score_topk, MFMA scores, no [B, T] matrix)."""
        return score_topk(session_embeddings, self.get_item_embeddings(), k)[0]

    def compute_loss(self, session_embeddings: torch.Tensor, target_items: torch.Tensor,
                     negative_items: torch.Tensor) -> torch.Tensor:
        """BPR: -mean(log(sigmoid(pos - neg) + 1e-8)) over B x n (base.py:80-113)."""
        return score_loss(session_embeddings, target_items, negative_items, self.item_embedding.weight, "bpr")


class SessionReadout(nn.Module):
    """Session readout (base.py:116-193).  Inside GraphTransformer the ``mean``
    readout is fused into the HIP readout/loss kernel; this module is the
    stand-alone API (vectorised, no per-session Python loop)."""

    def __init__(self, hidden_dim: int = 256, readout_type: str = "mean"):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.readout_type = readout_type
        if readout_type == "attention":
            self.attention = nn.Linear(hidden_dim, 1)
            nn.init.xavier_uniform_(self.attention.weight)
            nn.init.zeros_(self.attention.bias)
        elif readout_type not in ("mean", "max", "last"):
            # the reference raises at forward time; raising early is stricter but the same type
            raise ValueError(f"Unknown readout type: {readout_type}")

    def forward(self, node_embeddings: torch.Tensor, batch_indices: torch.Tensor) -> torch.Tensor:
        B = int(batch_indices.max().item()) + 1
        x = node_embeddings
        idx = batch_indices.long()
        if self.readout_type == "mean":
            s = torch.zeros(B, x.shape[1], dtype=x.dtype, device=x.device).index_add(0, idx, x)
            cnt = torch.bincount(idx, minlength=B).clamp(min=1).to(x.dtype).unsqueeze(1)
            return s / cnt
        if self.readout_type == "max":
            out = torch.full((B, x.shape[1]), float("-inf"), dtype=x.dtype, device=x.device)
            return out.scatter_reduce(0, idx.unsqueeze(1).expand_as(x), x, reduce="amax", include_self=True)
        if self.readout_type == "last":
            pos = torch.arange(x.shape[0], device=x.device)
            last = torch.zeros(B, dtype=torch.long, device=x.device).scatter_reduce(0, idx, pos, reduce="amax")
            return x[last]
        scores = self.attention(x).squeeze(-1)
        m = torch.full((B,), float("-inf"), dtype=x.dtype, device=x.device).scatter_reduce(
            0, idx, scores.detach(), reduce="amax")
        w = (scores - m[idx]).exp()
        z = torch.zeros(B, dtype=x.dtype, device=x.device).index_add(0, idx, w)
        w = w / z[idx]
        return torch.zeros(B, x.shape[1], dtype=x.dtype, device=x.device).index_add(0, idx, w.unsqueeze(1) * x)
