"""Loss functions — API of etpgt/train/losses.py (reference, :8-228).

Each ``forward(session_embeddings, target_items, negative_items, item_embeddings)``
stays a plain Python method with that signature (the reference Trainer dispatches
on ``loss_fn.forward.__code__.co_varnames``, trainer.py:96).  The arithmetic runs
in the fused HIP scoring kernel (forward and backward in one launch).
"""

from __future__ import annotations

import torch
import torch.nn as nn

from etpgt.backend.ops import score_loss


class BPRLoss(nn.Module):
    """-mean(log(sigmoid(pos - neg) + 1e-8)) over B x n (losses.py:8-53)."""

    kind = "bpr"

    def __init__(self):
        super().__init__()

    def forward(self, session_embeddings: torch.Tensor, target_items: torch.Tensor,
                negative_items: torch.Tensor, item_embeddings: nn.Embedding) -> torch.Tensor:
        return score_loss(session_embeddings, target_items, negative_items, item_embeddings, "bpr")


class ListwiseLoss(nn.Module):
    """Softmax cross-entropy over [pos, neg_1..n] / temperature, target 0 (losses.py:56-111)."""

    kind = "listwise"

    def __init__(self, temperature: float = 1.0):
        super().__init__()
        self.temperature = temperature

    def forward(self, session_embeddings: torch.Tensor, target_items: torch.Tensor,
                negative_items: torch.Tensor, item_embeddings: nn.Embedding) -> torch.Tensor:
        return score_loss(session_embeddings, target_items, negative_items, item_embeddings, "listwise",
                          temperature=self.temperature)


class DualLoss(nn.Module):
    """alpha * listwise + (1 - alpha) * BPR; returns (loss, components) (losses.py:114-164)."""

    kind = "dual"

    def __init__(self, alpha: float = 0.7, temperature: float = 1.0):
        super().__init__()
        self.alpha = alpha
        self.temperature = temperature
        self.listwise_loss = ListwiseLoss(temperature=temperature)
        self.bpr_loss = BPRLoss()

    def forward(self, session_embeddings: torch.Tensor, target_items: torch.Tensor,
                negative_items: torch.Tensor, item_embeddings: nn.Embedding):
        listwise = self.listwise_loss(session_embeddings, target_items, negative_items, item_embeddings)
        bpr = self.bpr_loss(session_embeddings, target_items, negative_items, item_embeddings)
        total = self.alpha * listwise + (1 - self.alpha) * bpr
        return total, {"total": total.item(), "listwise": listwise.item(), "bpr": bpr.item()}


class SampledSoftmaxLoss(nn.Module):
    """Identical to ListwiseLoss (losses.py:167-201)."""

    kind = "sampled_softmax"

    def __init__(self, temperature: float = 1.0):
        super().__init__()
        self.temperature = temperature

    def forward(self, session_embeddings: torch.Tensor, target_items: torch.Tensor,
                negative_items: torch.Tensor, item_embeddings: nn.Embedding) -> torch.Tensor:
        return score_loss(session_embeddings, target_items, negative_items, item_embeddings, "listwise",
                          temperature=self.temperature)


def create_loss_function(loss_type: str = "dual", alpha: float = 0.7, temperature: float = 1.0) -> nn.Module:
    if loss_type == "bpr":
        return BPRLoss()
    if loss_type == "listwise":
        return ListwiseLoss(temperature=temperature)
    if loss_type == "dual":
        return DualLoss(alpha=alpha, temperature=temperature)
    if loss_type == "sampled_softmax":
        return SampledSoftmaxLoss(temperature=temperature)
    raise ValueError(f"Unknown loss type: {loss_type}")
