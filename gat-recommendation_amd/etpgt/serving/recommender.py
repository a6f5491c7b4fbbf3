"""Recommender — API of etpgt/serving/recommender.py (reference, :25-145) on MI355X.

Same behaviour: the architecture is read off the checkpoint tensors (optimized model,
2 heads, LapPE; a checkpoint with FFN layers is refused), the co-occurrence graph is
loaded without self-loops, a session's induced subgraph (sorted unique items, stored
edges item_i -> item_j with both ends in the session) goes through the model, every
item is scored by dot product with the session embedding, the session's own items and
the padding row 0 are never recommended, and the top-k come back best first.

MI355X path: the forward is the HIP layer stack (eval mode) and the masked full-catalog
scoring + top-k is ``gtr_score_topk_masked`` (MFMA scores in registers, the exclusion
applied before selection) — no [T] score vector is materialised.  Checkpoints load with
``torch.load(weights_only=True)``.
"""

from __future__ import annotations

from collections import defaultdict
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np
import pandas as pd
import torch

from etpgt.backend.ops import score_topk
from etpgt.data.batch import SessionBatch
from etpgt.model import create_graph_transformer_optimized


@dataclass
class ValidatedRequest:
    """The reference's validated request (etpgt/serving/validation.py:20-36)."""

    session_items: list[int]
    k: int
    dropped_items: list[int] = field(default_factory=list)
    truncated: bool = False


class Recommender:
    def __init__(self, checkpoint_path: Path | str, graph_edges_path: Path | str, device: str = "cuda"):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("the Recommender runs on the MI355X HIP path only (device='cuda')")
        self._load_model(Path(checkpoint_path))
        self._load_graph(Path(graph_edges_path))

    def _load_model(self, checkpoint_path: Path) -> None:
        checkpoint = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        sd = checkpoint["model_state_dict"]
        if any(key.startswith("ffns.") for key in sd):
            raise RuntimeError(
                "This Recommender targets the optimized (no-FFN) checkpoint, but the "
                "given checkpoint has FFN layers. Load the optimized model instead."
            )
        self.num_items, self.embedding_dim = (int(v) for v in sd["item_embedding.weight"].shape)
        hidden_dim = int(sd["batch_norms.0.weight"].shape[0])
        laplacian_k = int(sd["laplacian_pe.projection.weight"].shape[1])
        num_layers = len({key.split(".")[1] for key in sd if key.startswith("convs.")})
        model = create_graph_transformer_optimized(
            num_items=self.num_items, embedding_dim=self.embedding_dim, hidden_dim=hidden_dim,
            num_layers=num_layers, num_heads=2, use_laplacian_pe=True, laplacian_k=laplacian_k,
        )
        model.laplacian_pe._cached_pe = torch.empty_like(sd["laplacian_pe._cached_pe"])
        result = model.load_state_dict(sd, strict=False)
        if result.missing_keys or result.unexpected_keys:
            raise RuntimeError(
                f"checkpoint does not match model: missing={result.missing_keys[:4]} "
                f"unexpected={result.unexpected_keys[:4]}"
            )
        self.model = model.to(self.device).eval()
        self.item_embeddings = self.model.get_item_embeddings().detach()
        self.checkpoint_epoch = int(checkpoint.get("epoch", -1))
        self.val_recall_at_10 = float(checkpoint.get("best_val_metric", float("nan")))

    def _load_graph(self, graph_edges_path: Path) -> None:
        edges = pd.read_csv(graph_edges_path, usecols=["item_i", "item_j"])
        adjacency: dict[int, set[int]] = defaultdict(set)
        for i, j in edges.itertuples(index=False):
            if i != j:  # no self-loops for serving message passing (recommender.py:95)
                adjacency[int(i)].add(int(j))
        self._adjacency = adjacency

    def _build_session_graph(self, items: list[int]) -> SessionBatch:
        seen = set(int(v) for v in items)
        unique = sorted(seen)
        local = {g: i for i, g in enumerate(unique)}
        pairs = sorted((i, j) for i in seen for j in self._adjacency.get(i, ()) if j in seen)
        x = torch.tensor(unique, dtype=torch.long)
        if pairs:
            ei = torch.tensor([[local[i], local[j]] for i, j in pairs], dtype=torch.long).t()
        else:
            ei = torch.zeros((2, 0), dtype=torch.long)
        return SessionBatch(x, ei, torch.zeros(len(unique), dtype=torch.long), num_graphs=1)

    @torch.no_grad()
    def recommend(self, request) -> tuple[list[int], list[float]]:
        """(item_ids, scores) of the top-k, best first (recommender.py:115-131)."""
        if not request.session_items:
            raise ValueError("session_items must not be empty.")
        batch = self._build_session_graph(request.session_items)
        se = self.model(batch.to(self.device))  # [1, hidden_dim]
        excl = sorted(set(int(v) for v in request.session_items if 0 <= int(v) < self.num_items) | {0})
        k = int(request.k)
        if k > self.num_items:
            raise RuntimeError("selected index k out of range")
        # the reference scores excluded items -inf and takes torch.topk over all T, so a k
        # past the unmasked count (validation clamps k to num_items - 1 only) returns the
        # masked ids after every finite score.  torch.topk leaves the order among equal
        # -inf scores unspecified; they come back here in ascending id order.
        live = min(k, self.num_items - len(excl))
        idx, sc = (score_topk(se, self.item_embeddings, live, exclude=[excl]) if live > 0
                   else (torch.empty(1, 0, dtype=torch.int64), torch.empty(1, 0)))
        ids = [int(v) for v in idx[0].tolist()]
        scores = [float(v) for v in sc[0].tolist()]
        if k > live:
            ids += excl[: k - live]
            scores += [float("-inf")] * (k - live)
        return ids, scores

    def health(self) -> dict:
        return {
            "num_items": self.num_items,
            "embedding_dim": self.embedding_dim,
            "checkpoint_epoch": self.checkpoint_epoch,
            "val_recall_at_10": self.val_recall_at_10,
        }
