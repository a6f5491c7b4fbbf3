"""GraphTransformer — API of etpgt/model/graph_transformer.py (reference), MI355X path.

Same constructor, factories, attributes and state_dict keys as the reference
(``item_embedding.weight``, ``laplacian_pe.projection.{weight,bias}``,
``laplacian_pe._cached_pe``, ``convs.{l}.lin_{key,query,value,skip}.{weight,bias}``,
``convs.{l}.lin_beta.weight``, ``batch_norms.{l}.*``), so checkpoints interchange
with the reference (recommender.py:61-85 reads them).

``forward(batch)`` runs the whole layer stack on libgtr_hip (one fused kernel per
layer + one readout kernel; graph_transformer.py:126-182 semantics with PyG
TransformerConv(beta=True)).  There is no CPU path: a
model on the CPU raises.  Scope: the optimized variant
(use_ffn=False) with the mean readout is the hot path.  use_ffn=True (the
feed-forward block of graph_transformer.py:88-100,160-170) runs on the split layer
kernels plus gtr_ffn_fwd / gtr_ffn_bwd / gtr_ffn_wgrad at hidden_dim 64 / 128 / 256 with
ffn_expansion 1 / 2 / 4 (the reference's create_graph_transformer default d = 256, x 4 and
the optimized factory's x 2 included); the max/last/attention readouts raise
NotImplementedError.
"""

from __future__ import annotations

import torch
import torch.nn as nn

from etpgt.encodings.laplacian_pe import LaplacianPECached
from etpgt.model.base import BaseRecommendationModel, SessionReadout


class TransformerConv(nn.Module):
    """Parameter container with PyG ``TransformerConv(in, C, heads=H, concat=True,
    beta=True, dropout=p)`` names and shapes (lin_key/query/value/skip biased
    [H*C, in]; lin_beta [1, 3*H*C] without bias).  Its arithmetic is executed by
    the fused layer kernel of the enclosing GraphTransformer."""

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, dropout: float = 0.0,
                 concat: bool = True, beta: bool = True):
        super().__init__()
        if not (concat and beta):
            raise NotImplementedError("only concat=True, beta=True (the reference configuration) is supported")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.heads = heads
        self.dropout = dropout
        hc = heads * out_channels
        self.lin_key = nn.Linear(in_channels, hc)
        self.lin_query = nn.Linear(in_channels, hc)
        self.lin_value = nn.Linear(in_channels, hc)
        self.lin_skip = nn.Linear(in_channels, hc, bias=True)
        self.lin_beta = nn.Linear(3 * hc, 1, bias=False)

    def forward(self, x, edge_index):  # pragma: no cover - guarded
        raise RuntimeError("TransformerConv runs fused inside GraphTransformer.forward on the HIP path")


class GraphTransformer(BaseRecommendationModel):
    def __init__(
        self,
        num_items: int,
        embedding_dim: int = 256,
        hidden_dim: int = 256,
        num_layers: int = 3,
        num_heads: int = 4,
        dropout: float = 0.1,
        readout_type: str = "mean",
        use_laplacian_pe: bool = True,
        laplacian_k: int = 16,
        use_ffn: bool = True,
        ffn_expansion: int = 4,
    ):
        super().__init__(num_items, embedding_dim, hidden_dim, num_layers, dropout)
        self.num_heads = num_heads
        self.readout_type = readout_type
        self.use_laplacian_pe = use_laplacian_pe
        self.laplacian_k = laplacian_k
        self.use_ffn = use_ffn
        self.ffn_expansion = ffn_expansion
        if use_laplacian_pe:
            self.laplacian_pe = LaplacianPECached(k=laplacian_k, embedding_dim=embedding_dim)
        self.convs = nn.ModuleList()
        self.batch_norms = nn.ModuleList()
        self.ffns = nn.ModuleList() if use_ffn else None
        for d_in in [embedding_dim] + [hidden_dim] * (num_layers - 1):
            self.convs.append(TransformerConv(d_in, hidden_dim // num_heads, heads=num_heads, dropout=dropout))
            self.batch_norms.append(nn.BatchNorm1d(hidden_dim))
            if use_ffn:
                self.ffns.append(self._make_ffn(hidden_dim))
        self.dropout_layer = nn.Dropout(dropout)
        self.readout = SessionReadout(hidden_dim, readout_type)
        self._engine = None

    def _make_ffn(self, hidden_dim: int) -> nn.Module:
        return nn.Sequential(
            nn.Linear(hidden_dim, hidden_dim * self.ffn_expansion),
            nn.GELU(),
            nn.Dropout(self.dropout),
            nn.Linear(hidden_dim * self.ffn_expansion, hidden_dim),
            nn.Dropout(self.dropout),
        )

    # ------------------------------------------------------------------ HIP binding
    def hip_engine(self):
        from etpgt.backend.engine import Engine

        dev = self.item_embedding.weight.device
        eng = self._engine
        if eng is None or eng.device != dev or not eng.flat.intact():
            self._check_supported()
            eng = Engine(self, dev)
            self.__dict__["_engine"] = eng  # not a submodule / not in state_dict
        return eng

    def _check_supported(self):
        if self.embedding_dim != self.hidden_dim:
            raise ValueError("embedding_dim must equal hidden_dim (residual at graph_transformer.py:176)")
        if self.use_ffn and (self.hidden_dim not in (64, 128, 256) or self.ffn_expansion not in (1, 2, 4)):
            raise NotImplementedError(f"use_ffn=True runs on the split-layer FFN kernels: hidden_dim 64 / 128 / 256 "
                                      f"with ffn_expansion 1 / 2 / 4 (got {self.hidden_dim}, {self.ffn_expansion})")
        if self.readout_type != "mean":
            raise NotImplementedError(f"readout '{self.readout_type}' is outside the HIP hot path (mean only)")

    def forward(self, batch):
        """Session embeddings [B, hidden_dim] for a PyG-style batch (graph_transformer.py:126-182)."""
        from etpgt.backend.ops import GraphTransformerFn

        self._sync_lazy()
        dev = self.item_embedding.weight.device
        if dev.type != "cuda":
            raise RuntimeError("GraphTransformer runs on the MI355X HIP path only; move the model to 'cuda'")
        if self.use_laplacian_pe and getattr(batch, "laplacian_pe", None) is None and self.laplacian_pe._cached_pe is None:
            raise RuntimeError("Laplacian PE not precomputed. Call precompute() first.")
        eng = self.hip_engine()
        caps, blob, node_pe = eng.prepare(batch)
        B = int(batch.num_graphs) if hasattr(batch, "num_graphs") else int(batch.batch.max()) + 1
        if self.training and int(batch.x.shape[0]) <= 1:
            raise ValueError("Expected more than 1 value per channel when training (BatchNorm1d)")
        params = eng.flat.params()
        need_grad = torch.is_grad_enabled() and (self.item_embedding.weight.requires_grad
                                                  or any(p.requires_grad for p in params))
        if not self.training and not need_grad:  # inference: the registered op etpgt::graph_transformer_eval
            from etpgt.backend.ops import engine_handle

            return torch.ops.etpgt.graph_transformer_eval(blob, node_pe, self.item_embedding.weight, list(params),
                                                          engine_handle(eng), caps.n_cap, caps.b_cap, caps.e_cap,
                                                          caps.n_neg, B)
        return GraphTransformerFn.apply(eng, caps, blob, node_pe, B, self.training, need_grad,
                                        self.item_embedding.weight, *params)


def create_graph_transformer(num_items: int, embedding_dim: int = 256, hidden_dim: int = 256,
                             num_layers: int = 3, num_heads: int = 4, dropout: float = 0.1,
                             readout_type: str = "mean", use_laplacian_pe: bool = True,
                             laplacian_k: int = 16, use_ffn: bool = True, ffn_expansion: int = 4) -> GraphTransformer:
    return GraphTransformer(num_items=num_items, embedding_dim=embedding_dim, hidden_dim=hidden_dim,
                            num_layers=num_layers, num_heads=num_heads, dropout=dropout,
                            readout_type=readout_type, use_laplacian_pe=use_laplacian_pe,
                            laplacian_k=laplacian_k, use_ffn=use_ffn, ffn_expansion=ffn_expansion)


def create_graph_transformer_optimized(num_items: int, embedding_dim: int = 256, hidden_dim: int = 256,
                                       num_layers: int = 2, num_heads: int = 2, dropout: float = 0.1,
                                       readout_type: str = "mean", use_laplacian_pe: bool = True,
                                       laplacian_k: int = 16, use_ffn: bool = False,
                                       ffn_expansion: int = 2) -> GraphTransformer:
    """Defaults of graph_transformer.py:231-280 (L=2, H=2, no FFN)."""
    return GraphTransformer(num_items=num_items, embedding_dim=embedding_dim, hidden_dim=hidden_dim,
                            num_layers=num_layers, num_heads=num_heads, dropout=dropout,
                            readout_type=readout_type, use_laplacian_pe=use_laplacian_pe,
                            laplacian_k=laplacian_k, use_ffn=use_ffn, ffn_expansion=ffn_expansion)
