"""Models (reference: etpgt/model/__init__.py).  GAT / GraphSAGE baselines are
outside the hot-path scope and are not provided."""

from etpgt.model.base import BaseRecommendationModel, SessionReadout
from etpgt.model.graph_transformer import (
    GraphTransformer,
    TransformerConv,
    create_graph_transformer,
    create_graph_transformer_optimized,
)

__all__ = [
    "BaseRecommendationModel",
    "SessionReadout",
    "GraphTransformer",
    "TransformerConv",
    "create_graph_transformer",
    "create_graph_transformer_optimized",
]
