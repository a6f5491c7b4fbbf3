"""Models (reference: etpgt/model/__init__.py).  The GAT / GraphSAGE baselines are
outside the hot-path scope: their names are exported so that
callers' imports resolve, and constructing them raises NotImplementedError."""

from etpgt.model.base import BaseRecommendationModel, SessionReadout
from etpgt.model.gat import GAT, create_gat
from etpgt.model.graph_transformer import (
    GraphTransformer,
    TransformerConv,
    create_graph_transformer,
    create_graph_transformer_optimized,
)
from etpgt.model.graphsage import GraphSAGE, create_graphsage

__all__ = [
    "BaseRecommendationModel",
    "SessionReadout",
    "GraphSAGE",
    "create_graphsage",
    "GAT",
    "create_gat",
    "GraphTransformer",
    "TransformerConv",
    "create_graph_transformer",
    "create_graph_transformer_optimized",
]
