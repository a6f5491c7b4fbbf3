"""Laplacian positional encoding — API of etpgt/encodings/laplacian_pe.py (reference).

``compute_laplacian_pe`` (laplacian_pe.py:19-66) is a one-time host precompute
(sparse sym-normalised Laplacian -> k+1 smallest eigenvectors, drop the first,
abs): PyG ``get_laplacian(normalization="sym")`` is restated with scipy (PyG is
not a dependency).  The per-step cached gather + projection (laplacian_pe.py:
181-199) is fused into the layer-0 prologue of the HIP conv kernel when the
module lives inside a GraphTransformer; ``forward``/``project`` here are the
stand-alone API.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn


def sym_laplacian(edge_index, num_nodes: int):
    import scipy.sparse as sp

    ei = edge_index.detach().cpu().numpy() if isinstance(edge_index, torch.Tensor) else np.asarray(edge_index)
    row, col = ei[0].astype(np.int64), ei[1].astype(np.int64)
    keep = row != col
    row, col = row[keep], col[keep]
    w = np.ones(row.shape[0], dtype=np.float32)
    deg = np.bincount(row, weights=w, minlength=num_nodes).astype(np.float32)
    with np.errstate(divide="ignore"):
        dis = np.where(deg > 0, deg ** -0.5, 0.0).astype(np.float32)
    vals = np.concatenate([-dis[row] * w * dis[col], np.ones(num_nodes, np.float32)])
    r = np.concatenate([row, np.arange(num_nodes)])
    c = np.concatenate([col, np.arange(num_nodes)])
    return sp.coo_matrix((vals, (r, c)), shape=(num_nodes, num_nodes)).tocsr()


def compute_laplacian_pe(edge_index, num_nodes: int, k: int = 16, normalization: str = "sym") -> torch.Tensor:
    if normalization != "sym":
        raise NotImplementedError("only the 'sym' normalisation used by the reference is provided")
    from scipy.sparse.linalg import eigsh

    L = sym_laplacian(edge_index, num_nodes)
    # fixed ARPACK start vector: without one, eigsh draws it from a generator whose state
    # persists across calls in the process, so the result (its eigenvector signs, and on the
    # reference's non-symmetric directed input the vectors themselves) depended on how many
    # solves ran before -- data-parallel ranks and repeated runs must get the same table
    v0 = np.random.default_rng(0).random(num_nodes)
    try:
        _, vecs = eigsh(L, k=k + 1, which="SM", return_eigenvectors=True, v0=v0)
    except Exception:
        _, vt = torch.linalg.eigh(torch.from_numpy(L.toarray()).float())
        vecs = vt.numpy()
    return torch.from_numpy(np.ascontiguousarray(vecs[:, 1 : k + 1])).float().abs()


class LaplacianPE(nn.Module):
    """Uncached variant (laplacian_pe.py:69-121)."""

    def __init__(self, k: int = 16, embedding_dim: int = 256, normalization: str = "sym"):
        super().__init__()
        self.k, self.embedding_dim, self.normalization = k, embedding_dim, normalization
        self.projection = nn.Linear(k, embedding_dim)
        nn.init.xavier_uniform_(self.projection.weight)
        nn.init.zeros_(self.projection.bias)

    def forward(self, data) -> torch.Tensor:
        pe = compute_laplacian_pe(data.edge_index, data.num_nodes, k=self.k, normalization=self.normalization)
        return self.projection(pe.to(self.projection.weight.device))


class LaplacianPECached(nn.Module):
    """Cached variant (laplacian_pe.py:124-199); ``_cached_pe`` is a buffer."""

    def __init__(self, k: int = 16, embedding_dim: int = 256, normalization: str = "sym"):
        super().__init__()
        self.k, self.embedding_dim, self.normalization = k, embedding_dim, normalization
        self.projection = nn.Linear(k, embedding_dim)
        nn.init.xavier_uniform_(self.projection.weight)
        nn.init.zeros_(self.projection.bias)
        self.register_buffer("_cached_pe", None)

    def precompute(self, data) -> None:
        pe = compute_laplacian_pe(data.edge_index, data.num_nodes, k=self.k, normalization=self.normalization)
        self._cached_pe = pe.to(self.projection.weight.device)

    def project(self, pe: torch.Tensor) -> torch.Tensor:
        return self.projection(pe)

    def forward(self, node_indices: torch.Tensor) -> torch.Tensor:
        if self._cached_pe is None:
            raise RuntimeError("Laplacian PE not precomputed. Call precompute() first.")
        return self.projection(self._cached_pe[node_indices])
