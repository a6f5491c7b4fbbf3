"""CPU ORACLE for the GraphTransformer training hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain-PyTorch (CPU, fp32 unless asked otherwise) restatement of
the reference's training hot path.  It is imported ONLY by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` — as the
checker / the timed reference CPU path, never as the thing measured or shipped.
The product path (``gat-recommendation_amd/etpgt``) never imports it.

What it restates (reference = /root/reference, file:line):

* ``etpgt/model/base.py:35-37``       item table, padding row 0, xavier on rows 1..
* ``etpgt/model/base.py:80-113``      BPR ``compute_loss``
* ``etpgt/model/base.py:136-193``     ``SessionReadout`` (Python loop, all 4 modes)
* ``etpgt/model/graph_transformer.py:23-182``  layer stack (no-FFN and FFN branches)
* PyG ``TransformerConv(in, C, heads=H, concat=True, beta=True, dropout=p)`` and
  ``torch_geometric.utils.softmax`` — third-party, NOT installed here; restated
  from its published algorithm.  Call sites:
  ``graph_transformer.py:73-82,89-98,174``.
* ``etpgt/encodings/laplacian_pe.py:19-66,124-199``  LapPE (PyG ``get_laplacian``
  sym normalisation restated with scipy), cached gather + projection
* ``etpgt/train/losses.py:8-228``     BPR / Listwise / Dual / SampledSoftmax / factory
* ``etpgt/train/trainer.py:80-133``   one training step (zero_grad/backward/step)
* ``scripts/train/train_baseline.py:252-256``  AdamW(lr=1e-3, wd=1e-5)

Parity pinning: the pieces that live in the reference's own importable files
(readout, BPR, losses, metrics, the trainer loop) are pinned against golden
vectors produced by importing those files (``oracle/gen_golden.py`` →
``tests/golden/``).  The TransformerConv arithmetic lives in PyG, which is absent
from this container: it is pinned only structurally (parameter-count known
answers, 36,800 / 45,952 / 112,128, and the reference tests' shape/finiteness
checks).  TransformerConv numerics: PARITY UNPINNED against PyG itself.
"""

from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

# --------------------------------------------------------------------------------------
# PyG semantics restated
# --------------------------------------------------------------------------------------


def pyg_softmax(src: torch.Tensor, index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """torch_geometric.utils.softmax(src, index, num_nodes=N) restated.

    max-shift on the detached logits, ``+1e-16`` in the denominator.
    src: [E, H]; index: [E] (destination node of each edge).
    """
    H = src.shape[1]
    idx = index.view(-1, 1).expand(-1, H)
    src_max = torch.full((num_nodes, H), float("-inf"), dtype=src.dtype)
    src_max = src_max.scatter_reduce(0, idx, src.detach(), reduce="amax", include_self=True)
    out = (src - src_max.index_select(0, index)).exp()
    out_sum = torch.zeros((num_nodes, H), dtype=src.dtype).index_add(0, index, out) + 1e-16
    return out / out_sum.index_select(0, index)


class RefTransformerConv(nn.Module):
    """PyG ``TransformerConv(in_channels, out_channels=C, heads=H, concat=True,
    beta=True, dropout=p, edge_dim=None, bias=True, root_weight=True)`` restated.

    Parameter layout (and registration order) follows PyG: lin_key, lin_query,
    lin_value, lin_skip (all biased, [H*C, in]) and lin_beta ([1, 3*H*C], no bias).
    """

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, dropout: float = 0.0):
        super().__init__()
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

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        H, C = self.heads, self.out_channels
        N = x.shape[0]
        q = self.lin_query(x).view(-1, H, C)
        k = self.lin_key(x).view(-1, H, C)
        v = self.lin_value(x).view(-1, H, C)
        src, dst = edge_index[0], edge_index[1]  # flow source_to_target
        alpha = (q[dst] * k[src]).sum(dim=-1) / math.sqrt(C)  # [E, H]
        alpha = pyg_softmax(alpha, dst, N)
        mask = getattr(self, "attn_mask", None)
        if mask is not None and self.training:  # injected mask (hip_dropout_masks), else torch's RNG
            alpha = alpha * mask
        else:
            alpha = F.dropout(alpha, p=self.dropout, training=self.training)
        msg = v[src] * alpha.view(-1, H, 1)
        out = torch.zeros((N, H, C), dtype=x.dtype).index_add(0, dst, msg)
        out = out.view(-1, H * C)
        x_r = self.lin_skip(x)
        beta = self.lin_beta(torch.cat([out, x_r, out - x_r], dim=-1)).sigmoid()
        return beta * x_r + (1 - beta) * out


# --------------------------------------------------------------------------------------
# LapPE (laplacian_pe.py:19-66 with PyG get_laplacian(normalization="sym"))
# --------------------------------------------------------------------------------------


def ref_sym_laplacian(edge_index: np.ndarray, num_nodes: int):
    """PyG ``get_laplacian(edge_index, normalization='sym', num_nodes)`` restated
    (remove self loops; deg = scatter-sum over row; L = I - D^-1/2 A D^-1/2;
    duplicates summed by the COO->CSR conversion, as ``to_scipy_sparse_matrix``)."""
    import scipy.sparse as sp

    row, col = np.asarray(edge_index[0]), np.asarray(edge_index[1])
    keep = row != col
    row, col = row[keep], col[keep]
    w = np.ones(row.shape[0], dtype=np.float32)
    deg = np.zeros(num_nodes, dtype=np.float32)
    np.add.at(deg, row, w)
    with np.errstate(divide="ignore"):
        dis = deg ** -0.5
    dis[np.isinf(dis)] = 0.0
    w = -dis[row] * w * dis[col]
    loops = np.arange(num_nodes)
    r = np.concatenate([row, loops])
    c = np.concatenate([col, loops])
    vals = np.concatenate([w, np.ones(num_nodes, dtype=np.float32)])
    return sp.coo_matrix((vals, (r, c)), shape=(num_nodes, num_nodes)).tocsr()


def ref_compute_laplacian_pe(edge_index, num_nodes: int, k: int = 16) -> torch.Tensor:
    """``compute_laplacian_pe`` (laplacian_pe.py:19-66): eigsh(k+1, 'SM'), dense
    eigh fallback, drop column 0, abs, float32."""
    from scipy.sparse.linalg import eigsh

    ei = edge_index.numpy() if isinstance(edge_index, torch.Tensor) else np.asarray(edge_index)
    L = ref_sym_laplacian(ei, num_nodes)
    try:
        _, vecs = eigsh(L, k=k + 1, which="SM", return_eigenvectors=True)
    except Exception:
        _, vecs_t = torch.linalg.eigh(torch.from_numpy(L.toarray()).float())
        vecs = vecs_t.numpy()
    return torch.from_numpy(np.ascontiguousarray(vecs[:, 1 : k + 1])).float().abs()


class RefLaplacianPECached(nn.Module):
    """``LaplacianPECached`` (laplacian_pe.py:124-199)."""

    def __init__(self, k: int = 16, embedding_dim: int = 256):
        super().__init__()
        self.k = k
        self.embedding_dim = embedding_dim
        self.projection = nn.Linear(k, embedding_dim)
        nn.init.xavier_uniform_(self.projection.weight)
        nn.init.zeros_(self.projection.bias)
        self.register_buffer("_cached_pe", None)

    def precompute_from_edges(self, edge_index, num_nodes: int) -> None:
        self._cached_pe = ref_compute_laplacian_pe(edge_index, num_nodes, self.k)

    def project(self, pe: torch.Tensor) -> torch.Tensor:
        return self.projection(pe)

    def forward(self, node_indices: torch.Tensor) -> torch.Tensor:
        if self._cached_pe is None:
            raise RuntimeError("Laplacian PE not precomputed. Call precompute() first.")
        return self.projection(self._cached_pe[node_indices])


# --------------------------------------------------------------------------------------
# Readout (base.py:116-193) — the reference's Python loop, kept as a loop
# --------------------------------------------------------------------------------------


class RefSessionReadout(nn.Module):
    def __init__(self, hidden_dim: int = 256, readout_type: str = "mean"):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.readout_type = readout_type
        if readout_type == "attention":
            self.attention = nn.Linear(hidden_dim, 1)
            nn.init.xavier_uniform_(self.attention.weight)
            nn.init.zeros_(self.attention.bias)

    def forward(self, node_embeddings: torch.Tensor, batch_indices: torch.Tensor) -> torch.Tensor:
        B = int(batch_indices.max().item()) + 1
        dt = node_embeddings.dtype
        if self.readout_type in ("mean", "max", "last"):
            se = torch.zeros(B, self.hidden_dim, dtype=dt)
            for i in range(B):
                rows = node_embeddings[batch_indices == i]
                if self.readout_type == "mean":
                    se[i] = rows.mean(dim=0)
                elif self.readout_type == "max":
                    se[i] = rows.max(dim=0)[0]
                else:
                    se[i] = rows[-1]
            return se
        if self.readout_type == "attention":
            scores = self.attention(node_embeddings).squeeze(-1)
            w = torch.zeros(B, node_embeddings.size(0), dtype=dt)
            for i in range(B):
                m = batch_indices == i
                w[i, m] = torch.softmax(scores[m], dim=0)
            return w @ node_embeddings
        raise ValueError(f"Unknown readout type: {self.readout_type}")


# --------------------------------------------------------------------------------------
# Model (graph_transformer.py:23-182 on base.py:9-113)
# --------------------------------------------------------------------------------------


class RefGraphTransformer(nn.Module):
    """Same attribute names (hence state_dict keys) as the reference GraphTransformer."""

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
        super().__init__()
        self.num_items = num_items
        self.embedding_dim = embedding_dim
        self.hidden_dim = hidden_dim
        self.num_layers = num_layers
        self.dropout = dropout
        self.item_embedding = nn.Embedding(num_items, embedding_dim, padding_idx=0)
        nn.init.xavier_uniform_(self.item_embedding.weight[1:])
        self.num_heads = num_heads
        self.readout_type = readout_type
        self.use_laplacian_pe = use_laplacian_pe
        self.laplacian_k = laplacian_k
        self.use_ffn = use_ffn
        self.ffn_expansion = ffn_expansion
        if use_laplacian_pe:
            self.laplacian_pe = RefLaplacianPECached(k=laplacian_k, embedding_dim=embedding_dim)
        self.convs = nn.ModuleList()
        self.batch_norms = nn.ModuleList()
        self.ffns = nn.ModuleList() if use_ffn else None
        dims = [embedding_dim] + [hidden_dim] * (num_layers - 1)
        for d_in in dims:
            self.convs.append(RefTransformerConv(d_in, hidden_dim // num_heads, num_heads, dropout))
            self.batch_norms.append(nn.BatchNorm1d(hidden_dim))
            if use_ffn:
                self.ffns.append(
                    nn.Sequential(
                        nn.Linear(hidden_dim, hidden_dim * ffn_expansion),
                        nn.GELU(),
                        nn.Dropout(dropout),
                        nn.Linear(hidden_dim * ffn_expansion, hidden_dim),
                        nn.Dropout(dropout),
                    )
                )
        self.dropout_layer = nn.Dropout(dropout)
        self.readout = RefSessionReadout(hidden_dim, readout_type)

    def forward(self, batch) -> torch.Tensor:
        x = self.item_embedding(batch.x)
        edge_index = batch.edge_index
        if self.use_laplacian_pe:
            pe = getattr(batch, "laplacian_pe", None)
            x = x + (self.laplacian_pe.project(pe) if pe is not None else self.laplacian_pe(batch.x))
        if self.use_ffn:
            masks = getattr(self, "drop_masks", None) if self.training else None
            for l, (conv, bn, ffn) in enumerate(zip(self.convs, self.batch_norms, self.ffns)):
                r = x
                if masks is not None:  # graph_transformer.py:160-170 with the HIP path's masks
                    conv.attn_mask = masks["attn"][l]
                    x = (bn(conv(x, edge_index)) + r) * masks["out"][l]
                    conv.attn_mask = None
                    r = x
                    h = ffn[1](ffn[0](x)) * masks["ffn_h"][l]
                    x = ffn[3](h) * masks["ffn_o"][l] + r
                else:
                    x = self.dropout_layer(bn(conv(x, edge_index)) + r)
                    r = x
                    x = ffn(x) + r
        else:
            masks = getattr(self, "drop_masks", None) if self.training else None
            for l, (conv, bn) in enumerate(zip(self.convs, self.batch_norms)):
                r = x
                if masks is not None:
                    conv.attn_mask = masks["attn"][l]
                    x = (bn(conv(x, edge_index)) + r) * masks["out"][l]
                    conv.attn_mask = None
                else:
                    x = self.dropout_layer(bn(conv(x, edge_index)) + r)
        return self.readout(x, batch.batch)

    def get_item_embeddings(self) -> torch.Tensor:
        return self.item_embedding.weight

    def predict(self, session_embeddings: torch.Tensor, k: int = 20) -> torch.Tensor:
        scores = session_embeddings @ self.item_embedding.weight.t()
        return torch.topk(scores, k=k, dim=1)[1]

    def compute_loss(self, se, target_items, negative_items):
        return ref_bpr(se, target_items, negative_items, self.item_embedding)


def ref_create_graph_transformer_optimized(num_items, **kw) -> RefGraphTransformer:
    """graph_transformer.py:231-280 defaults."""
    d = dict(
        embedding_dim=256, hidden_dim=256, num_layers=2, num_heads=2, dropout=0.1,
        readout_type="mean", use_laplacian_pe=True, laplacian_k=16, use_ffn=False,
        ffn_expansion=2,
    )
    d.update(kw)
    return RefGraphTransformer(num_items, **d)


# --------------------------------------------------------------------------------------
# The HIP path's dropout stream, restated so that the oracle can apply the SAME masks
# (value-level parity at p > 0; torch's CPU generator cannot be reproduced on the device)
# --------------------------------------------------------------------------------------

_M32 = np.uint64(0xFFFFFFFF)


def _u32(x):
    return np.asarray(x, np.uint64) & _M32


def hip_mix3(a, b, c) -> np.ndarray:
    """gtr_common.cuh ``mix3`` (32-bit wrap-around arithmetic) over numpy arrays."""
    a, b, c = _u32(a), _u32(b), _u32(c)
    h = (a * np.uint64(0x9E3779B1)) & _M32
    h ^= (b + np.uint64(0x7F4A7C15) + ((h << np.uint64(6)) & _M32) + (h >> np.uint64(2))) & _M32
    h = (h * np.uint64(0x85EBCA77)) & _M32
    h ^= (c * np.uint64(0xC2B2AE3D)) & _M32
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x7FEB352D)) & _M32
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x846CA68B)) & _M32
    h ^= h >> np.uint64(16)
    return h


def hip_drop_stream(kind: int, layer: int, ctr: int) -> int:
    """gtr_common.cuh ``drop_stream``: kind 0 = attention probabilities of a layer,
    kind 1 = the layer's output (BN + residual), kind 2 / 3 = its feed-forward block's
    hidden / output dropout (gtr.h gtr_ffn)."""
    return int(((kind << 28) ^ (layer << 20) ^ ((ctr * 0x632BE5AB) & 0xFFFFFFFF)) & 0xFFFFFFFF)


def hip_dropout_masks(seed: int, ctr: int, p: float, num_layers: int, edge_index, num_nodes: int, dim: int,
                      heads: int, ffn_expansion: int = 0) -> dict:
    """The masks (0 or 1/(1-p)) the HIP step applies at dropout ``p`` with stream counter
    ``ctr``: {"attn": [L] x [E, H] in edge_index order, "out": [L] x [N, D]}.

    Element indices follow the kernels: attention (edge, head) pairs are numbered in the
    packed batch's destination order (a stable sort of edge_index by destination,
    etpgt/data/batch.py build_csr) as e*H + h; output elements as row*D + j.  Keep iff
    mix3(seed, stream, idx) >= uint32(p * 2^32) (p as the fp32 config value).
    ``ffn_expansion`` > 0 adds the feed-forward blocks' masks: "ffn_h" [N, F] (kind 2,
    row*F + j, after GELU) and "ffn_o" [N, D] (kind 3, row*D + j, after the second Linear)."""
    pf = float(np.float32(p))
    thresh = np.uint64(int(pf * 4294967296.0))
    scale = float(np.float32(1.0 / (1.0 - pf)))
    dst = np.asarray(edge_index[1], np.int64)
    E = dst.shape[0]
    order = np.argsort(dst, kind="stable")
    pos = np.empty(E, np.int64)
    pos[order] = np.arange(E)
    idx_attn = pos[:, None] * heads + np.arange(heads)[None, :]
    idx_out = np.arange(num_nodes * dim, dtype=np.int64).reshape(num_nodes, dim)
    out = {"attn": [], "out": []}
    for l in range(num_layers):
        ha = hip_mix3(seed, hip_drop_stream(0, l, ctr), idx_attn)
        ho = hip_mix3(seed, hip_drop_stream(1, l, ctr), idx_out)
        out["attn"].append(torch.from_numpy(np.where(ha >= thresh, scale, 0.0).astype(np.float32)))
        out["out"].append(torch.from_numpy(np.where(ho >= thresh, scale, 0.0).astype(np.float32)))
        if ffn_expansion > 0:
            F = ffn_expansion * dim
            idx_h = np.arange(num_nodes * F, dtype=np.int64).reshape(num_nodes, F)
            hh = hip_mix3(seed, hip_drop_stream(2, l, ctr), idx_h)
            hf = hip_mix3(seed, hip_drop_stream(3, l, ctr), idx_out)
            out.setdefault("ffn_h", []).append(torch.from_numpy(np.where(hh >= thresh, scale, 0.0).astype(np.float32)))
            out.setdefault("ffn_o", []).append(torch.from_numpy(np.where(hf >= thresh, scale, 0.0).astype(np.float32)))
    return out


# --------------------------------------------------------------------------------------
# Losses (losses.py:8-228; base.py:97-111)
# --------------------------------------------------------------------------------------


def _scores(se, target_items, negative_items, emb):
    t = emb(target_items)
    n = emb(negative_items)
    pos = (se * t).sum(dim=1)
    neg = torch.bmm(n, se.unsqueeze(2)).squeeze(2)
    return pos, neg


def ref_bpr(se, target_items, negative_items, emb):
    pos, neg = _scores(se, target_items, negative_items, emb)
    return -torch.log(torch.sigmoid(pos.unsqueeze(1) - neg) + 1e-8).mean()


def ref_listwise(se, target_items, negative_items, emb, temperature: float = 1.0):
    pos, neg = _scores(se, target_items, negative_items, emb)
    logits = torch.cat([pos.unsqueeze(1), neg], dim=1) / temperature
    return F.cross_entropy(logits, torch.zeros(logits.size(0), dtype=torch.long))


def ref_dual(se, target_items, negative_items, emb, alpha: float = 0.7, temperature: float = 1.0):
    lw = ref_listwise(se, target_items, negative_items, emb, temperature)
    bpr = ref_bpr(se, target_items, negative_items, emb)
    return alpha * lw + (1 - alpha) * bpr


def ref_loss(kind: str, se, target_items, negative_items, emb, alpha=0.7, temperature=1.0):
    if kind == "bpr":
        return ref_bpr(se, target_items, negative_items, emb)
    if kind in ("listwise", "sampled_softmax"):
        return ref_listwise(se, target_items, negative_items, emb, temperature)
    if kind == "dual":
        return ref_dual(se, target_items, negative_items, emb, alpha, temperature)
    raise ValueError(f"Unknown loss type: {kind}")


# --------------------------------------------------------------------------------------
# Batch (duck-typed PyG Batch; dataloader.py:157-202 layout)
# --------------------------------------------------------------------------------------


class RefBatch:
    """x [N] global ids, edge_index [2,E] (offset), batch [N], target_item [B],
    negative_items [B*n]; optional laplacian_pe [N,k]."""

    def __init__(self, x, edge_index, batch, target_item=None, negative_items=None, laplacian_pe=None):
        self.x = x
        self.edge_index = edge_index
        self.batch = batch
        self.target_item = target_item
        self.negative_items = negative_items
        self.laplacian_pe = laplacian_pe

    @property
    def num_graphs(self) -> int:
        return int(self.batch.max().item()) + 1

    def to(self, device):
        return self


def ref_batch_from(sb) -> RefBatch:
    """Build a CPU RefBatch from any object exposing the Batch contract fields."""
    def c(t):
        return None if t is None else t.detach().cpu().long()

    pe = getattr(sb, "laplacian_pe", None)
    return RefBatch(
        c(sb.x), c(sb.edge_index), c(sb.batch), c(sb.target_item), c(sb.negative_items),
        None if pe is None else pe.detach().cpu().float(),
    )


# --------------------------------------------------------------------------------------
# One training step (trainer.py:80-133)
# --------------------------------------------------------------------------------------


def ref_train_step(model, batch, optimizer, loss_kind: str = "bpr", alpha=0.7, temperature=1.0):
    """trainer.py:80-133: forward, reshape negatives, loss, zero_grad, backward, step."""
    model.train()
    se = model(batch)
    B = batch.target_item.shape[0]
    n = batch.negative_items.numel() // B
    neg = batch.negative_items.view(B, n)
    if loss_kind == "model":
        loss = model.compute_loss(se, batch.target_item, neg)
    else:
        loss = ref_loss(loss_kind, se, batch.target_item, neg, model.item_embedding, alpha, temperature)
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    return loss.detach()
