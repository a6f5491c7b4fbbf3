"""FFN variant, host side (no GPU): the flat parameter layout covers every FFN parameter
under the reference's state_dict names, the oracle's FFN dropout masks, and the entry
points that must refuse FFN models."""

from __future__ import annotations

import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import etpgt_ref as R  # noqa: E402
from etpgt.backend.engine import ParamLayout, model_param_map  # noqa: E402
from etpgt.model import create_graph_transformer  # noqa: E402


def test_ffn_state_dict_keys_match_reference_layout():
    torch.manual_seed(0)
    m = create_graph_transformer(50, embedding_dim=64, hidden_dim=64, num_layers=3, num_heads=2, use_ffn=True)
    ref = R.RefGraphTransformer(50, embedding_dim=64, hidden_dim=64, num_layers=3, num_heads=2, use_ffn=True)
    assert set(m.state_dict()) == set(ref.state_dict())
    assert "ffns.2.0.weight" in m.state_dict() and tuple(m.ffns[0][3].weight.shape) == (64, 256)


def test_ffn_param_layout_covers_every_dense_parameter():
    m = create_graph_transformer(50, embedding_dim=128, hidden_dim=128, num_layers=2, num_heads=4, use_ffn=True,
                                 use_laplacian_pe=True, laplacian_k=16)
    lay = ParamLayout(128, 2, 16, ffn=True)
    mp = model_param_map(m)
    covered = {id(p) for _, p, _ in mp}
    dense = [p for n, p in m.named_parameters() if n != "item_embedding.weight"]
    assert {id(p) for p in dense} == covered
    for name, p, row in mp:
        s = lay.seg(name)
        assert s.begin % 256 == 0
        if name.endswith("ffn_w1"):
            assert s.shape == (512, 128) and p.shape == (512, 128)
        if name.endswith("ffn_w2"):
            assert s.shape == (128, 512) and p.shape == (128, 512)
    assert lay.ffn_block == 8 * 128 * 128 + 5 * 128 and lay.ffn_stride % 256 == 0
    segs = sorted((s.begin, s.begin + s.numel) for s in lay.segs.values())
    assert all(a[1] <= b[0] for a, b in zip(segs, segs[1:])), "segments overlap"


def test_oracle_ffn_masks_shapes_and_rate():
    rng = np.random.default_rng(0)
    N, D, H, p = 40, 64, 2, 0.25
    ei = rng.integers(0, N, size=(2, 120))
    mk = R.hip_dropout_masks(987654321, 3, p, 2, ei, N, D, H, ffn_expansion=4)
    assert len(mk["ffn_h"]) == 2 and tuple(mk["ffn_h"][0].shape) == (N, 4 * D)
    assert tuple(mk["ffn_o"][1].shape) == (N, D)
    scale = np.float32(1.0 / (1.0 - np.float32(p)))
    for t in mk["ffn_h"] + mk["ffn_o"]:
        vals = set(np.unique(t.numpy()).tolist())
        assert vals <= {0.0, float(scale)}
        keep = float((t > 0).float().mean())
        assert abs(keep - (1 - p)) < 0.05
    # the four streams of a layer differ
    assert not torch.equal(mk["ffn_o"][0], mk["out"][0])
    assert "ffn_h" not in R.hip_dropout_masks(987654321, 3, p, 2, ei, N, D, H)


def test_ffn_models_refuse_unsupported_fused_steps_and_shapes(monkeypatch):
    from etpgt.train.fused import FusedTrainStep

    # data parallel on the replicated or row-sharded table, with or without SyncBN, is
    # supported (tests/test_gpu_ffn_dp.py); GTR_TAILW and SyncBN outside dim 64 / 128 at
    # expansion 4 refuse up front
    m = create_graph_transformer(50, embedding_dim=64, hidden_dim=64, num_layers=2, num_heads=2, use_ffn=True)
    monkeypatch.setenv("GTR_TAILW", "1")
    with pytest.raises(NotImplementedError, match="use_ffn"):
        FusedTrainStep(m)
    monkeypatch.delenv("GTR_TAILW")
    m2 = create_graph_transformer(50, embedding_dim=64, hidden_dim=64, num_layers=2, num_heads=2, use_ffn=True,
                                  ffn_expansion=2)
    with pytest.raises(NotImplementedError, match="ffn_expansion 4"):
        FusedTrainStep(m2, data_parallel=True, sync_bn=True)
    # the reference's create_graph_transformer defaults (d = 256, FFN x 4) and the optimized
    # factory's FFN x 2 are supported (gtr_gemm_gen.hip); other widths / expansions refuse
    create_graph_transformer(50)._check_supported()
    create_graph_transformer(50, embedding_dim=64, hidden_dim=64, num_layers=2, num_heads=2, use_ffn=True,
                             ffn_expansion=2)._check_supported()
    bad = create_graph_transformer(50, embedding_dim=96, hidden_dim=96, num_layers=2, num_heads=4, use_ffn=True)
    with pytest.raises(NotImplementedError, match="hidden_dim 64 / 128 / 256"):
        bad._check_supported()
    odd = create_graph_transformer(50, embedding_dim=64, hidden_dim=64, num_layers=2, num_heads=2, use_ffn=True,
                                   ffn_expansion=3)
    with pytest.raises(NotImplementedError, match="ffn_expansion 1 / 2 / 4"):
        odd._check_supported()
    ok = create_graph_transformer(50, embedding_dim=128, hidden_dim=128, num_layers=2, num_heads=4, use_ffn=True)
    ok._check_supported()
