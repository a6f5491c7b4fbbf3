"""GPU: weight gradients folded into the fused backward (gtr_layer.wfold, gtr_config.
wfold_stride): every row group of gtr_conv_bwd writes its split-K partial of dW_all, db_all
and dW_beta (the gtr_wgrad jobs of the layer over the group's rows), and the optimizer tail
sums the batch's live groups (gtr_segment.live_groups).  Against gtr_wgrad's chunked
partials (GTR_WFOLD=0) on the same step: the summed gradients agree to fp32 summation-order
noise, and three steps of training agree with the oracle-grade bar."""

from __future__ import annotations

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

from gpu_helpers import batches, make_pair, small_data  # noqa: E402

from etpgt.train.fused import FusedTrainStep  # noqa: E402


@pytest.mark.parametrize("D,H,K,loss,B", [(64, 1, 0, "bpr", 32), (64, 4, 16, "listwise", 32),
                                          (32, 2, 0, "bpr", 96), (64, 2, 0, "dual", 200)])
def test_folded_weight_gradients_equal_wgrad(D, H, K, loss, B, monkeypatch):
    data = small_data()
    T = data.table_rows
    m1, _ = make_pair(T, D, H, K=K, seed=81)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    n = 100 if loss != "bpr" else 5
    bl = batches(data, B, n, 3, seed=82)
    monkeypatch.setenv("GTR_WFOLD", "1")
    f1 = FusedTrainStep(m1, lr=1e-3, weight_decay=1e-5, loss=loss, use_graph=False)
    l1 = float(f1(bl[0].to("cuda")))
    monkeypatch.setenv("GTR_WFOLD", "0")
    f2 = FusedTrainStep(m2, lr=1e-3, weight_decay=1e-5, loss=loss, use_graph=False)
    l2 = float(f2(bl[0].to("cuda")))
    assert f1.wfold and not f2.wfold and not f1.split
    assert l1 == l2  # the forward and the loss do not depend on the weight-gradient path
    G = int(f1.blob[0:8].cpu()[4])  # live row groups (hdr[4])
    stride_cols = 4 * D * D + 7 * D
    for l in range(2):
        fold = f1.ws.wfold[l, :G, :stride_cols].double().sum(0)
        chunk = f2.ws.slabs[l, :, :stride_cols].double().sum(0)
        scale = float(chunk.abs().max())
        err = float((fold - chunk).abs().max())
        assert err <= 1e-5 * scale, (l, err, scale)
    for sb in bl[1:]:
        dsb = sb.to("cuda")
        a, b = float(f1(dsb)), float(f2(dsb))
        assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), (a, b)
    for (name, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        if name.endswith("lin_key.bias"):
            continue
        assert float((a - b).norm()) <= 1e-4 * float(b.norm()) + 1e-7, name
