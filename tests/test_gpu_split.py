"""GPU: the large-batch ("split") layer path -- gtr_qkvs_fwd + gtr_attn_fwd and
gtr_attn_bwd + gtr_qkvs_bwd (csrc/gtr_gemm.hip) -- against the fused layer kernels and the
oracle.

The split path runs the same arithmetic in the same k order (the GEMMs keep the fused
kernels' mfma4 chains), so every forward activation (xin, qkvs, alpha, agg, gate, out),
the loss and the last layer's dQKVS are BITWISE those of the fused kernels; only the
BatchNorm backward sums of the layers below are summed in another fixed order (per GEMM
workgroup instead of per row group), which moves the rest by float rounding.  Against
the CPU oracle it is held to the usual 1e-3 bar."""

from __future__ import annotations

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

import etpgt_ref as R  # noqa: E402
from gpu_helpers import OracleTrio, assert_close, batches, make_pair, small_data  # noqa: E402

from etpgt.train.fused import FusedTrainStep  # noqa: E402

CASES = [  # (D, H, K, loss, B)
    (64, 1, 0, "bpr", 256),
    (128, 4, 16, "listwise", 256),
    (128, 4, 16, "dual", 2100),
]


def _step(m, loss, split, monkeypatch, **kw):
    monkeypatch.setenv("GTR_SPLIT", "1" if split else "0")
    # producer-finalized BatchNorm statistics on both sides (the split path's mode): the
    # same partial grouping, so the same sums
    monkeypatch.setenv("GTR_CONSUMER_REDUCE", "0")
    f = FusedTrainStep(m, lr=1e-2, weight_decay=1e-2, loss=loss, use_graph=False, **kw)
    return f


@pytest.mark.parametrize("D,H,K,loss,B", CASES)
def test_split_forward_bitwise_equals_fused(D, H, K, loss, B, monkeypatch):
    """GTR_ATTN=group: the split path's attention on the fused kernels' row-group body --
    bitwise the fused step (see the module docstring)."""
    monkeypatch.setenv("GTR_ATTN", "group")
    data = small_data()
    T = data.table_rows
    m1, _ = make_pair(T, D, H, K=K, seed=61)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    p0 = {k: v.detach().clone() for k, v in m1.named_parameters()}
    n = 100 if loss != "bpr" else 5
    sb = batches(data, B, n, 1, seed=62)[0]
    f1 = _step(m1, loss, False, monkeypatch)
    l1 = float(f1(sb.to("cuda")))
    f2 = _step(m2, loss, True, monkeypatch)
    l2 = float(f2(sb.to("cuda")))
    assert not f1.split and f2.split
    assert l1 == l2, (l1, l2)
    N, E = sb.num_nodes, sb.num_edges
    for l in range(2):
        a, b = f1.ws.layers[l], f2.ws.layers[l]
        for name, rows in (("xin", N), ("qkvs", N), ("agg", N), ("out", N), ("gate", N), ("alpha", E)):
            assert torch.equal(a[name][:rows], b[name][:rows]), (l, name)
    assert torch.equal(f1.ws.se[:B], f2.ws.se[:B])
    top = f1.ws.layers[1]["dqkvs"][:N], f2.ws.layers[1]["dqkvs"][:N]
    assert torch.equal(*top)  # its BatchNorm sums come from the readout in both paths
    assert_close(f2.ws.layers[0]["dqkvs"][:N], f1.ws.layers[0]["dqkvs"][:N], rtol=1e-4, name="dqkvs layer 0")
    assert_close(f2.ws.dx0[:N], f1.ws.dx0[:N], rtol=1e-4, name="dx0")
    # one AdamW step (lr 1e-2) on gradients that differ by rounding only.  A first Adam
    # step moves an element by lr * g / (|g| + eps): by lr exactly unless |g| is near eps,
    # i.e. a gradient that cancels to rounding noise, whose update then depends on that
    # noise -- such elements (fused update visibly shorter than lr) are bounded by 2 lr,
    # every other element is held to 1e-3
    for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        if n1.endswith("lin_key.bias"):
            continue
        step = (p1.detach() - p0[n1] * (1.0 - 1e-2 * 1e-2)).abs()
        noise = step < 0.99e-2
        assert float((p2.detach() - p1.detach())[noise].abs().max()) <= 2e-2 + 1e-7 if bool(noise.any()) else True
        assert_close(p2.detach()[~noise], p1.detach()[~noise], rtol=1e-3, name=n1)


@pytest.mark.parametrize("D,H,K,loss,B", CASES[:2])
def test_split_training_matches_oracle(D, H, K, loss, B, monkeypatch):
    """Three AdamW steps on the split path (captured hipGraph) against the CPU oracle."""
    monkeypatch.setenv("GTR_SPLIT", "1")
    data = small_data()
    T = data.table_rows
    m, ref = make_pair(T, D, H, K=K, seed=63, pe_table=torch.rand(T, max(K, 1)) if K else None)
    m.train(); ref.train()
    f = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, loss=loss)
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-3, weight_decay=1e-5))
    n = 100 if loss != "bpr" else 5
    for sb in batches(data, B, n, 3, seed=64):
        l = float(f(sb.to("cuda")))
        rb = R.ref_batch_from(sb)
        rl = float(trio.step(lambda mod, o: R.ref_train_step(mod, rb, o, loss)))
        assert abs(l - rl) <= 1e-3 * abs(rl), (l, rl)
    assert f.split
    trio.compare({k: v.detach().cpu() for k, v in m.named_parameters()}, lr=1e-3)


def test_split_eval_forward_matches_oracle(monkeypatch):
    """model(batch) in eval mode (running statistics) through the split path."""
    monkeypatch.setenv("GTR_SPLIT", "1")
    data = small_data()
    T = data.table_rows
    m, ref = make_pair(T, 128, 4, seed=65)
    with torch.no_grad():
        for bn, rb in zip(m.batch_norms, ref.batch_norms):
            bn.running_mean.uniform_(-0.1, 0.1)
            bn.running_var.uniform_(0.5, 2.0)
            rb.running_mean.copy_(bn.running_mean.cpu())
            rb.running_var.copy_(bn.running_var.cpu())
    m.eval(); ref.eval()
    sb = batches(data, 512, 5, 1, seed=66)[0]
    with torch.no_grad():
        se = m(sb.to("cuda"))
        rse = ref(R.ref_batch_from(sb))
    assert m.hip_engine().workspace(m.hip_engine().prepare(sb)[0]).split
    assert_close(se, rse, rtol=1e-3, name="session embeddings (eval)")


@pytest.mark.parametrize("D,H,K,loss,B", CASES)
def test_split_row_attention_equals_fused(D, H, K, loss, B, monkeypatch):
    """The default split path: row-parallel attention kernels (one wave per destination /
    source row, k_attn_rows*).  The projection is still bitwise the fused one; attention,
    softmax and BatchNorm partials are summed in another order, so the rest agrees to
    float rounding (1e-4 relative) -- and the whole step to the oracle in
    test_split_training_matches_oracle."""
    monkeypatch.delenv("GTR_ATTN", raising=False)
    data = small_data()
    T = data.table_rows
    m1, _ = make_pair(T, D, H, K=K, seed=67)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    n = 100 if loss != "bpr" else 5
    sb = batches(data, B, n, 1, seed=68)[0]
    f1 = _step(m1, loss, False, monkeypatch)
    l1 = float(f1(sb.to("cuda")))
    f2 = _step(m2, loss, True, monkeypatch)
    l2 = float(f2(sb.to("cuda")))
    assert abs(l1 - l2) <= 1e-5 * abs(l1), (l1, l2)
    N, E = sb.num_nodes, sb.num_edges
    a, b = f1.ws.layers[0], f2.ws.layers[0]
    assert torch.equal(a["xin"][:N], b["xin"][:N]) and torch.equal(a["qkvs"][:N], b["qkvs"][:N])
    for l in range(2):
        a, b = f1.ws.layers[l], f2.ws.layers[l]
        for name, rows in (("xin", N), ("qkvs", N), ("agg", N), ("out", N), ("gate", N), ("alpha", E),
                           ("dqkvs", N), ("du", N)):  # (the fused fast path keeps dlogit in LDS)
            assert_close(b[name][:rows], a[name][:rows], rtol=1e-4, name=f"layer {l} {name}")
    assert_close(f2.ws.dx0[:N], f1.ws.dx0[:N], rtol=1e-4, name="dx0")
    _params_after_one_adam_step(m1, m2, lr=1e-2)


def _params_after_one_adam_step(m1, m2, lr):
    """One AdamW step from equal parameters: the update is lr * g / (|g| + eps) per element,
    so gradients equal to float rounding give equal parameters -- except where |g| is at
    the eps floor and the rounding moves the update by up to 2 lr.  Elementwise 1e-3, and
    at most one element in 1,000 per tensor inside 2 lr instead."""
    for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        if n1.endswith("lin_key.bias"):
            continue
        a, b = p2.detach().float().cpu(), p1.detach().float().cpu()
        tol = 1e-3 * (b.abs() + 1e-2 * float(b.abs().max()))
        miss = (a - b).abs() > tol
        assert float(miss.float().mean()) <= 1e-3, (n1, int(miss.sum()))
        if bool(miss.any()):
            assert float((a - b).abs()[miss].max()) <= 2 * lr, n1
