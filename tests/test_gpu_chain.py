"""The fused middle of the step (gtr_chain_mid): conv_fwd(1..L-1) -> readout + loss ->
conv_bwd(L-1..0) in ONE launch with in-launch barriers, against the same step as separate
launches (GTR_CHAIN_MID=0).  Same layer bodies, same row groups, same summation orders,
so the trained state must be equal BIT FOR BIT: losses, every parameter, the BatchNorm
buffers, the table and both AdamW moments.  The separate launches are themselves held to
the oracle by test_gpu_parity.py / test_gpu_fullsize.py."""

from __future__ import annotations

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

from gpu_helpers import batches, make_pair, small_data  # noqa: E402

from etpgt.data.synthetic import make_sessions_and_graph  # noqa: E402
from etpgt.train.fused import FusedTrainStep  # noqa: E402

_DATA = {}


def data(full: bool):
    if full not in _DATA:
        _DATA[full] = make_sessions_and_graph(seed=42) if full else small_data()
    return _DATA[full]


def _chain_vs_split(monkeypatch, D, H, K, loss, dropout, n, steps, full=False, B=32):
    d = data(full)
    T = d.table_rows
    m1, _ = make_pair(T, D, H, K=K, dropout=dropout, seed=21)
    m2 = copy.deepcopy(m1)
    m1.cuda().train()
    m2.cuda().train()
    bl = batches(d, B, n, steps, seed=31)
    monkeypatch.setenv("GTR_CHAIN_MID", "0")
    f1 = FusedTrainStep(m1, lr=1e-3, weight_decay=1e-5, loss=loss)
    f1(bl[0].to("cuda"))
    monkeypatch.setenv("GTR_CHAIN_MID", "1")
    f2 = FusedTrainStep(m2, lr=1e-3, weight_decay=1e-5, loss=loss)
    l2 = [float(f2(bl[0].to("cuda")))]
    for sb in bl[1:]:
        dsb = sb.to("cuda")
        assert float(f1(dsb)) == float(f2(dsb))
    assert not f1.chain_mid and f2.chain_mid
    for (n1, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n1
    for (n1, a), (_, b) in zip(m1.named_buffers(), m2.named_buffers()):
        if a is not None:
            assert torch.equal(a, b), n1
    for name in ("m_tab", "v_tab", "m_flat", "v_flat"):
        assert torch.equal(getattr(f1, name), getattr(f2, name)), name
    assert f2.chain_bar.tolist() == [0, 0, 0, 0], "barrier counters re-armed, no timeout"
    return l2, f2


@pytest.mark.parametrize("D,H,K,loss,dropout,n", [(64, 1, 0, "bpr", 0.1, 5), (128, 4, 16, "listwise", 0.1, 100),
                                                  (32, 2, 0, "dual", 0.0, 7), (64, 2, 8, "bpr", 0.0, 5)])
def test_chain_mid_bitwise_equals_separate_launches(monkeypatch, D, H, K, loss, dropout, n):
    _chain_vs_split(monkeypatch, D, H, K, loss, dropout, n, steps=5)


def test_chain_mid_full_c2_table(monkeypatch):
    """C2 shape on the full 82,174-row table (the merged sweep slice covers slots 1..2L of
    the whole table), dropout 0.1, 6 steps."""
    _, f2 = _chain_vs_split(monkeypatch, 64, 1, 0, "bpr", 0.1, 5, steps=6, full=True)
    assert f2.sweep is not None


def test_chain_mid_not_taken_past_its_limits(monkeypatch):
    """Batches with more than 32 row groups keep the separate launches."""
    d = data(False)
    m1, _ = make_pair(d.table_rows, 64, 1, K=0, seed=3)
    m1.cuda().train()
    f = FusedTrainStep(m1, loss="bpr")
    f(batches(d, 300, 5, 1, seed=5)[0].to("cuda"))
    assert not f.chain_mid
