"""FFN variant (use_ffn=True, graph_transformer.py:88-100,160-170) on the HIP split layer
kernels + gtr_ffn_fwd / gtr_ffn_bwd / gtr_ffn_wgrad, against the CPU oracle
(oracle/etpgt_ref.py RefGraphTransformer(use_ffn=True): torch nn.Linear / nn.GELU).

Tolerances: the same bar as the optimized model's autograd tests (test_gpu_parity.py
test_train_grads): session embeddings, loss and running statistics within 1e-3 relative
(assert_close), every parameter gradient within 2e-3 relative with an absolute floor of
1e-6 of the largest gradient; trained parameters after AdamW steps within 1e-3 relative
(assert_close, plus the tensor-norm bar).  Dropout p > 0 is checked value for value with
the oracle applying the HIP path's own masks (hip_dropout_masks, kinds 0-3).
"""

from __future__ import annotations

import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import etpgt_ref as R  # noqa: E402
from etpgt.model import create_graph_transformer  # noqa: E402
from gpu_helpers import (OracleTrio, assert_close, batches, edge_case_batch, ref_batch,  # noqa: E402
                         small_data)

pytestmark = pytest.mark.gpu

_DATA = None


def data():
    global _DATA
    if _DATA is None:
        _DATA = small_data()
    return _DATA


def make_ffn_pair(T, D, H, L=2, K=0, dropout=0.0, seed=0, expansion=4):
    """HIP FFN model (cuda) + oracle FFN model (cpu) with identical parameters."""
    torch.manual_seed(seed)
    m = create_graph_transformer(T, embedding_dim=D, hidden_dim=D, num_layers=L, num_heads=H, dropout=dropout,
                                 use_laplacian_pe=K > 0, laplacian_k=max(K, 1), use_ffn=True,
                                 ffn_expansion=expansion)
    if K > 0:
        m.laplacian_pe._cached_pe = torch.rand(T, K)
    with torch.no_grad():
        for bn in m.batch_norms:
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
    ref = R.RefGraphTransformer(T, embedding_dim=D, hidden_dim=D, num_layers=L, num_heads=H, dropout=dropout,
                                use_laplacian_pe=K > 0, laplacian_k=max(K, 1), use_ffn=True, ffn_expansion=expansion)
    if K > 0:
        ref.laplacian_pe._cached_pe = torch.zeros(T, K)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    assert set(sd) == set(ref.state_dict()), "state_dict keys differ from the reference layout"
    ref.load_state_dict(sd)
    return m.cuda(), ref


def _grads_vs_oracle(m, ref, sb, n, masks=None):
    dsb = sb.to("cuda")
    B = sb.num_graphs
    se = m(dsb)
    L_hip = m.compute_loss(se, dsb.target_item, dsb.negative_items.view(B, n))
    m.zero_grad()
    L_hip.backward()
    rb = ref_batch(sb)
    ref.drop_masks = masks
    se_ref = ref(rb)
    ref.drop_masks = None
    L_ref = R.ref_loss("bpr", se_ref, rb.target_item, rb.negative_items.view(B, n), ref.item_embedding)
    ref.zero_grad()
    L_ref.backward()
    assert_close(se, se_ref, name="se")
    assert_close(L_hip.reshape(1), L_ref.reshape(1), name="loss")
    hp = dict(m.named_parameters())
    gscale = max(float(p.grad.abs().max()) for p in ref.parameters())
    for name, p in ref.named_parameters():
        assert hp[name].grad is not None, name
        assert_close(hp[name].grad, p.grad, rtol=2e-3, name=f"grad {name}", floor=1e-6 * gscale)
    hb = dict(m.named_buffers())
    for name, b in ref.named_buffers():
        if "running" in name:
            assert_close(hb[name], b, name=name)


@pytest.mark.parametrize("D,H,K,B", [(64, 1, 0, 32), (64, 2, 0, 600), (128, 4, 16, 32), (128, 4, 16, 400)])
def test_ffn_train_grads(D, H, K, B):
    """Train mode, dropout 0: loss, session embeddings, every gradient (FFN weights and
    biases included) and the BatchNorm running statistics.  B = 400 / 600 spans several
    GEMM tiles and weight-gradient chunks."""
    T = data().table_rows
    m, ref = make_ffn_pair(T, D, H, K=K, seed=3)
    m.train(); ref.train()
    sb = batches(data(), B, 5, 1, seed=11 + D)[0]
    _grads_vs_oracle(m, ref, sb, 5)


@pytest.mark.parametrize("D,H,K,B,E,L", [(256, 4, 16, 32, 4, 3), (256, 4, 16, 300, 4, 2), (128, 4, 16, 200, 2, 2),
                                         (64, 2, 0, 64, 2, 3), (256, 4, 0, 48, 2, 2)])
def test_ffn_reference_default_shapes_train_grads(D, H, K, B, E, L):
    """The FFN shapes the register-resident GEMMs do not cover, on the LDS-staged GEMMs
    (gtr_gemm_gen.hip): create_graph_transformer's own defaults -- d = 256, 4 heads, FFN x 4,
    LapPE k = 16, 3 layers (graph_transformer.py:185-197) -- and ffn_expansion = 2 (the
    optimized factory's default when its FFN is on, :231-280).  Train mode, dropout 0: the
    loss, the session embeddings, every gradient and the running statistics."""
    T = data().table_rows
    m, ref = make_ffn_pair(T, D, H, L=L, K=K, seed=3 + D + E, expansion=E)
    m.train(); ref.train()
    sb = batches(data(), B, 5, 1, seed=13 + D)[0]
    _grads_vs_oracle(m, ref, sb, 5)


def test_ffn_reference_defaults_fused_steps_match_oracle():
    """create_graph_transformer(num_items) at its defaults (d = 256, L = 3, H = 4, FFN x 4,
    LapPE k = 16) through the fused step: five steps against the oracle trainer, every
    trained parameter elementwise (gpu_helpers.close_trained)."""
    from etpgt.train.fused import FusedTrainStep

    T = data().table_rows
    m, ref = make_ffn_pair(T, 256, 4, L=3, K=16, seed=23)
    m.train(); ref.train()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, loss="bpr")
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-3, weight_decay=1e-5))
    for i, sb in enumerate(batches(data(), 32, 5, 5, seed=41)):
        hl = float(step(sb.to("cuda")))
        rb_ = ref_batch(sb)
        rl = trio.step(lambda mod, o: R.ref_train_step(mod, rb_, o, "bpr"))
        assert abs(hl - float(rl)) <= 1e-3 * max(1.0, abs(float(rl))), (i, hl, float(rl))
    trio.compare(dict(m.named_parameters()), lr=1e-3)


def test_ffn_eval_forward_d256():
    """Eval forward of the reference-default FFN model (the registered op
    etpgt::graph_transformer_eval)."""
    T = data().table_rows
    m, ref = make_ffn_pair(T, 256, 4, L=3, K=16, dropout=0.1, seed=9)
    with torch.no_grad():
        for bn, rb_ in zip(m.batch_norms, ref.batch_norms):
            bn.running_mean.uniform_(-0.1, 0.1)
            bn.running_var.uniform_(0.5, 2.0)
            rb_.running_mean.copy_(bn.running_mean.cpu())
            rb_.running_var.copy_(bn.running_var.cpu())
    m.eval(); ref.eval()
    sb = batches(data(), 40, 5, 1, seed=27)[0]
    with torch.no_grad():
        se = m(sb.to("cuda"))
        se_ref = ref(ref_batch(sb))
    assert_close(se, se_ref, name="se eval d256")


def test_ffn_three_layers_edge_cases():
    """L = 3 (the FFN factory's default depth; the middle layer reads an FFN output and
    writes d/dz of another) on the edge-case batch: nodes without in-edges, a single-node
    session, a session without edges, a dense session with self loops."""
    m, ref = make_ffn_pair(300, 64, 2, L=3, seed=5)
    m.train(); ref.train()
    _grads_vs_oracle(m, ref, edge_case_batch(), 5)


def test_ffn_dropout_values_with_hip_masks():
    """p = 0.1: the oracle applies the HIP path's own masks (attention, layer output, FFN
    hidden, FFN output) -- value-level parity of the forward and every gradient."""
    T = data().table_rows
    D, H, p = 64, 2, 0.1
    m, ref = make_ffn_pair(T, D, H, dropout=p, seed=7)
    m.train(); ref.train()
    sb = batches(data(), 64, 5, 1, seed=19)[0]
    eng = m.hip_engine()
    ctr = int(eng.rng_ctr.item())
    masks = R.hip_dropout_masks(eng.seed, ctr, p, 2, sb.edge_index.numpy(), int(sb.x.shape[0]), D, H,
                                ffn_expansion=4)
    _grads_vs_oracle(m, ref, sb, 5, masks=masks)


@pytest.mark.parametrize("D,H,K", [(64, 2, 0), (128, 4, 16)])
def test_ffn_eval_forward(D, H, K):
    """Eval mode: running statistics, no dropout; the readout's identity view of the last
    block's output."""
    T = data().table_rows
    m, ref = make_ffn_pair(T, D, H, K=K, dropout=0.1, seed=9)
    with torch.no_grad():
        for bn, rb_ in zip(m.batch_norms, ref.batch_norms):
            bn.running_mean.uniform_(-0.1, 0.1)
            bn.running_var.uniform_(0.5, 2.0)
            rb_.running_mean.copy_(bn.running_mean.cpu())
            rb_.running_var.copy_(bn.running_var.cpu())
    m.eval(); ref.eval()
    sb = batches(data(), 48, 5, 1, seed=23)[0]
    with torch.no_grad():
        se = m(sb.to("cuda"))
        se_ref = ref(ref_batch(sb))
    assert_close(se, se_ref, name="se eval")


def test_ffn_adamw_steps_match_oracle():
    """Five AdamW steps (torch.optim.AdamW on both sides, the Trainer's autograd path for
    FFN models): losses every step and every trained parameter."""
    T = data().table_rows
    m, ref = make_ffn_pair(T, 64, 2, seed=13)
    m.train(); ref.train()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-5)
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-3, weight_decay=1e-5))
    for i, sb in enumerate(batches(data(), 32, 5, 5, seed=29)):
        dsb = sb.to("cuda")
        B = sb.num_graphs
        loss = m.compute_loss(m(dsb), dsb.target_item, dsb.negative_items.view(B, 5))
        opt.zero_grad()
        loss.backward()
        opt.step()
        rb_ = ref_batch(sb)
        rl = trio.step(lambda mod, o: R.ref_train_step(mod, rb_, o, "bpr"))
        assert abs(float(loss) - float(rl)) <= 1e-4 * max(1.0, abs(float(rl))), (i, float(loss), float(rl))
    # every trained parameter ELEMENTWISE against the oracle trio (fp32 / fp32 one thread /
    # fp64): 1e-3 relative, or no further from fp64 than the fp32 oracle's own noise
    trio.compare(dict(m.named_parameters()), lr=1e-3)


@pytest.mark.parametrize("D,H,K,B,loss", [(64, 2, 0, 32, "bpr"), (128, 4, 16, 300, "listwise")])
def test_ffn_fused_step_matches_oracle(D, H, K, B, loss):
    """The fused (captured) training step on an FFN model: five steps of the whole step
    (forward, loss, backward, dense-equivalent AdamW on the table, the FFN weights among
    the small parameters) against the oracle trainer, losses every step and every trained
    parameter."""
    from etpgt.train.fused import FusedTrainStep

    T = data().table_rows
    n = 5 if loss == "bpr" else 20
    m, ref = make_ffn_pair(T, D, H, K=K, seed=21)
    m.train(); ref.train()
    step = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, loss=loss)
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-3, weight_decay=1e-5))
    for i, sb in enumerate(batches(data(), B, n, 5, seed=37)):
        hl = float(step(sb.to("cuda")))
        rb_ = ref_batch(sb)
        rl = trio.step(lambda mod, o: R.ref_train_step(mod, rb_, o, loss))
        assert abs(hl - float(rl)) <= 1e-4 * max(1.0, abs(float(rl))), (i, hl, float(rl))
    step.sync_table()
    trio.compare(dict(m.named_parameters()), lr=1e-3)


def test_ffn_trainer_runs_autograd_path(tmp_path):
    """The drop-in Trainer trains an FFN model on the autograd path (fused=False) for one
    epoch on device."""
    from etpgt.train.trainer import Trainer

    data_ = data()
    T = data_.table_rows
    m, _ = make_ffn_pair(T, 64, 2, seed=17)
    loader = [sb for sb in batches(data_, 32, 5, 4, seed=31)]
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-5)
    tr = Trainer(m, loader, loader, opt, device="cuda", output_dir=tmp_path, max_epochs=1, fused=False)
    loss = tr.train_epoch()
    assert tr._fused is None
    assert loss == loss and loss > 0
