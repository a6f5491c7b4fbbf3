"""GPU parity: the HIP path (libgtr_hip via etpgt) against the CPU oracle.

Tolerance (BASELINE.json north star): 1e-3 relative, fp32 — see gpu_helpers.assert_close.
Dropout is 0 in every value-level comparison (the HIP dropout stream cannot
reproduce the CPU generator); dropout > 0 is covered by determinism/finiteness.
"""

import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

import etpgt_ref as R  # noqa: E402
from gpu_helpers import (OracleTrio, assert_close, batches, close_trained, edge_case_batch,  # noqa: E402
                         long_session_batch, make_pair, ref_batch, small_data)

from etpgt.train.fused import FusedTrainStep  # noqa: E402
from etpgt.train.losses import create_loss_function  # noqa: E402

DATA = None


def data():
    global DATA
    if DATA is None:
        DATA = small_data()
    return DATA


CONFIGS = [
    # (D, H, K)
    (32, 2, 0),
    (64, 1, 0),
    (64, 2, 8),
    (128, 4, 16),
    (256, 2, 0),
]


def test_device_is_gfx950():
    from etpgt.backend import _lib as L

    L.check(L.lib().gtr_device_check(0), "device check")


@pytest.mark.parametrize("D,H,K", CONFIGS)
def test_forward_eval(D, H, K):
    T = data().table_rows
    m, ref = make_pair(T, D, H, K=K, seed=1)
    m.eval(); ref.eval()
    for sb in batches(data(), 32, 5, 2, seed=D) + [edge_case_batch(5, T)]:
        with torch.no_grad():
            se = m(sb.to("cuda"))
            se_ref = ref(ref_batch(sb))
        assert_close(se, se_ref, name=f"se D={D} H={H}")


@pytest.mark.parametrize("D,H,K", CONFIGS)
@pytest.mark.parametrize("loss", ["model_bpr", "listwise", "dual"])
def test_train_grads(D, H, K, loss):
    """Train mode (batch BN stats), dropout 0: loss, session embeddings and every
    parameter gradient (dense table gradient included) against oracle autograd."""
    T = data().table_rows
    n = 5 if loss != "listwise" else 20
    m, ref = make_pair(T, D, H, K=K, seed=2)
    m.train(); ref.train()
    sb = batches(data(), 32, n, 1, seed=7 + D)[0]
    if loss == "model_bpr":
        sb2 = sb
    else:
        sb2 = sb
    dsb = sb2.to("cuda")
    se = m(dsb)
    B = sb.num_graphs
    neg = dsb.negative_items.view(B, n)
    if loss == "model_bpr":
        L_hip = m.compute_loss(se, dsb.target_item, neg)
    else:
        fn = create_loss_function(loss, alpha=0.7, temperature=0.5)
        out = fn(se, dsb.target_item, neg, m.item_embedding)
        L_hip = out[0] if isinstance(out, tuple) else out
    m.zero_grad()
    L_hip.backward()
    rb = ref_batch(sb)
    se_ref = ref(rb)
    kind = "bpr" if loss == "model_bpr" else loss
    L_ref = R.ref_loss(kind, se_ref, rb.target_item, rb.negative_items.view(B, n), ref.item_embedding, 0.7, 0.5)
    ref.zero_grad()
    L_ref.backward()
    assert_close(se, se_ref, name="se")
    assert_close(L_hip.reshape(1), L_ref.reshape(1), name="loss")
    hp = dict(m.named_parameters())
    gscale = max(float(p.grad.abs().max()) for p in ref.parameters())
    for name, p in ref.named_parameters():
        assert hp[name].grad is not None, name
        assert_close(hp[name].grad, p.grad, rtol=2e-3, name=f"grad {name}", floor=1e-6 * gscale)
    for name, b in ref.named_buffers():
        if "running" in name:
            assert_close(dict(m.named_buffers())[name], b, name=name)


@pytest.mark.parametrize("split", ["0", "1"])
def test_edge_cases_train(split, monkeypatch):
    """split "1": the same edge cases on the split layer path (row-parallel attention
    kernels: rows without in-edges, single-node sessions, dense sessions)."""
    monkeypatch.setenv("GTR_SPLIT", split)
    T = data().table_rows
    m, ref = make_pair(T, 64, 2, K=0, seed=3)
    m.train(); ref.train()
    sb = edge_case_batch(5, T)
    dsb = sb.to("cuda")
    se = m(dsb)
    L_hip = m.compute_loss(se, dsb.target_item, dsb.negative_items.view(sb.num_graphs, 5))
    L_hip.backward()
    rb = ref_batch(sb)
    se_ref = ref(rb)
    L_ref = ref.compute_loss(se_ref, rb.target_item, rb.negative_items.view(sb.num_graphs, 5))
    L_ref.backward()
    assert_close(L_hip.reshape(1), L_ref.reshape(1), name="loss")
    hp = dict(m.named_parameters())
    gscale = max(float(p.grad.abs().max()) for p in ref.parameters())
    for name, p in ref.named_parameters():
        assert_close(hp[name].grad, p.grad, rtol=2e-3, name=f"grad {name}", floor=1e-6 * gscale)


@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("D,H", [(64, 2), (128, 4)])
def test_long_sessions_general_path_train(D, H, split, monkeypatch):
    """Row groups beyond the LDS carve (70-row session, 1600-edge session) run the
    general global-memory path next to fast-path groups of the same batch; split "1":
    the row-parallel attention kernels' hub pairs (more than 64 in-edges per row pair,
    ids per round, logits parked in the alpha buffer)."""
    monkeypatch.setenv("GTR_SPLIT", split)
    T = data().table_rows
    m, ref = make_pair(T, D, H, K=0, seed=4)
    m.train(); ref.train()
    sb = long_session_batch(5, T)
    dsb = sb.to("cuda")
    se = m(dsb)
    L_hip = m.compute_loss(se, dsb.target_item, dsb.negative_items.view(sb.num_graphs, 5))
    L_hip.backward()
    rb = ref_batch(sb)
    se_ref = ref(rb)
    L_ref = ref.compute_loss(se_ref, rb.target_item, rb.negative_items.view(sb.num_graphs, 5))
    L_ref.backward()
    assert_close(se, se_ref, name="se")
    assert_close(L_hip.reshape(1), L_ref.reshape(1), name="loss")
    hp = dict(m.named_parameters())
    gscale = max(float(p.grad.abs().max()) for p in ref.parameters())
    for name, p in ref.named_parameters():
        assert_close(hp[name].grad, p.grad, rtol=2e-3, name=f"grad {name}", floor=1e-6 * gscale)


@pytest.mark.parametrize("D,H,K,loss,opt", [
    (64, 1, 0, "bpr", "adamw"),        # config C2 shape
    (128, 4, 16, "listwise", "adamw"),  # config C3 shape
    (64, 2, 0, "dual", "adam"),
])
@pytest.mark.parametrize("use_graph", [False, True])
def test_fused_steps(D, H, K, loss, opt, use_graph):
    """k fused steps (forward+loss+backward+optimizer, hipGraph replay) == k
    reference trainer steps (trainer.py:80-133) with torch.optim.AdamW/Adam."""
    _fused_vs_reference(D, H, K, loss, opt, use_graph, B=32, steps=4)


def test_fused_steps_last_arriver_reductions(monkeypatch):
    """The large-grid BatchNorm reduction mode (last arriving workgroup combines the
    partials, agent-scope fences) on the C2 shape."""
    monkeypatch.setenv("GTR_CONSUMER_REDUCE", "0")
    _fused_vs_reference(64, 1, 0, "bpr", "adamw", True, B=32, steps=3)


def test_fused_steps_large_batch():
    """B = 1400: > 64 row groups (last-arriver reductions), > 8192 table-gradient
    contributions (prep + radix-sort begin path), readout grid-stride over sessions."""
    _fused_vs_reference(64, 2, 0, "bpr", "adamw", True, B=1400, steps=2)


@pytest.mark.parametrize("wgrad", ["default", "valu"])
def test_fused_steps_large_batch_c3_shape(wgrad, monkeypatch):
    """The C3 / C5 layer shape (D = 128, 4 heads, LapPE k = 16, listwise) at a batch whose
    node capacity passes 8192 rows: row groups of R = 16 rows (hundreds of groups), the
    bucketed last-arriver merges of the forward (count, mean, M2) and backward sums.  The
    weight gradients run on MFMA tiles there by default (>= 128 rows per split-K chunk:
    QKVS weight with the bias column sums folded in, narrow LapPE projection tiles);
    GTR_WGRAD=valu forces the register-tile path."""
    if wgrad != "default":
        monkeypatch.setenv("GTR_WGRAD", wgrad)
    _fused_vs_reference(128, 4, 16, "listwise", "adamw", True, B=2400, steps=2, expect_ncap=8192)


@pytest.mark.parametrize("D,H,K,loss,wgrad", [(64, 1, 0, "bpr", "default"), (128, 4, 16, "listwise", "default"),
                                               (128, 4, 16, "listwise", "mfma"), (32, 2, 8, "dual", "default")])
def test_tail_wgrad_bitwise_equals_separate_launches(D, H, K, loss, wgrad, monkeypatch):
    """gtr_step_tail_wgrad (opt-in GTR_TAILW=1: weight-gradient tiles and the
    optimizer tail in one launch, each tile's last arriving chunk summing the split-K
    partials in chunk order and applying AdamW) against gtr_wgrad + gtr_step_tail
    (GTR_TAILW=0): losses, parameters, buffers and moments bit for bit, dropout on."""
    if wgrad != "default":
        monkeypatch.setenv("GTR_WGRAD", wgrad)
    monkeypatch.setenv("GTR_WFOLD", "0")  # the reference: gtr_wgrad's split-K chunks
    T = data().table_rows
    n = 100 if loss == "listwise" else 5
    m1, _ = make_pair(T, D, H, K=K, dropout=0.1, seed=9)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    bl = batches(data(), 32, n, 4, seed=17)
    monkeypatch.setenv("GTR_TAILW", "0")
    f1 = FusedTrainStep(m1, loss=loss)
    first = float(f1(bl[0].to("cuda")))
    monkeypatch.setenv("GTR_TAILW", "1")
    f2 = FusedTrainStep(m2, loss=loss)
    assert first == float(f2(bl[0].to("cuda")))
    assert not f1.tail_wgrad and f2.tail_wgrad
    for sb in bl[1:]:
        dsb = sb.to("cuda")
        assert float(f1(dsb)) == float(f2(dsb))
    for (name, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), name
    for (name, a), (_, b) in zip(m1.named_buffers(), m2.named_buffers()):
        if a is not None:
            assert torch.equal(a, b), name
    for name in ("m_tab", "v_tab", "m_flat", "v_flat"):
        assert torch.equal(getattr(f1, name), getattr(f2, name)), name
    assert int(f2.tile_cnt.abs().sum()) == 0  # every tile's counter re-armed


@pytest.mark.parametrize("mode", ["mfma", "valu"])
def test_fused_steps_wgrad_tiles_forced(mode, monkeypatch):
    """Both weight-gradient tile forms at a small batch (B = 32: VALU by default) and the
    C3 layer shape: GTR_WGRAD=mfma forces the MFMA tiles onto 32-row chunks."""
    monkeypatch.setenv("GTR_WGRAD", mode)
    _fused_vs_reference(128, 4, 16, "listwise", "adamw", True, B=32, steps=3)


def _fused_vs_reference(D, H, K, loss, opt, use_graph, B, steps, expect_ncap=0):
    T = data().table_rows
    n = 5 if loss != "listwise" else 100
    m, ref = make_pair(T, D, H, K=K, seed=4)
    m.train(); ref.train()
    lr, wd = 1e-3, 1e-2
    fused = FusedTrainStep(m, lr=lr, weight_decay=wd if opt == "adamw" else 0.0, decoupled=opt == "adamw",
                           loss=loss, temperature=1.0, alpha=0.7, use_graph=use_graph)
    if opt == "adamw":
        trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=lr, weight_decay=wd))
    else:
        trio = OracleTrio(ref, lambda ps: torch.optim.Adam(ps, lr=lr))
    bl = batches(data(), B, n, steps, seed=11)
    losses, rlosses = [], []
    for sb in bl:
        losses.append(float(fused(sb.to("cuda"))))
        rb = ref_batch(sb)
        rlosses.append(float(trio.step(lambda mod, o: R.ref_train_step(mod, rb, o, loss))))
    np.testing.assert_allclose(losses, rlosses, rtol=2e-3)
    if expect_ncap:
        assert fused.caps.n_cap > expect_ncap and fused.ws.R == 16, (fused.caps, fused.ws.R)
    # every trained parameter ELEMENTWISE (gpu_helpers.close_trained; the key bias, whose
    # gradient is exactly 0 -- softmax over a destination's in-edges is shift invariant --
    # is noise-driven on both sides and bounded by 2 lr per step instead)
    fused.flush()
    trio.compare(dict(m.named_parameters()), lr=lr)
    b64 = dict(trio.ref64.named_buffers())
    b1 = dict(trio.ref1.named_buffers())
    for name, b in ref.named_buffers():
        if "running" in name:
            close_trained(dict(m.named_buffers())[name], b, b64[name], torch.zeros_like(b, dtype=torch.bool), 0.0,
                          name, b1[name])
    assert int(dict(m.named_buffers())["batch_norms.0.num_batches_tracked"]) == len(bl)
    return fused


def test_fused_dropout_deterministic_and_finite():
    T = data().table_rows
    m, _ = make_pair(T, 64, 2, K=0, dropout=0.1, seed=5)
    m2 = copy.deepcopy(m)
    m.train(); m2.train()
    bl = batches(data(), 32, 5, 3, seed=12)
    f1 = FusedTrainStep(m, loss="bpr")
    f2 = FusedTrainStep(m2, loss="bpr", use_graph=False)
    l1 = [float(f1(sb.to("cuda"))) for sb in bl]
    l2 = [float(f2(sb.to("cuda"))) for sb in bl]
    assert all(np.isfinite(l1))
    # graph replay and eager launches draw the same dropout masks
    np.testing.assert_allclose(l1, l2, rtol=1e-5)
    assert torch.equal(m.item_embedding.weight, m2.item_embedding.weight) or torch.allclose(
        m.item_embedding.weight, m2.item_embedding.weight, rtol=1e-5, atol=1e-7)


def test_table_untouched_rows_follow_dense_adamw():
    """Rows not in the batch still decay / move with their moments (dense AdamW)."""
    T = data().table_rows
    m, ref = make_pair(T, 64, 1, K=0, seed=6)
    m.train(); ref.train()
    fused = FusedTrainStep(m, lr=1e-2, weight_decay=1e-1, loss="bpr")
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=1e-1))
    bl = batches(data(), 16, 5, 3, seed=13)
    for sb in bl:
        fused(sb.to("cuda"))
        rb = ref_batch(sb)
        trio.step(lambda mod, o: R.ref_train_step(mod, rb, o, "bpr"))
    trio.compare(dict(m.named_parameters()), lr=1e-2)  # the whole table (and the rest) elementwise
    untouched = torch.ones(T, dtype=torch.bool)
    for sb in bl:
        for t in (sb.x, sb.target_item, sb.negative_items):
            untouched[t] = False
    # rows never in a batch: pure decay + zero-gradient moment updates, elementwise
    assert_close(m.item_embedding.weight[untouched.cuda()], ref.item_embedding.weight[untouched], rtol=1e-5,
                 name="untouched rows")


@pytest.mark.parametrize("D,H,K,loss", [(64, 1, 0, "model_bpr"), (128, 4, 16, "listwise"), (32, 2, 0, "dual")])
def test_train_grads_wave_readout(D, H, K, loss, monkeypatch):
    """The large-batch readout kernel (wave per session, online listwise softmax),
    forced at B = 32: forward (RO_FWD), loss (RO_LOSS) and readout backward (RO_BWD)
    as separate launches of the autograd path."""
    monkeypatch.setenv("GTR_RO_WAVE_MIN_B", "1")
    test_train_grads(D, H, K, loss)


@pytest.mark.parametrize("D,H,K,loss", [(64, 1, 0, "bpr"), (128, 4, 16, "listwise"), (32, 2, 0, "dual")])
def test_fused_steps_wave_readout(D, H, K, loss, monkeypatch):
    """Fused steps through the wave-per-session readout (FWD|LOSS|BWD in one launch)."""
    monkeypatch.setenv("GTR_RO_WAVE_MIN_B", "1")
    _fused_vs_reference(D, H, K, loss, "adamw", True, B=64, steps=3)


def test_fused_steps_wave_readout_large_batch(monkeypatch):
    """B = 2100 at the default switch-over: > 64 row groups, radix-sort begin, wave readout
    with several sessions per wave (grid-stride), 100 listwise negatives."""
    monkeypatch.delenv("GTR_RO_WAVE_MIN_B", raising=False)
    _fused_vs_reference(64, 2, 0, "listwise", "adamw", True, B=2100, steps=2)


def _lazy_vs_eager(D, H, K, loss, opt, B, steps, dropout=0.1, use_graph=True, dp=None, cap=None, lagged=False):
    T = data().table_rows
    n = 5 if loss != "listwise" else 100
    m1, _ = make_pair(T, D, H, K=K, dropout=dropout, seed=7)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    kw = dict(lr=1e-3, weight_decay=1e-2, decoupled=opt == "adamw", loss=loss, use_graph=use_graph,
              data_parallel=dp)
    f1 = FusedTrainStep(m1, **kw)
    f2 = FusedTrainStep(m2, lazy=not lagged, lagged=lagged, **kw)
    if cap is not None:
        f2._lazy_alloc(cap)
    for sb in batches(data(), B, n, steps, seed=13):
        l1 = float(f1(sb.to("cuda")))
        l2 = float(f2(sb.to("cuda")))
        assert l1 == l2
    sd1, sd2 = m1.state_dict(), m2.state_dict()  # state_dict() flushes the lazy table
    for k in sd1:
        assert torch.equal(sd1[k], sd2[k]), k
    assert torch.equal(f1.m_tab, f2.m_tab) and torch.equal(f1.v_tab, f2.v_tab)
    assert torch.equal(f1.m_flat, f2.m_flat) and torch.equal(f1.v_flat, f2.v_flat)
    return f2


@pytest.mark.parametrize("D,H,K,loss,opt", [(64, 1, 0, "bpr", "adamw"), (128, 4, 16, "listwise", "adam"),
                                            (32, 2, 0, "dual", "adamw")])
def test_lazy_table_bitwise_equals_dense_adamw(D, H, K, loss, opt):
    """Deferred zero-gradient AdamW (gtr_step_begin_lazy / gtr_lazy_flush): after k steps
    the table, its moments and every parameter equal the eager dense update bit for bit
    (dropout on: both use the same device streams)."""
    _lazy_vs_eager(D, H, K, loss, opt, B=32, steps=5)


def test_lazy_table_large_batch_and_capacity_growth():
    """Radix-sort begin path (B = 1400) + consts table growth (capacity 4 -> 8 -> 16)."""
    _lazy_vs_eager(64, 2, 0, "bpr", "adamw", B=1400, steps=2)
    _lazy_vs_eager(64, 1, 0, "bpr", "adamw", B=32, steps=10, cap=4)


def test_lazy_table_data_parallel_world1():
    """Data-parallel tail in lazy mode (catch-up of union rows in gtr_dp_tail)."""
    _lazy_vs_eager(64, 2, 0, "bpr", "adamw", B=32, steps=4, dp=True)


@pytest.mark.parametrize("dp", [False, True])
def test_lagged_sweep_bitwise_equals_dense_adamw(dp):
    """Lagged sweep (gtr_sweep.lag): the chain's launches bring the previous step's
    untouched rows forward; single GPU and the data-parallel step (world 1), 12 steps so
    rows go untouched, get read again and get touched again."""
    f2 = _lazy_vs_eager(64, 1, 0, "bpr", "adamw", B=32, steps=12, dp=dp, lagged=True)
    assert f2.sweep is not None and f2.sweep.lag == 1
    # after the flush every row is current through the last step
    assert int(f2.stamp.min()) == f2.steps


def test_lagged_sweep_consts_growth_and_listwise():
    """Lagged mode with the consts table growing under it (capacity 4), D = 128 / 4 heads /
    LapPE / listwise, and a large batch where the chain carries no sweep (g_cap > 128:
    rows then fall further behind and are caught up on read)."""
    _lazy_vs_eager(64, 1, 0, "bpr", "adamw", B=32, steps=10, cap=4, lagged=True)
    _lazy_vs_eager(128, 4, 16, "listwise", "adam", B=32, steps=4, lagged=True)
    _lazy_vs_eager(64, 2, 0, "bpr", "adamw", B=1400, steps=3, lagged=True)


def test_lazy_table_flushes_before_eval_forward():
    """model(batch) in eval mode after lazy steps sees the up-to-date table (forward hook)."""
    f2 = _lazy_vs_eager(64, 1, 0, "bpr", "adamw", B=32, steps=3)
    m2 = f2.model
    sb = batches(data(), 32, 5, 1, seed=99)[0]
    f2(sb.to("cuda"))  # dirty again
    assert f2._dirty
    m2.eval()
    with torch.no_grad():
        m2(sb.to("cuda"))
    assert not f2._dirty


@pytest.mark.parametrize("lazy", [False, True])
def test_resident_images_equal_copied_blob(lazy):
    """bind_resident / run_resident (one captured graph per resident batch image, no copy
    into the step's blob; bench.py's one-GPU default) trains bit for bit like load + run,
    images reused included, with the eager sweep and with the lazy table."""
    from etpgt.data.batch import Caps

    T = data().table_rows
    m1, _ = make_pair(T, 64, 2, K=0, dropout=0.1, seed=8)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    bl = batches(data(), 32, 5, 3, seed=14)
    caps = Caps(max(b.num_nodes for b in bl), 32, max(b.num_edges for b in bl), 5)
    f1 = FusedTrainStep(m1, loss="bpr", caps=caps, lazy=lazy)
    f2 = FusedTrainStep(m2, loss="bpr", caps=caps, lazy=lazy)
    staged = [torch.from_numpy(b.packed(f2.caps)[1]).cuda() for b in bl]
    f2.bind_resident(staged)
    order = [0, 1, 2, 1, 0, 2]
    for i in order[:2]:
        assert float(f1(bl[i].to("cuda"))) == float(f2.run_resident(i))
    f2.prepare_resident()
    for i in order[2:]:
        assert float(f1(bl[i].to("cuda"))) == float(f2.run_resident(i))
    if lazy:
        f1.flush()
        f2.flush()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(a, b)


@pytest.mark.parametrize("lazy", [False, True])
def test_multi_step_graph_equals_per_step_graphs(lazy):
    """capture_steps / run_steps (bench.py's timed loop: K steps as ONE hipGraph over the
    resident images) trains bit for bit like K run_resident calls (one graph launch per
    step): losses of every replay, parameters, AdamW moments, with the eager sweep and
    the lazy table; a replay after a reallocation of the lazy constants is refused."""
    from etpgt.data.batch import Caps

    T = data().table_rows
    m1, _ = make_pair(T, 64, 2, K=0, dropout=0.1, seed=9)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    bl = batches(data(), 32, 5, 3, seed=15)
    caps = Caps(max(b.num_nodes for b in bl), 32, max(b.num_edges for b in bl), 5)
    f1 = FusedTrainStep(m1, loss="bpr", caps=caps, lazy=lazy)
    f2 = FusedTrainStep(m2, loss="bpr", caps=caps, lazy=lazy)
    st1 = [torch.from_numpy(b.packed(f1.caps)[1]).cuda() for b in bl]
    st2 = [torch.from_numpy(b.packed(f2.caps)[1]).cuda() for b in bl]
    f1.bind_resident(st1)
    f2.bind_resident(st2)
    for i in range(2):
        assert float(f1.run_resident(i)) == float(f2.run_resident(i))
    f1.prepare_resident()
    f2.prepare_resident()
    h = f2.capture_steps(2, 4)  # images 2, 0, 1, 2
    for rep in range(3):
        for k in range(4):
            l1 = float(f1.run_resident((2 + k) % 3))
        assert l1 == float(f2.run_steps(h)), rep
    assert f1.steps == f2.steps == 14
    f1.flush()
    f2.flush()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    assert torch.equal(f1.m_tab, f2.m_tab) and torch.equal(f1.v_tab, f2.v_tab)
    if lazy:
        f2._lazy_alloc(2 * f2.lz.cap)
        with pytest.raises(RuntimeError, match="capture the steps again"):
            f2.run_steps(h)
    # any rebind (here: the resident images) makes the handle stale; the refused
    # replay changes no host state
    h = f2.capture_steps(0, 2)
    steps_before = f2._host_steps
    f2.bind_resident(st2)
    with pytest.raises(RuntimeError, match="capture the steps again"):
        f2.run_steps(h)
    assert f2._host_steps == steps_before


@pytest.mark.parametrize("gemm,D,H,K,loss", [("split", 64, 1, 0, "model_bpr"), ("split", 128, 4, 16, "listwise"),
                                             ("split", 32, 2, 0, "dual"), ("f32", 128, 4, 16, "listwise")])
def test_train_grads_gemm_modes(gemm, D, H, K, loss, monkeypatch):
    """The layer GEMMs in the opt-in split-bf16 mode (GTR_GEMM=split) and forced exact f32:
    single-step gradients against the oracle at 2e-3."""
    monkeypatch.setenv("GTR_GEMM", gemm)
    test_train_grads(D, H, K, loss)


@pytest.mark.parametrize("rg", ["8", "16"])
def test_row_group_widths_match_oracle(rg, monkeypatch):
    """Both row-group widths the step picks (8 rows for <= 32 groups, 16 above) on the same
    C2- and C3-shaped batches: per-step losses and trained parameters against the oracle."""
    monkeypatch.setenv("GTR_ROW_GROUP", rg)
    _fused_vs_reference(64, 1, 0, "bpr", "adamw", True, B=32, steps=3)
    _fused_vs_reference(128, 4, 16, "listwise", "adamw", True, B=32, steps=3)


@pytest.mark.parametrize("B", [32, 700])
def test_dropin_default_config_fused_steps(B):
    """The drop-in's default model: ``train_baseline.py --model graph_transformer_optimized``
    at its default flags builds create_graph_transformer_optimized with d = 256, 3 layers,
    4 heads and LapPE k = 16 (train_baseline.py:39-42,220-232), trained by the Trainer's
    default BPR loss with 5 negatives.  Five fused steps against the oracle trainer, every
    trained parameter ELEMENTWISE (gpu_helpers.close_trained), at B = 32 and at B = 700
    (> 128 row groups at d = 256)."""
    from gpu_helpers import OracleTrio

    T = data().table_rows
    m, ref = make_pair(T, 256, 4, L=3, K=16, seed=41)
    m.train(); ref.train()
    fused = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, loss="bpr")
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-3, weight_decay=1e-5))
    for i, sb in enumerate(batches(data(), B, 5, 5, seed=43)):
        hl = float(fused(sb.to("cuda")))
        rb = ref_batch(sb)
        rl = trio.step(lambda mod, o: R.ref_train_step(mod, rb, o, "bpr"))
        assert abs(hl - float(rl)) <= 1e-3 * max(1.0, abs(float(rl))), (i, hl, float(rl))
    if B == 700:
        assert fused.ws.g_cap > 128, fused.ws.g_cap
    trio.compare(dict(m.named_parameters()), lr=1e-3)
    bufs = dict(m.named_buffers())
    from gpu_helpers import close_trained

    b64, b1 = dict(trio.ref64.named_buffers()), dict(trio.ref1.named_buffers())
    for name, b in ref.named_buffers():
        if "running" in name:
            close_trained(bufs[name], b, b64[name], torch.zeros_like(b, dtype=torch.bool), 0.0, name, b1[name])
