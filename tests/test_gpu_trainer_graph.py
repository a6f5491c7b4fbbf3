"""GPU: the drop-in Trainer's device-built epochs as multi-step hipGraphs.

``Trainer._train_epoch_device_batches`` runs an epoch's full batches in chunks of
``steps_per_graph`` consecutive steps captured as ONE hipGraph
(``FusedTrainStep.capture_steps_built``), the leftover full batches one step graph each
and the partial last batch eagerly; the epoch loss is the tail's device-side running sum
(``gtr_tail.loss_acc``).  Every step is still the full step of ``run()``, so two epochs
with chunks must equal two epochs with one graph per batch BIT FOR BIT: epoch losses,
every parameter, the AdamW moments and the BatchNorm running statistics -- with dropout
on (the masks come from the device counter the tail advances).  The second epoch checks
that the chunk graph, captured in epoch 1, reads epoch 2's order (the builder rewrites its
order buffer in place) -- reference trainer.py:80-133 driven by
scripts/train/train_baseline.py:260-274."""

from __future__ import annotations

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

from dropin_helpers import write_csvs  # noqa: E402

from etpgt.model import create_graph_transformer_optimized  # noqa: E402
from etpgt.train.dataloader import DeviceSessionLoader, SessionDataset  # noqa: E402
from etpgt.train.trainer import Trainer  # noqa: E402


def _trainer(model, loader, tmp_path, tag, steps_per_graph, loss_fn=None):
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-5)
    tr = Trainer(model, loader, None, opt, device="cuda", output_dir=tmp_path / tag, max_epochs=2,
                 loss_fn=loss_fn)
    tr.steps_per_graph = steps_per_graph
    return tr


@pytest.mark.parametrize("D,H,K,loss", [(64, 1, 0, None), (128, 4, 16, "listwise")])
def test_trainer_epoch_chunk_graphs_bitwise_equal_per_step_graphs(tmp_path, D, H, K, loss):
    from etpgt.train.losses import create_loss_function

    d = write_csvs(tmp_path)
    ds = SessionDataset(d / "train.csv", d / "graph_edges.csv", 5, 50)
    T = ds.num_items
    torch.manual_seed(3)
    m1 = create_graph_transformer_optimized(T, embedding_dim=D, hidden_dim=D, num_layers=2, num_heads=H,
                                            dropout=0.1, use_laplacian_pe=K > 0, laplacian_k=max(K, 1))
    if K > 0:
        torch.manual_seed(4)
        m1.laplacian_pe._cached_pe = torch.rand(T, K)
    m2 = copy.deepcopy(m1)
    lf = None if loss is None else create_loss_function(loss)
    B = 8  # 150 sessions: 18 full batches + a partial one of 6
    l1 = DeviceSessionLoader(ds, B, 5, shuffle=True, seed=11)
    l2 = DeviceSessionLoader(ds, B, 5, shuffle=True, seed=11)
    t1 = _trainer(m1, l1, tmp_path, "a", 1, lf)
    t2 = _trainer(m2, l2, tmp_path, "b", 4, lf)
    losses1, losses2 = [], []
    for ep in range(2):
        g = torch.random.get_rng_state()
        losses1.append(t1.train_epoch())
        torch.random.set_rng_state(g)  # both loaders draw the same epoch order
        losses2.append(t2.train_epoch())
    assert t2._chunk_graph is not None and t2._chunk_graph["n"] == 4  # the chunks ran
    assert t1._chunk_graph is None
    assert losses1 == losses2, (losses1, losses2)
    f1, f2 = t1._fused, t2._fused
    assert f1.steps == f2.steps == 2 * 19
    f1.flush()
    f2.flush()
    for (n, a), (_, b) in zip(m1.named_parameters(), m2.named_parameters()):
        assert torch.equal(a, b), n
    for (n, a), (_, b) in zip(m1.named_buffers(), m2.named_buffers()):
        assert torch.equal(a, b), n
    assert torch.equal(f1.m_tab, f2.m_tab) and torch.equal(f1.v_tab, f2.v_tab)
    assert torch.equal(f1.m_flat, f2.m_flat) and torch.equal(f1.v_flat, f2.v_flat)


def test_trainer_epoch_loss_is_the_mean_of_the_step_losses(tmp_path):
    """The device running sum divided by the batch count equals the mean of the per-step
    losses read one by one (the reference's ``loss.item()`` per step, trainer.py:130)."""
    d = write_csvs(tmp_path)
    ds = SessionDataset(d / "train.csv", d / "graph_edges.csv", 5, 50)
    T = ds.num_items
    torch.manual_seed(5)
    m1 = create_graph_transformer_optimized(T, embedding_dim=64, hidden_dim=64, num_layers=2, num_heads=1,
                                            dropout=0.0, use_laplacian_pe=False)
    m2 = copy.deepcopy(m1)
    l1 = DeviceSessionLoader(ds, 16, 5, shuffle=False, seed=2)
    t1 = _trainer(m1, l1, tmp_path, "a", 4)
    got = t1.train_epoch()
    # the same epoch step by step, reading each step's loss
    l2 = DeviceSessionLoader(ds, 16, 5, shuffle=False, seed=2)
    t2 = _trainer(m2, l2, tmp_path, "b", 1)
    f = t2._fused_step()
    l2.start_epoch()
    sizes = l2.batch_sizes()
    f.attach_builder(l2.builder, num_batches=sum(1 for b in sizes if b == 16),
                     extra=[(l2.batch_start(i), b) for i, b in enumerate(sizes) if b != 16])
    per = []
    for i, b in enumerate(sizes):
        l2.builder.seek(l2.batch_start(i))
        per.append(float(f.run_partial(b) if b != 16 else f.run()))
    want = sum(per) / len(per)
    assert abs(got - want) <= 1e-6 * abs(want), (got, want)
