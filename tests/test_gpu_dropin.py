"""GPU: the train_baseline.py drop-in end to end.

The counterpart script (scripts/train/train_baseline.py, the reference's flags) trains
one epoch on tiny reference-format CSVs with batches built on the GPU inside the
captured step; the oracle trainer replays the same epoch -- the same initial weights
(set_seed(42) + the factory), the same session order (the DataLoader iterator's
_base_seed and RandomSampler draws), the same per-session examples and negatives
(oracle/batch_ref.py restates the device stream) -- and the epoch loss, every trained
parameter ELEMENTWISE (gpu_helpers.close_trained) and the validation Recall@10 must
agree."""

from __future__ import annotations

import importlib.util
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

import batch_ref as BR  # noqa: E402
import etpgt_ref as R  # noqa: E402
from dropin_helpers import write_csvs  # noqa: E402
from gpu_helpers import OracleTrio, close_trained  # noqa: E402

from etpgt.data.batch import collate_sessions  # noqa: E402
from etpgt.model import create_graph_transformer_optimized  # noqa: E402
from etpgt.train.dataloader import SessionDataset  # noqa: E402
from etpgt.utils.metrics import compute_recall_at_k  # noqa: E402
from etpgt.utils.seed import set_seed  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script():
    spec = importlib.util.spec_from_file_location("train_baseline_cp",
                                                  os.path.join(ROOT, "scripts", "train", "train_baseline.py"))
    tb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tb)
    return tb


@pytest.mark.parametrize("D,H,L,B", [(32, 2, 2, 16), (256, 4, 3, 32)])
def test_train_baseline_counterpart_one_epoch_matches_oracle(tmp_path, D, H, L, B):
    """(256, 4, 3, 32): the reference script's own defaults -- embedding / hidden 256, 3
    layers, 4 heads, batch 32, 5 negatives (train_baseline.py:39-42,63-64) -- with
    dropout 0 so that the oracle can replay the epoch."""
    d = write_csvs(tmp_path)
    n = 5
    args = ["--model", "graph_transformer_optimized", "--train-sessions", str(d / "train.csv"),
            "--val-sessions", str(d / "val.csv"), "--graph-edges", str(d / "graph_edges.csv"),
            "--embedding-dim", str(D), "--hidden-dim", str(D), "--num-layers", str(L), "--num-heads", str(H),
            "--dropout", "0", "--batch-size", str(B), "--num-negatives", str(n), "--max-epochs", "1",
            "--num-workers", "0", "--output-dir", str(tmp_path / "out")]
    trainer = _script().main(args)
    from etpgt.train.dataloader import DeviceSessionLoader

    assert isinstance(trainer.train_loader, DeviceSessionLoader)
    assert trainer._fused is not None and trainer._fused.builder is trainer.train_loader.builder
    with open(tmp_path / "out" / "graph_transformer_optimized" / "history.json") as f:
        hist = json.load(f)
    ck = torch.load(tmp_path / "out" / "graph_transformer_optimized" / "checkpoint_latest.pt", map_location="cpu",
                    weights_only=True)
    sd = ck["model_state_dict"]

    # ---- the oracle replays the epoch
    tr = SessionDataset(d / "train.csv", d / "graph_edges.csv", n, 50)
    va = SessionDataset(d / "val.csv", d / "graph_edges.csv", n, 50)
    T = max(tr.num_items, va.num_items)
    set_seed(42)
    init = create_graph_transformer_optimized(T, embedding_dim=D, hidden_dim=D, num_layers=L, num_heads=H,
                                              dropout=0.0, use_laplacian_pe=True, use_ffn=False, ffn_expansion=2)
    torch.empty((), dtype=torch.int64).random_()  # the epoch iterator's _base_seed draw
    seed = int(torch.empty((), dtype=torch.int64).random_().item())  # the epoch's RandomSampler draw
    g = torch.Generator()
    g.manual_seed(seed)
    order = torch.randperm(len(tr), generator=g).numpy()
    ref = R.ref_create_graph_transformer_optimized(T, embedding_dim=D, hidden_dim=D, num_layers=L, num_heads=H,
                                                   dropout=0.0, use_laplacian_pe=True)
    isd = {k: v.clone() for k, v in init.state_dict().items()}
    isd["laplacian_pe._cached_pe"] = sd["laplacian_pe._cached_pe"].clone()  # eigsh result of the run
    ref.laplacian_pe._cached_pe = isd["laplacian_pe._cached_pe"]
    ref.load_state_dict(isd)
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-3, weight_decay=1e-5))
    ei = tr.edge_index.numpy()
    keys = np.unique(ei[0].astype(np.int64) * tr.num_items + ei[1].astype(np.int64))
    S = len(tr)
    losses = []
    for i in range(-(-S // B)):
        b = min(B, S - i * B)
        ex = BR.build_batch(tr._ptr, tr._items, keys, tr.num_items, order, i * B, b, 50, n, 42)
        rb = R.ref_batch_from(collate_sessions(ex))
        losses.append(float(trio.step(lambda mod, o: R.ref_train_step(mod, rb, o, "bpr"))))
    want = float(np.mean(losses))
    assert abs(hist["train_loss"][0] - want) <= 1e-3 * abs(want), (hist["train_loss"][0], want)
    # every trained parameter ELEMENTWISE (gpu_helpers.close_trained: 1e-3 relative, or within
    # the fp32 oracle's own distance to fp64 where a gradient nearly cancels)
    trio.compare({k: sd[k] for k, _ in ref.named_parameters()}, lr=1e-3)
    for k, b in ref.named_buffers():
        if "num_batches_tracked" in k:
            assert int(sd[k]) == int(b)
        elif "running" in k:
            b64 = dict(trio.ref64.named_buffers())[k]
            close_trained(sd[k], b, b64, torch.zeros_like(b, dtype=torch.bool), 0.0, k,
                          dict(trio.ref1.named_buffers())[k])
    # validation Recall@10 of the trained model (shuffle=False order, eval mode)
    ref.eval()
    vkeys = np.unique(va.edge_index.numpy()[0].astype(np.int64) * va.num_items + va.edge_index.numpy()[1])
    preds, tg = [], []
    Sv = len(va)
    with torch.no_grad():
        for i in range(-(-Sv // B)):
            b = min(B, Sv - i * B)
            ex = BR.build_batch(va._ptr, va._items, vkeys, va.num_items, np.arange(Sv), i * B, b, 50, n, 42)
            rb = R.ref_batch_from(collate_sessions(ex))
            preds.append(ref.predict(ref(rb), k=20))
            tg.append(rb.target_item)
    r10 = compute_recall_at_k(torch.cat(preds)[:, :10], torch.cat(tg), k=10)
    got = hist["val_metrics"][0]["recall@10"]
    assert abs(got - r10) <= 1.0 / Sv + 1e-9, (got, r10)


def test_train_baseline_reference_default_flags_one_epoch(tmp_path):
    """``train_baseline.py --model graph_transformer_optimized`` with NO model / training
    flags: the reference defaults (d = 256, 3 layers, 4 heads, dropout 0.1, batch 32, 5
    negatives, AdamW 1e-3 / 1e-5).  One epoch through the fused step: finite loss, the
    validation metrics, a checkpoint with the reference's state-dict keys."""
    d = write_csvs(tmp_path)
    args = ["--model", "graph_transformer_optimized", "--train-sessions", str(d / "train.csv"),
            "--val-sessions", str(d / "val.csv"), "--graph-edges", str(d / "graph_edges.csv"), "--max-epochs", "1",
            "--num-workers", "0", "--output-dir", str(tmp_path / "out")]
    trainer = _script().main(args)
    m = trainer.model
    assert trainer._fused is not None
    assert m.item_embedding.weight.shape[1] == 256 and m.num_layers == 3 and m.num_heads == 4
    with open(tmp_path / "out" / "graph_transformer_optimized" / "history.json") as f:
        hist = json.load(f)
    assert len(hist["train_loss"]) == 1 and np.isfinite(hist["train_loss"][0])
    assert 0.0 <= hist["val_metrics"][0]["recall@10"] <= 1.0
    ck = torch.load(tmp_path / "out" / "graph_transformer_optimized" / "checkpoint_latest.pt", map_location="cpu",
                    weights_only=True)
    sd = ck["model_state_dict"]
    for k in ("item_embedding.weight", "laplacian_pe.projection.weight", "convs.2.lin_query.weight",
              "convs.2.lin_beta.weight", "batch_norms.2.running_var"):
        assert k in sd, k


def test_train_baseline_ffn_model_trains_one_epoch(tmp_path):
    """``--model graph_transformer`` (the FFN variant, create_graph_transformer defaults
    apart from the dimensions) trains through the Trainer's fused step on the HIP split
    layer + FFN kernels: one epoch, finite loss, a checkpoint with the reference keys."""
    d = write_csvs(tmp_path)
    args = ["--model", "graph_transformer", "--train-sessions", str(d / "train.csv"),
            "--val-sessions", str(d / "val.csv"), "--graph-edges", str(d / "graph_edges.csv"),
            "--embedding-dim", "64", "--hidden-dim", "64", "--num-layers", "2", "--num-heads", "2",
            "--batch-size", "16", "--num-negatives", "5", "--max-epochs", "1",
            "--num-workers", "0", "--output-dir", str(tmp_path / "out")]
    trainer = _script().main(args)
    assert trainer._fused is not None and trainer.model.use_ffn
    with open(tmp_path / "out" / "graph_transformer" / "history.json") as f:
        hist = json.load(f)
    assert len(hist["train_loss"]) == 1 and np.isfinite(hist["train_loss"][0])
    ck = torch.load(tmp_path / "out" / "graph_transformer" / "checkpoint_latest.pt", map_location="cpu",
                    weights_only=True)
    assert "ffns.1.3.weight" in ck["model_state_dict"]


def test_train_baseline_graph_transformer_reference_default_flags(tmp_path):
    """``train_baseline.py --model graph_transformer`` with NO model flags: the reference
    defaults build create_graph_transformer with d = 256, 3 layers, 4 heads, FFN x 4 and
    LapPE (train_baseline.py:39-42,198-208; graph_transformer.py:185-197).  One epoch
    through the Trainer's fused step on the LDS-staged d = 256 GEMMs."""
    d = write_csvs(tmp_path)
    args = ["--model", "graph_transformer", "--train-sessions", str(d / "train.csv"),
            "--val-sessions", str(d / "val.csv"), "--graph-edges", str(d / "graph_edges.csv"), "--max-epochs", "1",
            "--num-workers", "0", "--output-dir", str(tmp_path / "out")]
    trainer = _script().main(args)
    m = trainer.model
    assert trainer._fused is not None and m.use_ffn and m.ffn_expansion == 4
    assert m.item_embedding.weight.shape[1] == 256 and m.num_layers == 3 and m.num_heads == 4
    with open(tmp_path / "out" / "graph_transformer" / "history.json") as f:
        hist = json.load(f)
    assert len(hist["train_loss"]) == 1 and np.isfinite(hist["train_loss"][0])
    ck = torch.load(tmp_path / "out" / "graph_transformer" / "checkpoint_latest.pt", map_location="cpu",
                    weights_only=True)
    assert ck["model_state_dict"]["ffns.2.0.weight"].shape == (1024, 256)
