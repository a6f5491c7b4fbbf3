#!/usr/bin/env python3 -B
"""Generate the golden fixtures under tests/golden/ — TEST INFRASTRUCTURE ONLY.

Runs in the build container only (``/root/reference`` does not exist on the GPU
box).  It imports the reference's own pure-torch files BY FILE PATH, with
bytecode writing disabled so nothing lands in the read-only tree:

* ``etpgt/model/base.py``   -> SessionReadout (all modes), BaseRecommendationModel.compute_loss
* ``etpgt/train/losses.py`` -> BPR / Listwise / Dual / SampledSoftmax
* ``etpgt/utils/metrics.py``-> compute_recall_at_k / compute_ndcg_at_k
* ``etpgt/train/trainer.py``-> Trainer.train_epoch / Trainer.evaluate (the step loop)
* ``scripts/data/00_generate_synthetic_data.py``, ``02_sessionize.py``,
  ``04_build_graph.py`` -> config C1's events, sessions and co-event graph

PyG (``torch_geometric``) is not installed here, so the model's TransformerConv
arithmetic inside the trainer fixture is the oracle restatement
(``oracle/etpgt_ref.py``); the fixture pins the trainer loop, AdamW and losses
around it.  Outputs are small ``.npz`` files of inputs and expected outputs.

Usage:  python -B oracle/gen_golden.py [--ref /root/reference] [--out tests/golden]
"""

from __future__ import annotations

import argparse
import importlib.util
import os
import sys
import tempfile

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import etpgt_ref as R  # noqa: E402


def load_by_path(name: str, path: str):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def t2n(t):
    return t.detach().cpu().numpy().copy()


def gen_readout(ref_base, out):
    torch.manual_seed(1)
    N, d = 11, 8
    x = torch.randn(N, d)
    batch = torch.tensor([0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2])
    res = {"x": t2n(x), "batch": t2n(batch)}
    for mode in ("mean", "max", "last", "attention"):
        torch.manual_seed(2)
        ro = ref_base.SessionReadout(hidden_dim=d, readout_type=mode)
        xi = x.clone().requires_grad_(True)
        se = ro(xi, batch)
        w = torch.linspace(-1, 1, se.numel()).view_as(se)
        (se * w).sum().backward()
        res[f"{mode}_se"] = t2n(se)
        res[f"{mode}_dx"] = t2n(xi.grad)
        if mode == "attention":
            res["attention_w"] = t2n(ro.attention.weight)
            res["attention_b"] = t2n(ro.attention.bias)
    np.savez(os.path.join(out, "readout.npz"), **res)


def gen_losses(ref_base, ref_losses, out):
    torch.manual_seed(3)
    B, n, T, d = 4, 5, 20, 8
    se0 = torch.randn(B, d)
    W0 = torch.randn(T, d) * 0.5
    W0[0] = 0
    tgt = torch.randint(1, T, (B,))
    neg = torch.randint(1, T, (B, n))
    res = {"se": t2n(se0), "W": t2n(W0), "target": t2n(tgt), "neg": t2n(neg)}
    cases = {
        "bpr": ref_losses.BPRLoss(),
        "listwise_t0.5": ref_losses.ListwiseLoss(temperature=0.5),
        "listwise_t1": ref_losses.ListwiseLoss(temperature=1.0),
        "listwise_t2": ref_losses.ListwiseLoss(temperature=2.0),
        "dual_a0.7": ref_losses.DualLoss(alpha=0.7, temperature=1.0),
        "sampled_softmax": ref_losses.SampledSoftmaxLoss(temperature=1.0),
    }
    for name, fn in cases.items():
        se = se0.clone().requires_grad_(True)
        emb = torch.nn.Embedding(T, d, padding_idx=0)
        with torch.no_grad():
            emb.weight.copy_(W0)
        outv = fn(se, tgt, neg, emb)
        loss = outv[0] if isinstance(outv, tuple) else outv
        loss.backward()
        res[f"{name}_loss"] = np.array(loss.item(), dtype=np.float64)
        res[f"{name}_dse"] = t2n(se.grad)
        res[f"{name}_dW"] = t2n(emb.weight.grad)

    # BaseRecommendationModel.compute_loss (base.py:80-113) via a minimal concrete subclass
    class _M(ref_base.BaseRecommendationModel):
        def forward(self, batch):  # pragma: no cover - abstract filler
            return None

    torch.manual_seed(4)
    m = _M(num_items=T, embedding_dim=d, hidden_dim=d)
    with torch.no_grad():
        m.item_embedding.weight.copy_(W0)
    se = se0.clone().requires_grad_(True)
    loss = m.compute_loss(se, tgt, neg)
    loss.backward()
    res["model_bpr_loss"] = np.array(loss.item(), dtype=np.float64)
    res["model_bpr_dse"] = t2n(se.grad)
    res["model_bpr_dW"] = t2n(m.item_embedding.weight.grad)

    # table init statistics (base.py:35-37): row 0 zero, xavier bound on rows 1..
    torch.manual_seed(5)
    m2 = _M(num_items=1000, embedding_dim=32, hidden_dim=32)
    Wi = m2.item_embedding.weight.detach()
    res["init_row0_absmax"] = np.array(float(Wi[0].abs().max()))
    res["init_absmax"] = np.array(float(Wi[1:].abs().max()))
    res["init_bound"] = np.array(float(np.sqrt(6.0 / (999 + 32))))
    np.savez(os.path.join(out, "losses.npz"), **res)


def gen_metrics(ref_metrics, out):
    g = torch.Generator().manual_seed(6)
    B, K, T = 64, 20, 50
    preds = torch.stack([torch.randperm(T, generator=g)[:K] for _ in range(B)])
    tgts = torch.randint(0, T, (B,), generator=g)
    res = {"preds": t2n(preds), "targets": t2n(tgts)}
    for k in (1, 5, 10, 20):
        res[f"recall@{k}"] = np.array(ref_metrics.compute_recall_at_k(preds, tgts, k))
        res[f"ndcg@{k}"] = np.array(ref_metrics.compute_ndcg_at_k(preds, tgts, k))
    np.savez(os.path.join(out, "metrics.npz"), **res)


def _tiny_sessions(seed, n_sessions, T, max_len=6):
    """A tiny deterministic session set + batch list in the training layout."""
    rng = np.random.default_rng(seed)
    sess = []
    for _ in range(n_sessions):
        L = int(rng.integers(3, max_len + 1))
        items = rng.integers(1, T, size=L)
        sess.append(items)
    return sess


def _collate(sessions, T, n_neg, rng):
    """dataloader.py:64-202 semantics on in-memory sessions: context = all but last,
    nodes = sorted unique context ids, edges = canonical (i<=j) pairs that co-occur
    within a +-5 window in the session (the 04_build_graph rule), directed small->large,
    self loops kept; negatives uniform in [1,T) excluding the session's items."""
    xs, srcs, dsts, bvec, tg, ng = [], [], [], [], [], []
    off = 0
    for b, items in enumerate(sessions):
        ctx = items[:-1]
        uniq = np.unique(ctx)
        loc = {int(v): i for i, v in enumerate(uniq)}
        pairs = set()
        for i in range(len(ctx)):
            for j in range(i + 1, min(i + 6, len(ctx))):
                a, c = int(ctx[i]), int(ctx[j])
                pairs.add((min(a, c), max(a, c)))
        for a, c in sorted(pairs):
            srcs.append(loc[a] + off)
            dsts.append(loc[c] + off)
        xs.extend(int(v) for v in uniq)
        bvec.extend([b] * len(uniq))
        off += len(uniq)
        tg.append(int(items[-1]))
        s = set(int(v) for v in items)
        negs = []
        while len(negs) < n_neg:
            v = int(rng.integers(1, T))
            if v not in s:
                negs.append(v)
        ng.extend(negs)
    return dict(
        x=np.array(xs, np.int64), edge_index=np.array([srcs, dsts], np.int64).reshape(2, -1),
        batch=np.array(bvec, np.int64), target_item=np.array(tg, np.int64),
        negative_items=np.array(ng, np.int64),
    )


def gen_trainer(ref_trainer, ref_losses, out):
    """Drive the REFERENCE Trainer (trainer.py:80-173) over oracle-restated models."""
    T, d, H, L, n = 40, 16, 2, 2, 5
    rng = np.random.default_rng(7)
    sessions = _tiny_sessions(8, 12, T)
    batches_np = [_collate(sessions[i : i + 4], T, n, rng) for i in range(0, 12, 4)]
    res = {}
    for bi, bn in enumerate(batches_np):
        for k, v in bn.items():
            res[f"b{bi}_{k}"] = v

    def mk_batches():
        return [
            R.RefBatch(*(torch.from_numpy(bn[k]) for k in ("x", "edge_index", "batch", "target_item", "negative_items")))
            for bn in batches_np
        ]

    for tag, loss_fn, kw in (
        ("bpr", None, dict(use_laplacian_pe=False)),
        ("listwise", ref_losses.ListwiseLoss(temperature=1.0), dict(use_laplacian_pe=True, laplacian_k=4)),
        ("dual", ref_losses.DualLoss(alpha=0.7), dict(use_laplacian_pe=False)),
    ):
        torch.manual_seed(9)
        model = R.ref_create_graph_transformer_optimized(
            T, embedding_dim=d, hidden_dim=d, num_layers=L, num_heads=H, dropout=0.0, **kw
        )
        if kw.get("use_laplacian_pe"):
            g = torch.Generator().manual_seed(10)
            model.laplacian_pe._cached_pe = torch.rand(T, kw["laplacian_k"], generator=g)
        init = {k: t2n(v) for k, v in model.state_dict().items()}
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=1e-5)
        with tempfile.TemporaryDirectory() as td:
            tr = ref_trainer.Trainer(
                model, mk_batches(), mk_batches(), opt, device="cpu", output_dir=td,
                max_epochs=1, loss_fn=loss_fn,
            )
            avg = tr.train_epoch()
            metrics = tr.evaluate()
        res[f"{tag}_avg_loss"] = np.array(avg)
        for k, v in init.items():
            res[f"{tag}_init.{k}"] = v
        for k, v in model.state_dict().items():
            res[f"{tag}_final.{k}"] = t2n(v)
        for k, v in metrics.items():
            res[f"{tag}_metric.{k}"] = np.array(v)
    np.savez(os.path.join(out, "trainer.npz"), **res)


def gen_c1(ref_root, out):
    """BASELINE.json configs[0] inputs from the reference's own data scripts, imported by
    path: scripts/data/00_generate_synthetic_data.py (seed 42, 100 sessions, 1k items),
    02_sessionize.py (30-minute gap, >= 3 events) and 04_build_graph.py (+-5 window).
    The temporal split (03) is skipped: it keeps ~70 of the 100 sessions, while C1 names
    100 (run_full_pipeline.py's 100-session subset of them is all of them).  Events,
    sessions and graph edges go to tests/golden/c1_data.npz (strings as category codes)."""
    gen = load_by_path("ref_gen00", os.path.join(ref_root, "scripts/data/00_generate_synthetic_data.py"))
    ses = load_by_path("ref_ses02", os.path.join(ref_root, "scripts/data/02_sessionize.py"))
    grf = load_by_path("ref_grf04", os.path.join(ref_root, "scripts/data/04_build_graph.py"))
    ev = gen.generate_synthetic_events(num_sessions=100, num_items=1000, seed=42)
    sd = ses.sessionize_events(ev)
    edges, _ = grf.build_co_event_graph(sd)
    code = {"view": 0, "addtocart": 1, "transaction": 2}
    res = {
        "ev_timestamp": ev["timestamp"].to_numpy(np.int64),
        "ev_visitor": ev["visitorid"].str.replace("visitor_", "").astype(np.int64).to_numpy(),
        "ev_event": ev["event"].map(code).to_numpy(np.int64),
        "ev_itemid": ev["itemid"].to_numpy(np.int64),
        "ev_txn": ev["transactionid"].notna().to_numpy(),
        "sd_timestamp": sd["timestamp"].to_numpy(np.int64),
        "sd_itemid": sd["itemid"].to_numpy(np.int64),
        "sd_session": sd["session_id"].str.replace("sess_", "").astype(np.int64).to_numpy(),
        "sd_index": sd.index.to_numpy(np.int64),
        "g_item_i": edges["item_i"].to_numpy(np.int64),
        "g_item_j": edges["item_j"].to_numpy(np.int64),
        "g_count": edges["count"].to_numpy(np.int64),
        "g_last_ts": edges["last_ts"].to_numpy(np.int64),
    }
    np.savez_compressed(os.path.join(out, "c1_data.npz"), **res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(HERE), "tests", "golden"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    sys.path.insert(0, a.ref)  # for trainer.py's `from etpgt.utils.metrics import ...`
    ref_base = load_by_path("ref_base", os.path.join(a.ref, "etpgt/model/base.py"))
    ref_losses = load_by_path("ref_losses", os.path.join(a.ref, "etpgt/train/losses.py"))
    ref_metrics = load_by_path("ref_metrics", os.path.join(a.ref, "etpgt/utils/metrics.py"))
    ref_trainer = load_by_path("ref_trainer", os.path.join(a.ref, "etpgt/train/trainer.py"))
    torch.set_num_threads(1)
    gen_readout(ref_base, a.out)
    gen_losses(ref_base, ref_losses, a.out)
    gen_metrics(ref_metrics, a.out)
    gen_trainer(ref_trainer, ref_losses, a.out)
    gen_c1(a.ref, a.out)
    for f in sorted(os.listdir(a.out)):
        print(f, os.path.getsize(os.path.join(a.out, f)))


if __name__ == "__main__":
    main()
