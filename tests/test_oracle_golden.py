"""The CPU oracle (oracle/etpgt_ref.py) pinned against golden vectors produced by
the reference's own files (oracle/gen_golden.py: base.py, losses.py, metrics.py,
trainer.py imported by path) and against the reference's known answers."""

import os

import numpy as np
import pytest
import torch

import etpgt_ref as R


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


@pytest.mark.parametrize("mode", ["mean", "max", "last", "attention"])
def test_readout_matches_reference(golden_dir, mode):
    g = load(golden_dir, "readout.npz")
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    ro = R.RefSessionReadout(hidden_dim=x.shape[1], readout_type=mode)
    if mode == "attention":
        with torch.no_grad():
            ro.attention.weight.copy_(torch.from_numpy(g["attention_w"]))
            ro.attention.bias.copy_(torch.from_numpy(g["attention_b"]))
    se = ro(x, torch.from_numpy(g["batch"]))
    w = torch.linspace(-1, 1, se.numel()).view_as(se)
    (se * w).sum().backward()
    np.testing.assert_allclose(se.detach().numpy(), g[f"{mode}_se"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(x.grad.numpy(), g[f"{mode}_dx"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("case", ["bpr", "listwise_t0.5", "listwise_t1", "listwise_t2", "dual_a0.7",
                                  "sampled_softmax", "model_bpr"])
def test_losses_match_reference(golden_dir, case):
    g = load(golden_dir, "losses.npz")
    se = torch.from_numpy(g["se"]).requires_grad_(True)
    T, d = g["W"].shape
    emb = torch.nn.Embedding(T, d, padding_idx=0)
    with torch.no_grad():
        emb.weight.copy_(torch.from_numpy(g["W"]))
    tgt, neg = torch.from_numpy(g["target"]), torch.from_numpy(g["neg"])
    kind, kw = {
        "bpr": ("bpr", {}), "model_bpr": ("bpr", {}), "listwise_t0.5": ("listwise", {"temperature": 0.5}),
        "listwise_t1": ("listwise", {"temperature": 1.0}), "listwise_t2": ("listwise", {"temperature": 2.0}),
        "dual_a0.7": ("dual", {"alpha": 0.7}), "sampled_softmax": ("sampled_softmax", {}),
    }[case]
    loss = R.ref_loss(kind, se, tgt, neg, emb, **kw)
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(g[f"{case}_loss"]), rtol=1e-6)
    np.testing.assert_allclose(se.grad.numpy(), g[f"{case}_dse"], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(emb.weight.grad.numpy(), g[f"{case}_dW"], rtol=1e-5, atol=1e-8)


def test_table_init_matches_reference(golden_dir):
    g = load(golden_dir, "losses.npz")
    torch.manual_seed(5)
    m = R.RefGraphTransformer(1000, 32, 32, 1, 1, use_laplacian_pe=False, use_ffn=False)
    W = m.item_embedding.weight.detach()
    assert float(W[0].abs().max()) == float(g["init_row0_absmax"]) == 0.0
    assert float(W[1:].abs().max()) <= float(g["init_bound"]) + 1e-7


def test_metrics_known_answers(golden_dir):
    # tests/test_utils.py:62-93 of the reference
    from etpgt.utils.metrics import compute_ndcg_at_k, compute_recall_at_k

    p = torch.tensor([[1, 2, 3, 4, 5], [6, 7, 8, 9, 10], [11, 12, 13, 14, 15]])
    assert compute_recall_at_k(p, torch.tensor([2, 9, 20]), 5) == pytest.approx(2 / 3, abs=1e-6)
    assert compute_recall_at_k(p, torch.tensor([2, 9, 20]), 2) == pytest.approx(1 / 3, abs=1e-6)
    assert compute_ndcg_at_k(p, torch.tensor([1, 9, 20]), 5) == pytest.approx(0.4769, abs=1e-4)
    g = load(golden_dir, "metrics.npz")
    preds, tg = torch.from_numpy(g["preds"]), torch.from_numpy(g["targets"])
    for k in (1, 5, 10, 20):
        assert compute_recall_at_k(preds, tg, k) == pytest.approx(float(g[f"recall@{k}"]), abs=1e-7)
        assert compute_ndcg_at_k(preds, tg, k) == pytest.approx(float(g[f"ndcg@{k}"]), abs=1e-7)


@pytest.mark.parametrize("tag,kind,kw", [
    ("bpr", "model", dict(use_laplacian_pe=False)),
    ("listwise", "listwise", dict(use_laplacian_pe=True, laplacian_k=4)),
    ("dual", "dual", dict(use_laplacian_pe=False)),
])
def test_oracle_step_matches_reference_trainer(golden_dir, tag, kind, kw):
    """oracle ref_train_step over 3 batches == the REFERENCE Trainer.train_epoch
    (trainer.py:80-133) driving the same restated model with AdamW."""
    g = load(golden_dir, "trainer.npz")
    T, d = 40, 16
    model = R.ref_create_graph_transformer_optimized(T, embedding_dim=d, hidden_dim=d, num_layers=2, num_heads=2,
                                                     dropout=0.0, **kw)
    if kw.get("use_laplacian_pe"):
        model.laplacian_pe._cached_pe = torch.zeros(T, kw["laplacian_k"])
    init = {k[len(tag) + 6:]: torch.from_numpy(g[k]) for k in g.files if k.startswith(f"{tag}_init.")}
    model.load_state_dict(init)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=1e-5)
    losses = []
    for bi in range(3):
        b = R.RefBatch(*(torch.from_numpy(g[f"b{bi}_{k}"]) for k in
                         ("x", "edge_index", "batch", "target_item", "negative_items")))
        losses.append(float(R.ref_train_step(model, b, opt, kind)))
    np.testing.assert_allclose(np.mean(losses), float(g[f"{tag}_avg_loss"]), rtol=1e-6)
    for k, v in model.state_dict().items():
        if k.endswith("lin_key.bias"):
            # exactly-zero gradient (softmax shift invariance): Adam turns the rounding
            # noise into +-lr steps, so only the bound is reproducible across thread counts
            assert float(np.abs(v.numpy() - g[f"{tag}_final.{k}"]).max()) <= 2 * 3 * 1e-2
            continue
        np.testing.assert_allclose(v.numpy(), g[f"{tag}_final.{k}"], rtol=1e-5, atol=1e-7, err_msg=k)


def test_param_count_known_answers():
    # notebooks/session_recsys_walkthrough.ipynb:1076,1091 and docs/EXPERIMENTS.md:87-88
    def count(m):
        return sum(p.numel() for p in m.parameters())

    assert count(R.ref_create_graph_transformer_optimized(36, embedding_dim=64, hidden_dim=64, laplacian_k=8)) == 36800
    assert count(R.ref_create_graph_transformer_optimized(188, embedding_dim=64, hidden_dim=64,
                                                          use_laplacian_pe=False)) == 45952
    assert count(R.RefGraphTransformer(188, 64, 64, 2, 2, use_laplacian_pe=False, use_ffn=True,
                                       ffn_expansion=4)) == 112128


def test_lappe_path_graph():
    # tests/test_models.py:232-239: 4-node path, shape (4,2), float32, non-negative
    ei = torch.tensor([[0, 1, 1, 2, 2, 3], [1, 0, 2, 1, 3, 2]])
    pe = R.ref_compute_laplacian_pe(ei, num_nodes=4, k=2)
    assert pe.shape == (4, 2) and pe.dtype == torch.float32 and bool((pe >= 0).all())
    # the sym-normalised path Laplacian's spectrum: 1 - cos(pi j / 3), j = 0..3
    import scipy.sparse.linalg  # noqa: F401

    L = R.ref_sym_laplacian(ei.numpy(), 4).toarray()
    np.testing.assert_allclose(np.sort(np.linalg.eigvalsh(L)), 1 - np.cos(np.pi * np.arange(4) / 3), atol=1e-6)


def test_cached_pe_raises_without_precompute():
    m = R.RefLaplacianPECached(k=2, embedding_dim=16)
    with pytest.raises(RuntimeError, match="not precomputed"):
        m(torch.tensor([0, 1]))


def test_hip_dropout_mask_restatement_keep_rate_and_scale():
    """The oracle's restatement of the HIP dropout stream (used for value-level parity at
    p = 0.1): keep rate 1 - p within 3 sigma, kept entries scaled by fp32 1/(1 - p),
    streams of different layers / kinds / counters independent, attention masks indexed
    in destination order."""
    import numpy as np
    import torch

    import etpgt_ref as R

    p, N, D, H = 0.1, 4000, 64, 4
    ei = np.stack([np.arange(3000) % N, (np.arange(3000) * 7) % N])
    m1 = R.hip_dropout_masks(123456789, 5, p, 2, ei, N, D, H)
    m2 = R.hip_dropout_masks(123456789, 6, p, 2, ei, N, D, H)
    scale = float(np.float32(1.0 / (1.0 - np.float32(p))))
    for k in ("attn", "out"):
        for l in range(2):
            m = m1[k][l].numpy()
            kept = m > 0
            n = m.size
            assert abs(kept.mean() - (1 - p)) <= 3 * np.sqrt(p * (1 - p) / n)
            assert np.all(m[kept] == np.float32(scale))
        # layers and counters draw different masks
        assert not torch.equal(m1[k][0], m1[k][1])
        assert not torch.equal(m1[k][0], m2[k][0])
    assert not torch.equal(m1["attn"][0][:, 0], m1["out"][0][:3000, 0])
    # attention element index = (destination-order position) * H + head
    dst = ei[1]
    order = np.argsort(dst, kind="stable")
    e = int(order[17])  # the edge at destination-order position 17
    want = R.hip_mix3(123456789, R.hip_drop_stream(0, 1, 5), np.array([17 * H + 2]))[0]
    thresh = int(float(np.float32(p)) * 4294967296.0)
    assert (m1["attn"][1][e, 2].item() > 0) == (int(want) >= thresh)
