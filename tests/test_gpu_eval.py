"""GPU parity of the evaluation path: full-catalog scoring + top-k (gtr_score_topk,
base.py:59-78 predict) and Recall@K / NDCG@K of Trainer.evaluate (trainer.py:138-173)
against the CPU oracle.

Tolerance: scores within 1e-5 of the score scale (fp32 dot products of <= 256 terms in
a different summation order); the selected ids must equal the exact (fp64) top-k except
where two candidates at the k-th boundary are closer than that tolerance (a near-tie
either implementation may break either way).
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

import etpgt_ref as R  # noqa: E402
from gpu_helpers import batches, make_pair, ref_batch, small_data  # noqa: E402

from etpgt.backend.ops import score_topk  # noqa: E402
from etpgt.train.fused import FusedTrainStep  # noqa: E402
from etpgt.train.trainer import Trainer  # noqa: E402
from etpgt.utils.metrics import compute_ndcg_at_k, compute_recall_at_k  # noqa: E402


def _check_topk(se, table, k, idx, sc):
    ref = se.double().cpu() @ table.double().cpu().t()
    B, T = ref.shape
    scale = float(ref.abs().max()) + 1e-30
    tol = 1e-5 * scale
    idx = idx.cpu()
    sc = sc.cpu().double()
    assert idx.shape == (B, k) and idx.dtype == torch.int64
    assert bool((idx >= 0).all()) and bool((idx < T).all())
    # reported scores are the scores of the reported ids, best first
    got = ref.gather(1, idx)
    assert float((got - sc).abs().max()) <= tol
    assert bool((sc[:, 1:] <= sc[:, :-1] + tol).all())
    # each row's ids are distinct and form an exact top-k up to near-ties at the boundary
    srt = torch.sort(ref, dim=1, descending=True).values
    kth = srt[:, k - 1]
    for b in range(B):
        ids = idx[b].tolist()
        assert len(set(ids)) == k
        assert float(got[b].min()) >= float(kth[b]) - tol
        exact = set(torch.topk(ref[b], k).indices.tolist())
        if set(ids) != exact:
            nxt = float(srt[b, k]) if k < T else -float("inf")
            assert float(kth[b]) - nxt <= tol, f"row {b}: wrong set without a near-tie"


@pytest.mark.parametrize("B,T,D,k", [
    (1, 300, 64, 20),
    (33, 1000, 128, 10),
    (100, 5000, 32, 128),
    (70, 82174, 64, 20),
    (16, 257, 256, 1),
    (200, 20000, 128, 64),
])
def test_score_topk_matches_exact(B, T, D, k):
    g = torch.Generator().manual_seed(B * 7 + D)
    se = torch.randn(B, D, generator=g)
    table = torch.randn(T, D, generator=g) * 0.1
    idx, sc = score_topk(se.cuda(), table.cuda(), k)
    _check_topk(se, table, k, idx, sc)


def test_score_topk_ties_prefer_lower_id_and_multi_pass_merge():
    """Duplicate rows tie exactly: the lower item id ranks first (deterministic).  A
    98k-row catalog with k = 128 needs two merge passes (384 chunks x 128 candidates)."""
    B, D, k = 5, 64, 128
    g = torch.Generator().manual_seed(3)
    base = torch.randn(1024, D, generator=g)
    table = base.repeat(96, 1)  # row r duplicates row r % 1024 (same lane / tile slot)
    se = torch.randn(B, D, generator=g)
    idx, sc = score_topk(se.cuda(), table.cuda(), k)
    idx = idx.cpu()
    ref = se.double() @ table.double().t()
    # the best 96 entries are the 96 copies of the best base row, in increasing id order
    best = int(torch.argmax(ref[0, :1024]))
    assert idx[0, :96].tolist() == [best + 1024 * j for j in range(96)]
    _check_topk(se, table, k, idx.cuda(), sc)


def test_score_topk_errors():
    se = torch.randn(4, 64, device="cuda")
    with pytest.raises(ValueError):
        score_topk(se, torch.randn(100, 32, device="cuda"), 5)
    with pytest.raises(RuntimeError):
        score_topk(se, torch.randn(100, 64, device="cuda"), 101)
    with pytest.raises(RuntimeError):
        score_topk(se, torch.randn(1000, 64, device="cuda"), 129)  # k <= 128 on the HIP kernel
    with pytest.raises(RuntimeError):
        score_topk(se.cpu(), torch.randn(100, 64), 5)


def _ref_eval(ref, vb, ks):
    ref.eval()
    preds, tg = [], []
    with torch.no_grad():
        for sb in vb:
            rb = ref_batch(sb)
            preds.append(ref.predict(ref(rb), k=max(ks)))
            tg.append(rb.target_item)
    preds, tg = torch.cat(preds), torch.cat(tg)
    out = {}
    for k in ks:
        out[f"recall@{k}"] = compute_recall_at_k(preds[:, :k], tg, k=k)
        out[f"ndcg@{k}"] = compute_ndcg_at_k(preds[:, :k], tg, k=k)
    return out, preds


def test_predict_same_weights_matches_oracle():
    """model.predict on the HIP path == oracle predict (torch matmul + topk) on the
    same weights, up to boundary near-ties."""
    data = small_data()
    T = data.table_rows
    m, ref = make_pair(T, 64, 2, seed=21)
    m.eval(); ref.eval()
    W = ref.item_embedding.weight.detach()
    for sb in batches(data, 48, 5, 3, seed=31):
        with torch.no_grad():
            se = m(sb.to("cuda"))
            p = m.predict(se, k=20)
            se_r = ref(ref_batch(sb))
        torch.testing.assert_close(se.cpu(), se_r, rtol=1e-3, atol=1e-5)
        idx, sc = score_topk(se, m.item_embedding.weight, 20)
        assert torch.equal(idx, p)
        _check_topk(se.cpu(), W, 20, idx, sc)
        # the oracle's own ranking (torch matmul + topk on its session embeddings)
        rp = ref.predict(se_r, k=20)
        agree = sum(len(set(a) & set(b)) for a, b in zip(p.cpu().tolist(), rp.tolist()))
        assert agree >= 0.99 * rp.numel()


def test_recall_parity_after_training(tmp_path):
    """Recall@10 parity: the HIP fused trainer and the oracle trainer start from the same
    weights, take the same 30 AdamW steps on the same batches (dropout 0), then
    Trainer.evaluate (HIP forward + HIP top-k) and the oracle evaluation agree."""
    data = small_data()
    T = data.table_rows
    m, ref = make_pair(T, 64, 2, seed=22)
    m.train(); ref.train()
    fused = FusedTrainStep(m, lr=3e-3, weight_decay=1e-5, loss="bpr")
    ropt = torch.optim.AdamW(ref.parameters(), lr=3e-3, weight_decay=1e-5)
    for sb in batches(data, 32, 5, 30, seed=41):
        fused(sb.to("cuda"))
        R.ref_train_step(ref, ref_batch(sb), ropt, "bpr")
    vb = batches(data, 64, 5, 4, seed=42)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    tr = Trainer(m, [], vb, opt, device="cuda", output_dir=tmp_path, k_values=[10, 20])
    got = tr.evaluate()
    want, _ = _ref_eval(ref, vb, [10, 20])
    n = 64 * 4
    for key in want:
        # one boundary flip changes recall by 1/n; allow two
        assert abs(got[key] - want[key]) <= 2.0 / n + 1e-9, (key, got[key], want[key])
    assert got["recall@20"] > 0.0


def test_score_topk_exclusion():
    """Masked top-k: excluded ids never come back; the rest is the exact top-k of the
    remaining catalogue; too few remaining ids pad with -1."""
    g = torch.Generator().manual_seed(5)
    B, T, D, k = 3, 3000, 64, 20
    se = torch.randn(B, D, generator=g)
    table = torch.randn(T, D, generator=g)
    ref = se.double() @ table.double().t()
    top = torch.topk(ref, 40, dim=1).indices
    excl = [top[0, :10].tolist() + [0], [], list(range(0, T, 2))]
    idx, sc = score_topk(se.cuda(), table.cuda(), k, exclude=excl)
    for b in range(B):
        r = ref[b].clone()
        r[excl[b]] = -float("inf")
        want = torch.topk(r, k).indices.tolist()
        assert idx[b].tolist() == want
        assert not set(idx[b].tolist()) & set(excl[b])
    idx, sc = score_topk(se[:1].cuda(), table[:25].cuda(), 20, exclude=[list(range(10))])
    assert idx[0, 15:].tolist() == [-1] * 5 and bool(torch.isinf(sc[0, 15:]).all())


def test_recommender_matches_oracle(tmp_path):
    """Single-session serving (recommender.py:115-131): checkpoint round trip, session
    subgraph without self-loops, HIP forward + masked top-k == the oracle forward +
    masked torch.topk."""
    import pandas as pd

    from etpgt.serving import Recommender, ValidatedRequest

    data = small_data()
    T = data.table_rows
    m, ref = make_pair(T, 64, 2, K=8, seed=23)
    torch.save({"epoch": 3, "model_state_dict": m.state_dict(), "best_val_metric": 0.25}, tmp_path / "ck.pt")
    ei = data.edge_index()
    pd.DataFrame({"item_i": ei[0], "item_j": ei[1]}).to_csv(tmp_path / "edges.csv", index=False)
    rec = Recommender(tmp_path / "ck.pt", tmp_path / "edges.csv", device="cuda")
    assert rec.health()["checkpoint_epoch"] == 3
    ref.laplacian_pe._cached_pe = m.laplacian_pe._cached_pe.detach().cpu().clone()
    ref.eval()
    adj = {}
    for i, j in zip(ei[0].tolist(), ei[1].tolist()):
        if i != j:
            adj.setdefault(i, set()).add(j)
    for s in range(0, 200, 17):
        items = data.session(s).tolist()
        ids, scores = rec.recommend(ValidatedRequest(items, 10))
        seen = set(items)
        uniq = sorted(seen)
        loc = {g: q for q, g in enumerate(uniq)}
        pairs = sorted((i, j) for i in seen for j in adj.get(i, ()) if j in seen)
        e = torch.tensor([[loc[i], loc[j]] for i, j in pairs], dtype=torch.long).t() if pairs else \
            torch.zeros((2, 0), dtype=torch.long)
        rb = R.RefBatch(torch.tensor(uniq), e, torch.zeros(len(uniq), dtype=torch.long))
        with torch.no_grad():
            se = ref(rb)
        sc = (se.double() @ ref.item_embedding.weight.detach().double().t()).squeeze(0)
        sc[list(seen)] = -float("inf")
        sc[0] = -float("inf")
        top = torch.topk(sc, 11)
        want = top.indices[:10].tolist()
        if ids != want:  # only a near-tie at the boundary may differ
            assert float(top.values[9] - top.values[10]) <= 1e-4 * float(top.values.abs().max())
        assert not set(ids) & (seen | {0})
        np.testing.assert_allclose(scores, sc[ids].numpy(), rtol=1e-3, atol=1e-5)


def test_recommender_k_past_the_unmasked_items(tmp_path):
    """A validated request near the catalog size (validation.py:89 clamps k to
    num_items - 1 only): the reference's torch.topk returns every finite score and then
    the masked ids at -inf; so does the Recommender (masked ids in ascending order)."""
    import pandas as pd

    from etpgt.serving import Recommender, ValidatedRequest

    T = 12
    m, _ = make_pair(T, 32, 2, K=4, seed=24)
    torch.save({"epoch": 0, "model_state_dict": m.state_dict()}, tmp_path / "ck.pt")
    pd.DataFrame({"item_i": [1, 2, 3, 5], "item_j": [2, 3, 5, 5]}).to_csv(tmp_path / "edges.csv", index=False)
    rec = Recommender(tmp_path / "ck.pt", tmp_path / "edges.csv", device="cuda")
    session = [3, 1, 5, 2]
    ids, scores = rec.recommend(ValidatedRequest(session, T - 1))
    live = T - len(set(session) | {0})
    assert len(ids) == T - 1 and len(set(ids)) == T - 1
    assert set(ids[:live]) == set(range(T)) - set(session) - {0}
    assert all(np.isfinite(scores[:live])) and scores[:live] == sorted(scores[:live], reverse=True)
    assert ids[live:] == sorted(set(session) | {0})[: T - 1 - live]
    assert all(s == float("-inf") for s in scores[live:])
    short, _ = rec.recommend(ValidatedRequest(session, live))
    assert short == ids[:live]


def test_registered_ops_pass_opcheck():
    """torch.library.opcheck of the registered HIP ops (schema, fake implementation vs the
    real kernel, autograd registration) on device tensors."""
    from etpgt.backend import ops  # noqa: F401

    g = torch.Generator().manual_seed(5)
    se = torch.randn(8, 64, generator=g).cuda().requires_grad_()
    tab = torch.randn(300, 64, generator=g).cuda().requires_grad_()
    t = torch.randint(1, 300, (8,), generator=g).cuda()
    n = torch.randint(1, 300, (8, 5), generator=g).cuda()
    torch.library.opcheck(torch.ops.etpgt.score_loss.default, (se, tab, t, n, 2, 1.0, 0.7),
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))
    torch.library.opcheck(torch.ops.etpgt.score_topk.default, (se.detach(), tab.detach(), 10, None, None),
                          test_utils=("test_schema", "test_faketensor"))
