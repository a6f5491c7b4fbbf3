"""GPU: the contribution-list sort of the large-batch step (gtr_contrib_sort): the own
10-bit LSD radix (default) and hipCUB's merge path (GTR_SORT=merge) both equal a stable
sort of the (row, slot) pairs -- ties keep slot order, which the segmented table-gradient
sums rely on for determinism -- at the C3 / C5 shapes (855k slots, rows < 2^17 / 2^20),
ragged sizes and the sentinel row T of unused slots."""

from __future__ import annotations

import ctypes as C

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

from etpgt.backend import _lib as L  # noqa: E402


def _sort(keys, T, mode, monkeypatch):
    monkeypatch.setenv("GTR_SORT", mode)
    n = keys.numel()
    vals = torch.arange(n, dtype=torch.int32, device="cuda")
    sk = torch.empty_like(keys)
    sv = torch.empty_like(vals)
    nb = C.c_size_t(0)
    L.check(L.lib().gtr_contrib_sort_bytes(n, T, C.byref(nb)), "sort_bytes")
    tmp = torch.zeros(int(nb.value), dtype=torch.uint8, device="cuda")  # zeroed once (gtr.h contract)
    L.check(L.lib().gtr_contrib_sort(keys.data_ptr(), vals.data_ptr(), sk.data_ptr(), sv.data_ptr(), n, T,
                                     tmp.data_ptr(), tmp.numel(), torch.cuda.current_stream().cuda_stream),
            "contrib_sort")
    torch.cuda.synchronize()
    return sk.cpu(), sv.cpu()


@pytest.mark.parametrize("n,T", [(855_000, 82_174), (107_000, 1_000_001), (8193, 300), (4096 * 3 + 17, 1 << 19)])
def test_contrib_sort_is_a_stable_sort(n, T, monkeypatch):
    g = torch.Generator().manual_seed(n)
    keys = torch.randint(1, T, (n,), generator=g, dtype=torch.int32)
    keys[torch.randint(0, n, (n // 50,), generator=g)] = T  # sentinel rows of unused slots
    hot = torch.randint(0, n, (n // 20,), generator=g)
    keys[hot] = 7  # a Zipf-hot row: long runs of equal keys
    order = torch.sort(keys.long() * (1 << 24) + torch.arange(n), stable=True).indices
    want_k, want_v = keys[order], order.to(torch.int32)
    for mode in ("radix", "merge"):
        sk, sv = _sort(keys.cuda(), T, mode, monkeypatch)
        assert torch.equal(sk, want_k), mode
        assert torch.equal(sv, want_v), mode
    # the same workspace reused by a second call (the digit totals must be left zeroed)
    monkeypatch.setenv("GTR_SORT", "radix")
    n2 = keys.numel()
    kd, vals = keys.cuda(), torch.arange(n2, dtype=torch.int32, device="cuda")
    nb = C.c_size_t(0)
    L.check(L.lib().gtr_contrib_sort_bytes(n2, T, C.byref(nb)), "sort_bytes")
    tmp = torch.zeros(int(nb.value), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        sk, sv = torch.empty_like(kd), torch.empty_like(vals)
        L.check(L.lib().gtr_contrib_sort(kd.data_ptr(), vals.data_ptr(), sk.data_ptr(), sv.data_ptr(), n2, T,
                                         tmp.data_ptr(), tmp.numel(), torch.cuda.current_stream().cuda_stream),
                "contrib_sort")
        torch.cuda.synchronize()
        assert torch.equal(sk.cpu(), want_k) and torch.equal(sv.cpu(), want_v)


def test_contrib_sort_rejects_a_short_workspace():
    n, T = 10_000, 300
    keys = torch.zeros(n, dtype=torch.int32, device="cuda")
    out = torch.empty_like(keys)
    with pytest.raises(RuntimeError, match="workspace"):
        L.check(L.lib().gtr_contrib_sort(keys.data_ptr(), keys.data_ptr(), out.data_ptr(), out.data_ptr(), n, T,
                                         out.data_ptr(), 16, torch.cuda.current_stream().cuda_stream), "contrib_sort")


@pytest.mark.parametrize("D,H,K,loss,B", [(128, 4, 16, "listwise", 2400), (64, 1, 0, "bpr", 32)])
def test_step_workspaces_do_not_overlap(D, H, K, loss, B):
    """Round-3 Onesweep question: every device buffer a fused step's kernels write (the
    contribution keys / values, their sorted copies, the sort scratch, the batch image, the
    carry scratch, the activations) occupies its own bytes -- checked on a large batch (the
    radix-sort begin path of C3 at B = 8192) and on C2's small one, after a step has run."""
    from gpu_helpers import batches, make_pair, small_data

    from etpgt.train.fused import FusedTrainStep

    data = small_data()
    m, _ = make_pair(data.table_rows, D, H, K=K, seed=3)
    m.train()
    f = FusedTrainStep(m, loss=loss)
    n = 100 if loss == "listwise" else 5
    f(batches(data, B, n, 1, seed=5)[0].to("cuda"))
    torch.cuda.synchronize()
    assert len(f.workspace_ranges()) > 20
    f.check_workspace_overlap()
