"""GPU batch constructor (gtr_build_batch, etpgt.data.gpu_batch) against the CPU
restatement of the reference's __getitem__ + collate_fn (oracle/batch_ref.py): the
packed batch images must be identical word for word (integer work: bit-exact), and a
fused training step fed by the device builder must equal the same step fed by the
host-packed batches."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

import batch_ref as BR  # noqa: E402
from gpu_helpers import make_pair, small_data  # noqa: E402

from etpgt.data.batch import collate_sessions  # noqa: E402
from etpgt.data.gpu_batch import GpuBatchBuilder, GpuSessionStore  # noqa: E402
from etpgt.data.synthetic import make_sessions_and_graph  # noqa: E402
from etpgt.train.fused import FusedTrainStep  # noqa: E402


def _ref_blob(data, order, start, B, n, seed, caps, max_len=50):
    ex = BR.build_batch(data.session_ptr, data.session_items, data.edge_keys, data.table_rows, order, start, B,
                        max_len, n, seed)
    return collate_sessions(ex).packed(caps)[1]


@pytest.mark.parametrize("B,n,max_len", [(32, 5, 50), (64, 100, 50), (300, 7, 6), (1, 3, 50)])
def test_gpu_batches_equal_reference(B, n, max_len):
    data = small_data()
    store = GpuSessionStore.from_synthetic(data, "cuda", max_session_length=max_len)
    # per-session counts against the restatement
    for s in range(0, data.num_sessions, 97):
        ex = BR.session_example(data.session_ptr, data.session_items, data.edge_keys, data.table_rows, s, max_len,
                                1, 0, 0)
        assert store.nodes[s] == ex["x"].size and store.edges[s] == ex["edge_index"].shape[1]
    bld = GpuBatchBuilder(store, B, n, seed=11)
    order = np.random.default_rng(B).permutation(data.num_sessions)
    bld.set_epoch_order(order, position=5)
    caps = bld.plan_caps(4, 5)
    for k in range(4):
        start = 5 + k * B
        assert int(bld.cursor.item()) == start
        _, blob = bld.build(caps)
        want = _ref_blob(data, order, start, B, n, 11, caps, max_len)
        got = blob.cpu().numpy()
        assert got.shape == want.shape
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"batch {k}: {bad.size} words differ, first at {bad[:5]}"


def test_gpu_batches_retailrocket_shape_wraparound():
    """RetailRocket-shaped store (82k items, 738k edges in the hash), B = 2048, an
    epoch order that wraps around the end."""
    data = make_sessions_and_graph(seed=42)
    store = GpuSessionStore.from_synthetic(data, "cuda")
    bld = GpuBatchBuilder(store, 2048, 100, seed=3)
    order = np.random.default_rng(0).permutation(data.num_sessions)
    pos = data.num_sessions - 1000
    bld.set_epoch_order(order, position=pos)
    caps = bld.plan_caps(1, pos)
    _, blob = bld.build(caps)
    want = _ref_blob(data, order, pos, 2048, 100, 3, caps)
    assert np.array_equal(blob.cpu().numpy(), want)


def test_capacity_overflow_reported():
    data = small_data()
    store = GpuSessionStore.from_synthetic(data, "cuda")
    bld = GpuBatchBuilder(store, 64, 5)
    caps = bld.plan_caps(1)
    from etpgt.data.batch import Caps

    small = Caps(max(16, caps.n_cap // 4), caps.b_cap, caps.e_cap, caps.n_neg)
    with pytest.raises(RuntimeError, match="capacities"):
        bld.build(small)


def test_store_rejects_short_sessions():
    with pytest.raises(ValueError):
        GpuSessionStore(np.array([0, 3, 4]), np.array([1, 2, 3, 4]), np.array([1 * 10 + 2]), 10, "cuda")


@pytest.mark.parametrize("use_graph", [False, True])
def test_fused_step_with_device_builder_equals_host_batches(use_graph):
    """attach_builder: the build runs inside the (captured) step.  Same weights, same
    batches (host-packed from the oracle restatement) -> identical losses and tables."""
    data = small_data()
    T = data.table_rows
    m1, _ = make_pair(T, 64, 2, seed=31)
    import copy

    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    store = GpuSessionStore.from_synthetic(data, "cuda")
    bld = GpuBatchBuilder(store, 32, 5, seed=5)
    order = np.random.default_rng(1).permutation(data.num_sessions)
    bld.set_epoch_order(order)
    f1 = FusedTrainStep(m1, lr=1e-3, weight_decay=1e-5, loss="bpr", use_graph=use_graph)
    f1.attach_builder(bld, num_batches=6)
    f2 = FusedTrainStep(m2, lr=1e-3, weight_decay=1e-5, loss="bpr", use_graph=use_graph, caps=f1.caps)
    for k in range(6):
        l1 = float(f1.run())
        ex = BR.build_batch(data.session_ptr, data.session_items, data.edge_keys, T, order, k * 32, 32, 50, 5, 5)
        l2 = float(f2(collate_sessions(ex)))
        assert l1 == l2, (k, l1, l2)
    assert torch.equal(m1.item_embedding.weight, m2.item_embedding.weight)


def test_negatives_reject_until_found_and_unsatisfiable_session_raises():
    """Negative sampling rejects session items for as long as it takes
    (dataloader.py:107-124), beyond the 64 rounds of the earlier builder: a session holding
    all but one catalog item gets that item n times, exactly as the oracle restatement.
    A session holding every item has no negative at all -- the reference would spin
    forever; the builder stops and the host raises."""
    T = 8  # items 1..7
    ptr = np.array([0, 7, 14])
    items = np.array([1, 2, 3, 4, 5, 6, 2, 1, 2, 3, 4, 5, 6, 7])  # session 1 holds all of 1..7
    keys = np.array([1 * T + 2, 2 * T + 3])
    store = GpuSessionStore(ptr, items, keys, T, "cuda")
    bld = GpuBatchBuilder(store, 1, 6, seed=4)
    bld.set_epoch_order(np.array([0, 1]))
    caps = bld.plan_caps(1, 0)
    _, blob = bld.build(caps)
    ex = BR.build_batch(ptr, items, keys, T, np.array([0, 1]), 0, 1, 50, 6, 4)
    assert ex[0]["negative_items"].tolist() == [7] * 6
    assert np.array_equal(blob.cpu().numpy(), collate_sessions(ex).packed(caps)[1])
    with pytest.raises(RuntimeError, match="negative sampling"):
        bld.build(caps)
    with pytest.raises(RuntimeError, match="negative sampling"):
        BR.build_batch(ptr, items, keys, T, np.array([0, 1]), 1, 1, 50, 6, 4)
