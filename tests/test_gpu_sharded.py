"""GPU: the row-sharded item table (etpgt.train.sharded, gtr_shard_* in include/gtr.h).

Rank p owns the rows r % P == p with their AdamW moments; rows are fetched and
gradients returned by all-to-all.  The arithmetic is the replicated data-parallel step's
with the lazy table (same per-rank segment sums, rank-ordered averaging, the same
zero-gradient catch-up), so the tests ask for bit equality:
  * one rank: the sharded step == the single-GPU fused step with the lazy table;
  * two and four ranks sharing the GPU (gloo transport): == the replicated data-parallel
    step, with and without SyncBN, with LapPE, and the replicas agree;
  * a batch that overflows an exchange block is reported, not silently trained on."""

from __future__ import annotations

import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

from gpu_helpers import collect, batches, make_pair, small_data  # noqa: E402

from etpgt.train.fused import FusedTrainStep  # noqa: E402

CASES = [  # (D, H, K, loss, steps, B)
    (64, 2, 0, "bpr", 6, 16),
    (128, 4, 16, "listwise", 4, 16),
]


def _state(m, f):
    return {n: p.detach().clone() for n, p in m.named_parameters()}, f.m_tab.clone(), f.v_tab.clone()


@pytest.mark.parametrize("D,H,K,loss,steps,B", CASES + [(64, 1, 0, "dual", 3, 2100)])
def test_shard_world1_bitwise_equals_lazy_step(D, H, K, loss, steps, B):
    data = small_data()
    T = data.table_rows
    m1, _ = make_pair(T, D, H, K=K, seed=41)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    # large batches (m_cap > 8192): the single-GPU tail sums a long segment in window
    # pieces; the data-parallel pack (like the shard pack) sums it in one pass -- compare
    # with the world-1 data-parallel step there
    f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss=loss, lazy=True, data_parallel=B > 1000)
    f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss=loss, shard_table=True)
    assert f2.world == 1 and f2.shard_state is not None
    for sb in batches(data, B, 5, steps, seed=42):
        l1 = float(f1(sb.to("cuda")))
        l2 = float(f2(sb.to("cuda")))
        assert l1 == l2, (l1, l2)
    assert f2.shard is not None and f2.graph is not None
    with pytest.raises(RuntimeError, match="row-sharded"):
        m2.state_dict()  # the model's table copy is stale until sync_table()
    f1.flush()
    f2.sync_table()
    p1, mt1, vt1 = _state(m1, f1)
    p2, mt2, vt2 = _state(m2, f2)
    for n in p1:
        assert torch.equal(p1[n], p2[n]), n
    assert torch.equal(mt1, mt2) and torch.equal(vt1, vt2)


def test_shard_overflow_is_reported(monkeypatch):
    monkeypatch.setenv("GTR_SHARD_SLACK", "0.0001")  # blocks of 64 rows: a B=16 batch needs more
    data = small_data()
    T = data.table_rows
    m, _ = make_pair(T, 64, 2, seed=43)
    m.train()
    f = FusedTrainStep(m, lr=1e-2, weight_decay=1e-2, loss="bpr", shard_table=True)
    for sb in batches(data, 16, 5, 2, seed=44):
        f(sb.to("cuda"))
    assert f.shard.cap <= 66
    with pytest.raises(RuntimeError, match="exchange capacity"):
        f.sync_table()


def test_shard_overflow_on_the_last_step_is_reported(monkeypatch):
    """an overflow on the FINAL step (no later step to carry the asynchronous
    status read) is still raised by sync_table(), and the flagged step is applied as a
    zero-gradient step (no partial update)."""
    monkeypatch.setenv("GTR_SHARD_SLACK", "0.0001")  # blocks of 64 rows
    data = small_data()
    T = data.table_rows
    m, _ = make_pair(T, 64, 2, seed=47)
    m.train()
    f = FusedTrainStep(m, lr=1e-2, weight_decay=1e-2, loss="bpr", shard_table=True)
    for sb in batches(data, 4, 5, 2, seed=48):  # B = 4: well under 64 distinct rows
        f(sb.to("cuda"))
    f.shard_state.check_status(block=True)  # nothing overflowed so far
    small_before = f.eng.flat.flat.clone()
    big = batches(data, 16, 5, 1, seed=49)[0]  # > 64 distinct rows from the one owner
    f(big.to("cuda"))
    with pytest.raises(RuntimeError, match="exchange capacity"):
        f.sync_table()
    assert int(f.shard_state.status[1].item()) & 2  # the owner saw the flag in the pack
    # the flagged step moved the small parameters by a zero-gradient AdamW update only
    assert torch.isfinite(f.eng.flat.flat).all()
    assert float((f.eng.flat.flat - small_before).abs().max()) < 0.05


def test_shard_table_never_takes_the_early_union_or_chain_sweep(monkeypatch):
    """GTR_DP_EARLY=1 must not install the chain sweep (whose table / moment
    pointers are the model's stale copy and 1-row placeholders) on a sharded step."""
    monkeypatch.setenv("GTR_DP_EARLY", "1")
    data = small_data()
    T = data.table_rows
    m1, _ = make_pair(T, 64, 2, seed=50)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss="bpr", lazy=True)
    f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss="bpr", shard_table=True)
    for sb in batches(data, 16, 5, 3, seed=51):
        assert float(f1(sb.to("cuda"))) == float(f2(sb.to("cuda")))
    assert not f2.early_union and f2.sweep is None
    f1.flush()
    f2.sync_table()
    assert torch.equal(m1.item_embedding.weight, m2.item_embedding.weight)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q, ncases):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        for (D, H, K, loss, steps, B), sync in list(zip(CASES, (False, True)))[:ncases]:
            data = small_data()
            T = data.table_rows
            m1, _ = make_pair(T, D, H, K=K, seed=45)
            m2 = copy.deepcopy(m1)
            m1.train(); m2.train()
            f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss=loss, lazy=True, sync_bn=sync,
                                data_parallel=True)
            f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss=loss, shard_table=True, sync_bn=sync)
            bl = batches(data, B, 5, steps * world, seed=46)
            same_loss = True
            static = None
            for s in range(steps):
                l1 = float(f1(bl[s * world + rank].to("cuda")))
                l2 = float(f2(bl[s * world + rank].to("cuda")))
                same_loss = same_loss and l1 == l2
                if s == 0 and sync:  # blocks sized to this run's batches from step 1 on
                    static = (f2.shard.cap, f2.shard.cap_s)
                    f2.fit_shard_blocks([bl[k * world + rank] for k in range(steps)])
            f1.flush()
            f2.sync_table()
            p1, mt1, vt1 = _state(m1, f1)
            p2, mt2, vt2 = _state(m2, f2)
            same = all(torch.equal(p1[n], p2[n]) for n in p1) and torch.equal(mt1, mt2) and torch.equal(vt1, vt2)
            bad = [n for n in p1 if not torch.equal(p1[n], p2[n])]
            vol = f2.shard.volume()
            vol["static"] = static
            out.append((same_loss, same, bad, {n: v.cpu().numpy() for n, v in p2.items()}, vol))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,ncases", [(2, 2), (4, 1)])
def test_shard_ranks_bitwise_equal_replicated_dp(world, ncases):
    """2 (4) ranks sharing the GPU over gloo: the sharded step equals the replicated
    data-parallel step (lazy table) bit for bit -- BPR at D=64, and (2 ranks) listwise at
    D=128 / 4 heads / LapPE with SyncBN, its exchange blocks refitted to the run's batches
    after the first step (FusedTrainStep.fit_shard_blocks) -- and the gathered tables agree
    across ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, ncases)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for item in collect(q, procs, world):
            rank, out = item
            res[rank] = out
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for case in range(ncases):
        for r in range(world):
            same_loss, same, bad, _, vol = res[r][case]
            assert same_loss, (case, r)
            assert same, (case, r, bad)
            if vol["static"] is not None:  # fitted blocks: smaller, and every rank agrees on them
                assert vol["cap"] <= vol["static"][0] and vol["cap_scoring"] < vol["static"][1], vol
                assert (vol["cap"], vol["cap_scoring"]) == (res[0][case][4]["cap"], res[0][case][4]["cap_scoring"])
        for r in range(1, world):
            for k, v in res[0][case][3].items():
                assert np.array_equal(v, res[r][case][3][k]), f"replicas diverged: {k}"
