"""GPU: the data-parallel step kernels (gtr_dp_pack / gtr_dp_tail) — world size 1
against the single-GPU fused step, and two ranks sharing the GPU over a gloo group
against the oracle's rank-averaged AdamW trajectory (replicas must stay identical)."""

from __future__ import annotations

import copy

import numpy as np
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

from gpu_helpers import (OracleTrio, batches, close_trained, collect, make_pair,  # noqa: E402
                         ref_batch, small_data)
import etpgt_ref as R  # noqa: E402

from etpgt.train.fused import FusedTrainStep  # noqa: E402

D, H, STEPS, B, NNEG = 64, 2, 3, 16, 5


def test_dp_world1_equals_fused_step():
    data = small_data()
    T = data.table_rows
    m1, _ = make_pair(T, D, H, K=0, seed=21)
    m2 = copy.deepcopy(m1)
    m1.train(); m2.train()
    f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss="bpr")
    f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss="bpr", data_parallel=True)
    assert f2.world == 1
    for sb in batches(data, B, NNEG, STEPS, seed=22):
        l1 = float(f1(sb.to("cuda")))
        l2 = float(f2(sb.to("cuda")))
        assert abs(l1 - l2) <= 1e-6 * max(1.0, abs(l1))
    assert f2.dp is not None
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7, msg=n)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    # exact f32-input MFMA: this test pins the averaging protocol against the oracle's
    # trajectory at lr 1e-2, where Adam turns 1e-5-relative GEMM differences on
    # near-zero gradient components into +-lr steps
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GTR_GEMM="f32")
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = small_data()
        T = data.table_rows
        m, _ = make_pair(T, D, H, K=0, seed=23)
        m.train()
        f = FusedTrainStep(m, lr=1e-2, weight_decay=1e-2, loss="bpr")
        assert f.data_parallel and f.world == world
        bl = batches(data, B, NNEG, STEPS * world, seed=24)
        losses = [float(f(bl[s * world + rank].to("cuda"))) for s in range(STEPS)]
        q.put((rank, losses, {n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()}))
    finally:
        dist.destroy_process_group()


def test_dp_two_ranks_match_oracle_average():
    import etpgt_ref as R

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for item in collect(q, procs, world):
            rank, losses, params = item
            res[rank] = (losses, {k: torch.from_numpy(v) for k, v in params.items()})
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for k, v in res[0][1].items():
        assert torch.equal(v, res[1][1][k]), f"replicas diverged: {k}"
    # oracle: per step, each rank's batch through its own BatchNorm statistics, the
    # gradients averaged, one AdamW step
    data = small_data()
    T = data.table_rows
    _, ref = make_pair(T, D, H, K=0, seed=23)
    lr = 1e-2
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=lr, weight_decay=1e-2))
    bl = batches(data, B, NNEG, STEPS * world, seed=24)
    for s in range(STEPS):
        rbs = [ref_batch(bl[s * world + r]) for r in range(world)]

        def dp_step(model, opt):
            gsum, ls = {}, []
            for rb in rbs:
                model.train()
                model.zero_grad()
                se = model(rb)
                loss = R.ref_loss("bpr", se, rb.target_item, rb.negative_items.view(B, NNEG), model.item_embedding)
                loss.backward()
                ls.append(float(loss))
                for n, p in model.named_parameters():
                    gsum[n] = gsum.get(n, 0) + p.grad.clone()
            for n, p in model.named_parameters():
                p.grad = gsum[n] / world
            opt.step()
            return sum(ls) / world

        lavg = trio.step(dp_step)
        assert abs(res[0][0][s] - lavg) <= 1e-3 * abs(lavg)
    # every parameter ELEMENTWISE against the oracle trio (fp32 / fp32 one thread / fp64)
    trio.compare(res[0][1], lr=lr)


def _concat(b0, b1):
    """The global batch: b0's sessions then b1's (PyG Batch.from_data_list order)."""
    from etpgt.data.batch import SessionBatch

    n0 = b0.num_nodes
    return SessionBatch(torch.cat([b0.x, b1.x]), torch.cat([b0.edge_index, b1.edge_index + n0], dim=1),
                        torch.cat([b0.batch, b1.batch + b0.num_graphs]),
                        torch.cat([b0.target_item, b1.target_item]),
                        torch.cat([b0.negative_items.reshape(-1), b1.negative_items.reshape(-1)]),
                        num_graphs=b0.num_graphs + b1.num_graphs)


def _sync_worker(rank, world, port, q, split="0"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GTR_SPLIT=split)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = small_data()
        T = data.table_rows
        m, _ = make_pair(T, D, H, K=0, seed=25)
        m.train()
        f = FusedTrainStep(m, lr=1e-2, weight_decay=1e-2, loss="listwise", sync_bn=True)
        assert f.data_parallel and f.world == world and f.sync_bn
        bl = batches(data, B, NNEG, STEPS * world, seed=26)
        losses = [float(f(bl[s * world + rank].to("cuda"))) for s in range(STEPS)]
        assert f.split == (split == "1")
        bufs = {n: b.detach().cpu().numpy().copy() for n, b in m.named_buffers() if "running" in n}
        q.put((rank, losses, {n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()}, bufs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("split", ["0", "1"])
def test_sync_bn_two_ranks_equal_one_gpu_on_the_global_batch(split, monkeypatch):
    """SyncBN data parallel (2 ranks sharing the GPU, gloo transport for the partials and
    the gradient packs) trains exactly like the single-GPU fused step on the
    concatenated global batch: same losses, parameters and BatchNorm running stats up to
    reduction order -- on the fused layer kernels (every row group's partials gathered)
    and on the split path (split = "1": one merged row per rank and BatchNorm,
    gtr_config.split_sync)."""
    monkeypatch.setenv("GTR_SPLIT", split)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sync_worker, args=(r, world, port, q, split)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for item in collect(q, procs, world):
            rank, losses, params, bufs = item
            res[rank] = (losses, params, bufs)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for k, v in res[0][1].items():
        assert np.array_equal(v, res[1][1][k]), f"replicas diverged: {k}"
    data = small_data()
    T = data.table_rows
    m, ref = make_pair(T, D, H, K=0, seed=25)
    m.train()
    ref.train()
    f = FusedTrainStep(m, lr=1e-2, weight_decay=1e-2, loss="listwise")
    bl = batches(data, B, NNEG, STEPS * world, seed=26)
    # the CPU oracle trains on the concatenated global batch (one-GPU semantics: BatchNorm
    # over all 2 x B sessions) -- the parameters and running statistics of rank 0 are held
    # to it ELEMENTWISE (gpu_helpers.close_trained); the single-GPU HIP step on the same
    # global batch gives the loss trajectory to 1e-5
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=1e-2))
    for s in range(STEPS):
        gb = _concat(bl[s * world], bl[s * world + 1])
        g = float(f(gb.to("cuda")))
        avg = (res[0][0][s] + res[1][0][s]) / 2
        assert abs(g - avg) <= 1e-5 * max(1.0, abs(g)), (s, g, res[0][0][s], res[1][0][s])
        rb = ref_batch(gb)
        lo = trio.step(lambda mod, o: R.ref_train_step(mod, rb, o, "listwise"))
        assert abs(avg - float(lo)) <= 1e-3 * abs(float(lo)), (s, avg, float(lo))
    trio.compare({n: torch.from_numpy(v) for n, v in res[0][1].items()}, lr=1e-2)
    b64 = dict(trio.ref64.named_buffers())
    b1 = dict(trio.ref1.named_buffers())
    for n, b in trio.ref.named_buffers():
        if "running" in n:  # SyncBN: statistics over the global batch
            close_trained(torch.from_numpy(res[0][2][n]), b, b64[n], torch.zeros_like(b, dtype=torch.bool), 0.0, n,
                          b1[n])


def _lagged_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = small_data()
        T = data.table_rows
        m1, _ = make_pair(T, D, H, K=0, seed=27)
        m2 = copy.deepcopy(m1)
        m1.train(); m2.train()
        f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss="bpr")
        f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss="bpr", lagged=True)
        bl = batches(data, B, NNEG, 6 * world, seed=28)
        for s in range(6):
            l1 = float(f1(bl[s * world + rank].to("cuda")))
            l2 = float(f2(bl[s * world + rank].to("cuda")))
            assert l1 == l2, (s, l1, l2)
        assert f2.sweep is not None and f2.sweep.lag == 1
        f2.flush()
        same = all(torch.equal(a, b) for a, b in zip(m1.parameters(), m2.parameters()))
        same = same and torch.equal(f1.m_tab, f2.m_tab) and torch.equal(f1.v_tab, f2.v_tab)
        q.put((rank, same, {n: p.detach().cpu().numpy().copy() for n, p in m2.named_parameters()}))
    finally:
        dist.destroy_process_group()


def test_dp_lagged_sweep_two_ranks_bitwise_equals_eager_dp():
    """Data parallel with the lagged sweep (each rank's chain sweeps the previous step's
    untouched rows; the union's rows are updated by gtr_dp_tail): on 2 ranks sharing the
    GPU it equals the eager data-parallel step bit for bit, and the replicas agree."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lagged_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for item in collect(q, procs, world):
            rank, same, params = item
            res[rank] = (same, params)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert res[0][0] and res[1][0]
    for k, v in res[0][1].items():
        assert np.array_equal(v, res[1][1][k]), f"replicas diverged: {k}"


def _rccl_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GTR_GRAPH_COLL="1")
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        data = small_data()
        T = data.table_rows
        m1, _ = make_pair(T, D, H, K=0, seed=29)
        m2 = copy.deepcopy(m1)
        m1.train(); m2.train()
        f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss="bpr")
        f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss="bpr", data_parallel=True, lagged=True)
        out = []
        for sb in batches(data, B, NNEG, 5, seed=30):
            out.append((float(f1(sb.to("cuda"))), float(f2(sb.to("cuda")))))
        f2.flush()
        ok_graph = f2._graph_collectives() and len(f2.graph) == 1
        diff = max(float((a - b).abs().max()) for a, b in zip(m1.parameters(), m2.parameters()))
        q.put((out, ok_graph, diff))
    finally:
        dist.destroy_process_group()


def test_dp_rccl_world1_graph_captured_collectives():
    """The RCCL transport (nccl backend, one rank): the data-parallel step with its
    all-gather captured inside the step's hipGraph and the lagged sweep equals the
    single-GPU fused step."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        out, ok_graph, diff = collect(q, [p], 1, 300)[0]
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0
    assert ok_graph
    for l1, l2 in out:
        assert abs(l1 - l2) <= 1e-6 * max(1.0, abs(l1))
    assert diff <= 1e-6


def _refuse_worker(port, q):
    # GTR_DP_NOALIAS: the one-rank all-gather stays a real RCCL collective (by default one
    # rank aliases the exchange and the step has no collective to refuse)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GTR_GRAPH_COLL="1", GTR_DP_NOALIAS="1")
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        data = small_data()
        T = data.table_rows
        m1, _ = make_pair(T, D, H, K=0, seed=31)
        m2 = copy.deepcopy(m1)
        m1.train(); m2.train()
        f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss="bpr", data_parallel=True, lagged=True)
        f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss="bpr", data_parallel=True, lagged=True)
        real = f2._capture
        calls = {"n": 0}

        def refuse_once(fn):
            calls["n"] += 1
            if calls["n"] == 1:
                raise RuntimeError("operation not permitted when stream is capturing")
            return real(fn)

        f2._capture = refuse_once
        out = []
        for sb in batches(data, B, NNEG, 4, seed=32):
            out.append((float(f1(sb.to("cuda"))), float(f2(sb.to("cuda")))))
        f1.flush(); f2.flush()
        same = all(torch.equal(a, b) for a, b in zip(m1.parameters(), m2.parameters()))
        q.put((out, same, f2._coll_capture_refused, len(f2.graph), f1._graph_collectives(),
               os.environ.get("GTR_GRAPH_COLL")))
    finally:
        dist.destroy_process_group()


def test_collective_capture_refusal_falls_back_per_instance():
    """A transport that refuses stream capture of the collectives: that step object falls
    back to one graph per piece (same numbers), without touching the environment or any
    other step object in the process."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_refuse_worker, args=(_free_port(), q))
    p.start()
    try:
        out, same, refused, pieces, other_captures, env = collect(q, [p], 1, 300)[0]
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0
    assert refused and pieces == 2
    assert other_captures and env == "1"
    assert same
    for l1, l2 in out:
        assert l1 == l2


def _resident_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from etpgt.data.batch import Caps

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = small_data()
        T = data.table_rows
        m1, _ = make_pair(T, D, H, K=0, dropout=0.1, seed=31)
        m2 = copy.deepcopy(m1)
        m1.train(); m2.train()
        bl = batches(data, B, NNEG, 3 * world, seed=32)[rank::world]
        caps = Caps(max(b.num_nodes for b in bl) * 2, B, max(b.num_edges for b in bl) * 2, NNEG)
        f1 = FusedTrainStep(m1, loss="bpr", caps=caps, data_parallel=True, lagged=True)
        f2 = FusedTrainStep(m2, loss="bpr", caps=caps, data_parallel=True, lagged=True)
        staged = [torch.from_numpy(b.packed(f2.caps)[1]).cuda() for b in bl]
        f2.bind_resident(staged)
        same = True
        for i in [0, 1, 2, 1, 0]:
            same = same and float(f1(bl[i].to("cuda"))) == float(f2.run_resident(i))
        f1.flush()
        f2.flush()
        same = same and all(torch.equal(a, b) for a, b in zip(m1.parameters(), m2.parameters()))
        q.put((rank, same))
    finally:
        dist.destroy_process_group()


def test_dp_resident_images_equal_copied_blob():
    """The data-parallel step (2 ranks sharing the GPU over gloo, lagged sweep, dropout on)
    launched on resident batch images (bind_resident / run_resident: one graph per image,
    no copy into the step's blob; bench.py's default at N > 1) trains bit for bit like
    load + run, images reused included."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_resident_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(collect(q, procs, world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert res[0] and res[1]


def _multi_worker(port, q):
    # a real one-rank RCCL all-gather captured in the step graph (GTR_DP_NOALIAS)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GTR_GRAPH_COLL="1", GTR_DP_NOALIAS="1")
    import torch.distributed as dist

    from etpgt.data.batch import Caps

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        data = small_data()
        T = data.table_rows
        m1, _ = make_pair(T, D, H, K=0, seed=33)
        m2 = copy.deepcopy(m1)
        m1.train(); m2.train()
        bl = batches(data, B, NNEG, 3, seed=34)
        caps = Caps(max(b.num_nodes for b in bl), B, max(b.num_edges for b in bl), NNEG)
        f1 = FusedTrainStep(m1, lr=1e-2, weight_decay=1e-2, loss="bpr", data_parallel=True, lagged=True, caps=caps)
        f2 = FusedTrainStep(m2, lr=1e-2, weight_decay=1e-2, loss="bpr", data_parallel=True, lagged=True, caps=caps)
        st1 = [torch.from_numpy(b.packed(f1.caps)[1]).cuda() for b in bl]
        st2 = [torch.from_numpy(b.packed(f2.caps)[1]).cuda() for b in bl]
        for i in range(2):  # eager first touch + per-step graph capture, both objects
            f1.load_blob(st1[i]); l1 = float(f1.run())
            f2.load_blob(st2[i]); l2 = float(f2.run())
            assert l1 == l2
        h = f2.capture_steps_copied(st2, 2, 4)  # images 2, 0, 1, 2
        out = []
        for rep in range(3):
            for k in range(4):
                f1.load_blob(st1[(2 + k) % 3])
                l1 = float(f1.run())
            out.append((l1, float(f2.run_steps(h))))
        f1.flush(); f2.flush()
        same = all(torch.equal(a, b) for a, b in zip(m1.parameters(), m2.parameters()))
        q.put((out, same, h is not None, f1.steps, f2.steps))
    finally:
        dist.destroy_process_group()


def test_dp_multi_step_graph_equals_per_step_launches():
    """bench.py's data-parallel timed loop at N > 1 (collectives inside the step graph):
    K image copies + steps captured as ONE hipGraph (capture_steps_copied) train bit for
    bit like K load_blob + run calls, over RCCL with one rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_multi_worker, args=(_free_port(), q))
    p.start()
    try:
        out, same, captured, s1, s2 = collect(q, [p], 1, 300)[0]
    finally:
        p.join(timeout=60)
    assert p.exitcode == 0
    assert captured and s1 == s2 == 14
    for l1, l2 in out:
        assert l1 == l2
    assert same


def _shard_multi_worker(port, q, two_class=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GTR_GRAPH_COLL="1")
    import torch.distributed as dist

    from etpgt.data.batch import Caps

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        data = small_data()
        T = data.table_rows
        m1, _ = make_pair(T, D, H, K=0, seed=35)
        m2 = copy.deepcopy(m1)
        m1.train(); m2.train()
        bl = batches(data, B, NNEG, 3, seed=36)
        caps = Caps(max(b.num_nodes for b in bl), B, max(b.num_edges for b in bl), NNEG)
        kw = dict(lr=1e-2, weight_decay=1e-2, loss="bpr", shard_table=True, sync_bn=True, caps=caps)
        f1 = FusedTrainStep(m1, **kw)
        if two_class:  # f2: two row classes, real RCCL copies, overlapped with forked compute
            os.environ.update(GTR_SHARD_SPLIT="1", GTR_SHARD_NOALIAS="1")
        f2 = FusedTrainStep(m2, **kw)
        os.environ.pop("GTR_SHARD_SPLIT", None)
        os.environ.pop("GTR_SHARD_NOALIAS", None)
        if two_class:
            assert f2.shard.cap_s > 0 and f2.shard.can_overlap and not f2.shard.alias
            assert f1.shard.cap_s == 0 and f1.shard.alias
        st1 = [torch.from_numpy(b.packed(f1.caps)[1]).cuda() for b in bl]
        st2 = [torch.from_numpy(b.packed(f2.caps)[1]).cuda() for b in bl]
        for i in range(2):
            f1.load_blob(st1[i]); l1 = float(f1.run())
            f2.load_blob(st2[i]); l2 = float(f2.run())
            assert l1 == l2
        h = f2.capture_steps_copied(st2, 2, 4, reserve=12)
        out = []
        for rep in range(3):
            for k in range(4):
                f1.load_blob(st1[(2 + k) % 3])
                l1 = float(f1.run())
            out.append((l1, float(f2.run_steps(h))))
        f1.sync_table(); f2.sync_table()
        same = all(torch.equal(a, b) for a, b in zip(m1.parameters(), m2.parameters()))
        q.put((out, same, h is not None, f1.steps, f2.steps))
        # the graphs that captured RCCL collectives pin the communicator: release them, or
        # destroy_process_group() below never returns (scripts/dbg/teardown_probe.py)
        h = None
        f1.close()
        f2.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("two_class", [False, True])
def test_sharded_multi_step_graph_equals_per_step_launches(two_class):
    """The strong-scaling legs' row-sharded step (all-to-alls and SyncBN gathers inside the
    step graph) as ONE multi-step hipGraph equals per-step launches bit for bit, over RCCL
    with one rank.  two_class: the second step exchanges its rows in two classes -- the
    scoring-only rows' all-to-all beside the forward (forked onto a compute stream), the
    gradient rows' beside the weight gradients (include/gtr.h gtr_shard) -- with real RCCL
    copies (no aliasing at one rank): bitwise the one-class step."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_shard_multi_worker, args=(_free_port(), q, two_class))
    p.start()
    try:
        out, same, captured, s1, s2 = collect(q, [p], 1, 300)[0]
    finally:
        p.join(timeout=60)
        if p.exitcode is None:  # the worker we started, stuck in teardown: fail, do not hang
            p.kill()
            p.join(10)
    assert p.exitcode == 0, f"worker exit code {p.exitcode} (teardown)"
    assert captured and s1 == s2 == 14
    for l1, l2 in out:
        assert l1 == l2
    assert same
    assert p.exitcode == 0
