"""GPU: the FFN variant (use_ffn=True, graph_transformer.py:88-100,160-170) trained data
parallel -- two ranks sharing the GPU over a gloo group, with SyncBN (the gathered merged
BatchNorm rows folded by each FFN's first GEMM, gtr_ffn_fwd) against the oracle on the
concatenated global batch, and without SyncBN against the oracle's rank-averaged AdamW
trajectory.  Replicas must stay identical; every trained parameter is held to the oracle
elementwise (gpu_helpers.close_trained through OracleTrio.compare)."""

from __future__ import annotations

import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

from gpu_helpers import OracleTrio, batches, close_trained, collect, ref_batch, small_data  # noqa: E402
import etpgt_ref as R  # noqa: E402

from etpgt.train.fused import FusedTrainStep  # noqa: E402

D, H, STEPS, B, NNEG = 64, 2, 3, 16, 5


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _pair(T, seed):
    from test_gpu_ffn import make_ffn_pair

    return make_ffn_pair(T, D, H, seed=seed)


def _concat(b0, b1):
    from test_gpu_distributed import _concat as cat

    return cat(b0, b1)


def _worker(rank, world, port, q, sync, shard=False):
    # exact f32-input MFMA (the averaging protocol is pinned at lr 1e-2, as test_gpu_distributed)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GTR_GEMM="f32")
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    f = None
    try:
        data = small_data()
        T = data.table_rows
        m, _ = _pair(T, 31)
        m.train()
        f = FusedTrainStep(m, lr=1e-2, weight_decay=1e-2, loss="listwise" if sync else "bpr", sync_bn=sync,
                           shard_table=shard)
        assert f.data_parallel and f.world == world and f.sync_bn == sync
        bl = batches(data, B, NNEG, STEPS * world, seed=32)
        losses = [float(f(bl[s * world + rank].to("cuda"))) for s in range(STEPS)]
        assert f.split  # the FFN blocks run on the split layer path
        assert (f.shard_state is not None) == shard
        f.sync_table()  # row-sharded: the shards back into the model's table (collective)
        bufs = {n: b.detach().cpu().numpy().copy() for n, b in m.named_buffers() if "running" in n}
        q.put((rank, losses, {n: p.detach().cpu().numpy().copy() for n, p in m.named_parameters()}, bufs))
    finally:
        if f is not None:
            f.close()
        dist.destroy_process_group()


def _run(sync, shard=False):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, sync, shard)) for r in range(world)]
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
    return res


@pytest.mark.parametrize("shard", [False, True], ids=["replicated", "row_sharded"])
def test_ffn_sync_bn_two_ranks_equal_oracle_on_the_global_batch(shard):
    """SyncBN: two ranks train the FFN model like one GPU on the concatenated global batch
    (BatchNorm over all 2 x B sessions, the FFN weights among the averaged small
    parameters): losses, every parameter and the running statistics against the oracle.
    ``row_sharded``: the item table and its moments row-sharded across the ranks."""
    world = 2
    res = _run(True, shard)
    data = small_data()
    T = data.table_rows
    _, ref = _pair(T, 31)
    ref.train()
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=1e-2))
    bl = batches(data, B, NNEG, STEPS * world, seed=32)
    for s in range(STEPS):
        rb = ref_batch(_concat(bl[s * world], bl[s * world + 1]))
        lo = trio.step(lambda mod, o: R.ref_train_step(mod, rb, o, "listwise"))
        avg = (res[0][0][s] + res[1][0][s]) / 2
        assert abs(avg - float(lo)) <= 1e-3 * abs(float(lo)), (s, avg, float(lo))
    trio.compare({n: torch.from_numpy(v) for n, v in res[0][1].items()}, lr=1e-2)
    b64 = dict(trio.ref64.named_buffers())
    b1 = dict(trio.ref1.named_buffers())
    for n, b in trio.ref.named_buffers():
        if "running" in n:
            close_trained(torch.from_numpy(res[0][2][n]), b, b64[n], torch.zeros_like(b, dtype=torch.bool), 0.0, n,
                          b1[n])


def test_ffn_dp_two_ranks_match_oracle_average():
    """Without SyncBN (per-rank BatchNorm statistics, torch DDP's default): each rank's
    batch through its own statistics, the gradients averaged, one AdamW step."""
    world = 2
    res = _run(False)
    data = small_data()
    T = data.table_rows
    _, ref = _pair(T, 31)
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=1e-2))
    bl = batches(data, B, NNEG, STEPS * world, seed=32)
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
        assert abs(res[0][0][s] - lavg) <= 1e-3 * abs(lavg), (s, res[0][0][s], lavg)
    trio.compare({n: torch.from_numpy(v) for n, v in res[0][1].items()}, lr=1e-2)
