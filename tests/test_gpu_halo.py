"""GPU: the halo step (etpgt.train.halo.HaloTrainStep) -- destination-range cuts that
split sessions, K / V rows of cross-cut sources fetched per layer and their dK / dV
returned, the straddling sessions read out by the rank of their first node.

2 and 4 ranks share the GPU over gloo; every rank steps the SAME global batches with
equal-node cuts (which split sessions: checked).  Against the single-GPU step on the
global batch (split layer path, GTR_SPLIT=1) the ranks must agree with each other bit for
bit and with the single GPU up to the order of the cross-rank sums: per-step losses to
1e-5 and every parameter tensor to 1e-4 in norm.  Against the CPU oracle trainer on the
global batch: losses to 1e-3, and every trained parameter ELEMENTWISE by the repository's
trained-parameter rule (gpu_helpers.close_trained: 1e-3 relative to the fp32 oracle, or
within the fp32 oracle's own distance to its fp64 replay where Adam turns a nearly
cancelling gradient's rounding into a visible update difference)."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

import etpgt_ref as R  # noqa: E402
from gpu_helpers import OracleTrio, batches, collect, make_pair, small_data  # noqa: E402

CASES = [  # (D, H, K, loss, B global, steps)
    (64, 2, 0, "listwise", 64, 3),
    (128, 4, 16, "bpr", 48, 3),
]
LR = 1e-2


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q, case):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.pop("GTR_ATTN", None)
    import torch.distributed as dist

    from etpgt.train.halo import HaloTrainStep

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        D, H, K, loss, B, steps = CASES[case]
        data = small_data()
        m, _ = make_pair(data.table_rows, D, H, K=K, seed=71)
        m.train()
        f = HaloTrainStep(m, lr=LR, weight_decay=1e-2, loss=loss)
        n = 100 if loss != "bpr" else 5
        losses, ghosts = [], []
        for sb in batches(data, B, n, steps, seed=72):
            losses.append(float(f(sb)))
            ghosts.append(f.halo.ghost_rows)
        assert f.split and f.world == world
        params = {k: v.detach().cpu().numpy() for k, v in m.named_parameters()}
        bufs = {k: v.detach().cpu().numpy() for k, v in m.named_buffers() if "running" in k}
        q.put((rank, losses, ghosts, params, bufs))
    finally:
        dist.destroy_process_group()


def _single(case, monkeypatch):
    """The single-GPU step on the global batches (split layer path) and the oracle trio."""
    from etpgt.train.fused import FusedTrainStep

    D, H, K, loss, B, steps = CASES[case]
    monkeypatch.setenv("GTR_SPLIT", "1")
    monkeypatch.delenv("GTR_ATTN", raising=False)
    data = small_data()
    m, ref = make_pair(data.table_rows, D, H, K=K, seed=71)
    if K > 0:
        ref.laplacian_pe._cached_pe = m.laplacian_pe._cached_pe.cpu().clone()
    m.train()
    ref.train()
    f = FusedTrainStep(m, lr=LR, weight_decay=1e-2, loss=loss, use_graph=False)
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=LR, weight_decay=1e-2))
    n = 100 if loss != "bpr" else 5
    losses, rlosses = [], []
    for sb in batches(data, B, n, steps, seed=72):
        losses.append(float(f(sb.to("cuda"))))
        rb = R.ref_batch_from(sb)
        rlosses.append(trio.step(lambda model, opt, rb=rb: float(R.ref_train_step(model, rb, opt, loss))))
    assert f.split
    return m, trio, losses, rlosses


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("case", [0, 1])
def test_halo_ranks_train_like_one_gpu(world, case, monkeypatch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for item in collect(q, procs, world):
            res[item[0]] = item[1:]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in range(1, world):  # replicas bit-identical
        assert res[r][0] == res[0][0]
        for k, v in res[0][2].items():
            assert np.array_equal(v, res[r][2][k]), f"replicas diverged: {k}"
    assert any(g > 0 for r in range(world) for g in res[r][1]), "the cuts split no session"
    m, trio, losses, rlosses = _single(case, monkeypatch)
    steps = len(losses)
    for s in range(steps):
        assert abs(res[0][0][s] - losses[s]) <= 1e-5 * max(1.0, abs(losses[s])), (s, res[0][0][s], losses[s])
        assert abs(res[0][0][s] - rlosses[s]) <= 1e-3 * abs(rlosses[s]), (s, res[0][0][s], rlosses[s])
    hip = {n: torch.from_numpy(v) for n, v in res[0][2].items()}
    for n, p in m.named_parameters():
        a, b = hip[n], p.detach().cpu()
        if not n.endswith("lin_key.bias"):  # exactly-zero gradient: Adam-amplified noise on both
            assert float((a - b).norm()) <= 1e-4 * float(b.norm()), n
    trio.compare(hip, LR)
    for n, b in m.named_buffers():
        if "running" in n:
            a = torch.from_numpy(res[0][3][n])
            assert torch.allclose(a, b.detach().cpu(), rtol=1e-4, atol=1e-6), n
