"""Data-parallel protocol on CPU (gloo, world size 2): the gradient pack / all-gather /
rank-average of etpgt.train.distributed, driven with the oracle's autograd gradients,
equals one AdamW step on the averaged gradients, and the replicas stay identical.
(The device kernels of the same protocol: tests/test_gpu_parity.py::test_dp_*.)"""

from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

T, D, H, L_, B, NNEG = 300, 32, 2, 2, 8, 5


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _model():
    import etpgt_ref as R

    torch.manual_seed(0)
    return R.ref_create_graph_transformer_optimized(T, embedding_dim=D, hidden_dim=D, num_layers=L_, num_heads=H,
                                                    dropout=0.0, use_laplacian_pe=False)


def _batches(world):
    from etpgt.data.synthetic import make_batches, make_sessions_and_graph

    data = make_sessions_and_graph(num_items=T, num_sessions=500, num_edges=1500, seed=3)
    return make_batches(data, B, world, NNEG, seed=7)


def _grads(model, sb):
    """Forward + loss + backward of one rank's batch (trainer.py:80-122, BPR)."""
    import etpgt_ref as R

    rb = R.ref_batch_from(sb)
    model.train()
    model.zero_grad()
    se = model(rb)
    loss = R.ref_loss("bpr", se, rb.target_item, rb.negative_items.view(B, NNEG), model.item_embedding)
    loss.backward()
    return loss.detach()


def _flat_grad(model, layout):
    from etpgt.backend.engine import model_param_map

    flat = torch.zeros(layout.total)
    for name, p, row in model_param_map(model):
        s = layout.seg(name)
        start = s.begin + row * (D if name.endswith("w_all") else 1)
        flat[start: start + p.numel()] = p.grad.reshape(-1)
    return flat


def _set_grads(model, layout, flat, rows):
    from etpgt.backend.engine import model_param_map

    for name, p, row in model_param_map(model):
        s = layout.seg(name)
        start = s.begin + row * (D if name.endswith("w_all") else 1)
        p.grad = flat[start: start + p.numel()].view(p.shape).clone()
    g = torch.zeros(T, D)
    for k, v in rows.items():
        g[k] = v
    model.item_embedding.weight.grad = g


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from etpgt.backend.engine import ParamLayout
    from etpgt.train import distributed as DP

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model()
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=1e-2)
        layout = ParamLayout(D, L_, 0)
        sb = _batches(world)[rank]
        m_cap = 64 + B * (1 + NNEG) + 64
        lay = DP.DpLayout(layout.total, m_cap, D, world)
        loss = _grads(model, sb)
        keys = torch.cat([torch.as_tensor(sb.x), torch.as_tensor(sb.target_item),
                          torch.as_tensor(sb.negative_items).reshape(-1)])
        pack = DP.pack_reference(lay, _flat_grad(model, layout), float(loss), model.item_embedding.weight.grad,
                                 keys, T)
        recv = torch.zeros(world, lay.words)
        DP.all_gather_packs(recv, pack)
        flat, rows, loss_avg = DP.combine_reference(lay, recv, T)
        _set_grads(model, layout, flat, rows)
        opt.step()
        # numpy payload: tensors would travel as shared-memory handles that die with the process
        q.put((rank, loss_avg, {k: v.detach().numpy().copy() for k, v in model.state_dict().items()}))
    finally:
        dist.destroy_process_group()


def test_dp_protocol_matches_averaged_step():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, loss, state = q.get(timeout=240)
        res[rank] = (loss, {k: torch.from_numpy(v) for k, v in state.items()})
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # replicas identical (parameters; BatchNorm running statistics are rank-local, as in
    # DistributedDataParallel without SyncBatchNorm / buffer broadcast)
    is_buffer = lambda k: "running_" in k or "num_batches" in k  # noqa: E731
    for k, v in res[0][1].items():
        if not is_buffer(k):
            assert torch.equal(v, res[1][1][k]), k
    # single process: average of the two ranks' gradients, one AdamW step
    model = _model()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=1e-2)
    bl = _batches(world)
    gsum = {}
    losses = []
    for sb in bl:
        losses.append(float(_grads(model, sb)))
        for n, p in model.named_parameters():
            gsum[n] = gsum.get(n, 0) + p.grad.clone()
    for n, p in model.named_parameters():
        p.grad = gsum[n] / world
    opt.step()
    assert abs(res[0][0] - sum(losses) / world) < 1e-6
    for k, v in model.state_dict().items():
        if not is_buffer(k):
            torch.testing.assert_close(res[0][1][k], v, rtol=1e-5, atol=1e-6, msg=k)


def test_dp_layout_is_aligned_and_packed():
    from etpgt.train.distributed import DpLayout

    for F, m, d, w in ((34000, 342, 64, 8), (1, 1, 32, 1), (133123, 3382, 128, 2)):
        lay = DpLayout(F, m, d, w)
        assert lay.loss_off == F and lay.keys_off == F + 1
        assert lay.rows_off % 4 == 0 and lay.rows_off >= lay.keys_off + m
        assert lay.words % 4 == 0 and lay.words >= lay.rows_off + m * d
        s = lay.struct()
        assert (s.flat_total, s.loss_off, s.keys_off, s.rows_off, s.words, s.m_cap, s.world) == (
            F, lay.loss_off, lay.keys_off, lay.rows_off, lay.words, m, w)


# ---- row-sharded table protocol (etpgt.train.sharded) on CPU ------------------------------
def _route_reference(keys: torch.Tensor, T: int, P: int, cap: int) -> torch.Tensor:
    """send_ids [P][cap] of gtr_shard_route: the distinct rows of a batch per owner r % P,
    ascending, count in slot 0."""
    out = torch.zeros(P, cap, dtype=torch.int32)
    u = torch.unique(keys[(keys >= 0) & (keys < T)])
    for q in range(P):
        mine = u[u % P == q]
        assert mine.numel() <= cap - 1
        out[q, 0] = mine.numel()
        out[q, 1 : 1 + mine.numel()] = mine.to(torch.int32)
    return out


def _shard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from etpgt.train.distributed import all_to_all
    from etpgt.train.sharded import shard_capacity

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model()
        sb = _batches(world)[rank]
        _grads(model, sb)
        tab_grad = model.item_embedding.weight.grad
        keys = torch.cat([sb.x.reshape(-1), sb.target_item.reshape(-1), sb.negative_items.reshape(-1)])
        m_cap = torch.tensor([keys.numel()])
        dist.all_reduce(m_cap, op=dist.ReduceOp.MAX)  # the ranks bind equal capacities (FusedTrainStep._agree)
        cap = shard_capacity(int(m_cap), T, world)
        send_ids = _route_reference(keys, T, world, cap)
        recv_ids = torch.zeros_like(send_ids)
        all_to_all(recv_ids, send_ids)
        # requester: the summed gradient row of each requested row, at its slot
        send_g = torch.zeros(world, cap, D)
        for o in range(world):
            for j in range(1, int(send_ids[o, 0]) + 1):
                send_g[o, j] = tab_grad[int(send_ids[o, j])]
        recv_g = torch.zeros_like(send_g)
        all_to_all(recv_g, send_g)
        # owner: rank-ordered sum / P of every requested row it owns
        got = {}
        for r in range(world):
            for j in range(1, int(recv_ids[r, 0]) + 1):
                k = int(recv_ids[r, j])
                assert k % world == rank
                got[k] = got.get(k, torch.zeros(D)) + recv_g[r, j]
        q.put((rank, {k: (v / world).numpy() for k, v in got.items()}, tab_grad.numpy()))
    finally:
        dist.destroy_process_group()


def test_shard_protocol_routes_rows_to_owners_and_averages():
    """gloo world 2: the all-to-all route of requested rows to their owners (r % P) and the
    owners' rank-ordered average equal the dense averaged table gradient on every touched
    row, each row updated by exactly one owner."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, got, g = q.get(timeout=300)
            res[rank] = (got, g)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    dense = (torch.from_numpy(res[0][1]) + torch.from_numpy(res[1][1])) / world
    touched = set(res[0][0]) | set(res[1][0])
    assert not (set(res[0][0]) & set(res[1][0]))
    assert touched == set(int(i) for i in torch.nonzero(dense.abs().sum(1)).reshape(-1)) - {0} | (touched & {0})
    for rank in range(world):
        for k, v in res[rank][0].items():
            torch.testing.assert_close(torch.from_numpy(v), dense[k], rtol=1e-6, atol=1e-7)


def test_shard_capacity_bounds():
    from etpgt.train.sharded import shard_capacity

    assert shard_capacity(1000, 300, 2) == 1 + 150            # exact bound: the owner's 150 rows
    assert shard_capacity(100, 10**6, 8) == 1 + 19 + 64       # 1.5 x the even share + 64 ...
    assert shard_capacity(40, 10**6, 8) == 1 + 40             # ... never above the batch's rows
    assert shard_capacity(107_000, 10**6, 8, slack=1.5) == 1 + 20_063 + 64  # 1.5 x the even share


def test_block_rows_counts_distinct_rows_per_owner_and_class():
    """block_rows (the fitted exchange blocks): per batch, the distinct rows of each owner
    (r % P) in class 0 (rows a node reads) and class 1 (rows only targets / negatives
    read), maximised over batches and owners -- checked against a brute-force count."""
    import numpy as np

    from etpgt.train.sharded import block_rows

    class B:
        def __init__(self, x, t, n):
            self.x, self.target_item, self.negative_items = torch.tensor(x), torch.tensor(t), torch.tensor(n)

    rng = np.random.default_rng(3)
    bl = [B(rng.integers(1, 200, 30), rng.integers(1, 200, 8), rng.integers(1, 200, (8, 12))) for _ in range(4)]
    for P in (1, 3, 8):
        w0 = w1 = wa = 0
        for b in bl:
            nodes = set(b.x.tolist())
            score = set(b.target_item.tolist()) | set(b.negative_items.reshape(-1).tolist())
            for q in range(P):
                w0 = max(w0, sum(1 for r in nodes if r % P == q))
                w1 = max(w1, sum(1 for r in score - nodes if r % P == q))
                wa = max(wa, sum(1 for r in nodes | score if r % P == q))
        assert block_rows(bl, P, True) == (w0, w1)
        assert block_rows(bl, P, False) == (wa, 0)


def _trainer_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import tempfile

    import torch.distributed as dist

    from etpgt.model import create_graph_transformer
    from etpgt.train import Trainer

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = create_graph_transformer(T, embedding_dim=64, hidden_dim=64)  # use_ffn=True
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
        with tempfile.TemporaryDirectory() as d:
            tr = Trainer(model, [], [], opt, device="cpu", output_dir=d, max_epochs=1)
            try:
                tr.train_epoch()
                q.put((rank, "no error"))
            except RuntimeError as e:
                q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_trainer_refuses_the_autograd_loop_under_data_parallel():
    """under a process group of more than one rank the generic autograd loop
    averages nothing across ranks (the replicas would drift apart), so Trainer raises
    instead of silently training P independent models (here: the FFN variant, which has
    no data-parallel fused step)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert "data-parallel training (2 ranks) needs the fused HIP step" in msgs[r], msgs[r]


def _trainer_sync_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from etpgt.model import create_graph_transformer, create_graph_transformer_optimized
        from etpgt.train.trainer import Trainer

        out = {}
        for name, m in (("opt64", create_graph_transformer_optimized(50, embedding_dim=64, hidden_dim=64)),
                        ("ffn64", create_graph_transformer(50, embedding_dim=64, hidden_dim=64, num_layers=2)),
                        ("ffn256", create_graph_transformer(50)),
                        ("ffn64x2", create_graph_transformer(50, embedding_dim=64, hidden_dim=64, ffn_expansion=2))):
            opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
            tr = Trainer(m, [], [], opt, device="cpu", output_dir=f"/tmp/_tr_sync_{port}_{rank}", max_epochs=1)
            out[name] = tr.sync_bn
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_trainer_sync_bn_default_at_two_ranks():
    """Trainer at world 2: SyncBN by default for the optimized model and for the FFN model
    at d 64 / 128 with expansion 4 (gtr_ffn_fwd folds the gathered rows); per-rank
    BatchNorm statistics for the FFN shapes the SyncBN fold does not cover."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_sync_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in range(world):
        assert res[r] == {"opt64": True, "ffn64": True, "ffn256": False, "ffn64x2": False}, res[r]
