"""GPU: configuration C4 (BASELINE.json configs[3]) at its real workload.

C4 is the C3 model -- d = 128, 2 layers, 4 heads, LapPE k = 16, listwise with 100 sampled
negatives -- on the full RetailRocket-shaped table (T = 82,174 rows), trained data
parallel with the item table ROW-SHARDED across the ranks (etpgt.train.sharded: rank p owns
rows r % P == p with their AdamW moments, rows fetched / row gradients returned by
all-to-all) and SyncBN (BatchNorm statistics over the global batch).  Here the ranks share
the one GPU over gloo (world 2 and 4), each on its slice of the same global batches:

* the sharded step equals the replicated data-parallel step (lazy table, SyncBN) BIT FOR
  BIT -- losses, every parameter, the AdamW moments -- and every replica agrees;
* the trained parameters and BatchNorm running statistics match the CPU oracle trainer
  (trainer.py:80-133 + AdamW, train_baseline.py:252-256) run on the CONCATENATED global
  batch ELEMENTWISE at the north star's 1e-3 relative fp32 bar (gpu_helpers.close_trained:
  the fp32 oracle, or within the fp32 oracle's own distance to its fp64 replay).

World 2 runs B = 1024 per rank (the per-rank batch of C4's global 8192 at N = 8; more than
128 row groups, so the split GEMM + attention layer path), world 4 runs B = 512 per rank --
both on the same 2048-session global batches, so one oracle run checks both."""

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

import etpgt_ref as R  # noqa: E402
from gpu_helpers import OracleTrio, assert_close, collect  # noqa: E402

GLOBAL_B = 2048
STEPS = 3
N_NEG = 100
LR = 1e-3
D, H, K = 128, 4, 16


def _data():
    from etpgt.data.synthetic import make_sessions_and_graph

    return make_sessions_and_graph(seed=42)  # the C2 / C3 / C4 RetailRocket shape


def _global_examples(data):
    """STEPS global batches of GLOBAL_B session examples (the bench's seeded shuffle)."""
    from etpgt.data.synthetic import session_example

    rng = np.random.default_rng(301)
    order = np.random.default_rng(300).permutation(data.num_sessions)
    return [[session_example(data, int(s), N_NEG, rng) for s in order[i * GLOBAL_B:(i + 1) * GLOBAL_B]]
            for i in range(STEPS)]


def _model(T):
    from etpgt.data.synthetic import random_pe_table
    from etpgt.model import create_graph_transformer_optimized

    torch.manual_seed(401)
    kw = dict(embedding_dim=D, hidden_dim=D, num_layers=2, num_heads=H, dropout=0.0, use_laplacian_pe=True,
              laplacian_k=K)
    m = create_graph_transformer_optimized(T, **kw)
    m.laplacian_pe._cached_pe = random_pe_table(T, K)
    with torch.no_grad():  # non-trivial BN affine parameters
        for bn in m.batch_norms:
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
    return m, kw


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from etpgt.data.batch import collate_sessions
    from etpgt.train.fused import FusedTrainStep

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = _data()
        T = data.table_rows
        m1, _ = _model(T)
        m2 = copy.deepcopy(m1)
        m1 = m1.cuda().train()
        m2 = m2.cuda().train()
        f1 = FusedTrainStep(m1, lr=LR, weight_decay=1e-5, loss="listwise", lazy=True, sync_bn=True,
                            data_parallel=True)
        f2 = FusedTrainStep(m2, lr=LR, weight_decay=1e-5, loss="listwise", shard_table=True, sync_bn=True)
        Bp = GLOBAL_B // world
        l1s, l2s = [], []
        for ex in _global_examples(data):
            sb = collate_sessions(ex[rank * Bp:(rank + 1) * Bp]).to("cuda")
            l1s.append(float(f1(sb)))
            l2s.append(float(f2(sb)))
        f1.flush()
        f2.sync_table()
        p1 = {n: p.detach() for n, p in m1.named_parameters()}
        p2 = {n: p.detach() for n, p in m2.named_parameters()}
        bad = [n for n in p1 if not torch.equal(p1[n], p2[n])]
        moments = torch.equal(f1.m_tab, f2.m_tab) and torch.equal(f1.v_tab, f2.v_tab)
        info = dict(split=bool(f2.split), world=f2.world, sharded=f2.shard_state is not None,
                    vol=f2.shard.volume())
        params = {n: p.cpu().numpy() for n, p in p2.items()}
        bufs = {n: b.detach().cpu().numpy() for n, b in m2.named_buffers() if "running" in n or "tracked" in n}
        q.put((rank, l1s, l2s, bad, moments, params, bufs, info))
    finally:
        dist.destroy_process_group()


_ORACLE = {}


def _oracle():
    """One oracle run (fp32, fp32 one thread, fp64) on the concatenated global batches."""
    if "trio" in _ORACLE:
        return _ORACLE["trio"]
    from etpgt.data.batch import collate_sessions

    data = _data()
    T = data.table_rows
    m, kw = _model(T)
    ref = R.ref_create_graph_transformer_optimized(T, **kw)
    ref.laplacian_pe._cached_pe = m.laplacian_pe._cached_pe.clone()
    ref.load_state_dict({k: v.detach().clone() for k, v in m.state_dict().items()})
    ref.train()
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=LR, weight_decay=1e-5))
    losses = []
    touched = torch.zeros(T, dtype=torch.bool)
    for ex in _global_examples(data):
        sb = collate_sessions(ex)
        rb = R.ref_batch_from(sb)
        for t in (sb.x, sb.target_item, sb.negative_items):
            touched[t.reshape(-1)] = True

        def fn(model, opt, rb=rb):
            se = model(rb)
            neg = rb.negative_items.view(se.shape[0], -1)
            loss = R.ref_loss("listwise", se, rb.target_item, neg, model.item_embedding)
            opt.zero_grad()
            loss.backward()
            opt.step()
            return float(loss.detach())

        losses.append(trio.step(fn))
    _ORACLE["trio"] = (trio, losses, touched)
    return _ORACLE["trio"]


@pytest.mark.parametrize("world", [2, 4])
def test_c4_sharded_full_table_bitwise_dp_and_matches_oracle(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for item in collect(q, procs, world, timeout=900.0):
            res[item[0]] = item[1:]
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in range(world):
        l1s, l2s, bad, moments, _, _, info = res[r]
        assert l1s == l2s, (r, l1s, l2s)  # sharded == replicated data parallel, bit for bit
        assert not bad, (r, bad)
        assert moments, r
        assert info["world"] == world and info["sharded"]
        if world == 2:  # B = 1024 per rank (C4's per-rank batch at N = 8): the split layer path
            assert info["split"], info
    for r in range(1, world):  # every replica holds the same parameters
        for k, v in res[0][4].items():
            assert np.array_equal(v, res[r][4][k]), f"replicas diverged: {k}"
    print(f"world {world}: exchange volume per step {res[0][6]['vol']}")

    trio, rlosses, touched = _oracle()
    for s in range(STEPS):  # the global loss is the mean of the equal-sized rank losses
        g = sum(res[r][0][s] for r in range(world)) / world
        print(f"step {s}: loss {g:.7f} oracle {rlosses[s]:.7f} rel {abs(g - rlosses[s]) / abs(rlosses[s]):.2e}")
        assert abs(g - rlosses[s]) <= 1e-3 * abs(rlosses[s]), (s, g, rlosses[s])
    hip = {n: torch.from_numpy(v) for n, v in res[0][4].items()}
    tab = "item_embedding.weight"
    p64 = dict(trio.ref64.named_parameters())
    p1 = dict(trio.ref1.named_parameters())
    from gpu_helpers import close_trained

    for n, p in trio.ref.named_parameters():
        if n == tab:
            close_trained(hip[n][touched], p.detach()[touched], p64[n].detach()[touched], trio.noise[n][touched],
                          2 * LR * STEPS, f"{n} touched rows ({int(touched.sum())})", p1[n].detach()[touched])
            assert_close(hip[n][~touched], p.detach()[~touched], name=f"{n} untouched rows ({int((~touched).sum())})")
        else:
            close_trained(hip[n], p.detach(), p64[n].detach(), trio.noise[n], 2 * LR * STEPS, n, p1[n].detach())
    b64 = dict(trio.ref64.named_buffers())
    b1 = dict(trio.ref1.named_buffers())
    for n, b in trio.ref.named_buffers():
        if "running" in n:  # SyncBN: statistics over the global batch
            close_trained(torch.from_numpy(res[0][5][n]), b, b64[n], torch.zeros_like(b, dtype=torch.bool), 0.0, n,
                          b1[n])
        if n.endswith("num_batches_tracked"):
            assert int(res[0][5][n]) == STEPS
