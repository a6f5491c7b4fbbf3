"""CPU: the halo cut planner and exchange protocol (etpgt.train.halo), no GPU.

* ``plan_halo`` cuts a global batch at destination-node ranges that split sessions: every
  rank's local + ghost rows reproduce the global graph exactly -- each local destination
  row sees the same in-edges in the same order, with sources resolved through the ghost
  rows; each session is read out by exactly one rank over a contiguous row range holding
  the session's own items; the packed images carry hdr[6] = local + ghost rows.
* ``HaloExchange.fetch`` / ``give_back`` over a 2- and 3-rank gloo group on CPU tensors:
  ghost slots receive their owners' rows; ghost gradients come back and are added to the
  owners' rows (readout rows assigned)."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from etpgt.data.batch import blob_layout
from etpgt.data.synthetic import make_batches, make_sessions_and_graph
from etpgt.train.halo import HaloExchange, halo_caps, pack_halo, plan_halo


def _batch(B=48, seed=5):
    data = make_sessions_and_graph(num_items=400, num_sessions=2000, num_edges=6000, seed=seed)
    return make_batches(data, B, 1, 5, seed=seed)[0]


@pytest.mark.parametrize("world", [2, 3, 4])
def test_cut_reproduces_the_global_graph(world):
    sb = _batch()
    N, B, E, n_neg = sb.sizes()
    parts = plan_halo(sb, world)
    x = sb.x.numpy()
    src, dst = sb.edge_index.numpy()
    ptr = sb.ptr.numpy()
    # destination ranges tile [0, N); the default cuts split sessions
    assert parts[0].lo == 0 and parts[-1].hi == N
    assert all(parts[r].hi == parts[r + 1].lo for r in range(world - 1))
    split = [int(np.searchsorted(ptr, p.lo, side="right")) for p in parts[1:]]
    assert any(ptr[s - 1] != p.lo for s, p in zip(split, parts[1:])), "no cut splits a session"
    owned = []
    for p in parts:
        ext_global = np.concatenate([np.arange(p.lo, p.hi), p.ghosts])
        assert np.array_equal(p.x, x[ext_global])
        # in-edges of every local destination row: the global row's, in the same order
        for t in range(p.n_local):
            g = p.lo + t
            want = src[dst == g]
            got = ext_global[p.in_src[p.in_ptr[t]:p.in_ptr[t + 1]]]
            assert np.array_equal(got, want), (p.rank, t)
        # CSR by source covers the local + ghost rows and lists exactly the local edges
        assert p.out_ptr.shape[0] == p.n_ext + 1 and p.out_ptr[-1] == p.num_edges
        for s in range(p.n_ext):
            e = p.out_edge[p.out_ptr[s]:p.out_ptr[s + 1]]
            assert np.all(p.in_src[e] == s)
        # owned sessions: contiguous local(+ghost) rows holding the session's items
        for k in range(p.num_sessions):
            a, b = p.node_ptr[k], p.node_ptr[k + 1]
            gs = int(np.searchsorted(ptr, p.lo + a, side="right")) - 1
            assert ptr[gs] == p.lo + a and ptr[gs + 1] == p.lo + b
            assert np.array_equal(p.x[a:b], x[ptr[gs]:ptr[gs + 1]])
            owned.append(gs)
        # ghosts never include own rows; the readout tail comes first
        assert not np.any((p.ghosts >= p.lo) & (p.ghosts < p.hi))
        assert np.array_equal(p.ghosts[:p.n_readout], np.arange(p.hi, p.hi + p.n_readout))
    assert sorted(owned) == list(range(B))  # every session read out by exactly one rank
    assert sum(p.num_edges for p in parts) == E
    caps = halo_caps(parts, n_neg)
    for p in parts:
        blob = pack_halo(p, caps)
        o = blob_layout(caps)["hdr"][0]
        assert list(blob[o:o + 7]) == [p.n_local, p.num_sessions, p.num_edges, n_neg,
                                       (p.n_local + caps.R - 1) // caps.R, caps.R, p.n_ext]


def test_cut_rejects_a_rank_without_a_session():
    sb = _batch(B=4)
    N = sb.num_nodes
    ptr = sb.ptr.numpy()
    with pytest.raises(ValueError):
        plan_halo(sb, 2, [0, N, N])
    long = int(np.argmax(np.diff(ptr)))
    if ptr[long + 1] - ptr[long] >= 3:
        with pytest.raises(ValueError, match="owns no session"):
            plan_halo(sb, 3, [0, int(ptr[long]) + 1, int(ptr[long]) + 2, N])


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sb = _batch()
        parts = plan_halo(sb, world)
        me = parts[rank]
        hx = HaloExchange(parts, rank, torch.device("cpu"))
        W = 4
        buf = torch.zeros(me.n_ext, W + 2)
        buf[: me.n_local, 1:W + 1] = torch.arange(me.lo, me.hi, dtype=torch.float32)[:, None] * 10 + torch.arange(W)
        hx.fetch(buf, 1, W + 1)
        want = torch.as_tensor(me.ghosts, dtype=torch.float32)[:, None] * 10 + torch.arange(W)
        ok_fetch = torch.equal(buf[me.n_local:, 1:W + 1], want) and bool((buf[:, 0] == 0).all())
        g = torch.zeros(me.n_ext, W)
        g[me.n_local:] = torch.as_tensor(me.ghosts, dtype=torch.float32)[:, None] + 0.5
        g[: me.n_local] = 1000.0
        hx.give_back(g, 0, W)
        q.put((rank, ok_fetch, g[: me.n_local].numpy(), me.lo, me.hi))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_over_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, ok, g, lo, hi = q.get(timeout=120)
        res[rank] = (ok, g, lo, hi)
    for p in procs:
        p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    parts = plan_halo(_batch(), world)
    for r in range(world):
        ok, g, lo, hi = res[r]
        assert ok, r
        # every owner row: 1000 + (global id + 0.5) once per rank holding it as a ghost
        cnt = np.zeros(hi - lo)
        for p in parts:
            if p.rank != r:
                gh = p.ghosts[(p.ghosts >= lo) & (p.ghosts < hi)]
                np.add.at(cnt, gh - lo, 1)
        want = 1000.0 + cnt[:, None] * (np.arange(lo, hi)[:, None] + 0.5)
        assert np.allclose(g, np.broadcast_to(want, g.shape)), r
