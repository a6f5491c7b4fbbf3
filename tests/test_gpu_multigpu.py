"""GPU: the multi-GPU entry points as the driver and a user reach them.

* ``bench.py --gpus N`` without a launcher starts N ranks itself (torch.distributed.run
  as a child process) and prints ONE line with ``n_gpus == N``; on the one-GPU box the
  ranks share cuda:0 over gloo (GTR_SHARE_DEVICE=1), on an 8-GPU node they are RCCL
  ranks.  The default C2 (replicated data parallel) and the C4 mode (row-sharded table,
  SyncBN, fixed global batch) both report identical replicas.
* ``scripts/train/train_baseline.py`` under a 2-rank process group trains like ONE GPU on
  the global batch (device-built batches sharded per rank, SyncBN, averaged gradients).
"""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - collected only on the GPU box
    pytest.skip("no GPU", allow_module_level=True)

from gpu_helpers import collect  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEAN = ["--cpu-seconds", "0", "--gather-batch", "0", "--recall-steps", "0", "--e2e-steps", "0", "--c1-reps", "0",
        "--tail-probe", "0"]
NO_STRONG = ["--strong-batches", "0"]


def _bench(args, timeout=420):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["GTR_SHARE_DEVICE"] = "1"
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *args, *LEAN], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]  # the bench line is the only stdout line
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    """The default line at N = 2, with its strong-scaling leg: the C4 mode (row-sharded
    table, SyncBN) at a fixed global batch over the same two ranks, launched as a child
    after the main line's process group is gone."""
    out = _bench(["--gpus", "2", "--steps", "4", "--warmup", "2", "--num-batches", "4", "--strong-batches", "512",
                  "--strong-steps", "3"])
    assert out["n_gpus"] == 2
    cfg = out["config"]
    assert cfg["process_group_world"] == 2 and cfg["launcher"].startswith("bench.py --gpus")
    assert cfg["replicas_identical"] is True
    assert cfg["parallelism"] == "dp2" and cfg["global_batch"] == 64 and out["scaling"] == "weak"
    assert out["value"] > 0
    ss = out["strong_scaling"]
    assert ss["config"] == "c4" and ss["n_gpus"] == 2 and len(ss["legs"]) == 1
    leg = ss["legs"][0]
    assert "error" not in leg, leg
    assert leg["global_batch"] == 512 and leg["per_gpu_batch"] == 256 and leg["process_group_world"] == 2
    assert leg["parallelism"] == "dp2+rowshard" and leg["sync_bn"] is True and leg["replicas_identical"] is True
    assert leg["value"] > 0


def test_bench_one_gpu_strong_leg_reports_the_unsharded_step_beside_it():
    out = _bench(["--steps", "3", "--warmup", "1", "--num-batches", "2", "--strong-batches", "256",
                  "--strong-steps", "3"])
    leg = out["strong_scaling"]["legs"][0]
    assert "error" not in leg, leg
    assert leg["parallelism"] == "dp1+rowshard" and leg["process_group_world"] is None
    assert leg["unsharded_single_gpu"]["value"] > 0


def test_bench_c4_gpus2_sharded_strong():
    out = _bench(["--config", "c4", "--gpus", "2", "--global-batch", "512", "--steps", "3", "--warmup", "1",
                  "--num-batches", "2", *NO_STRONG])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    cfg = out["config"]
    assert cfg["global_batch"] == 512 and cfg["per_gpu_batch"] == 256
    assert cfg["parallelism"] == "dp2+rowshard" and cfg["sync_bn"] is True
    assert cfg["replicas_identical"] is True


def test_bench_c4_one_gpu_line():
    """N = 1 of the C4 mode: the same sharded step at world 1 (the curve's first point)."""
    out = _bench(["--config", "c4", "--global-batch", "256", "--steps", "3", "--warmup", "1", "--num-batches", "2",
                  *NO_STRONG])
    assert out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1+rowshard"
    assert out["config"]["process_group_world"] is None


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _script():
    import importlib.util

    spec = importlib.util.spec_from_file_location("train_baseline_cp",
                                                  os.path.join(ROOT, "scripts", "train", "train_baseline.py"))
    tb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tb)
    return tb


EPOCHS = 2


def _args(d, out, B, shard, model="graph_transformer_optimized", dim=32):
    return ["--model", model, "--train-sessions", str(d / "train.csv"),
            "--val-sessions", str(d / "val.csv"), "--graph-edges", str(d / "graph_edges.csv"),
            "--embedding-dim", str(dim), "--hidden-dim", str(dim), "--num-layers", "2", "--num-heads", "2",
            "--dropout", "0", "--batch-size", str(B), "--num-negatives", "5", "--max-epochs", str(EPOCHS),
            "--num-workers", "0", "--output-dir", str(out), "--shard-table", "on" if shard else "off"]


def _rank_main(rank, world, port, d, out, B, q, shard, model="graph_transformer_optimized", dim=32):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), GTR_SHARE_DEVICE="1")
    # main() releases the captured graphs and destroys the process group itself
    tr = _script().main(_args(d, out, B, shard, model, dim))
    import torch.distributed as dist

    assert not dist.is_initialized()
    sd = {k: v.detach().cpu().numpy() for k, v in tr.model.state_dict().items()}
    q.put((rank, tr.history, sd, tr.shard_table, tr._fused.shard_state is not None))


@pytest.mark.parametrize("shard,model", [(False, "graph_transformer_optimized"), (True, "graph_transformer_optimized"),
                                         (False, "graph_transformer"), (True, "graph_transformer")],
                         ids=["replicated", "row_sharded", "ffn_replicated", "ffn_row_sharded"])
def test_train_baseline_two_ranks_match_oracle_on_the_global_batch(tmp_path, shard, model):
    """Two ranks of the drop-in train_baseline.py (SyncBN data parallel, B = 8 per rank,
    sharing the GPU over gloo) for two epochs against the CPU ORACLE replaying them on the
    global batches of 16 sessions (one-GPU semantics): the same initial weights
    (set_seed(42) + the factory), the same epoch orders (per epoch the DataLoader
    iterator's _base_seed and RandomSampler draws; the validation pass between the epochs
    draws one _base_seed), the same per-session examples and position-keyed negatives
    (oracle/batch_ref.py restates the device stream; rank r builds sessions [16 i + 8 r, +8)
    of global batch i).  ``row_sharded``: ``--shard-table on``, the item table and its
    moments row-sharded across the two ranks (SURVEY §8e ii).  ``ffn_replicated``: the
    reference's ``--model graph_transformer`` (use_ffn=True, FFN x 4) at d = 64, SyncBN
    folded by each FFN's first GEMM.  Replicas are bit-identical;
    each epoch's loss and every trained parameter match the oracle ELEMENTWISE
    (gpu_helpers.close_trained), the running statistics too; the ranks leave through
    ``destroy_process_group`` (exit code 0)."""
    import batch_ref as BR
    import etpgt_ref as R

    from dropin_helpers import write_csvs
    from gpu_helpers import OracleTrio, close_trained

    from etpgt.data.batch import collate_sessions
    from etpgt.model import create_graph_transformer, create_graph_transformer_optimized
    from etpgt.train.dataloader import SessionDataset
    from etpgt.utils.seed import set_seed

    d = write_csvs(tmp_path, num_train=150)  # 150 sessions: 9 global batches of 16 + a last one of 6
    world, B, n = 2, 8, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ffn = model == "graph_transformer"
    dim = 64 if ffn else 32  # the FFN kernels cover d 64 / 128 / 256
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, d, tmp_path / "dp", B, q, shard, model, dim))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for item in collect(q, procs, world):
            rank, hist, sd, tr_shard, st_shard = item
            assert tr_shard == st_shard == shard
            res[rank] = (hist, sd)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for k, v in res[0][1].items():
        assert np.array_equal(v, res[1][1][k]), f"replicas diverged: {k}"
    assert os.path.exists(tmp_path / "dp" / model / "history.json")
    hist, sd = res[0]
    # ---- the oracle replays the epoch on the global batches
    tr = SessionDataset(d / "train.csv", d / "graph_edges.csv", n, 50)
    va = SessionDataset(d / "val.csv", d / "graph_edges.csv", n, 50)
    T = max(tr.num_items, va.num_items)
    set_seed(42)
    if ffn:
        init = create_graph_transformer(T, embedding_dim=dim, hidden_dim=dim, num_layers=2, num_heads=2, dropout=0.0,
                                        readout_type="mean", use_laplacian_pe=True)
    else:
        init = create_graph_transformer_optimized(T, embedding_dim=dim, hidden_dim=dim, num_layers=2, num_heads=2,
                                                  dropout=0.0, use_laplacian_pe=True, use_ffn=False, ffn_expansion=2)
    orders = []
    for e in range(EPOCHS):
        if e > 0:
            torch.empty((), dtype=torch.int64).random_()  # the validation pass's iterator (shuffle=False)
        torch.empty((), dtype=torch.int64).random_()  # the epoch iterator's _base_seed draw
        seed = int(torch.empty((), dtype=torch.int64).random_().item())  # the epoch's RandomSampler draw
        g = torch.Generator()
        g.manual_seed(seed)
        orders.append(torch.randperm(len(tr), generator=g).numpy())
    if ffn:
        ref = R.RefGraphTransformer(T, embedding_dim=dim, hidden_dim=dim, num_layers=2, num_heads=2, dropout=0.0,
                                    use_laplacian_pe=True, use_ffn=True, ffn_expansion=4)
    else:
        ref = R.ref_create_graph_transformer_optimized(T, embedding_dim=dim, hidden_dim=dim, num_layers=2,
                                                       num_heads=2, dropout=0.0, use_laplacian_pe=True)
    isd = {k: v.clone() for k, v in init.state_dict().items()}
    isd["laplacian_pe._cached_pe"] = torch.from_numpy(sd["laplacian_pe._cached_pe"]).clone()
    ref.laplacian_pe._cached_pe = isd["laplacian_pe._cached_pe"]
    ref.load_state_dict(isd)
    trio = OracleTrio(ref, lambda ps: torch.optim.AdamW(ps, lr=1e-3, weight_decay=1e-5))
    ei = tr.edge_index.numpy()
    keys = np.unique(ei[0].astype(np.int64) * tr.num_items + ei[1].astype(np.int64))
    S, GB = len(tr), world * B
    assert len(hist["train_loss"]) == EPOCHS
    for e, order in enumerate(orders):
        losses = []
        for i in range(-(-S // GB)):
            b = min(GB, S - i * GB)
            ex = BR.build_batch(tr._ptr, tr._items, keys, tr.num_items, order, e * S + i * GB, b, 50, n, 42)
            rb = R.ref_batch_from(collate_sessions(ex))
            losses.append(float(trio.step(lambda mod, o: R.ref_train_step(mod, rb, o, "bpr"))))
        want = float(np.mean(losses))
        assert abs(hist["train_loss"][e] - want) <= 1e-3 * abs(want), (e, hist["train_loss"][e], want)
    trio.compare({k: torch.from_numpy(sd[k]) for k, _ in ref.named_parameters()}, lr=1e-3)
    b64 = dict(trio.ref64.named_buffers())
    b1 = dict(trio.ref1.named_buffers())
    for k, b in ref.named_buffers():
        if "num_batches_tracked" in k:
            assert int(sd[k]) == int(b), k
        elif "running" in k:  # SyncBN: statistics over the global batch
            close_trained(torch.from_numpy(sd[k]), b, b64[k], torch.zeros_like(b, dtype=torch.bool), 0.0, k, b1[k])


def test_rank_sharded_device_loader_equals_the_global_batch(tmp_path):
    """DeviceSessionLoader(rank, world): rank r's batch i is sessions [i*P*B + r*B, +B) of
    the epoch order with the negatives a single GPU draws for global batch i (positions),
    the last global batch split evenly -- in one process, no process group needed."""
    from dropin_helpers import write_csvs

    from etpgt.train.dataloader import DeviceSessionLoader, SessionDataset

    d = write_csvs(tmp_path, num_train=150)
    ds = SessionDataset(d / "train.csv", d / "graph_edges.csv", 5, 50)

    def epoch(loader):
        out = []
        for b in loader:
            ptr = b.ptr.cpu()
            x = b.x.cpu()
            out.append([(x[ptr[s]:ptr[s + 1]].tolist(), int(b.target_item[s]), b.negative_items.view(-1, 5)[s].tolist())
                        for s in range(b.num_graphs)])
        return out

    torch.manual_seed(3)
    one = epoch(DeviceSessionLoader(ds, 16, 5, shuffle=True, seed=42))
    ranks = []
    for r in range(2):
        torch.manual_seed(3)
        ranks.append(epoch(DeviceSessionLoader(ds, 8, 5, shuffle=True, seed=42, rank=r, world=2)))
    assert [len(b) for b in one] == [16] * 9 + [6]
    assert [len(b) for b in ranks[0]] == [8] * 9 + [3]
    for i, g in enumerate(one):
        assert ranks[0][i] + ranks[1][i] == g, i
