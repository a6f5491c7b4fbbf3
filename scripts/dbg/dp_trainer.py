"""Diagnostic: train_baseline counterpart, 2 ranks (gloo, shared cuda:0) vs one GPU on the
global batch; prints per-epoch losses for a few model widths / datasets."""
import os
import socket
import sys
import tempfile
from pathlib import Path

import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "gat-recommendation_amd"))
sys.path.insert(0, str(ROOT / "oracle"))


def script():
    import importlib.util

    spec = importlib.util.spec_from_file_location("tb", ROOT / "scripts" / "train" / "train_baseline.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def args(d, out, B, D, ep, extra):
    return ["--model", "graph_transformer_optimized", "--train-sessions", str(d / "train.csv"),
            "--val-sessions", str(d / "val.csv"), "--graph-edges", str(d / "graph_edges.csv"),
            "--embedding-dim", str(D), "--hidden-dim", str(D), "--num-layers", "2", "--num-heads", "2",
            "--dropout", "0", "--batch-size", str(B), "--num-negatives", "5", "--max-epochs", str(ep),
            "--num-workers", "0", "--output-dir", str(out)] + extra


def rank_main(rank, world, port, d, out, B, D, ep, extra, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), GTR_SHARE_DEVICE="1")
    tr = script().main(args(d, out, B, D, ep, extra))
    q.put((rank, tr.history["train_loss"], float(tr.model.item_embedding.weight.double().sum())))
    import torch.distributed as dist
    dist.destroy_process_group()


def run(ntrain, D, B, ep, extra=()):
    from dropin_helpers import write_csvs

    tmp = Path(tempfile.mkdtemp())
    d = write_csvs(tmp, num_train=ntrain)
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, 2, port, d, tmp / "dp", B, D, ep, list(extra), q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (l, w)) for r, l, w in [q.get(timeout=300) for _ in range(2)])
    for p in ps:
        p.join(60)
    tr = script().main(args(d, tmp / "one", 2 * B, D, ep, list(extra)))
    print(f"ntrain={ntrain} D={D} B={B} extra={extra}: dp {res[0][0]} (w {res[0][1]:.6f}) | one {tr.history['train_loss']} "
          f"(w {float(tr.model.item_embedding.weight.double().sum()):.6f})", flush=True)


if __name__ == "__main__":
    run(16, 64, 8, 2)
    run(32, 32, 8, 1)
    run(24, 32, 8, 1)
    run(48, 32, 8, 1)
    run(150, 32, 8, 1)
