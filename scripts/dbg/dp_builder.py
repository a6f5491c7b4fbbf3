"""Diagnostic: 2 DP ranks (gloo, shared cuda:0, SyncBN) with the device batch builder in the
fused step vs one GPU on the global batch -- per-step losses, graph and eager."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[2]
for p in ("tests", "gat-recommendation_amd", "oracle"):
    sys.path.insert(0, str(ROOT / p))

B, N_NEG, STEPS = 8, 5, 4


def setup(rank, world, graph, Bl, stride, pos):
    from gpu_helpers import make_pair, small_data

    from etpgt.data.gpu_batch import GpuBatchBuilder, GpuSessionStore
    from etpgt.train.fused import FusedTrainStep

    data = small_data()
    m, _ = make_pair(data.table_rows, 32, 2, seed=5)
    m.train()
    f = FusedTrainStep(m, lr=1e-2, weight_decay=1e-2, loss="bpr", sync_bn=world > 1, use_graph=graph)
    store = GpuSessionStore.from_synthetic(data, "cuda")
    bld = GpuBatchBuilder(store, Bl, N_NEG, seed=7, stride=stride)
    bld.set_epoch_order(np.random.default_rng(0).permutation(data.num_sessions), position=pos)
    f.attach_builder(bld, num_batches=STEPS)
    return f, m


def worker(rank, world, port, graph, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    f, m = setup(rank, world, graph, B, B * world, rank * B)
    losses = [float(f.run()) for _ in range(STEPS)]
    q.put((rank, losses, float(m.item_embedding.weight.double().sum())))
    dist.destroy_process_group()


def run(graph):
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, port, graph, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (l, w)) for r, l, w in [q.get(timeout=200) for _ in range(2)])
    for p in ps:
        p.join(60)
    f, m = setup(0, 1, graph, 2 * B, 2 * B, 0)
    one = [float(f.run()) for _ in range(STEPS)]
    print(f"graph={graph}: dp {res[0][0]} w {res[0][1]:.6f} | one {one} w {float(m.item_embedding.weight.double().sum()):.6f}",
          flush=True)


if __name__ == "__main__":
    run(False)
    run(True)
