"""Training throughput of the FFN variant (`create_graph_transformer`, use_ffn=True) on the
RetailRocket-shaped synthetic workload: the reference Trainer's autograd step (forward on
the split layer + FFN kernels, BPR loss, backward, torch.optim.AdamW) over pre-staged
device batches (built by gtr_build_batch, as the Trainer's DeviceSessionLoader yields them).  Prints one JSON line per configuration (sessions/s, ms/step).

usage: python scripts/ffn_bench.py [--steps 50] [--warmup 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))

import torch  # noqa: E402

from etpgt.data.gpu_batch import GpuBatchBuilder, GpuSessionStore  # noqa: E402
from etpgt.data.synthetic import make_sessions_and_graph  # noqa: E402
from etpgt.model import create_graph_transformer  # noqa: E402


def run(data, D, H, L, B, n_neg, steps, warmup):
    T = data.table_rows
    torch.manual_seed(0)
    m = create_graph_transformer(T, embedding_dim=D, hidden_dim=D, num_layers=L, num_heads=H, dropout=0.1,
                                 use_laplacian_pe=False, use_ffn=True, ffn_expansion=4).cuda().train()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, weight_decay=1e-5)
    bld = GpuBatchBuilder(GpuSessionStore.from_synthetic(data, "cuda"), B, n_neg, seed=5)
    batches = [bld.build_device_batch() for _ in range(8)]

    def step(b):
        se = m(b)
        loss = m.compute_loss(se, b.target_item, b.negative_items.view(b.num_graphs, n_neg))
        opt.zero_grad(set_to_none=False)
        loss.backward()
        opt.step()
        return loss

    for i in range(warmup):
        step(batches[i % len(batches)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(batches[i % len(batches)])
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    out = {"model": "graph_transformer (use_ffn=True, ffn_expansion=4)", "dim": D, "heads": H, "layers": L,
           "batch": B, "negatives": n_neg, "ms_per_step": round(ms, 4), "sessions_per_s": round(B / ms * 1e3, 1),
           "final_loss": round(float(loss), 5), "path": "autograd (GraphTransformerFn) + torch.optim.AdamW"}
    # the fused step (one captured hipGraph per step, the batch built inside it: the Trainer's
    # path with a DeviceSessionLoader)
    from etpgt.train.fused import FusedTrainStep

    fs = FusedTrainStep(m, lr=1e-3, weight_decay=1e-5, loss="bpr")
    fbld = GpuBatchBuilder(GpuSessionStore.from_synthetic(data, "cuda"), B, n_neg, seed=6)
    fs.attach_builder(fbld, num_batches=steps + warmup)
    for _ in range(warmup):
        fs.run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fl = fs.run()
    torch.cuda.synchronize()
    fms = 1e3 * (time.perf_counter() - t0) / steps
    out["fused"] = {"ms_per_step": round(fms, 4), "sessions_per_s": round(B / fms * 1e3, 1),
                    "final_loss": round(float(fl), 5), "path": "FusedTrainStep (captured step, device-built batches)"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    args = ap.parse_args()
    data = make_sessions_and_graph(seed=42)
    for D, H, L, B in ((64, 2, 3, 32), (128, 4, 3, 32), (128, 4, 3, 1024), (256, 4, 3, 32)):
        print(json.dumps(run(data, D, H, L, B, 5, args.steps, args.warmup)), flush=True)


if __name__ == "__main__":
    main()
