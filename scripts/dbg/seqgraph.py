"""Probe: K training steps as K graph launches (one captured graph per resident image)
against ONE captured K-step graph (FusedTrainStep.capture_steps), HIP events and host
clock.  usage: python scripts/dbg/seqgraph.py [config] [batch] [K]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))

import bench  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3, a.elapsed_time(b)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    dev = torch.device("cuda", 0)
    w = bench.build_workload(cfg, B, 4, dev, 0, use_graph=True, lazy=bool(bench.CONFIGS[cfg].get("lazy")))
    step, staged = w["step"], w["staged"]
    step.bind_resident(staged)
    for i in range(5):
        step.run_resident(i % len(staged))
    step.prepare_resident()
    h = step.capture_steps(5, K)
    for rep in range(3):
        host1, ev1 = timed(lambda: [step.run_resident((5 + i) % len(staged)) for i in range(K)])
        host2, ev2 = timed(lambda: step.run_steps(h))
        print(f"{cfg} B {B} K {K} rep {rep}: per-step graphs host {host1 / K:.4f} ms events {ev1 / K:.4f} ms | "
              f"one {K}-step graph host {host2 / K:.4f} ms events {ev2 / K:.4f} ms")


if __name__ == "__main__":
    main()
