"""Host enqueue cost of one bench step (load_blob + graph replay) while the GPU is held
busy by a long sleep kernel: if it approaches the GPU step time, the step is host-bound."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

for cfg in ("c2", "c3"):
    dev = torch.device("cuda", 0)
    w = bench.build_workload(cfg, 32, 64, dev)
    step, staged = w["step"], w["staged"]
    for i in range(30):
        step.load_blob(staged[i % 64])
        step.run()
    torch.cuda.synchronize()
    for variant in ("copy+replay", "replay only", "resident"):
        if variant == "resident":
            step.bind_resident(staged)
            for i in range(64):
                step.run_resident(i)
            step.prepare_resident()
            torch.cuda.synchronize()
        n = 200
        torch.cuda._sleep(int(2.4e9 * 0.2))  # ~200 ms of GPU time ahead of the enqueues
        t0 = time.perf_counter()
        for i in range(n):
            if variant == "copy+replay":
                step.load_blob(staged[i % 64])
                step.run()
            elif variant == "replay only":
                step.run()
            else:
                step.run_resident(i % 64)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        print(cfg, variant, f"host enqueue {1e6 * (t1 - t0) / n:.1f} us/step", flush=True)
