"""Diagnostics: time gtr_wgrad alone (HIP events) on the bench workload, per variant.

python scripts/wgrad_probe.py CONFIG BATCH  -- after a few real steps, re-launches the
weight-gradient kernel with GTR_WGRAD=valu|mfma and GTR_WGRAD_JOBS masks (1: QKVS weight,
2: gate, 4: bias column sums, 8: LapPE projection; timing only, the slabs are scratch)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    cfg_name, B = sys.argv[1], int(sys.argv[2])
    dev = torch.device("cuda", 0)
    w = bench.build_workload(cfg_name, B, 4, dev, 0, use_graph=True, data_parallel=None, lazy=False,
                             sync_bn=False, lagged=False, shard_table=False)
    step, staged = w["step"], w["staged"]
    for i in range(6):
        step.load_blob(staged[i % len(staged)])
        step.run()
    torch.cuda.synchronize()
    eng = step.eng
    bs = step.bs
    main_s = torch.cuda.current_stream()
    variants = [("valu", None), ("mfma", None)] + [("mfma", m) for m in ("1", "2", "4", "8")] + \
               [("valu", m) for m in ("1", "2", "8")]
    for mode, mask in variants:
        os.environ["GTR_WGRAD"] = mode
        if mask is None:
            os.environ.pop("GTR_WGRAD_JOBS", None)
        else:
            os.environ["GTR_WGRAD_JOBS"] = mask
        ev = []
        for _ in range(30):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            eng._wgrad(step.ws, step.cfg, bs, 0, eng.L, main_s.cuda_stream)
            e1.record(main_s)
            ev.append((e0, e1))
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) for a, b in ev[5:])
        print(f"{cfg_name} B={B} wgrad {mode:5s} jobs={mask or 'all':4s} P={step.ws.P} median {t[len(t)//2]*1e3:8.1f} us",
              flush=True)
    os.environ.pop("GTR_WGRAD_JOBS", None)
    os.environ.pop("GTR_WGRAD", None)


if __name__ == "__main__":
    main()
