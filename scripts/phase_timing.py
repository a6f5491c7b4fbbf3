#!/usr/bin/env python3
"""Diagnostic: per-workgroup phase stamps of the layer kernels inside one fused step.

Needs the timing build (``make -C gat-recommendation_amd/csrc timing``) loaded via
GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so.  Runs C2 steps (graph
replay), reads the s_memrealtime stamps (100 MHz) after each step and prints, per
kernel, the span from the first workgroup start to the last workgroup end, the
dispatch skew of workgroup starts, and the mean duration of each phase.
"""

from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

K, G, S = 32, 4096, 16
FWD_NAMES = {0: "conv_fwd L0", 1: "conv_fwd L1", 16: "readout"}
BWD_NAMES = {0: "conv_bwd L0", 1: "conv_bwd L1"}
FWD_PHASES = ["stage", "proj", "attn", "bnpart"]
BWD_PHASES = ["stage", "dst", "src", "dX"]
RO_PHASES = ["prologue", "sessions", "partials"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--batch-size", type=int, default=32)
    ap.add_argument("--out", default=None, help="also save the raw stamps (npz)")
    args = ap.parse_args()
    # stamps are indexed by hardware block: keep row group g on block g (no XCD packing)
    os.environ.setdefault("GTR_XCD_PACK", "0")
    dev = torch.device("cuda", 0)
    sys.path.insert(0, ROOT)
    import bench

    w = bench.build_workload(args.config, args.batch_size, 64, dev)
    step, staged, caps = w["step"], w["staged"], w["caps"]
    from etpgt.backend import _lib as L

    h = L.lib()
    for fn in ("gtr_dbg_fwd_phases", "gtr_dbg_bwd_phases"):
        getattr(h, fn).restype = C.c_int
        getattr(h, fn).argtypes = [C.c_void_p, C.c_size_t]
    fwd = np.zeros((K, G, S), np.uint64)
    bwd = np.zeros((K, G, S), np.uint64)
    for i in range(5):
        step.load_blob(staged[i % len(staged)])
        step.run()
    torch.cuda.synchronize()
    rows = {}
    detail = {}
    for i in range(args.steps):
        b = staged[i % len(staged)]
        step.load_blob(b)
        step.run()
        torch.cuda.synchronize()
        Gn = int(b[4].item())
        assert h.gtr_dbg_fwd_phases(fwd.ctypes.data, fwd.nbytes) == 0
        assert h.gtr_dbg_bwd_phases(bwd.ctypes.data, bwd.nbytes) == 0
        t_ref = int(fwd[0, :Gn, 0].min())
        ro_grid = max(1, min(caps.b_cap, 256))  # gtr_readout_grid
        for arr, names, nph, kind in ((fwd, FWD_NAMES, 5, "f"), (bwd, BWD_NAMES, 5, "b")):
            for kid, name in names.items():
                ng = ro_grid if kid == 16 else Gn
                last = 4 if kid != 16 else 3
                st = arr[kid, :ng, : last + 1].astype(np.int64)
                start, end = st[:, 0], st[:, last]
                rec = rows.setdefault(name, {"begin": [], "span": [], "skew": [], "ph": [], "mhz": []})
                if kind == "f" and kid != 16:
                    cyc = arr[kid, :ng, 7].astype(np.int64) - arr[kid, :ng, 6].astype(np.int64)
                    rt = (end - start).astype(np.float64)
                    rec["mhz"].append(float(np.median(cyc / np.maximum(rt, 1) * 100.0)))
                rec["begin"].append((start.min() - t_ref) * 10e-3)
                rec["span"].append((end.max() - start.min()) * 10e-3)
                rec["skew"].append((start.max() - start.min()) * 10e-3)
                rec["ph"].append(np.diff(st, axis=1).mean(0) * 10e-3)
                if kind == "b":  # dX then the folded weight gradients (stamp 9 between them)
                    sub = arr[kid, :ng][:, [3, 9, 4]].astype(np.int64)
                    detail.setdefault(name, []).append(np.diff(sub, axis=1).mean(0) * 10e-3)
                if kind == "f" and kid != 16:
                    cols = [0, 10, 12, 13, 14, 15, 1, 11, 2, 5, 8, 3, 4]
                    sub = arr[kid, :ng][:, cols].astype(np.int64)
                    detail.setdefault(name, []).append(np.diff(sub, axis=1).mean(0) * 10e-3)
    if detail:  # forward sub-phases from the fast path's extra stamps
        seq = [(0, "ranges"), (10, "csr_ld"), (12, "w_ld"), (13, "rows_ld"), (14, "bn+csr_st"), (15, "sync"), (1, "rows"), (11, "mfma"), (2, "logits"), (5, "softmax"), (8, "agg+gate"),
               (3, "bnpart"), (4, None)]
        for name, d in detail.items():
            m = np.median(np.stack(d), axis=0)
            if "bwd" in name:
                print(f"{name:14s} detail: dX={m[0]:.2f} wfold={m[1]:.2f}")
                continue
            print(f"{name:14s} detail: " + " ".join(f"{seq[i][1]}={m[i]:.2f}" for i in range(len(seq) - 1)))
    print(f"{'kernel':14s} {'begin_us':>9s} {'span_us':>8s} {'skew_us':>8s}  phases (mean us per workgroup)")
    order = sorted(rows, key=lambda n: np.median(rows[n]["begin"]))
    for name in order:
        r = rows[name]
        phn = RO_PHASES if name == "readout" else (FWD_PHASES if "fwd" in name else BWD_PHASES)
        ph = np.median(np.stack(r["ph"]), axis=0)
        print(f"{name:14s} {np.median(r['begin']):9.2f} {np.median(r['span']):8.2f} {np.median(r['skew']):8.2f}  "
              + " ".join(f"{n}={v:.2f}" for n, v in zip(phn, ph))
              + (f"  clk~{np.median(r['mhz']):.0f}MHz" if r["mhz"] else ""))


if __name__ == "__main__":
    main()
