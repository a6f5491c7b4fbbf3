#!/usr/bin/env python3
"""Diagnostic: per-workgroup phase stamps of the split path's row kernels (k_attn_rows,
kid 20 + layer; k_readout_wave, kid 26) inside one step, from the timing build
(``make -C gat-recommendation_amd/csrc timing``; GTR_LIB=.../build/timing/libgtr_hip.so).

Prints per kernel: the span from the first workgroup start to the last stamp, the
dispatch skew of the starts, the mean duration of each phase, and the last arriver's
tail (the largest final-phase duration).  usage: split_phases.py CONFIG BATCH [steps]"""

from __future__ import annotations

import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

K, G, S = 32, 4096, 16
KERNELS = {20: ("attn_rows L0", 4), 21: ("attn_rows L1", 4), 26: ("readout_wave", 6)}
# detail stamps: (name, from slot, to slot); only workgroups that reached both
DETAIL = {20: [("csr offsets", 0, 8), ("ids+K/V rows", 8, 9), ("K rest", 9, 10), ("softmax z", 10, 11),
               ("aggregate", 11, 12), ("gate+stores", 12, 13), ("other waves", 13, 1),
               ("bucket arrive", 2, 4), ("bucket merge", 4, 5), ("top arrive", 5, 6), ("top merge", 6, 7)],
          26: [("se (node rows)", 1, 6), ("scoring rounds", 6, 7), ("lse + coefs", 7, 8), ("bwd node rows", 8, 9)]}
DETAIL[21] = DETAIL[20]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    os.environ.setdefault("GTR_XCD_PACK", "0")
    import bench
    from etpgt.backend import _lib as L

    dev = torch.device("cuda", 0)
    w = bench.build_workload(cfg, B, 2, dev, 0, use_graph=False)
    step, staged = w["step"], w["staged"]
    h = L.lib()
    h.gtr_dbg_fwd_phases.restype = C.c_int
    h.gtr_dbg_fwd_phases.argtypes = [C.c_void_p, C.c_size_t]
    arr = np.zeros((K, G, S), np.uint64)
    rec = {}
    for i in range(steps + 2):
        step.load_blob(staged[i % 2])
        step.run()
        torch.cuda.synchronize()
        if i < 2:
            continue
        arr[:] = 0
        assert h.gtr_dbg_fwd_phases(arr.ctypes.data, arr.nbytes) == 0
        for kid, (name, nst) in KERNELS.items():
            st = arr[kid].astype(np.int64)
            live = st[:, 0] > 0
            if not live.any():
                continue
            # stamps are not cleared between steps: keep this step's workgroups (a batch with
            # fewer row groups than an earlier one leaves the extra slots' old stamps behind)
            med = np.median(st[live, 0])
            live &= np.abs(st[:, 0] - med) < 50000  # 500 us at the 100 MHz stamp clock
            st = st[live]
            start = st[:, 0]
            last = np.where(st[:, 1:nst] > 0, st[:, 1:nst], 0).max(1)
            r = rec.setdefault(name, {"span": [], "skew": [], "ph": [], "n": [], "tail": []})
            r["span"].append((last.max() - start.min()) * 10e-3)
            r["skew"].append((start.max() - start.min()) * 10e-3)
            r["n"].append(int(live.sum()))
            ph = []
            for k in range(1, nst):
                ok = st[:, k] > 0
                ph.append(float(((st[ok, k] - st[ok, k - 1]) * 10e-3).mean()) if ok.any() else 0.0)
            r["ph"].append(ph)
            tails = [(st[st[:, k] > 0, k] - st[st[:, k] > 0, k - 1]).max() * 10e-3 if (st[:, k] > 0).any() else 0.0
                     for k in range(1, nst)]
            r["tail"].append(tails)
            # when workgroups start and finish their main phase (relative to the first start)
            t0 = start.min()
            fin = np.where(st[:, 1] > 0, st[:, 1], last)
            r.setdefault("gen", []).append([np.percentile(start - t0, q) * 10e-3 for q in (50, 90, 100)]
                                           + [np.percentile(fin - t0, q) * 10e-3 for q in (50, 90, 100)])
            for dn, a0, a1 in DETAIL.get(kid, []):
                ok = (st[:, a0] > 0) & (st[:, a1] >= st[:, a0])
                if ok.any():
                    d = (st[ok, a1] - st[ok, a0]) * 10e-3
                    r.setdefault("det", {}).setdefault(dn, []).append((float(d.mean()), float(d.max()), int(ok.sum())))
    print(f"config {cfg} B {B} split {step.split} N {int(staged[0][0].item())}")
    for name, r in rec.items():
        print(f"{name:14s} wgs {int(np.median(r['n'])):5d} span {np.median(r['span']):7.2f} us  skew "
              f"{np.median(r['skew']):6.2f}  phase means " + " ".join(f"{v:6.2f}" for v in np.median(r['ph'], axis=0))
              + "  phase max " + " ".join(f"{v:6.2f}" for v in np.median(r['tail'], axis=0)))
        if "gen" in r:
            g = np.median(np.array(r["gen"]), axis=0)
            print(f"    starts p50/p90/max {g[0]:6.2f} {g[1]:6.2f} {g[2]:6.2f}   main done p50/p90/max "
                  f"{g[3]:6.2f} {g[4]:6.2f} {g[5]:6.2f} us")
        for dn, v in r.get("det", {}).items():
            v = np.array(v)
            print(f"    {dn:16s} mean {np.median(v[:, 0]):7.2f}  max {np.median(v[:, 1]):7.2f}  (wgs {int(np.median(v[:, 2]))})")


if __name__ == "__main__":
    main()
