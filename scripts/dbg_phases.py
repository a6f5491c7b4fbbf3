#!/usr/bin/env python3
"""Diagnostic: fine phase stamps of conv_fwd (layers 0 and 1) in captured C2 steps.
Slots (s_memrealtime, 100 MHz, thread 0): 0 start, 10 group ranges loaded, 1 staged
(CSR / items / BN stats), 11 input rows in LDS, 2 projection done, 5 logits, 8 softmax,
3 aggregation + gate, 4 BN partial.  Timing build:
GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so python3 scripts/dbg_phases.py"""
from __future__ import annotations

import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from etpgt.backend import _lib as L  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
# XCD-packed roles (GTR_XCD_PACK, default on): row group g runs on hardware block 8g
stride = 8 if os.environ.get("GTR_XCD_PACK", "1") != "0" else 1
dev = torch.device("cuda", 0)
w = bench.build_workload(cfg, 32, 16, dev)
step, staged = w["step"], w["staged"]
h = L.lib()
for fn in ("gtr_dbg_fwd_phases", "gtr_dbg_bwd_phases"):
    getattr(h, fn).restype = C.c_int
    getattr(h, fn).argtypes = [C.c_void_p, C.c_size_t]
ph = np.zeros((32, 1024, 16), np.uint64)
pb = np.zeros((32, 1024, 16), np.uint64)
bnames = ["stage", "dst", "src", "dX"]
bacc = {0: [], 1: []}
order = [0, 10, 1, 11, 2, 5, 8, 3, 4]
names = ["ranges", "staged", "rows", "proj", "logits", "softmax", "agg+gate", "bnpart"]
acc = {0: [], 1: []}
for i in range(40):
    step.load_blob(staged[i % len(staged)])
    step.run()
    torch.cuda.synchronize()
    if i < 5:
        continue
    assert h.gtr_dbg_fwd_phases(ph.ctypes.data, ph.nbytes) == 0
    assert h.gtr_dbg_bwd_phases(pb.ctypes.data, pb.nbytes) == 0
    G = int(staged[i % len(staged)][4].item())
    for l in (0, 1):
        a = ph[l, : G * stride : stride][:, order].astype(np.int64)
        ok = (a > 0).all(axis=1)
        acc[l].append(np.median(np.diff(a[ok], axis=1), axis=0) * 10e-3)
        b = pb[l, : G * stride : stride][:, :5].astype(np.int64)
        okb = (b > 0).all(axis=1)
        bacc[l].append(np.median(np.diff(b[okb], axis=1), axis=0) * 10e-3)
for l in (0, 1):
    m = np.median(np.stack(acc[l]), axis=0)
    print(f"conv_fwd L{l}: " + " ".join(f"{n}={v:.2f}" for n, v in zip(names, m)) + f"  total={m.sum():.2f} us")
for l in (1, 0):
    m = np.median(np.stack(bacc[l]), axis=0)
    print(f"conv_bwd L{l}: " + " ".join(f"{n}={v:.2f}" for n, v in zip(bnames, m)) + f"  total={m.sum():.2f} us")
