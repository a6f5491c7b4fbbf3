#!/usr/bin/env python3
"""Diagnostic: phase stamps of conv_fwd(layer 0) launched twice back to back (idempotent:
the same outputs) inside an eager C2 step -- the second launch runs with warm instruction
cache / L2, the first as inside the captured chain.  Timing build:
GTR_LIB=gat-recommendation_amd/build/timing/libgtr_hip.so python3 scripts/dbg_warm.py"""
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

dev = torch.device("cuda", 0)
w = bench.build_workload("c2", 32, 16, dev)
step, staged = w["step"], w["staged"]
h = L.lib()
h.gtr_dbg_fwd_phases.restype = C.c_int
h.gtr_dbg_fwd_phases.argtypes = [C.c_void_p, C.c_size_t]
for i in range(10):
    step.load_blob(staged[i % len(staged)])
    step.run()
torch.cuda.synchronize()
eng, ws, cfg = step.eng, step.ws, step.cfg
st = torch.cuda.current_stream().cuda_stream
ph = np.zeros((32, 1024, 8), np.uint64)
res = {"cold": [], "warm": [], "cold_ev": [], "warm_ev": []}
for it in range(20):
    step.load_blob(staged[it % len(staged)])
    step._begin(step.bs, st)
    for tag in ("cold", "warm"):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        L.check(h.gtr_conv_fwd(C.byref(cfg), C.byref(step.bs), C.byref(eng.fill_embed()), ws.structs, 0, st), "fwd")
        e1.record()
        torch.cuda.synchronize()
        assert h.gtr_dbg_fwd_phases(ph.ctypes.data, ph.nbytes) == 0
        Gn = int(staged[it % len(staged)][4].item())
        a = ph[0, :Gn, :5].astype(np.int64)
        res[tag].append(np.diff(a, axis=1).mean(0) * 10e-3)
        res[tag + "_ev"].append(e0.elapsed_time(e1) * 1e3)
    # finish the step so state stays consistent
    eng.run_forward(ws, cfg, step.bs, L.RO_FWD | L.RO_LOSS | L.RO_BWD, step.loss_kind)
    eng.run_backward(ws, cfg, step.bs)
    step._launch_b(False)
torch.cuda.synchronize()
for tag in ("cold", "warm"):
    p = np.median(np.stack(res[tag]), axis=0)
    print(f"{tag}: event {np.median(res[tag + '_ev']):.2f} us  stage={p[0]:.2f} proj={p[1]:.2f} attn={p[2]:.2f} "
          f"bnpart={p[3]:.2f}")
