"""Diagnostic: per-workgroup phase stamps of the projection GEMM (k_proj, kid 10 + layer)
from the timing build (GTR_LIB=.../build/timing/libgtr_hip.so): kernel start -> prologue
done (W_all in registers, first tile built, barrier) -> first tile's MFMA chain -> its
epilogue -> barrier -> the remaining tiles.  usage: gemm_phases.py CONFIG BATCH"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))

import bench  # noqa: E402
from etpgt.backend import _lib as L  # noqa: E402

K, G, S = 32, 4096, 16


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    dev = torch.device("cuda", 0)
    w = bench.build_workload(cfg, B, 2, dev, 0, use_graph=False)
    step, staged = w["step"], w["staged"]
    h = L.lib()
    h.gtr_dbg_gemm_phases.restype = C.c_int
    h.gtr_dbg_gemm_phases.argtypes = [C.c_void_p, C.c_size_t]
    arr = np.zeros((K, G, S), np.uint64)
    rows = {10: [], 11: []}
    for i in range(8):
        step.load_blob(staged[i % 2])
        step.run()
        torch.cuda.synchronize()
        if i < 2:
            continue
        arr[:] = 0
        assert h.gtr_dbg_gemm_phases(arr.ctypes.data, arr.nbytes) == 0
        for kid in rows:
            st = arr[kid].astype(np.int64)
            live = (st[:, 0] > 0) & (st[:, 1] > 0)
            st = st[live]
            if not len(st):
                continue
            t0 = st[:, 0].min()
            d = lambda a, b: (st[:, b] - st[:, a]) * 10e-3  # noqa: E731
            rows[kid].append([(st[:, 1].max() - t0) * 10e-3, (st[:, 0].max() - t0) * 10e-3, d(0, 2).mean(),
                              d(0, 2).max(), d(2, 3).mean(), d(3, 4).mean(), d(4, 5).mean(), d(5, 1).mean(),
                              len(st)])
    print(f"config {cfg} B {B} split {step.split}")
    for kid, r in rows.items():
        if not r:
            continue
        m = np.median(np.array(r), axis=0)
        print(f"k_proj layer {kid - 10}: span {m[0]:6.2f} us, start skew {m[1]:5.2f}; prologue (W + first tile) mean "
              f"{m[2]:5.2f} max {m[3]:5.2f}; first MFMA chain {m[4]:5.2f}; its epilogue {m[5]:5.2f}; barrier "
              f"{m[6]:5.2f}; remaining tiles {m[7]:6.2f} (wgs {int(m[8])})")


if __name__ == "__main__":
    main()
