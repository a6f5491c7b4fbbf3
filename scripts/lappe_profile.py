"""Where a GPU LOBPCG iteration's time goes (LapPE precompute): GPU work up to the Gram
transfer, the host Rayleigh-Ritz, the update; on the RetailRocket-shaped graph's LCC."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gat-recommendation_amd"))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import scipy.sparse.csgraph as cg  # noqa: E402
import torch  # noqa: E402

from etpgt.data.synthetic import make_sessions_and_graph  # noqa: E402
from etpgt.encodings.laplacian_gpu import LaplacianOperator  # noqa: E402

data = make_sessions_and_graph(seed=42)
ei = data.edge_index()
ei = ei[:, ei[0] != ei[1]]
sym = np.concatenate([ei, ei[::-1]], axis=1)
n = data.table_rows
A = sp.coo_matrix((np.ones(sym.shape[1]), (sym[0], sym[1])), shape=(n, n))
_, lab = cg.connected_components(A)
keep = lab == np.bincount(lab).argmax()
remap = -np.ones(n, np.int64)
remap[keep] = np.arange(keep.sum())
sym = remap[sym[:, keep[sym[0]]]]
n = int(keep.sum())
op = LaplacianOperator(torch.from_numpy(sym), n, "cuda")
b = 21
dev = op.device
S = torch.linalg.qr(torch.randn(n, 3 * b, device=dev))[0]
tg = th = tu = 0.0
reps = 20
print("threads", torch.get_num_threads(), os.environ.get("OMP_NUM_THREADS"), flush=True)
for r in range(reps + 3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    AS = op(S)
    Sd = S.double()
    GH = torch.stack([Sd.T @ Sd, Sd.T @ AS.double()]).cpu().numpy()
    t1 = time.perf_counter()
    G, H = GH[0], (GH[1] + GH[1].T) / 2
    d = 1.0 / np.sqrt(np.diag(G))
    sg, U = np.linalg.eigh(G * d[:, None] * d[None, :])
    T = U / np.sqrt(sg)
    w, W = np.linalg.eigh(T.T @ (H * d[:, None] * d[None, :]) @ T)
    V = d[:, None] * (T @ W[:, :b])
    t2 = time.perf_counter()
    Vt = torch.from_numpy(V).float().to(dev)
    X = S @ Vt
    P = S[:, b:] @ Vt[b:]
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    if r >= 3:
        tg += t1 - t0; th += t2 - t1; tu += t3 - t2
print(f"gpu+gram transfer {1e3*tg/reps:.3f} ms, host rayleigh-ritz {1e3*th/reps:.3f} ms, update {1e3*tu/reps:.3f} ms")
for nt in (1, 4):
    torch.set_num_threads(nt)
    t0 = time.perf_counter()
    for _ in range(reps):
        np.linalg.eigh(G)
    print(f"numpy eigh 63x63 ({nt} torch threads): {1e3*(time.perf_counter()-t0)/reps:.3f} ms")
