"""GPU Laplacian positional-encoding precompute.

``compute_laplacian_pe`` (etpgt/encodings/laplacian_pe.py:19-66) takes the k+1 smallest
eigenvectors of the sym-normalised Laplacian L = I - D^-1/2 A D^-1/2 (PyG
``get_laplacian(normalization="sym")``), drops the first and returns their absolute
values.  The reference calls scipy ``eigsh(L, k+1, which="SM")`` on the host, which is
slow on catalogue-sized graphs (and its dense fallback is infeasible there).

Here L lives on the GPU as CSR (values from ``gtr_lap_build``) and the eigenpairs come
from block LOBPCG whose only O(nnz) work is the HIP SpMM ``gtr_lap_spmm`` (a wave per
work item of <= 128 nonzeros of one row -- hub rows are split and their partials summed in
order -- lanes over the block's columns).  Per iteration: the block [X, R, P] is
multiplied by L, its fp64 Gram matrices go to the host in one transfer, and a
Rayleigh-Ritz step on the 3b x 3b generalized problem (fp64) picks the b smallest Ritz
pairs; P carries the search direction.  b = k + 1 + ``extra`` guard vectors speed up convergence of the wanted k+1.

Scope: the solver needs a symmetric adjacency (every i -> j with its j -> i) -- then L
is symmetric and its eigenvectors are well defined.  The reference's training script
(train_baseline.py:236-242) feeds the graph CSV's one-directional edges item_i -> item_j
(item_i < item_j once self loops are dropped) with num_nodes = num_items.  Then
D^-1/2 A D^-1/2 is strictly upper triangular, so L = I - D^-1/2 A D^-1/2 is UNIT upper
triangular: every eigenvalue is exactly 1 and L is defective.  ``eigsh`` (symmetric
Lanczos) on it returns Ritz pairs of a symmetry it assumes, not eigenpairs: on such
inputs its values lie in (-0.1, 1), its residuals ||L v - lambda v|| are 0.2-0.6, and two
calls give different vectors (ARPACK's random start; tests/test_host.py pins all three).
There is no answer to reproduce.  ``directed="reject"`` (default) raises on such input
(the host ``compute_laplacian_pe`` keeps the reference's behaviour);
``directed="symmetrize"`` takes the PE of the undirected graph (PyG ``to_undirected``:
each edge in both directions, duplicates merged), the well-defined spectrum the
positional encoding is meant to carry.  As with eigsh, eigenvectors of repeated
eigenvalues (e.g. one zero eigenvalue per connected component) are only defined up to a
rotation inside their eigenspace.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from etpgt.backend import _lib as L


def to_undirected(edge_index, n: int) -> np.ndarray:
    """PyG ``to_undirected`` without edge attributes: every edge in both directions,
    duplicates merged, sorted by (row, col); [2, E'] int64."""
    ei = edge_index.detach().cpu().numpy() if isinstance(edge_index, torch.Tensor) else np.asarray(edge_index)
    row, col = ei[0].astype(np.int64), ei[1].astype(np.int64)
    key = np.unique(np.concatenate([row * n + col, col * n + row]))
    return np.stack([key // n, key % n])


def _csr(edge_index, n: int, directed: str = "reject"):
    if directed not in ("reject", "symmetrize"):
        raise ValueError("directed must be 'reject' or 'symmetrize'")
    ei = edge_index.detach().cpu().numpy() if isinstance(edge_index, torch.Tensor) else np.asarray(edge_index)
    row, col = ei[0].astype(np.int64), ei[1].astype(np.int64)
    if row.size and (min(row.min(), col.min()) < 0 or max(row.max(), col.max()) >= n):
        raise IndexError("edge_index outside [0, num_nodes)")
    if directed == "symmetrize":
        row, col = to_undirected(np.stack([row, col]), n)
    keep = row != col
    r, c = row[keep], col[keep]
    if not np.array_equal(np.sort(r * n + c), np.sort(c * n + r)):
        raise NotImplementedError(
            "the GPU LapPE solver needs a symmetric adjacency (each i->j with its j->i); the reference's "
            "one-directional edge list gives a unit upper-triangular (non-symmetric) Laplacian whose eigsh output "
            "is not an eigen-decomposition -- pass directed='symmetrize' for the undirected graph's PE, or use "
            "compute_laplacian_pe (host eigsh) for the reference's behaviour")
    order = np.argsort(row, kind="stable")
    ptr = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(row, minlength=n), out=ptr[1:])
    if ptr[-1] >= 2**31:
        raise ValueError("more than 2^31 Laplacian entries")
    return ptr.astype(np.int32), col[order].astype(np.int32)


class LaplacianOperator:
    """X -> L X for [n, b] blocks by the HIP SpMM (gtr_lap_spmm) over an nnz-balanced
    work list (gtr_lap_plan: rows longer than ``chunk`` nonzeros are split)."""

    def __init__(self, edge_index, num_nodes: int, device="cuda", chunk: int = 128, directed: str = "reject"):
        self.n = int(num_nodes)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("LaplacianOperator runs on the GPU (HIP kernels); got device %s" % self.device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        ptr, col = _csr(edge_index, self.n, directed)
        self.nnz = int(col.size)
        lib = L.lib()
        ni, ns, npart = C.c_int64(), C.c_int64(), C.c_int64()
        L.check(lib.gtr_lap_plan(ptr.ctypes.data, self.n, chunk, None, C.byref(ni), None, C.byref(ns),
                                 C.byref(npart)), "lap_plan")
        items = np.empty((ni.value, 4), np.int32)
        splits = np.empty((max(ns.value, 1), 4), np.int32)
        L.check(lib.gtr_lap_plan(ptr.ctypes.data, self.n, chunk, items.ctypes.data, C.byref(ni),
                                 splits.ctypes.data, C.byref(ns), C.byref(npart)), "lap_plan")
        self.n_items, self.n_splits, self.n_parts = ni.value, ns.value, npart.value
        self.items = torch.from_numpy(items).to(self.device)
        self.splits = torch.from_numpy(splits).to(self.device)
        self.part = torch.empty(max(self.n_parts, 1) * 256, dtype=torch.float32, device=self.device)
        self.ptr = torch.from_numpy(ptr).to(self.device)
        # an edgeless graph (L = I) still passes non-null buffers; ptr keeps every row empty
        self.col = torch.from_numpy(col if col.size else np.zeros(1, np.int32)).to(self.device)
        self.dis = torch.empty(self.n, dtype=torch.float32, device=self.device)
        self.val = torch.empty(max(int(col.size), 1), dtype=torch.float32, device=self.device)
        L.check(lib.gtr_lap_build(self.ptr.data_ptr(), self.col.data_ptr(), self.n, self.dis.data_ptr(),
                                  self.val.data_ptr(), self._stream()), "lap_build")

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    GRAM_CHUNKS = 256

    def gram(self, S: torch.Tensor, Y: torch.Tensor) -> np.ndarray:
        """[2, m, m] fp64 host array (S^T S, S^T Y) for fp32 [n, m] blocks, m <= 64
        (HIP kernel gtr_lap_gram: fp64 accumulation, fixed summation order)."""
        m = S.shape[1]
        if S.shape != Y.shape or S.shape[0] != self.n or m > 64:
            raise ValueError("gram: S and Y must be [n, m <= 64]")
        if getattr(self, "_gpart", None) is None:
            self._gpart = torch.empty(self.GRAM_CHUNKS * 8192, dtype=torch.float64, device=self.device)
            self._gout = torch.empty(8192, dtype=torch.float64, device=self.device)
        S, Y = S.contiguous(), Y.contiguous()
        L.check(L.lib().gtr_lap_gram(S.data_ptr(), Y.data_ptr(), self.n, m, self._gpart.data_ptr(),
                                     self.GRAM_CHUNKS, self._gout.data_ptr(), self._stream()), "lap_gram")
        return self._gout.view(2, 64, 64)[:, :m, :m].cpu().numpy()

    def _spmm(self, X: torch.Tensor, Y: torch.Tensor, alpha: float = 1.0, beta: float = 0.0):
        L.check(L.lib().gtr_lap_spmm(self.col.data_ptr(), self.val.data_ptr(), self.n, X.shape[1],
                                     self.items.data_ptr(), self.n_items, self.splits.data_ptr(), self.n_splits,
                                     self.part.data_ptr(), X.data_ptr(), Y.data_ptr(), alpha, beta,
                                     self._stream()), "lap_spmm")

    def __call__(self, X: torch.Tensor) -> torch.Tensor:
        if X.dtype != torch.float32 or X.device != self.device or X.dim() != 2 or X.shape[0] != self.n:
            raise ValueError(f"expected fp32 [{self.n}, b] on {self.device}")
        b = X.shape[1]
        if b <= 256:
            X = X.contiguous()
            Y = torch.empty_like(X)
            self._spmm(X, Y)
            return Y
        Y = torch.empty_like(X)
        for c0 in range(0, b, 256):  # the kernel takes <= 256 columns
            xs = X[:, c0:c0 + 256].contiguous()
            ys = torch.empty_like(xs)
            self._spmm(xs, ys)
            Y[:, c0:c0 + 256] = ys
        return Y


def _gram_torch(S: torch.Tensor, Y: torch.Tensor) -> np.ndarray:
    Sd = S.double()
    return torch.stack([Sd.T @ Sd, Sd.T @ Y.double()]).cpu().numpy()


def lobpcg_smallest(op: LaplacianOperator, nev: int, extra: int = 4, tol: float = 1e-5, maxiter: int = 2000,
                    seed: int = 0, drop: float = 1e-7):
    """The ``nev`` smallest eigenpairs of the symmetric operator (ascending).  Returns
    (eigenvalues [nev] fp64 numpy, eigenvectors [n, nev] fp32 tensor, iterations).

    Block LOBPCG without explicit orthonormalisation: per iteration the basis
    S = [X, R, P] and L S (one SpMM) stay on the GPU, their Gram matrices S^T S and
    S^T L S are formed there in fp64 and cross to the host together (the iteration's one
    synchronisation), and the Rayleigh-Ritz step solves the generalized problem on the
    host in fp64: columns scaled to unit norm, directions of S^T S below ``drop``
    (relative) discarded so a (near-)dependent basis never breaks it, then the b
    smallest Ritz pairs.  The residual norms come from the same Gram diagonal."""
    n = op.n
    b = min(nev + extra, n)
    dev = op.device
    g = torch.Generator(device="cpu").manual_seed(seed)
    X, _ = torch.linalg.qr(torch.randn(n, b, generator=g, dtype=torch.float32).to(dev))
    AX = op(X)
    def gram(S, Y):  # the HIP Gram kernel takes blocks of <= 64 columns
        return op.gram(S, Y) if hasattr(op, "gram") and S.shape[1] <= 64 else _gram_torch(S, Y)

    H = gram(X, AX)[1]
    lam, Cm = np.linalg.eigh((H + H.T) / 2)
    Ct = torch.from_numpy(Cm).float().to(dev)
    X, AX = X @ Ct, AX @ Ct
    P = None
    it = 0
    for it in range(1, maxiter + 1):
        R = AX - X * torch.from_numpy(lam[:b]).float().to(dev)
        S = torch.cat([X, R] if P is None else [X, R, P], dim=1)
        AS = op(S)
        GH = gram(S, AS)
        G, H = GH[0], (GH[1] + GH[1].T) / 2
        dg = np.diag(G).copy()
        if np.sqrt(dg[b:b + nev].max()) < tol:
            break
        d = 1.0 / np.sqrt(np.where(dg > 0, dg, 1.0))
        Gs, Hs = G * d[:, None] * d[None, :], H * d[:, None] * d[None, :]
        sg, U = np.linalg.eigh((Gs + Gs.T) / 2)
        keep = sg > drop * sg.max()
        T = U[:, keep] / np.sqrt(sg[keep])
        w, W = np.linalg.eigh(T.T @ Hs @ T)
        V = d[:, None] * (T @ W[:, :b])  # coefficients of the b smallest Ritz vectors in S
        Vt = torch.from_numpy(V).float().to(dev)
        X, AX = S @ Vt, AS @ Vt
        P = S[:, b:] @ Vt[b:]  # search direction: the R and P parts of the update
        lam = w[:b]
    return lam[:nev], X[:, :nev], it


def compute_laplacian_pe_gpu(edge_index, num_nodes: int, k: int = 16, device="cuda", tol: float = 1e-5,
                             maxiter: int = 2000, extra: int = 4, seed: int = 0,
                             directed: str = "reject") -> torch.Tensor:
    """``compute_laplacian_pe`` (laplacian_pe.py:19-66) for a symmetric graph on the GPU:
    the k+1 smallest eigenvectors of the sym-normalised Laplacian, the first dropped,
    abs, fp32 [num_nodes, k] on ``device``.  ``directed="symmetrize"``: one-directional
    input (the reference training script's) is made undirected first (module doc)."""
    op = LaplacianOperator(edge_index, num_nodes, device, directed=directed)
    _, vecs, _ = lobpcg_smallest(op, k + 1, extra=extra, tol=tol, maxiter=maxiter, seed=seed)
    return vecs[:, 1:k + 1].abs().contiguous()
