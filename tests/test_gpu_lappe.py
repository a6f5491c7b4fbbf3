"""GPU LapPE precompute (gtr_lap_build / gtr_lap_spmm + block LOBPCG in
etpgt.encodings.laplacian_gpu) against the oracle's restatement of
``compute_laplacian_pe`` (laplacian_pe.py:19-66: scipy eigsh(k+1, 'SM') of the PyG
sym-normalised Laplacian, column 0 dropped, abs).

Eigenvectors are compared column by column only where the eigenvalue is separated
from its neighbours (gap >= 1e-3): inside a (near-)repeated eigenspace neither eigsh
nor any other solver defines a unique basis, so those columns are checked through
the subspace they span instead (projector distance).  Tolerance 2e-3 absolute on
unit-norm eigenvectors of an fp32 operator.
"""

import numpy as np
import pytest
import torch

import oracle.etpgt_ref as R

pytestmark = pytest.mark.gpu

from etpgt.encodings.laplacian_gpu import (  # noqa: E402
    LaplacianOperator,
    compute_laplacian_pe_gpu,
    lobpcg_smallest,
)


def _graph(n, chords, seed):
    """Connected ring + random chords, both directions, plus a few self loops
    (which get_laplacian removes)."""
    rng = np.random.default_rng(seed)
    a = np.arange(n)
    src = np.concatenate([a, rng.integers(0, n, chords)])
    dst = np.concatenate([(a + 1) % n, rng.integers(0, n, chords)])
    keep = src != dst
    src, dst = src[keep], dst[keep]
    loops = rng.integers(0, n, 5)
    ei = np.stack([np.concatenate([src, dst, loops]), np.concatenate([dst, src, loops])])
    return torch.from_numpy(ei.astype(np.int64))


def _check_columns(got, want, lam, atol=2e-3):
    """got/want [n, m] eigenvector columns (unsigned); lam [m + 2] eigenvalues around them."""
    m = got.shape[1]
    checked = 0
    for j in range(m):
        gap = min(abs(lam[j + 1] - lam[j]), abs(lam[j + 2] - lam[j + 1]))
        if gap < 1e-3:
            continue
        np.testing.assert_allclose(got[:, j], want[:, j], atol=atol, err_msg=f"column {j}")
        checked += 1
    return checked


def test_reference_path_graph():
    # tests/test_models.py:232-239: 4-node path, k=2 -> shape (4, 2), float32, non-negative
    ei = torch.tensor([[0, 1, 1, 2, 2, 3], [1, 0, 2, 1, 3, 2]])
    pe = compute_laplacian_pe_gpu(ei, num_nodes=4, k=2)
    assert pe.shape == (4, 2) and pe.dtype == torch.float32 and pe.device.type == "cuda"
    assert bool((pe >= 0).all())
    want = R.ref_compute_laplacian_pe(ei, num_nodes=4, k=2).numpy()
    # spectrum 1 - cos(pi j / 3): all simple, so every column is defined up to sign
    np.testing.assert_allclose(pe.cpu().numpy(), want, atol=1e-4)


def test_spmm_matches_scipy_laplacian():
    n = 3000
    ei = _graph(n, 9000, seed=3)
    op = LaplacianOperator(ei, n, "cuda")
    Lm = R.ref_sym_laplacian(ei.numpy(), n)
    g = torch.Generator().manual_seed(0)
    for b in (1, 7, 64, 300):  # 300 > 256 exercises the column chunking
        X = torch.randn(n, b, generator=g)
        Y = op(X.cuda()).cpu().numpy()
        np.testing.assert_allclose(Y, Lm @ X.numpy(), rtol=1e-4, atol=1e-5)


def test_spmm_isolated_nodes():
    # nodes with no edges: degree 0 -> D^-1/2 := 0, so their L row is the identity row
    n = 50
    ei = torch.tensor([[0, 1, 10, 11], [1, 0, 11, 10]])
    op = LaplacianOperator(ei, n, "cuda")
    X = torch.randn(n, 5)
    Y = op(X.cuda()).cpu().numpy()
    np.testing.assert_allclose(Y, R.ref_sym_laplacian(ei.numpy(), n) @ X.numpy(), rtol=1e-5, atol=1e-6)
    # no edges at all: L = I
    op0 = LaplacianOperator(torch.zeros(2, 0, dtype=torch.long), 7, "cuda")
    X = torch.randn(7, 3)
    np.testing.assert_array_equal(op0(X.cuda()).cpu().numpy(), X.numpy())


@pytest.mark.parametrize("n,chords,k", [(400, 600, 8), (1500, 4000, 16)])
def test_lappe_gpu_matches_eigsh(n, chords, k):
    ei = _graph(n, chords, seed=n)
    Lm = R.ref_sym_laplacian(ei.numpy(), n)
    dense = Lm.toarray().astype(np.float64)
    lam_all, vec_all = np.linalg.eigh(dense)

    op = LaplacianOperator(ei, n, "cuda")
    lam, X, it = lobpcg_smallest(op, k + 1, tol=1e-5)
    np.testing.assert_allclose(lam, lam_all[: k + 1], atol=1e-5)
    Xn = X.cpu().numpy().astype(np.float64)
    # orthonormal, and each column an eigenvector: ||L x - lam x|| small
    np.testing.assert_allclose(Xn.T @ Xn, np.eye(k + 1), atol=1e-4)
    assert np.abs(dense @ Xn - Xn * lam).max() < 1e-4

    pe = compute_laplacian_pe_gpu(ei, n, k=k, tol=1e-5).cpu().numpy()
    assert pe.shape == (n, k) and pe.dtype == np.float32 and (pe >= 0).all()
    want = R.ref_compute_laplacian_pe(ei, n, k=k).numpy()
    lam_ctx = np.concatenate([lam_all[: k + 2], [np.inf]])
    # columns 1..k of the spectrum; lam index j+1 is the eigenvalue of pe column j
    checked = _check_columns(pe, want, lam_ctx)
    assert checked >= k // 2, f"only {checked} well-separated columns"
    # the whole span agrees too (projector distance), repeated eigenvalues included
    # when the cut after column k falls in a gap
    if lam_all[k + 1] - lam_all[k] > 1e-3:
        Vg = Xn[:, : k + 1]
        Vr = vec_all[:, : k + 1]
        assert np.abs(Vg @ Vg.T - Vr @ Vr.T).max() < 1e-3


def test_lappe_gpu_rejects_one_directional_edges():
    ei = torch.tensor([[0, 1, 2], [1, 2, 3]])
    with pytest.raises(NotImplementedError, match="symmetric"):
        compute_laplacian_pe_gpu(ei, num_nodes=4, k=2)


def _one_directional(n, m, seed):
    """The reference training script's LapPE input (train_baseline.py:236-242): the graph
    CSV's canonical edges item_i -> item_j with item_i <= item_j, self loops included."""
    rng = np.random.default_rng(seed)
    i, j = rng.integers(0, n, m), rng.integers(0, n, m)
    return torch.from_numpy(np.stack([np.minimum(i, j), np.maximum(i, j)]).astype(np.int64))


@pytest.mark.parametrize("n,m,k", [(4, 6, 2), (1500, 9000, 16)])
def test_lappe_gpu_symmetrizes_the_reference_input(n, m, k):
    """directed='symmetrize': the reference's one-directional input gives the PE of its
    undirected graph (PyG to_undirected), checked against the oracle restatement on the
    symmetrized edges (eigenvalues vs dense eigh, well-separated columns, the span)."""
    from etpgt.encodings.laplacian_gpu import to_undirected

    ei = _one_directional(n, m, seed=n) if n > 4 else torch.tensor([[0, 0, 1, 1, 2, 2], [1, 2, 2, 3, 3, 2]])
    und = torch.from_numpy(to_undirected(ei, n))
    Lm = R.ref_sym_laplacian(und.numpy(), n)
    lam_all, vec_all = np.linalg.eigh(Lm.toarray().astype(np.float64))
    pe = compute_laplacian_pe_gpu(ei, n, k=k, tol=1e-5, directed="symmetrize").cpu().numpy()
    assert pe.shape == (n, k) and (pe >= 0).all()
    want = R.ref_compute_laplacian_pe(und, n, k=k).numpy()
    lam_ctx = np.concatenate([lam_all[: k + 2], [np.inf]])
    checked = _check_columns(pe, want, lam_ctx)
    assert checked >= 1
    op = LaplacianOperator(ei, n, "cuda", directed="symmetrize")
    lam, X, _ = lobpcg_smallest(op, k + 1, tol=1e-5)
    np.testing.assert_allclose(lam, lam_all[: k + 1], atol=1e-5)
    if lam_all[k + 1] - lam_all[k] > 1e-3:
        Xn = X.cpu().numpy().astype(np.float64)
        Vr = vec_all[:, : k + 1]
        assert np.abs(Xn @ Xn.T - Vr @ Vr.T).max() < 1e-3


def test_lappe_gpu_rejects_out_of_range():
    ei = torch.tensor([[0, 5], [5, 0]])
    with pytest.raises(IndexError):
        LaplacianOperator(ei, 4, "cuda")


@pytest.mark.parametrize("n,m", [(1000, 1), (12345, 21), (3000, 63), (777, 64)])
def test_gram_kernel_matches_fp64(n, m):
    """gtr_lap_gram (the solver's S^T S | S^T Y in fp64) against numpy in fp64."""
    ei = _graph(n, n, seed=1)
    op = LaplacianOperator(ei, n, "cuda")
    g = torch.Generator().manual_seed(m)
    S = torch.randn(n, m, generator=g)
    Y = torch.randn(n, m, generator=g)
    GH = op.gram(S.cuda(), Y.cuda())
    Sd, Yd = S.double().numpy(), Y.double().numpy()
    np.testing.assert_allclose(GH[0], Sd.T @ Sd, rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(GH[1], Sd.T @ Yd, rtol=1e-12, atol=1e-9)
