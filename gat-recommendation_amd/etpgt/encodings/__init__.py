"""Positional encoding modules (reference: etpgt/encodings/__init__.py)."""

from etpgt.encodings.laplacian_pe import LaplacianPE, LaplacianPECached, compute_laplacian_pe

__all__ = ["compute_laplacian_pe", "LaplacianPE", "LaplacianPECached"]
