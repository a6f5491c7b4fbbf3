"""ETP-GT hot path on MI355X (gfx950): the reference's etpgt.model / etpgt.train /
etpgt.encodings API over hand-written HIP kernels (libgtr_hip.so)."""

__version__ = "0.1.0"
