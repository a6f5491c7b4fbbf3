"""Hash of libgtr_hip's sources (csrc/*.hip, csrc/*.cuh, include/gtr.h).  The Makefile
compiles it into the library (gtr_source_hash) and profiles record it, so a stale binary
or a measurement taken on other kernels is recognisable.  Standalone (no torch): the
Makefile runs this file."""

from __future__ import annotations

import glob
import hashlib
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def source_hash() -> str:
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(PKG_ROOT, "csrc", "*.hip")) + glob.glob(os.path.join(PKG_ROOT, "csrc", "*.cuh"))
                   + [os.path.join(os.path.dirname(PKG_ROOT), "include", "gtr.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())
