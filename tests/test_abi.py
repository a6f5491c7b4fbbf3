"""The C-ABI library: builds, loads without a GPU, and exports every symbol that
include/gtr.h declares (no compute calls here)."""

import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gtr.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gtr_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def libpath():
    from etpgt.backend import _lib

    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(ROOT, "gat-recommendation_amd", "csrc"), "-j8"], check=True)
    return _lib.LIB_PATH


def test_header_declares_the_boundary():
    fns = header_functions()
    for required in ("gtr_conv_fwd", "gtr_conv_bwd", "gtr_readout_loss", "gtr_wgrad", "gtr_adamw_small",
                     "gtr_adamw_rows", "gtr_adamw_sweep", "gtr_contrib_prep", "gtr_contrib_sort",
                     "gtr_version", "gtr_device_check", "gtr_last_error"):
        assert required in fns


def test_library_exports_every_header_symbol(libpath):
    h = ctypes.CDLL(libpath)
    missing = [f for f in header_functions() if not hasattr(h, f)]
    assert not missing, missing


def test_python_binding_matches_header(libpath):
    from etpgt.backend import _lib

    assert set(_lib.EXPORTS) == set(header_functions())
    lib = _lib.lib()
    assert lib.gtr_abi_version() == _lib.ABI_VERSION == 8
    assert lib.gtr_version() >= 100


def test_struct_layouts_match_header():
    """ctypes mirrors of the ABI structs: field order/count as declared in gtr.h."""
    from etpgt.backend import _lib

    src = open(HEADER).read()
    for cname, py in (("gtr_batch", _lib.GtrBatch), ("gtr_config", _lib.GtrConfig), ("gtr_layer", _lib.GtrLayer), ("gtr_ffn", _lib.GtrFfn),
                      ("gtr_embed", _lib.GtrEmbed), ("gtr_head", _lib.GtrHead), ("gtr_segment", _lib.GtrSegment),
                      ("gtr_adam", _lib.GtrAdam), ("gtr_tail", _lib.GtrTail), ("gtr_dp_layout", _lib.GtrDpLayout),
                      ("gtr_sweep", _lib.GtrSweep), ("gtr_sessions", _lib.GtrSessions),
                      ("gtr_lazy", _lib.GtrLazy)):
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), src, re.S).group(1)
        body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
        names = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            parts = [t for t in decl.replace("*", " ").split() if t not in ("struct", "const")]
            # "int32_t n_cap, b_cap, e_cap" declares several fields
            tail = " ".join(parts[1:])
            names += [n.split("[")[0].strip() for n in tail.split(",") if n.strip()]  # arrays: name only
        assert [f[0] for f in py._fields_] == names, cname


def test_status_codes_raise(libpath):
    from etpgt.backend import _lib

    lib = _lib.lib()
    rc = lib.gtr_conv_fwd(None, None, None, None, 0, None)
    assert rc != 0
    with pytest.raises(RuntimeError, match="bad arguments"):
        _lib.check(rc, "conv_fwd")


def test_split_gemms_refuse_rows_past_the_buffer_offset_reach(libpath):
    """The split-path GEMMs store through raw buffers with 32-bit byte offsets: a batch whose
    n_cap rows of 4D floats exceed 4 GB is refused before any device work (argument check
    only, no GPU needed)."""
    from etpgt.backend import _lib

    lib = _lib.lib()
    cfg = _lib.GtrConfig(num_items=100, dim=128, heads=4, num_layers=2, training=1, row_group=16)
    bt = _lib.GtrBatch(n_cap=(1 << 32) // (4 * 128 * 4), b_cap=1, e_cap=1, n_neg=1)
    layers = (_lib.GtrLayer * 2)()
    emb = _lib.GtrEmbed()
    rc = lib.gtr_qkvs_fwd(ctypes.byref(cfg), ctypes.byref(bt), ctypes.byref(emb), layers, 1, None)
    assert rc != 0
    assert "4 GB" in lib.gtr_last_error().decode()
    rc = lib.gtr_qkvs_bwd(ctypes.byref(cfg), ctypes.byref(bt), layers, 1, None, None)
    assert rc != 0
    assert "4 GB" in lib.gtr_last_error().decode()


def test_lap_plan_is_nnz_balanced(libpath):
    """gtr_lap_plan (host-only): every nonzero lands in exactly one item of <= chunk
    nonzeros, in row order; split rows list their consecutive partial slots."""
    import numpy as np

    from etpgt.backend import _lib

    rng = np.random.default_rng(0)
    deg = rng.integers(0, 40, 500)
    deg[[3, 77, 499]] = [1000, 129, 128]  # hub rows, one just over / at the chunk
    ptr = np.zeros(501, np.int32)
    np.cumsum(deg, out=ptr[1:])
    lib = _lib.lib()
    ni, ns, npart = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    assert lib.gtr_lap_plan(ptr.ctypes.data, 500, 128, None, ctypes.byref(ni), None, ctypes.byref(ns),
                            ctypes.byref(npart)) == 0
    items = np.empty((ni.value, 4), np.int32)
    splits = np.empty((ns.value, 4), np.int32)
    assert lib.gtr_lap_plan(ptr.ctypes.data, 500, 128, items.ctypes.data, ctypes.byref(ni), splits.ctypes.data,
                            ctypes.byref(ns), ctypes.byref(npart)) == 0
    assert ns.value == 2 and npart.value == 8 + 2 and ni.value == 498 + 10
    assert (items[:, 2] - items[:, 1] <= 128).all() and (items[:, 2] >= items[:, 1]).all()
    assert np.array_equal(items[:, 1][1:], items[:, 2][:-1])  # contiguous cover of [0, nnz)
    assert items[0, 1] == 0 and items[-1, 2] == ptr[-1]
    assert np.array_equal(np.unique(items[:, 0]), np.arange(500))
    assert splits[:, 0].tolist() == [3, 77] and splits[:, 1:3].tolist() == [[0, 8], [8, 10]]
    split_items = items[items[:, 3] >= 0]
    assert split_items[:, 3].tolist() == list(range(10))
    assert (items[~np.isin(items[:, 0], [3, 77]), 3] == -1).all()
    bad = np.array([0, 5, 3], np.int32)
    assert lib.gtr_lap_plan(bad.ctypes.data, 2, 128, None, ctypes.byref(ni), None, ctypes.byref(ns),
                            ctypes.byref(npart)) != 0


def test_library_built_from_this_tree(libpath):
    """The loaded libgtr_hip.so carries the hash of the sources it was compiled from
    (Makefile -> gtr_source_hash): it must be this tree's, so a stale binary never runs
    the tests or the bench (rebuild: make -C gat-recommendation_amd/csrc)."""
    from etpgt.backend import _lib

    assert _lib.library_source_hash() == _lib.source_hash()


def test_kernels_are_registered_torch_library_ops():
    """the HIP entry points are torch.library ops of the ``etpgt`` namespace
    (FX / torch.compile / fake-tensor tracing see them), each with a fake implementation
    for shape inference -- checked here without a GPU (no kernel runs under FakeTensorMode)."""
    import torch
    from torch._subclasses.fake_tensor import FakeTensorMode

    from etpgt.backend import ops  # noqa: F401  (registers the ops)

    for name in ("score_loss", "score_rows_grad", "score_topk", "graph_transformer_eval"):
        assert hasattr(torch.ops.etpgt, name), name
    with FakeTensorMode():
        se, tab = torch.empty(4, 64), torch.empty(100, 64)
        t, n = torch.zeros(4, dtype=torch.long), torch.zeros(4, 5, dtype=torch.long)
        loss, dse, ct, cn = torch.ops.etpgt.score_loss(se, tab, t, n, 2, 1.0, 0.7)
        assert loss.shape == () and dse.shape == (4, 64) and ct.shape == (4,) and cn.shape == (20,)
        assert torch.ops.etpgt.score_rows_grad(se, ct, cn, t, n, 100).shape == (100, 64)
        idx, sc = torch.ops.etpgt.score_topk(se, tab, 10, None, None)
        assert idx.shape == (4, 10) and idx.dtype == torch.int64 and sc.shape == (4, 10)
        blob = torch.zeros(64, dtype=torch.int32)
        out = torch.ops.etpgt.graph_transformer_eval(blob, None, tab, [tab], 0, 16, 4, 16, 5, 4)
        assert out.shape == (4, 64)
