"""ctypes binding of libgtr_hip.so (the C ABI declared in include/gtr.h).

This is the FFI a maintainer of the reference would add: plain
pointers, int sizes and a hipStream_t; non-zero status -> RuntimeError with the
library's message.  The library is built in-tree (``gat-recommendation_amd/build``)
by ``__graft_entry__.build()`` / ``make -C gat-recommendation_amd/csrc``.  There is
no fallback: if the library is missing, every compute call raises.
"""

from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(os.path.dirname(_HERE))  # gat-recommendation_amd/
LIB_PATH = os.environ.get("GTR_LIB", os.path.join(PKG_ROOT, "build", "libgtr_hip.so"))

P = C.c_void_p
i32 = C.c_int32
i64 = C.c_int64
f32 = C.c_float
u32 = C.c_uint32


class GtrBatch(C.Structure):
    _fields_ = [
        ("hdr", P), ("node_item", P), ("node_ptr", P), ("in_ptr", P), ("in_src", P),
        ("out_ptr", P), ("out_edge", P), ("out_dst", P), ("target", P), ("negatives", P),
        ("node_pe", P), ("grp_row", P), ("grp_edge", P),
        ("n_cap", i32), ("b_cap", i32), ("e_cap", i32), ("n_neg", i32),
    ]


class GtrConfig(C.Structure):
    _fields_ = [
        ("num_items", i32), ("dim", i32), ("heads", i32), ("pe_k", i32), ("num_layers", i32),
        ("row_group", i32), ("training", i32), ("dropout", f32), ("bn_eps", f32),
        ("bn_momentum", f32), ("seed", u32), ("rng_ctr", P), ("consumer_reduce", i32), ("sync_bn", i32),
        ("sweep", P), ("begin", P), ("ctr_add", i32), ("split_sync", i32), ("loss_batch", f32),
        ("wfold_stride", i64),
    ]


class GtrBegin(C.Structure):
    _fields_ = [("skeys", P), ("svals", P), ("stamp", P), ("step_dev", P), ("num_items", i32), ("pad", i32)]


class GtrLayer(C.Structure):
    _fields_ = [
        ("w_all", P), ("b_all", P), ("w_beta", P), ("bn_gamma", P), ("bn_beta", P),
        ("bn_rmean", P), ("bn_rvar", P), ("bn_nbt", P),
        ("xin", P), ("qkvs", P), ("alpha", P), ("agg", P), ("gate", P), ("out", P),
        ("bn_stats", P), ("bn_part", P), ("bn_gsum", P), ("bn_gpart", P), ("cnt", P),
        ("dy", P), ("dqkvs", P), ("du", P), ("dlogit", P), ("dagg", P),
        ("bn_part_all", P), ("bn_gpart_all", P), ("nparts_fwd", i32), ("nparts_bwd", i32), ("wfold", P),
        ("ffn", P),
    ]


class GtrFfn(C.Structure):
    _fields_ = [
        ("w1", P), ("b1", P), ("w2", P), ("b2", P), ("y", P), ("a", P), ("z", P), ("dz", P), ("g2", P), ("da", P),
        ("expansion", i32), ("pad", i32),
    ]


class GtrEmbed(C.Structure):
    _fields_ = [("table", P), ("pe_tab", P), ("wpe", P), ("bpe", P)]


class GtrHead(C.Structure):
    _fields_ = [
        ("flags", i32), ("loss_kind", i32), ("temperature", f32), ("dual_alpha", f32),
        ("se", P), ("dse_in", P), ("dse_out", P), ("coef_tgt", P), ("coef_neg", P),
        ("loss_part", P), ("loss_out", P), ("cnt", P),
    ]


class GtrSegment(C.Structure):
    _fields_ = [
        ("begin", i64), ("len", i64), ("src", P), ("pstride", i64), ("nparts", i32), ("live_groups", i32),
    ]


class GtrAdam(C.Structure):
    _fields_ = [
        ("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("weight_decay", f32),
        ("decoupled", i32), ("step_offset", i32), ("step_dev", P),
    ]


class GtrTail(C.Structure):
    _fields_ = [
        ("skeys", P), ("svals", P), ("dx0", P), ("se", P), ("coef_tgt", P), ("coef_neg", P),
        ("table", P), ("table_m", P), ("table_v", P), ("stamp", P),
        ("flat", P), ("flat_m", P), ("flat_v", P), ("flat_total", i64),
        ("loss_part", P), ("loss_out", P), ("loss_nparts", i32), ("pad0", i32), ("carry", P),
        ("sweep_from", i64), ("lazy_consts", P), ("rng_inc", P), ("loss_acc", P),
    ]


SWEEP_SLOTS = 8
ABI_VERSION = 8  # GTR_ABI_VERSION of include/gtr.h


class GtrLazy(C.Structure):
    _fields_ = [
        ("consts", P), ("cap", i32), ("pad", i32), ("cnt", P), ("table", P), ("m", P), ("v", P), ("opt", GtrAdam),
    ]


class GtrSessions(C.Structure):
    _fields_ = [
        ("sess_ptr", P), ("sess_items", P), ("sess_nodes", P), ("sess_edges", P),
        ("num_sessions", i32), ("num_items", i32),
    ]


class GtrSweep(C.Structure):
    _fields_ = [
        ("table", P), ("m", P), ("v", P), ("stamp", P), ("opt", GtrAdam), ("bounds", i64 * (SWEEP_SLOTS + 1)),
        ("dim", i32), ("blocks", i32), ("consts", P), ("lag", i32), ("pad", i32),
    ]


class GtrDpLayout(C.Structure):
    _fields_ = [
        ("flat_total", i64), ("loss_off", i64), ("keys_off", i64), ("rows_off", i64), ("words", i64),
        ("m_cap", i32), ("world", i32),
    ]


class GtrShard(C.Structure):
    _fields_ = [
        ("num_items", i32), ("world", i32), ("rank", i32), ("cap", i32), ("local_rows", i32), ("dim", i32),
        ("table", P), ("m", P), ("v", P), ("stamp", P), ("consts", P), ("consts_cap", i32), ("cap_s", i32),
        ("status", P), ("opt", GtrAdam), ("node_mark", P), ("grad_stride", i64), ("small_stride", i64),
        ("pack_parts", i32), ("pad1", i32),
    ]


GTR_LOSS = {"none": 0, "bpr": 1, "listwise": 2, "sampled_softmax": 2, "dual": 3}
RO_FWD, RO_LOSS, RO_BWD = 1, 2, 4
SMALL_MAX_SEG = 48

# name -> (restype, argtypes)
_SIGS = {
    "gtr_version": (C.c_int, []),
    "gtr_abi_version": (C.c_int, []),
    "gtr_source_hash": (C.c_char_p, []),
    "gtr_last_error": (C.c_char_p, []),
    "gtr_device_check": (C.c_int, [C.c_int]),
    "gtr_conv_fwd": (C.c_int, [P, P, P, P, C.c_int, P]),
    "gtr_readout_loss": (C.c_int, [P, P, P, P, P, P]),
    "gtr_conv_bwd": (C.c_int, [P, P, P, C.c_int, P, P]),
    "gtr_qkvs_fwd": (C.c_int, [P, P, P, P, C.c_int, P]),
    "gtr_attn_fwd": (C.c_int, [P, P, P, C.c_int, P]),
    "gtr_attn_bwd": (C.c_int, [P, P, P, C.c_int, P]),
    "gtr_qkvs_bwd": (C.c_int, [P, P, P, C.c_int, P, P]),
    "gtr_ffn_fwd": (C.c_int, [P, P, P, C.c_int, P]),
    "gtr_ffn_bwd": (C.c_int, [P, P, P, C.c_int, P]),
    "gtr_ffn_wgrad": (C.c_int, [P, P, P, C.c_int, P, C.c_int, i64, P]),
    "gtr_wgrad": (C.c_int, [P, P, P, P, P, P, P, C.c_int, i64, C.c_int, C.c_int, P]),
    "gtr_adamw_small": (C.c_int, [P, P, P, P, i64, P, C.c_int, P, P]),
    "gtr_contrib_prep": (C.c_int, [P, C.c_int, P, P, P, P, P]),
    "gtr_contrib_sort_bytes": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_size_t)]),
    "gtr_contrib_sort": (C.c_int, [P, P, P, P, C.c_int, C.c_int, P, C.c_size_t, P]),
    "gtr_adamw_rows": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P, P, P, P, P, P, P, P]),
    "gtr_adamw_sweep": (C.c_int, [C.c_int, C.c_int, P, P, P, P, P, P]),
    "gtr_scatter_rows": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P]),
    "gtr_step_end": (C.c_int, [P, P, P, C.c_int, P, P]),
    "gtr_readout_grid": (C.c_int, [C.c_int]),
    "gtr_dp_pack": (C.c_int, [P, C.c_int, C.c_int, P, P, C.c_int, P, P, P]),
    "gtr_dp_tail": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P, P]),
    "gtr_dp_union_stamp": (C.c_int, [P, i64, C.c_int, P, P, P]),
    "gtr_step_begin": (C.c_int, [P, C.c_int, P, P, P, P, P, P, P, P, C.c_size_t, P]),
    "gtr_step_tail": (C.c_int, [P, C.c_int, C.c_int, P, P, C.c_int, P, P]),
    "gtr_step_tail_wgrad": (C.c_int, [P, P, P, P, P, P, C.c_int, C.c_int64, P, P, C.c_int, P, P, C.c_int, P, P,
                                      C.c_int, P]),
    "gtr_step_begin_lazy": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P, P, P, P, C.c_size_t, P, P]),
    "gtr_lazy_flush": (C.c_int, [C.c_int, C.c_int, P, P, P, P]),
    "gtr_tail_carry_floats": (C.c_int, [C.c_int, C.c_int]),
    "gtr_edge_hash_slots": (C.c_int, [i64, C.POINTER(i64)]),
    "gtr_edge_hash_build": (C.c_int, [P, i64, P, i64, P]),
    "gtr_session_counts": (C.c_int, [P, P, i64, C.c_int, P, P, P]),
    "gtr_build_batch": (C.c_int, [P, P, i64, C.c_int, P, P, C.c_int, C.c_int, u32, P, P, P, P, P]),
    "gtr_build_batch_strided": (C.c_int, [P, P, i64, C.c_int, P, P, C.c_int, i64, C.c_int, u32, P, P, P, P, P]),
    "gtr_lap_build": (C.c_int, [P, P, C.c_int, P, P, P]),
    "gtr_lap_plan": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P]),
    "gtr_lap_spmm": (C.c_int, [P, P, C.c_int, C.c_int, P, i64, P, i64, P, P, P, f32, f32, P]),
    "gtr_lap_gram": (C.c_int, [P, P, C.c_int, C.c_int, P, C.c_int, P, P]),
    "gtr_shard_route_scratch": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_size_t)]),
    "gtr_shard_route": (C.c_int, [P, P, P, P, P, P, P, P, P, P, C.c_int, P, P, C.c_size_t, P]),
    "gtr_shard_serve": (C.c_int, [P, P, P, P]),
    "gtr_shard_pack": (C.c_int, [P, P, P, P, P, C.c_int, P, P, P]),
    "gtr_shard_update": (C.c_int, [P, P, P, P, P, i64, P]),
    "gtr_topk_workspace_bytes": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_size_t)]),
    "gtr_score_topk": (C.c_int, [P, C.c_int, C.c_int, P, C.c_int, C.c_int, P, P, P, C.c_size_t, P]),
    "gtr_score_topk_masked": (C.c_int, [P, C.c_int, C.c_int, P, C.c_int, C.c_int, P, P, P, P, P, C.c_size_t, P]),
}

EXPORTS = tuple(_SIGS)

_lib = None


class GtrLibraryMissing(RuntimeError):
    pass


def lib():
    """Load libgtr_hip.so once; raise loudly if it is absent (no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GtrLibraryMissing(
                f"libgtr_hip.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or "
                "`make -C gat-recommendation_amd/csrc` (hipcc --offload-arch=gfx950)"
            )
        h = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        if h.gtr_abi_version() != ABI_VERSION:
            raise RuntimeError("libgtr_hip.so ABI version mismatch")
        _lib = h
    return _lib


def source_hash() -> str:
    """Hash of the library's sources (csrc/*.hip, *.cuh, include/gtr.h).  Profiles
    record it, so a measurement taken on other kernels is recognisable as stale; the
    library carries the hash of the sources it was built from (gtr_source_hash)."""
    from etpgt.backend._srchash import source_hash as _h

    return _h()


def library_source_hash() -> str:
    """The source hash compiled into the loaded libgtr_hip.so."""
    return lib().gtr_source_hash().decode()


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().gtr_last_error().decode(errors="replace")
        raise RuntimeError(f"libgtr_hip {what} failed (status {status}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()
