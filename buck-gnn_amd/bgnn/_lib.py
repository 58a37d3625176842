"""ctypes binding of libbgnn.so (declared in include/bgnn.h).

This is the drop-in boundary: every GPU computation of the package goes through
these C-ABI entry points. There is no CPU fallback — if the library cannot be
loaded, or a tensor is not on a ROCm device, the call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# BGNN_LIBRARY: a measurement build of the same ABI (make -C buck-gnn_amd m16), for tools/ only
LIB_PATH = os.environ.get("BGNN_LIBRARY") or os.path.join(_HERE, "_lib", "libbgnn.so")
ABI_VERSION = 13

_lock = threading.Lock()
_lib = None

c_p = ctypes.c_void_p
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_u64 = ctypes.c_uint64
c_sz = ctypes.c_size_t


class CsrStruct(ctypes.Structure):
    """Mirror of `bgnn_csr_t` (include/bgnn.h)."""

    _fields_ = [
        ("rowptr", c_p),
        ("col", c_p),
        ("heavy_row", c_p),
        ("heavy_chunk0", c_p),
        ("chunk_heavy", c_p),
        ("n_rows", c_i64),
        ("nnz", c_i64),
        ("n_heavy", c_i32),
        ("n_chunks", c_i32),
        ("chunk", c_i32),
        ("ranges_all", c_i32),
        ("gsrc", c_p),
        ("gmask", c_p),
        ("gcnt", c_p),
        ("grow", c_p),
        ("n_groups", c_i64),
        ("group_rows", c_i32),
        ("_pad2", c_i32),
        ("ranges", c_p),
    ]


# name -> (restype, argtypes)
SIGNATURES = {
    "bgnn_abi_version": (c_i32, []),
    "bgnn_last_error_string": (ctypes.c_char_p, []),
    "bgnn_store_gather_graph": (c_i32, [c_p, c_i32, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p,
                                        c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "bgnn_store_gather_rows": (c_i32, [c_p, c_i32, c_i32, c_i64, c_p, c_i64, c_p, c_p]),
    "bgnn_get_tuning": (c_i32, [c_i32]),
    "bgnn_heavy_timing": (c_i32, [c_i32]),
    "bgnn_gemm_w_tile": (c_i32, [c_i64, c_i64, c_i64]),
    "bgnn_gemm_wsplit_bytes": (c_sz, [c_i64, c_i64]),
    "bgnn_gemm_wsplit": (c_i32, [c_p, c_i32, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_i32, c_p]),
    "bgnn_gemm_f32_w": (c_i32, [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i32, c_p, c_i64, c_p, c_i32, c_p, c_p, c_p,
                                c_p, c_i64, c_f32, c_u64, c_p]),
    "bgnn_heavy_timing_read": (c_i32, [c_i32, c_p, c_p]),
    "bgnn_set_tuning": (c_i32, [c_i32, c_i32]),
    "bgnn_graph_build_ws_bytes": (c_sz, [c_i64, c_i64]),
    "bgnn_graph_build": (c_i32, [c_p, c_i64, c_i64, c_p, c_p, c_p, c_p, c_p, c_p, c_sz, c_p, c_p]),
    "bgnn_index_csr_build": (c_i32, [c_p, c_i64, c_i64, c_p, c_p, c_p, c_sz, c_p, c_p]),
    "bgnn_heavy_plan_ws_bytes": (c_sz, [c_i64]),
    "bgnn_heavy_plan": (c_i32, [c_p, c_i64, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "bgnn_spmm_fwd": (c_i32, [ctypes.POINTER(CsrStruct), c_p, c_i64, c_i32, c_i32, c_p, c_i64, c_p, c_p, c_p]),
    "bgnn_spmm_bwd": (c_i32, [ctypes.POINTER(CsrStruct), c_p, c_p, c_p, c_i64, c_i32, c_i32, c_p, c_i64, c_p, c_p,
                              c_i32, c_p]),
    "bgnn_heavy_ranges_bytes": (c_sz, [c_i32]),
    "bgnn_heavy_ranges": (c_i32, [ctypes.POINTER(CsrStruct), c_p, c_p]),
    "bgnn_range_partial_bytes": (c_sz, [c_i64, c_i32]),
    "bgnn_range_sums_finish": (c_i32, [c_p, c_i64, c_i32, ctypes.POINTER(CsrStruct), c_i32, c_p, c_i64, c_p, c_p,
                                       c_p]),
    "bgnn_bn_slots": (c_i32, [c_i64, c_i32]),
    "bgnn_bn_stats": (c_i32, [c_p, c_i64, c_i32, c_p, c_p]),
    "bgnn_bn_apply": (c_i32, [c_p, c_i64, c_i32, c_p, c_p, c_p, c_p]),
    "bgnn_bn_bwd_stats": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_i32, c_p, c_p]),
    "bgnn_bn_bwd_dx": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_i32, c_p, c_p]),
    "bgnn_spmm_bwd_add": (c_i32, [ctypes.POINTER(CsrStruct), c_p, c_p, c_p, c_i64, c_i32, c_i32, c_p, c_i64, c_p,
                                  c_i64, c_p, c_p, c_p]),
    "bgnn_spmm_bwd_max": (c_i32, [ctypes.POINTER(CsrStruct), c_p, c_p, c_i64, c_p, c_i64, c_i32, c_p, c_p, c_i64, c_p,
                                  c_i64, c_p, c_p, c_p]),
    "bgnn_spmm_max_arg_bytes": (c_sz, [c_i64, c_i32, c_i32]),
    "bgnn_sage_fwd_slots": (c_i32, [ctypes.POINTER(CsrStruct)]),
    "bgnn_group_plan": (c_i32, [c_p, c_p, c_i64, c_i32, c_i32, c_p, c_i64, c_p, c_p, c_p, c_p]),
    "bgnn_store_gather_groups": (c_i32, [c_p, c_i32, c_i32, c_i64, c_i64, c_i64, c_i64] + [c_p] * 14),
    "bgnn_sage_fwd": (c_i32, [ctypes.POINTER(CsrStruct), c_p, c_i64, c_p, c_i64, c_p, c_i32, c_i32, c_p, c_p, c_p,
                              c_p, c_p, c_i64, c_p]),
    "bgnn_bn_finalize": (c_i32, [c_p, c_i32, c_i32, c_i64, c_p, c_p, c_f32, c_f32, c_p, c_p, c_p, c_p, c_p, c_p,
                                 c_p]),
    "bgnn_bn_finalize_shifted": (c_i32, [c_p, c_i32, c_i32, c_i64, c_p, c_p, c_p, c_f32, c_f32, c_p, c_p, c_p, c_p, c_p, c_p,
                                 c_p]),
    "bgnn_bn_eval_coeffs": (c_i32, [c_i32, c_p, c_p, c_f32, c_p, c_p, c_p, c_p, c_p]),
    "bgnn_sage_apply": (c_i32, [c_p, c_p, c_p, c_p, c_i32, c_f32, c_u64, c_i64, c_i32, c_p, c_p, c_p, c_p, c_p]),
    "bgnn_rows_slots": (c_i32, [c_i64]),
    "bgnn_sage_bwd_stats": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f32, c_u64, c_i64, c_i32, c_p, c_p]),
    "bgnn_reduce_partials": (c_i32, [c_p, c_i32, c_i32, c_p, c_p, c_i32, c_p]),
    "bgnn_linear_bwd_prep_slots": (c_i32, []),
    "bgnn_linear_bwd_prep": (c_i32, [c_p, c_p, c_i64, c_i32, c_p, c_p, c_p, c_p]),
    "bgnn_linear_bwd_prep_bf16": (c_i32, [c_p, c_p, c_i64, c_i32, c_p, c_p, c_p]),
    "bgnn_absmax_items_f32": (c_i32, [c_p, c_i32, c_i64, c_i64, c_i64, c_i64, c_p, c_i64, c_p]),
    "bgnn_add_dropped_bf16": (c_i32, [c_p, c_p, c_i64, c_f32, c_u64, c_p, c_p]),
    "bgnn_gemm_bf16_dropadd": (c_i32, [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_f32,
                                       c_u64, c_p]),
    "bgnn_rel_error_loss": (c_i32, [c_p, c_p, c_i64, c_f32, c_f32, c_f32, c_p, c_p, c_p]),
    "bgnn_small_linear_fwd": (c_i32, [c_p, c_i64, c_i32, c_p, c_p, c_i32, c_i32, c_p, c_p]),
    "bgnn_small_linear_bwd": (c_i32, [c_p, c_p, c_p, c_i64, c_i32, c_p, c_i32, c_p, c_p, c_p, c_p]),
    "bgnn_sage_bwd_rows": (c_i32, [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_f32, c_u64, c_i32, c_i64,
                                   c_i32, c_p, c_i64, c_p, c_p, c_p, c_p, c_i32, c_p, c_p, c_p, c_p]),
    "bgnn_l2norm_bwd": (c_i32, [c_p, c_p, c_p, c_i64, c_i32, c_p, c_i64, c_p, c_p, c_p]),
    "bgnn_gemm_bf16": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_f32, c_p, c_i64, c_p, c_i64, c_f32, c_p, c_i64,
                               c_p, c_i32, c_i32, c_p, c_sz, c_p]),
    "bgnn_gemm_gather_add_bf16": (c_i32, [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i32, c_p,
                                          c_p, c_i64, c_p, c_p, c_i64, c_i32, c_p, c_sz, c_p]),
    "bgnn_gemm_b16_variant": (c_i32, [c_i32]),
    "bgnn_add_dropout_bf16": (c_i32, [c_p, c_p, c_i64, c_f32, c_u64, c_p, c_p]),
    "bgnn_segment_sum_bf16": (c_i32, [c_p, c_p, c_i64, c_p, c_i64, c_i32, c_i32, c_p, c_i64, c_p]),
    "bgnn_segment_bcast_bf16": (c_i32, [c_p, c_p, c_i64, c_p, c_i64, c_i32, c_i32, c_p, c_i64, c_p]),
    "bgnn_gemm_ws_bytes": (c_sz, [c_i64, c_i64, c_i64, c_i32, c_i32]),
    "bgnn_gemm_set_cfg": (c_i32, [c_i32]),
    "bgnn_gemm_f32_planes": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_f32, c_p, c_i64, c_i64, c_i64, c_p, c_i64,
                                     c_f32, c_p, c_i64, c_i64, c_i64, c_p, c_i32, c_p, c_sz, c_p]),
    "bgnn_gemm_f32_scaled": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_f32, c_p, c_i64, c_i64, c_i64, c_p, c_i64,
                                     c_f32, c_p, c_i64, c_i64, c_i64, c_p, c_i32, c_p, c_p, c_p, c_i32, c_p, c_sz,
                                     c_p]),
    "bgnn_gemm_ws_bytes_ex": (c_sz, [c_i64, c_i64, c_i64, c_i32, c_i32, c_i32]),
    "bgnn_gemm_gather_add": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i32,
                                     c_p, c_p, c_i64, c_p, c_p, c_i64, c_i32, c_p, c_sz, c_p]),
    "bgnn_absmax_f32": (c_i32, [c_p, c_i64, c_i64, c_i64, c_p, c_i32, c_p]),
    "bgnn_gemm_f32_ex": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_f32, c_p, c_i64, c_p, c_i64, c_f32, c_p,
                                 c_i64, c_p, c_i32, c_p, c_sz, c_p]),
    "bgnn_topk_rank": (c_i32, [c_p, c_p, c_p, c_i64, c_p, c_p]),
    "bgnn_topk_select": (c_i32, [c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, c_p]),
    "bgnn_gather_scale": (c_i32, [c_p, c_i64, c_i32, c_p, c_p, c_i64, c_p, c_i64, c_p]),
    "bgnn_gather_scale_bwd": (c_i32, [c_p, c_i64, c_p, c_i64, c_i32, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p]),
    "bgnn_filter_edges_ws_bytes": (c_sz, [c_i64]),
    "bgnn_filter_edges": (c_i32, [c_p, c_i64, c_p, c_i64, c_p, c_p, c_p, c_p, c_sz, c_p]),
    "bgnn_mlp2_supported": (c_i32, [c_i32, c_i32, c_i32]),
    "bgnn_mlp2_fwd": (c_i32, [c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p]),
    "bgnn_mlp2_bwd_ws_bytes": (c_sz, [c_i64]),
    "bgnn_mlp2_bwd": (c_i32, [c_p, c_i64, c_i32, c_i32, c_i32, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p,
                              c_sz, c_p]),
    "bgnn_gemm_f32_dropadd": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p,
                                      c_p, c_p, c_i64, c_f32, c_u64, c_p, c_sz, c_p]),
    "bgnn_gemm_f32_dropadd_cols": (c_i32, [c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_p,
                                           c_i64, c_i64, c_f32, c_u64, c_p, c_sz, c_p]),
    "bgnn_add_dropout": (c_i32, [c_p, c_p, c_i64, c_f32, c_u64, c_p, c_p]),
    "bgnn_gemm_f32": (c_i32, [c_i32, c_i32, c_i64, c_i64, c_i64, c_f32, c_p, c_i64, c_p, c_i64, c_f32, c_p, c_i64,
                              c_p, c_sz, c_p]),
}


class BgnnError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed with code {code}: {msg}")
        self.code = code


def load():
    """Load libbgnn.so once; raises if it is missing or ABI-incompatible."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"bgnn: native library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C buck-gnn_amd`")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.bgnn_abi_version()
        if v != ABI_VERSION:
            raise ImportError(f"bgnn: ABI version mismatch (library {v}, python {ABI_VERSION})")
        _lib = lib
        return lib


def _checked(lib, name: str, args):
    """The entry point, after checking the argument count against its SIGNATURES entry (ctypes
    passes surplus arguments on as C varargs, which shifts nothing it can see but everything the
    callee reads: a stale caller would hand the kernels wrong pointers)."""
    fn = getattr(lib, name)
    sig = SIGNATURES.get(name)
    if sig is not None and len(args) != len(sig[1]):
        raise TypeError(f"bgnn: {name} takes {len(sig[1])} arguments, {len(args)} given")
    return fn


def call(name: str, *args):
    """Call a status-returning entry point and raise BgnnError on failure."""
    lib = load()
    rc = _checked(lib, name, args)(*args)
    if rc != 0:
        msg = lib.bgnn_last_error_string().decode(errors="replace")
        raise BgnnError(name, rc, msg)
    return rc


def query(name: str, *args):
    """Call a value-returning entry point (sizes, slot counts)."""
    lib = load()
    return _checked(lib, name, args)(*args)
