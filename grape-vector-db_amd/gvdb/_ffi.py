"""ctypes binding of libgvdb.so (the C ABI declared in include/gvdb.h).

The shared library is built in-tree (``grape-vector-db_amd/libgvdb.so``) by
``__graft_entry__.build()``.  There is no CPU fallback: if the library is
missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# GVDB_LIB_PATH: an alternative build (timing ablations only)
LIB_PATH = os.environ.get("GVDB_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "libgvdb.so")

# gvdb_status (include/gvdb.h)
GVDB_OK = 0
GVDB_ERR_INDEX_NOT_BUILT = 1
GVDB_ERR_DIMENSION_MISMATCH = 2
GVDB_ERR_INVALID_VECTOR_DIMENSION = 3
GVDB_ERR_QUANTIZATION = 4
GVDB_ERR_INDEX = 5
GVDB_ERR_INVALID_ARGUMENT = 6
GVDB_ERR_DEVICE = 7
GVDB_ERR_OUT_OF_MEMORY = 8
GVDB_ERR_STORAGE = 9

GVDB_METRIC_COSINE = 0
GVDB_METRIC_L2 = 1
GVDB_METRIC_COSINE_DISTANCE = 2
GVDB_SEARCH_BQ_RERANK = 0
GVDB_SEARCH_FLAT = 1
GVDB_N_POISONED = 0xFFFFFFFF
GVDB_COMM_ID_BYTES = 128


class gvdb_params(C.Structure):
    _fields_ = [
        ("dimension", C.c_uint32),
        ("bq_threshold", C.c_float),
        ("device", C.c_int32),
        ("reserved", C.c_uint32),
        ("capacity_hint", C.c_uint64),
    ]


class gvdb_search_params(C.Structure):
    _fields_ = [
        ("mode", C.c_uint32),
        ("metric", C.c_uint32),
        ("rescore_count", C.c_uint64),
        ("rescore_ratio", C.c_float),
        ("reserved", C.c_uint32),
    ]


class gvdb_index_stats(C.Structure):
    _fields_ = [
        ("vector_count", C.c_uint64),
        ("dimension", C.c_uint64),
        ("memory_usage", C.c_uint64),
        ("device_bytes", C.c_uint64),
    ]


class gvdb_bm25_params(C.Structure):
    _fields_ = [("k1", C.c_float), ("b", C.c_float), ("device", C.c_int32), ("reserved", C.c_uint32)]


class gvdb_bm25_stats(C.Structure):
    _fields_ = [
        ("total_documents", C.c_uint64),
        ("average_document_length", C.c_float),
        ("reserved", C.c_uint32),
        ("vocabulary_size", C.c_uint64),
        ("total_entries", C.c_uint64),
        ("dense_fallbacks", C.c_uint64),
    ]


class gvdb_persist_meta(C.Structure):
    _fields_ = [
        ("dimension", C.c_uint64),
        ("total_points", C.c_uint64),
        ("m", C.c_uint64),
        ("ef_construction", C.c_uint64),
        ("ef_search", C.c_uint64),
        ("max_layers", C.c_uint64),
        ("created_at", C.c_char * 64),
    ]


P = C.c_void_p
u32, u64, i32, f32 = C.c_uint32, C.c_uint64, C.c_int32, C.c_float
PU64, PU32, PF32 = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_float)

# name -> (restype, argtypes).  Every symbol include/gvdb.h declares.
SIGNATURES = {
    "gvdb_abi_version": (u32, []),
    "gvdb_last_error": (C.c_char_p, []),
    "gvdb_status_string": (C.c_char_p, [C.c_int]),
    "gvdb_last_dimension_mismatch": (None, [PU64, PU64]),
    "gvdb_device_count": (i32, []),
    "gvdb_timing_enable": (None, [i32]),
    "gvdb_timing_reset": (None, []),
    "gvdb_timing_read": (C.c_int, [u32, C.POINTER(C.c_double), PU64]),
    "gvdb_flat_fallback_count": (C.c_uint64, []),
    "gvdb_flat_i8_fallback_count": (C.c_uint64, []),
    "gvdb_index_create": (C.c_int, [C.POINTER(gvdb_params), C.POINTER(P)]),
    "gvdb_index_destroy": (None, [P]),
    "gvdb_index_add": (C.c_int, [P, P, u64, u32, P]),
    "gvdb_index_add_device": (C.c_int, [P, P, u64, u32, P, P]),
    "gvdb_index_build": (C.c_int, [P]),
    "gvdb_index_search": (C.c_int, [P, P, u64, u32, u64, C.POINTER(gvdb_search_params), P, P, P]),
    "gvdb_index_search_device": (C.c_int, [P, P, u64, u32, u64, C.POINTER(gvdb_search_params), P, P, P, P]),
    "gvdb_index_bq_topr_device": (C.c_int, [P, P, u64, u32, u64, P, P, P]),
    "gvdb_index_bq_candidates_device": (C.c_int, [P, P, u64, u32, u64, P, P, P, P]),
    "gvdb_index_search_filtered": (C.c_int, [P, P, u64, u32, u64, C.POINTER(gvdb_search_params), P, u64, P, P, P]),
    "gvdb_coalescer_create": (C.c_int, [P, u32, u64, C.POINTER(gvdb_search_params), u32, u32, C.POINTER(P)]),
    "gvdb_coalescer_search": (C.c_int, [P, P, P, P, P]),
    "gvdb_coalescer_stats": (C.c_int, [P, PU64, PU64, PU64]),
    "gvdb_coalescer_destroy": (None, [P]),
    "gvdb_index_remove": (C.c_int, [P, u64, C.POINTER(i32)]),
    "gvdb_index_len": (u64, [P]),
    "gvdb_index_is_empty": (i32, [P]),
    "gvdb_index_optimize": (C.c_int, [P]),
    "gvdb_index_clear": (None, [P]),
    "gvdb_index_get_stats": (C.c_int, [P, C.POINTER(gvdb_index_stats)]),
    "gvdb_index_device_rows": (P, [P]),
    "gvdb_index_export": (C.c_int, [P, P, P, u64, PU64]),
    "gvdb_persist_create": (C.c_int, [C.c_char_p, C.POINTER(gvdb_persist_meta), u64, i32, C.POINTER(P)]),
    "gvdb_persist_append": (C.c_int, [P, P, u64, u32, P, P]),
    "gvdb_persist_close": (C.c_int, [P]),
    "gvdb_persist_open": (C.c_int, [C.c_char_p, C.POINTER(gvdb_persist_meta), PU64, C.POINTER(P)]),
    "gvdb_persist_next": (C.c_int, [P, P, u32, u64, P, u64, P, PU64]),
    "gvdb_persist_free": (None, [P]),
    "gvdb_bq_quantize": (C.c_int, [P, u64, u32, f32, P]),
    "gvdb_bq_quantize_device": (C.c_int, [P, u64, u32, f32, P, P]),
    "gvdb_bq_hamming": (C.c_int, [P, P, u64, u32, P]),
    "gvdb_bq_multi_stage_search": (C.c_int, [P, u32, P, u32, u64, P, u64, P, u64, f32, P, P, PU64]),
    "gvdb_flat_search": (C.c_int, [P, u64, P, u64, u32, u64, u32, i32, f32, P, P, P]),
    "gvdb_topk_merge": (C.c_int, [P, P, P, u64, u64, u64, u64, i32, P, P, P]),
    "gvdb_topk_merge_device": (C.c_int, [P, P, P, u64, u64, u64, u64, i32, P, P, P, P]),
    "gvdb_bq_shard_merge": (C.c_int, [P, P, P, P, u64, u64, u64, u64, u64, P, P, P]),
    "gvdb_bq_shard_merge_device": (C.c_int, [P, P, P, P, u64, u64, u64, u64, u64, P, P, P, P]),
    "gvdb_bq_shard_merge_packed_device": (C.c_int, [P, P, u64, u64, u64, u64, P, P, P, P]),
    "gvdb_comm_get_unique_id": (C.c_int, [P]),
    "gvdb_comm_create": (C.c_int, [P, i32, i32, i32, C.POINTER(P)]),
    "gvdb_comm_destroy": (None, [P]),
    "gvdb_comm_info": (C.c_int, [P, C.POINTER(i32), C.POINTER(i32)]),
    "gvdb_index_search_sharded_device": (C.c_int, [P, P, P, u64, u32, u64, C.POINTER(gvdb_search_params), P, P, P,
                                                   P]),
    "gvdb_shard_sizes": (None, [u64, u64, u64, u32, PU64, PU64, PU64]),
    "gvdb_shard_flat_words": (u64, [u64, u64]),
    "gvdb_shard_stage1_device": (C.c_int, [P, P, u64, u32, u64, P, P, P]),
    "gvdb_shard_rerank_device": (C.c_int, [P, P, u64, u32, u64, u64, P, u64, u64, P, P, P]),
    "gvdb_shard_final_device": (C.c_int, [P, u64, u64, u64, P, P, P, P]),
    "gvdb_shard_flat_final_device": (C.c_int, [P, u64, u64, u64, u32, P, P, P, P]),
    "gvdb_shard_merge_host": (C.c_int, [P, u64, u64, u64, u64, P, P, P, P]),
    "gvdb_shard_deep_own_host": (C.c_int, [P, u64, u64, u64, u64, u32, P, P, P, P, P, P]),
    "gvdb_shard_local_topk_host": (C.c_int, [P, P, P, P, P, u64, u64, u64, u32, P]),
    "gvdb_shard_final_host": (C.c_int, [P, u64, u64, u64, P, P, P]),
    "gvdb_sparse_create": (C.c_int, [C.POINTER(gvdb_bm25_params), C.POINTER(P)]),
    "gvdb_sparse_destroy": (None, [P]),
    "gvdb_sparse_add_document": (C.c_int, [P, u64, P, P, u64, f32]),
    "gvdb_sparse_add_documents": (C.c_int, [P, P, P, P, P, P, u64]),
    "gvdb_sparse_remove_document": (C.c_int, [P, u64, C.POINTER(i32)]),
    "gvdb_sparse_get_stats": (C.c_int, [P, C.POINTER(gvdb_bm25_stats)]),
    "gvdb_sparse_clear": (None, [P]),
    "gvdb_sparse_search_bm25": (C.c_int, [P, P, P, P, u64, u64, P, P, P]),
    "gvdb_rrf_fuse": (C.c_int, [P, P, P, u32, P, P, P, u32, P, P, P, u32, u64, f32, u64, P, P, P, P]),
    "gvdb_rrf_fuse_device": (C.c_int, [P, P, P, u32, P, P, P, u32, P, P, P, u32, u64, f32, u64, P, P, P, P, P]),
}

_lib = None
_lock = threading.Lock()


def lib() -> C.CDLL:
    """Load libgvdb.so (fails loudly when the HIP build is missing)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"libgvdb.so not found at {LIB_PATH}: run __graft_entry__.build() "
                    "(there is no CPU fallback for the GPU search path)"
                )
            # One HIP runtime per process: PyTorch-ROCm bundles its own
            # libamdhip64 (SONAME libamdhip64.so.7, NEEDED as "libamdhip64.so").
            # Loading torch first makes libgvdb bind to that same copy; loading
            # libgvdb first would pull /opt/rocm's copy and torch would then
            # load a second runtime that sees no device.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            L = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def ptr(a) -> int:
    """Address of a numpy array / torch tensor / int."""
    if a is None:
        return None
    if isinstance(a, int):
        return a
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data
