"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over ``oracle/liboracle.so`` (built from gvdb_oracle.cpp: a
sequential C++ restatement of grape-vector-db's ANN hot path; see that
file's header for the parity status and the reference lines it follows).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline.  The
product path (grape-vector-db_amd/) never touches it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

P = C.c_void_p
u32, u64, i32, f32 = C.c_uint32, C.c_uint64, C.c_int32, C.c_float

_SIG = {
    "orc_rust_f32_as_usize": (u64, [f32]),
    "orc_bq_quantize": (None, [P, u64, u32, f32, P]),
    "orc_hamming": (u64, [P, P, u64]),
    "orc_similarity": (f32, [u64, u32]),
    "orc_cosine_manual": (f32, [P, u64, P, u64]),
    "orc_storage_cosine": (f32, [P, u64, P, u64]),
    "orc_cosine_distance": (f32, [P, u64, P, u64]),
    "orc_l2_distance": (f32, [P, u64, P, u64]),
    "orc_multi_stage_search": (C.c_int, [P, u32, P, u32, u64, P, u64, P, u64, f32, P, P, P, P, P]),
    "orc_multi_stage_search_batch": (C.c_int, [P, u32, P, u64, P, P, u64, f32, u64, P, P, P, C.c_int]),
    "orc_bq_topr_batch": (None, [P, P, u64, u32, u64, u64, P, P, C.c_int]),
    "orc_storage_vector_search": (None, [P, u64, P, u64, u64, u64, C.c_int, f32, P, P, P]),
    "orc_flat_cosine_distance_search": (None, [P, u64, P, u64, u64, u64, P, P, P]),
    "orc_exact_topk_cosine_batch": (None, [P, P, u64, u64, u64, u64, P, P, C.c_int]),
    "orc_ref_id_remap_seconds": (C.c_double, [u64, u64, u64, C.c_int]),
    "orc_flat_cosine_distance_batch": (None, [P, P, u64, u64, u64, u64, P, P, P, C.c_int]),
    "orc_shard_merge": (None, [P, P, P, u64, u64, u64, P, P, P]),
    "orc_row_norms": (None, [P, u64, u64, P]),
    "orc_bq_shard_merge": (None, [P, P, P, P, u64, u64, u64, u64, u64, P, P, P]),
    "orc_multi_stage_search_batch_r": (None, [P, u32, P, u64, P, P, u64, u64, C.c_int, P, P, C.c_int]),
    "hnsw_build": (C.c_void_p, [P, u64, u32, u32, u32, u64, C.c_int]),
    "bm25o_create": (C.c_void_p, [f32, f32]),
    "bm25o_free": (None, [C.c_void_p]),
    "bm25o_add": (None, [C.c_void_p, u64, P, P, u64, f32]),
    "bm25o_remove": (C.c_int, [C.c_void_p, u64]),
    "bm25o_stats": (None, [C.c_void_p, P, P, P]),
    "bm25o_search": (u64, [C.c_void_p, P, P, u64, u64, P, P]),
    "bm25o_rrf": (u64, [P, P, u64, P, P, u64, P, P, u64, f32, P, P, P, P, P]),
    "bm25o_search_batch": (None, [C.c_void_p, P, P, P, u64, u64, P, P, P, C.c_int]),
    "bm25o_add_csr": (None, [C.c_void_p, P, P, P, P, P, u64]),
    "hnsw_free": (None, [C.c_void_p]),
    "hnsw_build2": (C.c_void_p, [P, u64, u32, u32, u32, u64, C.c_int, C.c_int]),
    "hnsw_set_fast": (None, [C.c_void_p, C.c_int]),
    "hnsw_search": (C.c_int, [C.c_void_p, P, u64, u32, u32, C.c_int, P, P, P]),
}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        for n, (r, a) in _SIG.items():
            fn = getattr(L, n)
            fn.restype = r
            fn.argtypes = a
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if a is not None else None


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def rust_f32_as_usize(v: float) -> int:
    return int(lib().orc_rust_f32_as_usize(float(np.float32(v))))


def quantize(x, threshold: float = 0.0) -> np.ndarray:
    x = _f32(x)
    if x.ndim == 1:
        x = x.reshape(1, -1)
    n, D = x.shape
    out = np.zeros((n, (D + 7) // 8), np.uint8)
    lib().orc_bq_quantize(_p(x), n, D, threshold, _p(out))
    return out


def hamming(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    assert a.size == b.size  # hamming 0.1.3 asserts equal lengths
    return int(lib().orc_hamming(_p(a), _p(b), a.size))


def similarity(d: int, dim: int) -> float:
    return float(lib().orc_similarity(d, dim))


def cosine_manual(a, b) -> float:
    a, b = _f32(a), _f32(b)
    return float(lib().orc_cosine_manual(_p(a), a.size, _p(b), b.size))


def storage_cosine(a, b) -> float:
    a, b = _f32(a), _f32(b)
    return float(lib().orc_storage_cosine(_p(a), a.size, _p(b), b.size))


def cosine_distance(a, b) -> float:
    a, b = _f32(a), _f32(b)
    return float(lib().orc_cosine_distance(_p(a), a.size, _p(b), b.size))


def l2_distance(a, b) -> float:
    a, b = _f32(a), _f32(b)
    return float(lib().orc_l2_distance(_p(a), a.size, _p(b), b.size))


def multi_stage_search(q_bits, qdim, c_bits, cdim, q, cands, rescore_ratio=0.1, want_stage1=False):
    """quantization.rs:151-193.  Returns (idx[], cos[]) (+ stage-1 lists)."""
    c_bits = np.ascontiguousarray(c_bits, np.uint8)
    q_bits = np.ascontiguousarray(q_bits, np.uint8).reshape(-1)
    if q_bits.size == 0:
        q_bits = np.zeros(1, np.uint8)
    q = _f32(q).reshape(-1)
    cands = _f32(cands)
    N = cands.shape[0]
    clen = cands.shape[1] if cands.ndim == 2 else 0
    oi = np.zeros(max(N, 1), np.uint64)
    oc = np.zeros(max(N, 1), np.float32)
    n = C.c_uint64()
    s1i = np.zeros(max(N, 1), np.uint64) if want_stage1 else None
    s1s = np.zeros(max(N, 1), np.float32) if want_stage1 else None
    if c_bits.size == 0:
        c_bits = np.zeros((max(N, 1), 1), np.uint8)
    st = lib().orc_multi_stage_search(_p(q_bits), qdim, _p(c_bits), cdim, N, _p(q), q.size, _p(cands), clen,
                                      rescore_ratio, _p(oi), _p(oc), C.byref(n), _p(s1i), _p(s1s))
    if st != 0:
        raise RuntimeError(f"oracle multi_stage_search status {st}")
    r = n.value
    if want_stage1:
        return oi[:r], oc[:r], s1i[:N], s1s[:N]
    return oi[:r], oc[:r]


def multi_stage_search_batch(q_bits, c_bits, q, cands, rescore_ratio, R_cap, threads=0):
    q_bits = np.ascontiguousarray(q_bits, np.uint8)
    c_bits = np.ascontiguousarray(c_bits, np.uint8)
    q, cands = _f32(q), _f32(cands)
    B, D = q.shape
    N = cands.shape[0]
    oi = np.zeros((B, R_cap), np.uint64)
    oc = np.zeros((B, R_cap), np.float32)
    on = np.zeros(B, np.uint64)
    st = lib().orc_multi_stage_search_batch(_p(q_bits), D, _p(c_bits), N, _p(q), _p(cands), B, rescore_ratio, R_cap,
                                            _p(oi), _p(oc), _p(on), threads)
    if st != 0:
        raise RuntimeError(f"oracle multi_stage_search_batch status {st}")
    return oi, oc, on


def bq_topr_batch(q_bits, c_bits, dim, R, threads=0):
    q_bits = np.ascontiguousarray(q_bits, np.uint8)
    c_bits = np.ascontiguousarray(c_bits, np.uint8)
    B = q_bits.shape[0]
    N = c_bits.shape[0]
    r = min(R, N)
    oi = np.zeros((B, R), np.uint64)
    od = np.zeros((B, R), np.uint32)
    lib().orc_bq_topr_batch(_p(q_bits), _p(c_bits), N, dim, B, R, _p(oi), _p(od), threads)
    return oi[:, :r], od[:, :r]


def storage_vector_search(q, rows, limit, threshold=None):
    q, rows = _f32(q).reshape(-1), _f32(rows)
    N, D = rows.shape
    oi = np.zeros(max(limit, 1), np.uint64)
    os_ = np.zeros(max(limit, 1), np.float32)
    n = C.c_uint64()
    lib().orc_storage_vector_search(_p(q), q.size, _p(rows), N, D, limit, int(threshold is not None),
                                    float(threshold or 0.0), _p(oi), _p(os_), C.byref(n))
    return oi[:n.value], os_[:n.value]


def flat_cosine_distance_search(q, rows, k):
    q, rows = _f32(q).reshape(-1), _f32(rows)
    N, D = rows.shape
    oi = np.zeros(max(k, 1), np.uint64)
    os_ = np.zeros(max(k, 1), np.float32)
    n = C.c_uint64()
    lib().orc_flat_cosine_distance_search(_p(q), q.size, _p(rows), N, D, k, _p(oi), _p(os_), C.byref(n))
    return oi[:n.value], os_[:n.value]


def exact_topk_cosine_batch(q, rows, k, threads=0):
    q, rows = _f32(q), _f32(rows)
    B, D = q.shape
    N = rows.shape[0]
    oi = np.zeros((B, k), np.uint64)
    os_ = np.zeros((B, k), np.float32)
    lib().orc_exact_topk_cosine_batch(_p(q), _p(rows), N, D, B, k, _p(oi), _p(os_), threads)
    return oi, os_


def flat_cosine_distance_batch(q, rows, k, threads=0):
    """B independent flat_cosine_distance_search calls (one query per thread)."""
    q, rows = _f32(q), _f32(rows)
    B, D = q.shape
    N = rows.shape[0]
    oi = np.zeros((B, max(k, 1)), np.uint64)
    os_ = np.zeros((B, max(k, 1)), np.float32)
    on = np.zeros(B, np.uint64)
    lib().orc_flat_cosine_distance_batch(_p(q), _p(rows), N, D, B, k, _p(oi), _p(os_), _p(on), threads)
    return oi[:, :k], os_[:, :k], on


def ref_id_remap_seconds(N, k, nq, threads=0):
    """Mean seconds per query of HnswVectorIndex::search's O(N k) id remap
    (index.rs:219-228) restated with its string formatting (the ref-faithful
    variant's extra cost)."""
    return float(lib().orc_ref_id_remap_seconds(N, k, nq, threads))


def shard_merge(ids, scores, counts, limit):
    ids = np.ascontiguousarray(ids, np.uint64)
    scores = _f32(scores)
    counts = np.ascontiguousarray(counts, np.uint64)
    S, stride = ids.shape
    oi = np.zeros(max(limit, 1), np.uint64)
    os_ = np.zeros(max(limit, 1), np.float32)
    n = C.c_uint64()
    lib().orc_shard_merge(_p(ids), _p(scores), _p(counts), S, stride, limit, _p(oi), _p(os_), C.byref(n))
    return oi[:n.value], os_[:n.value]


def row_norms(rows):
    rows = _f32(rows)
    N, D = rows.shape
    out = np.zeros(N, np.float32)
    lib().orc_row_norms(_p(rows), N, D, _p(out))
    return out


def bq_shard_merge(gids, dist, cosv, counts, R, k):
    """gids/dist/cosv: [G, B, stride]; counts [G, B]."""
    gids = np.ascontiguousarray(gids, np.uint64)
    dist = np.ascontiguousarray(dist, np.uint32)
    cosv = _f32(cosv)
    counts = np.ascontiguousarray(counts, np.uint64)
    G, B, stride = gids.shape
    oi = np.zeros((B, max(k, 1)), np.uint64)
    os_ = np.zeros((B, max(k, 1)), np.float32)
    on = np.zeros(B, np.uint64)
    lib().orc_bq_shard_merge(_p(gids), _p(dist), _p(cosv), _p(counts), G, B, stride, R, k, _p(oi), _p(os_), _p(on))
    return oi[:, :k], os_[:, :k], on


def multi_stage_search_batch_r(q_bits, c_bits, q, cands, R, kind=0, threads=0):
    """Explicit-R multi-stage search (kind 0 cosine desc, 1 L2 asc, 2 cosine distance asc)."""
    q_bits = np.ascontiguousarray(q_bits, np.uint8)
    c_bits = np.ascontiguousarray(c_bits, np.uint8)
    q, cands = _f32(q), _f32(cands)
    B, D = q.shape
    N = cands.shape[0]
    r = min(R, N)
    oi = np.zeros((B, R), np.uint64)
    os_ = np.zeros((B, R), np.float32)
    lib().orc_multi_stage_search_batch_r(_p(q_bits), D, _p(c_bits), N, _p(q), _p(cands), B, R, kind, _p(oi), _p(os_),
                                         threads)
    return oi[:, :r], os_[:, :r]


class Hnsw:
    """instant-distance 0.6.1 restatement (oracle/hnsw_oracle.cpp): the CPU-HNSW
    baseline of HnswVectorIndex (index.rs:140-154, 212-231).  Distances are L2
    (index.rs:64-79).  Recall-only parity; the rows array must stay alive."""

    def __init__(self, rows, M=32, ef_construction=100, seed=0x6772617065, threads=0, fast=False):
        """fast=True builds with re-associated (AVX2) L2 sums instead of the
        reference's strict fold (hnsw_oracle.cpp, l2_fast)."""
        self.rows = _f32(rows)
        n, d = self.rows.shape
        self.d = d
        self.h = lib().hnsw_build2(_p(self.rows), n, d, M, ef_construction, seed, threads, int(fast))
        if not self.h:
            raise ValueError("hnsw_build failed")

    def search(self, q, k=10, ef_search=100, threads=0, fast=False):
        lib().hnsw_set_fast(self.h, int(fast))
        q = _f32(q).reshape(-1, self.d)
        B = q.shape[0]
        ids = np.zeros((B, k), dtype=np.uint64)
        dist = np.zeros((B, k), dtype=np.float32)
        n = np.zeros(B, dtype=np.uint32)
        if lib().hnsw_search(self.h, _p(q), B, k, ef_search, threads, _p(ids), _p(dist), _p(n)) != 0:
            raise ValueError("hnsw_search failed")
        return ids, dist, n

    def __del__(self):
        if getattr(self, "h", None):
            lib().hnsw_free(self.h)
            self.h = None


class Bm25:
    """SparseIndex restatement (oracle/bm25_oracle.cpp; sparse.rs:71-222): the
    checker for the GPU BM25 path.  Ties by document slot, avgdl folded in slot
    order (the reference leaves both to HashMap order)."""

    def __init__(self, k1=1.2, b=0.75):
        self.h = lib().bm25o_create(float(k1), float(b))

    def add_document(self, doc_id, terms, tfs, doc_length):
        t = np.ascontiguousarray(np.asarray(terms, dtype=np.uint32))
        v = _f32(tfs)
        lib().bm25o_add(self.h, int(doc_id), _p(t), _p(v), t.size, float(np.float32(doc_length)))

    def add_documents_csr(self, ids, doc_ptr, terms, tfs, doc_lengths):
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        dp = np.ascontiguousarray(doc_ptr, dtype=np.uint64)
        t = np.ascontiguousarray(terms, dtype=np.uint32)
        v, dl = _f32(tfs), _f32(doc_lengths)
        lib().bm25o_add_csr(self.h, _p(ids), _p(dp), _p(t), _p(v), _p(dl), ids.size)

    def remove_document(self, doc_id) -> bool:
        return bool(lib().bm25o_remove(self.h, int(doc_id)))

    def stats(self):
        n, v = np.zeros(1, np.uint64), np.zeros(1, np.uint64)
        a = np.zeros(1, np.float32)
        lib().bm25o_stats(self.h, _p(n), _p(a), _p(v))
        return int(n[0]), a[0], int(v[0])

    def search(self, terms, values, limit):
        t = np.ascontiguousarray(np.asarray(terms, dtype=np.uint32))
        v = _f32(values)
        ids = np.zeros(max(limit, 1), np.uint64)
        sc = np.zeros(max(limit, 1), np.float32)
        n = lib().bm25o_search(self.h, _p(t), _p(v), t.size, limit, _p(ids), _p(sc))
        return ids[:n], sc[:n]

    def search_batch(self, q_ptr, q_terms, q_values, limit, threads=0):
        qp = np.ascontiguousarray(q_ptr, dtype=np.uint64)
        qt = np.ascontiguousarray(q_terms, dtype=np.uint32)
        qv = _f32(q_values)
        B = qp.size - 1
        ids = np.zeros((B, max(limit, 1)), np.uint64)
        sc = np.zeros((B, max(limit, 1)), np.float32)
        n = np.zeros(B, np.uint64)
        lib().bm25o_search_batch(self.h, _p(qp), _p(qt), _p(qv), B, limit, _p(ids), _p(sc), _p(n), threads)
        return ids[:, :limit], sc[:, :limit], n

    def __del__(self):
        if getattr(self, "h", None):
            lib().bm25o_free(self.h)
            self.h = None


def rrf_fusion(dense, sparse, text, k=60.0):
    """hybrid.rs:422-488 restated: lists of (id, raw score) -> [(id, rrf score,
    dense, sparse, text)] sorted by score desc (ties: first appearance)."""
    def arr(lst):
        ids = np.ascontiguousarray(np.array([int(i) for i, _ in lst], dtype=np.uint64))
        sc = _f32([s for _, s in lst]) if lst else np.zeros(0, np.float32)
        return ids, sc
    (di, ds), (si, ss), (ti, ts) = arr(dense), arr(sparse), arr(text)
    n = len(dense) + len(sparse) + len(text)
    oi = np.zeros(max(n, 1), np.uint64)
    os_, od, osp, ot = (np.zeros(max(n, 1), np.float32) for _ in range(4))
    m = lib().bm25o_rrf(_p(di), _p(ds), di.size, _p(si), _p(ss), si.size, _p(ti), _p(ts), ti.size, float(k),
                        _p(oi), _p(os_), _p(od), _p(osp), _p(ot))
    return [(int(oi[i]), os_[i], od[i], osp[i], ot[i]) for i in range(m)]
