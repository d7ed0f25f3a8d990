"""Host mirror of grape-vector-db's sparse (BM25) search and hybrid RRF fusion
over the MI355X C ABI (include/gvdb.h: gvdb_sparse_*, gvdb_rrf_fuse).

Reference interfaces mirrored (reference snapshot 2025-08-24, Rust):
  * ``SparseVector``                  src/types.rs:15-90
  * ``DocumentSparseRepresentation``  src/types.rs:92-102
  * ``BM25Stats``                     src/types.rs:104-115
  * ``BM25Parameters``                src/sparse.rs:42-53
  * ``SparseIndex``                   src/sparse.rs:29-254  -> :class:`SparseIndex`
  * ``SimpleTokenizer``               src/sparse.rs:257-359 (host-side text
    processing; builds the term lists the GPU index consumes)
  * ``HybridSearchRequest``           src/types.rs:206-223
  * ``HybridSearchEngine::search``    src/hybrid.rs:286-356 with
    ``FusionStrategy::RRF`` (rrf_fusion 422-488) -> :class:`HybridSearchEngine`

Document ids are strings on the host; the GPU sees u64 handles.  Scoring,
selection and fusion run in libgvdb.so (gvdb_sparse.hip); there is no CPU
fallback.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _ffi
from ._ffi import lib, ptr

__all__ = ["SparseVector", "DocumentSparseRepresentation", "BM25Parameters", "BM25Stats", "SparseIndex",
           "SimpleTokenizer", "ScoreBreakdown", "HybridSearchRequest", "HybridSearchEngine", "rrf_fuse"]


def _check(status: int) -> None:
    from . import check

    check(status)


class ConfigError(ValueError):
    """VectorDbError::ConfigError (types.rs)."""


@dataclass
class SparseVector:
    """types.rs:15-90."""
    indices: List[int]
    values: List[float]
    dimension: int

    def __post_init__(self):
        if len(self.indices) != len(self.values):
            raise ConfigError("sparse vector: index and value counts differ")  # types.rs:33-37
        if any(int(i) >= self.dimension for i in self.indices):
            raise ConfigError("sparse vector: index out of range")  # types.rs:39-43

    def norm(self) -> float:
        s = np.float32(-0.0)
        for v in self.values:
            s = np.float32(s + np.float32(v) * np.float32(v))
        return float(np.sqrt(s, dtype=np.float32))

    def dot_product(self, other: "SparseVector") -> float:
        r, i, j = np.float32(0.0), 0, 0
        while i < len(self.indices) and j < len(other.indices):
            a, b = self.indices[i], other.indices[j]
            if a == b:
                r = np.float32(r + np.float32(self.values[i]) * np.float32(other.values[j]))
                i += 1
                j += 1
            elif a < b:
                i += 1
            else:
                j += 1
        return float(r)

    def cosine_similarity(self, other: "SparseVector") -> float:
        d = np.float32(self.dot_product(other))
        n = np.float32(np.float32(self.norm()) * np.float32(other.norm()))
        return 0.0 if n == 0.0 else float(np.float32(d / n))


@dataclass
class DocumentSparseRepresentation:
    """types.rs:92-102."""
    document_id: str
    sparse_vector: SparseVector
    document_length: float
    term_frequencies: Dict[int, float]


@dataclass
class BM25Parameters:
    k1: float = 1.2
    b: float = 0.75


@dataclass
class BM25Stats:
    total_documents: int
    average_document_length: float
    vocabulary_size: int
    total_entries: int = 0
    dense_fallbacks: int = 0


class SparseIndex:
    """GPU drop-in for SparseIndex (sparse.rs:29-254): an HBM forward index;
    BM25 scoring, selection and ordering on the MI355X (gvdb_sparse.hip)."""

    def __init__(self, params: Optional[BM25Parameters] = None, device: int = 0):
        self._lib = lib()
        self.params = params or BM25Parameters()
        h = C.c_void_p()
        p = _ffi.gvdb_bm25_params(self.params.k1, self.params.b, device, 0)
        _check(self._lib.gvdb_sparse_create(C.byref(p), C.byref(h)))
        self._h = h
        self._id_of: Dict[str, int] = {}
        self._str_of: List[str] = []

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.gvdb_sparse_destroy(h)
            self._h = None

    def _u64(self, sid: str) -> int:
        u = self._id_of.get(sid)
        if u is None:
            u = len(self._str_of)
            self._id_of[sid] = u
            self._str_of.append(sid)
        return u

    def _str(self, u: int) -> str:
        return self._str_of[u] if u < len(self._str_of) else str(u)

    def add_document(self, doc: DocumentSparseRepresentation) -> None:
        """sparse.rs:71-107 (one posting entry per term of term_frequencies)."""
        terms = np.array(sorted(doc.term_frequencies), dtype=np.uint32)
        tfs = np.array([doc.term_frequencies[int(t)] for t in terms], dtype=np.float32)
        _check(self._lib.gvdb_sparse_add_document(self._h, self._u64(doc.document_id), ptr(terms), ptr(tfs),
                                                  terms.size, float(np.float32(doc.document_length))))

    def add_documents_csr(self, doc_ids: Sequence[str], doc_ptr: np.ndarray, terms: np.ndarray, tfs: np.ndarray,
                          doc_lengths: np.ndarray) -> None:
        """Bulk form of add_document (document d = terms[doc_ptr[d]:doc_ptr[d+1]])."""
        ids = np.array([self._u64(s) for s in doc_ids], dtype=np.uint64)
        self.add_documents_u64(ids, doc_ptr, terms, tfs, doc_lengths)

    def add_documents_u64(self, ids: np.ndarray, doc_ptr: np.ndarray, terms: np.ndarray, tfs: np.ndarray,
                          doc_lengths: np.ndarray) -> None:
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        dp = np.ascontiguousarray(doc_ptr, dtype=np.uint64)
        t = np.ascontiguousarray(terms, dtype=np.uint32)
        v = np.ascontiguousarray(tfs, dtype=np.float32)
        dl = np.ascontiguousarray(doc_lengths, dtype=np.float32)
        _check(self._lib.gvdb_sparse_add_documents(self._h, ptr(ids), ptr(dp), ptr(t), ptr(v), ptr(dl), ids.size))

    def remove_document(self, document_id: str) -> bool:
        """sparse.rs:109-149."""
        u = self._id_of.get(document_id)
        if u is None:
            return False
        r = C.c_int32(0)
        _check(self._lib.gvdb_sparse_remove_document(self._h, u, C.byref(r)))
        return bool(r.value)

    def search_bm25(self, query: SparseVector, limit: int) -> List[Tuple[str, float]]:
        """sparse.rs:151-198."""
        ids, sc, n = self.search_bm25_batch([query], limit)
        return [(self._str(int(ids[0, i])), float(sc[0, i])) for i in range(int(n[0]))]

    def search_bm25_batch(self, queries: Sequence[SparseVector], limit: int):
        """B queries in one GPU pass: (u64 ids [B, limit], scores, counts)."""
        qp = np.zeros(len(queries) + 1, np.uint64)
        for i, q in enumerate(queries):
            qp[i + 1] = qp[i] + len(q.indices)
        qt = np.ascontiguousarray(np.concatenate([np.asarray(q.indices, np.uint32) for q in queries])
                                  if queries else np.zeros(0, np.uint32), dtype=np.uint32)
        qv = np.ascontiguousarray(np.concatenate([np.asarray(q.values, np.float32) for q in queries])
                                  if queries else np.zeros(0, np.float32), dtype=np.float32)
        return self.search_bm25_csr(qp, qt, qv, limit)

    def search_bm25_csr(self, q_ptr: np.ndarray, q_terms: np.ndarray, q_values: np.ndarray, limit: int):
        qp = np.ascontiguousarray(q_ptr, dtype=np.uint64)
        qt = np.ascontiguousarray(q_terms, dtype=np.uint32)
        qv = np.ascontiguousarray(q_values, dtype=np.float32)
        B = qp.size - 1
        ids = np.zeros((B, max(limit, 1)), np.uint64)
        sc = np.zeros((B, max(limit, 1)), np.float32)
        n = np.zeros(max(B, 1), np.uint32)
        _check(self._lib.gvdb_sparse_search_bm25(self._h, ptr(qp), ptr(qt), ptr(qv), B, limit, ptr(ids), ptr(sc),
                                                 ptr(n)))
        return ids[:, :limit], sc[:, :limit], n[:B]

    def get_stats(self) -> BM25Stats:
        s = _ffi.gvdb_bm25_stats()
        _check(self._lib.gvdb_sparse_get_stats(self._h, C.byref(s)))
        return BM25Stats(int(s.total_documents), float(s.average_document_length), int(s.vocabulary_size),
                         int(s.total_entries), int(s.dense_fallbacks))

    def clear(self) -> None:
        self._lib.gvdb_sparse_clear(self._h)

    def get_memory_usage_mb(self) -> float:
        """HBM held by the forward index (the reference estimates its HashMaps)."""
        s = self.get_stats()
        return (s.total_entries * 12 + (len(self._str_of) + 1) * 16) / (1024.0 * 1024.0)


_STOP_WORDS = {
    "a", "an", "and", "are", "as", "at", "be", "by", "for", "from", "has", "he", "in", "is", "it", "its", "of", "on",
    "that", "the", "to", "was", "will", "with", "的", "了", "在", "是", "有", "和", "与", "或", "但", "而", "这", "那",
    "一", "不", "也", "就",
}


class SimpleTokenizer:
    """sparse.rs:257-359.  NOT part of the GPU path: SURVEY §2 row 10 marks text
    processing out of scope; this host-side helper only turns the hybrid mirror's
    and the tests' text queries into the term lists the GPU BM25 index consumes
    (a deployment passes its own SparseVector terms).  Vocabulary ids are
    assigned in sorted term order (the reference enumerates a HashSet: arbitrary
    order)."""

    def __init__(self):
        self.stop_words = set(_STOP_WORDS)

    def tokenize(self, text: str) -> Dict[str, float]:
        toks = []
        for word in text.lower().split():
            w = "".join(c for c in word if c.isalnum())
            if w and len(w.encode("utf-8")) > 1 and w not in self.stop_words:
                toks.append(w)
        tf: Dict[str, float] = {}
        for t in toks:
            tf[t] = float(np.float32(tf.get(t, 0.0)) + np.float32(1.0))
        total = np.float32(len(toks))
        return {k: float(np.float32(v) / total) for k, v in tf.items()}

    def build_vocabulary(self, documents: Sequence[str]) -> Dict[str, int]:
        vocab = set()
        for d in documents:
            vocab.update(self.tokenize(d).keys())
        return {t: i for i, t in enumerate(sorted(vocab))}

    def document_to_sparse_vector(self, document_id: str, text: str,
                                  vocabulary: Dict[str, int]) -> DocumentSparseRepresentation:
        tf = self.tokenize(text)
        dl = np.float32(-0.0)
        for v in tf.values():  # .values().sum::<f32>() (HashMap order; here insertion order)
            dl = np.float32(dl + np.float32(v))
        pairs = sorted((vocabulary[t], f) for t, f in tf.items() if t in vocabulary)
        sv = SparseVector([i for i, _ in pairs], [f for _, f in pairs], len(vocabulary))
        return DocumentSparseRepresentation(document_id, sv, float(dl), {i: f for i, f in pairs})


@dataclass
class ScoreBreakdown:
    """hybrid.rs ScoreBreakdown: the raw score each list gave (None = absent)."""
    dense_score: Optional[float]
    sparse_score: Optional[float]
    text_score: Optional[float]
    final_score: float


@dataclass
class HybridSearchRequest:
    """types.rs:206-223 (the weights are unused by RRF)."""
    dense_vector: Optional[Sequence[float]] = None
    sparse_vector: Optional[SparseVector] = None
    text_query: Optional[str] = None
    limit: int = 10
    dense_weight: float = 0.7
    sparse_weight: float = 0.3
    text_weight: float = 0.0


def rrf_fuse(dense: Sequence[Sequence[Tuple[int, float]]], sparse: Sequence[Sequence[Tuple[int, float]]],
             text: Sequence[Sequence[Tuple[int, float]]], k: float, limit: int):
    """Batched rrf_fusion (hybrid.rs:422-488) on the GPU: per query three ranked
    lists of (u64 id, raw score) -> [(id, score, (dense, sparse, text))]."""
    B = max(len(dense), len(sparse), len(text))

    def pack(lists):
        if not any(len(x) for x in lists):
            return None, None, None, 0
        st = max(1, max(len(x) for x in lists))
        ids = np.zeros((B, st), np.uint64)
        sc = np.zeros((B, st), np.float32)
        n = np.zeros(B, np.uint32)
        for q, x in enumerate(lists):
            n[q] = len(x)
            for r, (i, s) in enumerate(x):
                ids[q, r] = i
                sc[q, r] = s
        return ids, sc, n, st

    d, s, t = pack(dense), pack(sparse), pack(text)
    oi = np.zeros((B, max(limit, 1)), np.uint64)
    os_ = np.zeros((B, max(limit, 1)), np.float32)
    ob = np.zeros((B, max(limit, 1), 3), np.float32)
    on = np.zeros(max(B, 1), np.uint32)
    _check(lib().gvdb_rrf_fuse(ptr(d[0]), ptr(d[1]), ptr(d[2]), d[3], ptr(s[0]), ptr(s[1]), ptr(s[2]), s[3],
                               ptr(t[0]), ptr(t[1]), ptr(t[2]), t[3], B, float(np.float32(k)), limit, ptr(oi),
                               ptr(os_), ptr(ob), ptr(on)))
    out = []
    for q in range(B):
        out.append([(int(oi[q, i]), float(os_[q, i]), tuple(None if math.isnan(v) else float(v) for v in ob[q, i]))
                    for i in range(int(on[q]))])
    return out


class HybridSearchEngine:
    """HybridSearchEngine (hybrid.rs:169-488) with FusionStrategy::RRF: dense
    top-2*limit from a :class:`gvdb.GpuVectorIndex` (HnswVectorIndex::search
    semantics: L2 distances ascending), BM25 top-2*limit from a
    :class:`SparseIndex`, RRF on the GPU.  ``simple_text_search`` (a scan of
    the document store, hybrid.rs:619-680) belongs to the storage layer and
    is out of scope: pass its ranked list as ``text_results`` if you have it."""

    def __init__(self, dense_engine, sparse_engine: SparseIndex, rrf_k: float = 60.0, dense_params=None):
        from . import SearchParams

        self.dense_engine = dense_engine
        self.sparse_engine = sparse_engine
        self.rrf_k = rrf_k
        self.tokenizer = SimpleTokenizer()
        self.vocabulary: Dict[str, int] = {}
        self.dense_params = dense_params or SearchParams(metric=_ffi.GVDB_METRIC_L2)

    def update_vocabulary(self, documents: Sequence[str]) -> None:
        self.vocabulary = self.tokenizer.build_vocabulary(documents)

    def search(self, request: HybridSearchRequest, text_results: Optional[Sequence[Tuple[str, float]]] = None):
        return self.search_batch([request], [text_results or []])[0]

    def search_batch(self, requests: Sequence[HybridSearchRequest],
                     text_results: Optional[Sequence[Sequence[Tuple[str, float]]]] = None):
        """hybrid.rs:286-356 for a batch: one GPU dense pass, one BM25 pass, one
        RRF pass.  Returns per request [(doc_id, score, ScoreBreakdown)]."""
        B = len(requests)
        limit = max((r.limit for r in requests), default=0)
        want = 2 * limit
        # one id space for the fusion: strings -> u64
        sid: Dict[str, int] = {}
        names: List[str] = []

        def u(s: str) -> int:
            if s not in sid:
                sid[s] = len(names)
                names.append(s)
            return sid[s]

        dense_lists: List[List[Tuple[int, float]]] = [[] for _ in range(B)]
        dq = [i for i, r in enumerate(requests) if r.dense_vector is not None]
        if dq and want:
            Q = np.stack([np.asarray(requests[i].dense_vector, np.float32) for i in dq])
            ids, sc, n = self.dense_engine.search_batch(Q, want, self.dense_params)
            for j, i in enumerate(dq):
                lim = 2 * requests[i].limit
                dense_lists[i] = [(u(self.dense_engine._str_of[int(ids[j, r])]), float(sc[j, r]))
                                  for r in range(min(int(n[j]), lim))]
        sparse_lists: List[List[Tuple[int, float]]] = [[] for _ in range(B)]
        svs, sq = [], []
        for i, r in enumerate(requests):
            if r.sparse_vector is not None:
                svs.append(r.sparse_vector)
                sq.append(i)
            elif r.text_query is not None and self.vocabulary:
                svs.append(self.tokenizer.document_to_sparse_vector("query", r.text_query, self.vocabulary).sparse_vector)
                sq.append(i)
        if svs and want:
            ids, sc, n = self.sparse_engine.search_bm25_batch(svs, want)
            for j, i in enumerate(sq):
                lim = 2 * requests[i].limit
                sparse_lists[i] = [(u(self.sparse_engine._str(int(ids[j, r]))), float(sc[j, r]))
                                   for r in range(min(int(n[j]), lim))]
        text_lists = [[(u(d), float(s)) for d, s in (text_results[i] if text_results else [])][:2 * requests[i].limit]
                      for i in range(B)]
        fused = rrf_fuse(dense_lists, sparse_lists, text_lists, self.rrf_k, limit) if B else []
        out = []
        for i, r in enumerate(requests):
            out.append([(names[d], s, ScoreBreakdown(bd[0], bd[1], bd[2], s)) for d, s, bd in fused[i][:r.limit]])
        return out
