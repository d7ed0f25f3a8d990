"""gvdb — host-side mirror of grape-vector-db's vector hot-path API over the
MI355X C ABI (include/gvdb.h, libgvdb.so).

Reference interfaces mirrored (reference snapshot 2025-08-24, Rust):
  * ``VectorIndex`` trait                    src/index.rs:35-62
    -> :class:`GpuVectorIndex` (alias ``HnswVectorIndex``: the drop-in for
       HnswVectorIndex, index.rs:91-310)
  * ``IndexStats``                           src/index.rs:83-88
  * ``BinaryQuantizationConfig``             src/quantization.rs:10-31
  * ``BinaryVector``                         src/quantization.rs:35-63
  * ``BinaryQuantizer``                      src/quantization.rs:67-216
  * ``VectorStore::vector_search`` (flat)    src/storage.rs:296-339 -> :func:`flat_search`
  * ``ShardManager::search_vectors`` merge   src/distributed/shard.rs:776-784 -> :func:`topk_merge`
  * ``VectorDbError``                        src/types.rs:859-920

String ids stay on the host: each distinct string gets a stable u64; the C
ABI reproduces HashMap-insert shadowing for a re-added id.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _ffi
from ._ffi import lib, ptr

__all__ = [
    "VectorDbError", "IndexNotBuilt", "DimensionMismatch", "InvalidVectorDimension", "QuantizationError",
    "IndexError_", "DeviceError", "BinaryQuantizationConfig", "BinaryVector", "BinaryQuantizer",
    "IndexStats", "GpuVectorIndex", "HnswVectorIndex", "SearchParams", "flat_search", "topk_merge", "lib",
    "BinaryVectorStore", "QueryEngineConfig", "QueryEngine",
]


# ---------------------------------------------------------------------------
# errors (VectorDbError, types.rs:859-920)
# ---------------------------------------------------------------------------
class VectorDbError(Exception):
    code = -1


class IndexNotBuilt(VectorDbError):
    code = _ffi.GVDB_ERR_INDEX_NOT_BUILT


class DimensionMismatch(VectorDbError):
    code = _ffi.GVDB_ERR_DIMENSION_MISMATCH

    def __init__(self, msg: str, expected: int = 0, actual: int = 0):
        super().__init__(msg)
        self.expected = expected
        self.actual = actual


class InvalidVectorDimension(VectorDbError):
    code = _ffi.GVDB_ERR_INVALID_VECTOR_DIMENSION


class QuantizationError(VectorDbError):
    code = _ffi.GVDB_ERR_QUANTIZATION


class IndexError_(VectorDbError):
    code = _ffi.GVDB_ERR_INDEX


class InvalidArgument(VectorDbError):
    code = _ffi.GVDB_ERR_INVALID_ARGUMENT


class DeviceError(VectorDbError):
    code = _ffi.GVDB_ERR_DEVICE


class OutOfMemory(DeviceError):
    code = _ffi.GVDB_ERR_OUT_OF_MEMORY


class StorageError(VectorDbError):
    """VectorDbError::Storage(String): index file IO / format errors."""
    code = _ffi.GVDB_ERR_STORAGE


_ERRORS = {c.code: c for c in (IndexNotBuilt, DimensionMismatch, InvalidVectorDimension, QuantizationError,
                               IndexError_, InvalidArgument, DeviceError, OutOfMemory, StorageError)}


def check(status: int) -> None:
    if status == _ffi.GVDB_OK:
        return
    L = lib()
    msg = (L.gvdb_last_error() or b"").decode(errors="replace")
    cls = _ERRORS.get(status, VectorDbError)
    if cls is DimensionMismatch:
        e, a = C.c_uint64(), C.c_uint64()
        L.gvdb_last_dimension_mismatch(C.byref(e), C.byref(a))
        raise DimensionMismatch(msg, e.value, a.value)
    raise cls(msg)


def _stream(stream: Optional[int]):
    """The HIP stream for a _device call: the given handle, else torch's current
    stream (the inputs were produced there)."""
    if stream is not None:
        return stream or None
    import torch

    return torch.cuda.current_stream().cuda_stream or None


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


# ---------------------------------------------------------------------------
# BinaryQuantizer (quantization.rs)
# ---------------------------------------------------------------------------
@dataclass
class BinaryQuantizationConfig:
    """quantization.rs:10-31 (defaults 22-30)."""
    threshold: float = 0.0
    enable_simd: bool = True
    rescore_ratio: float = 0.1
    enable_cache: bool = True


@dataclass
class BinaryVector:
    """quantization.rs:35-63: BitVec<u8, Msb0> bytes + original dimension."""
    data: bytes
    dimension: int

    def byte_size(self) -> int:
        return (self.dimension + 7) // 8

    def to_bytes(self) -> bytes:
        return bytes(self.data)

    @staticmethod
    def from_bytes(b: bytes, dimension: int) -> "BinaryVector":
        return BinaryVector(bytes(b), dimension)

    def bits(self) -> List[bool]:
        return [bool(self.data[i >> 3] & (0x80 >> (i & 7))) for i in range(self.dimension)]


class BinaryQuantizer:
    """quantization.rs:67-216, computed on the GPU through the C ABI.

    The reference's cache (89-109) memoises identical bits; it changes no
    result, so this mirror keeps only its statistics surface.
    """

    def __init__(self, config: Optional[BinaryQuantizationConfig] = None):
        self.config = config or BinaryQuantizationConfig()

    def quantize(self, vector: Sequence[float]) -> BinaryVector:
        v = _f32(vector).reshape(1, -1)
        return self.quantize_batch(v)[0]

    def quantize_batch(self, vectors) -> List[BinaryVector]:
        rows = [_f32(v).reshape(-1) for v in vectors]
        if not rows:
            return []
        dims = {len(r) for r in rows}
        out: List[BinaryVector] = []
        if len(dims) == 1:
            D = dims.pop()
            m = np.stack(rows) if D else np.zeros((len(rows), 0), np.float32)
            nb = (D + 7) // 8
            o = np.zeros((len(rows), nb), np.uint8)
            if D:
                check(lib().gvdb_bq_quantize(ptr(m), len(rows), D, self.config.threshold, ptr(o)))
            return [BinaryVector(o[i].tobytes(), D) for i in range(len(rows))]
        for r in rows:
            out.extend(self.quantize_batch([r]))
        return out

    def hamming_distance(self, a: BinaryVector, b: BinaryVector) -> float:
        """quantization.rs:130-141 (Err(InvalidVectorDimension) on mismatch)."""
        if a.dimension != b.dimension:
            raise InvalidVectorDimension("binary vectors of different dimension")
        nb = a.byte_size()
        if nb == 0:
            return 0.0
        A = np.frombuffer(a.data, np.uint8).copy()
        B = np.frombuffer(b.data, np.uint8).copy()
        out = np.zeros(1, np.uint32)
        check(lib().gvdb_bq_hamming(ptr(A), ptr(B), 1, a.dimension, ptr(out)))
        return float(np.float32(out[0]))

    def similarity(self, a: BinaryVector, b: BinaryVector) -> float:
        """quantization.rs:144-148: 1 - d/D in f32."""
        d = np.float32(self.hamming_distance(a, b))
        with np.errstate(invalid="ignore", divide="ignore"):
            return float(np.float32(1.0) - (d / np.float32(a.dimension)))

    def multi_stage_search(self, query_binary: BinaryVector, candidates_binary: Sequence[BinaryVector],
                           original_query: Sequence[float], original_candidates) -> List[Tuple[int, float]]:
        """quantization.rs:151-193 on the GPU: BQ stage 1 + exact cosine rescore."""
        if len(candidates_binary) != len(original_candidates):
            raise QuantizationError("Mismatch between binary and original candidate counts")
        N = len(candidates_binary)
        q = _f32(original_query).reshape(-1)
        if N == 0:
            return []
        cdims = {c.dimension for c in candidates_binary}
        if len(cdims) != 1:
            raise InvalidArgument("the C ABI takes candidates of one dimension")
        cdim = cdims.pop()
        nb = (cdim + 7) // 8
        cb = np.zeros((N, max(nb, 1)), np.uint8)
        for i, c in enumerate(candidates_binary):
            cb[i, :nb] = np.frombuffer(c.data[:nb], np.uint8)
        cb = np.ascontiguousarray(cb[:, :nb]) if nb else np.zeros((N, 1), np.uint8)
        cands = np.stack([_f32(c).reshape(-1) for c in original_candidates])
        qb = np.frombuffer(query_binary.data, np.uint8).copy() if query_binary.data else np.zeros(1, np.uint8)
        R = N  # capacity upper bound
        out_idx = np.zeros(R, np.uint64)
        out_cos = np.zeros(R, np.float32)
        n = C.c_uint64()
        check(lib().gvdb_bq_multi_stage_search(ptr(qb), query_binary.dimension, ptr(cb), cdim, N, ptr(q), q.size,
                                               ptr(cands), cands.shape[1], self.config.rescore_ratio, ptr(out_idx),
                                               ptr(out_cos), C.byref(n)))
        return [(int(out_idx[i]), float(out_cos[i])) for i in range(n.value)]

    def get_cache_stats(self):
        return {"enabled": self.config.enable_cache, "size": 0, "capacity": 10000 if self.config.enable_cache else 0}


class BinaryVectorStore:
    """quantization.rs:286-354: BinaryVectors with their string ids, plus the
    reference's validation and memory accounting.  Host-side bookkeeping: the
    GPU layout of the same codes is the word-major SoA plane set of a
    GpuVectorIndex; :meth:`to_index` builds one."""

    def __init__(self, config: Optional[BinaryQuantizationConfig] = None):
        self.config = config or BinaryQuantizationConfig()
        self.vectors: List[BinaryVector] = []
        self.metadata: List[str] = []

    def add_vector(self, vector: BinaryVector, id: str) -> None:  # 306-310
        self.vectors.append(vector)
        self.metadata.append(id)

    def get_vector(self, index: int) -> Optional[BinaryVector]:  # 313-315 (Option<&BinaryVector>)
        return self.vectors[index] if 0 <= index < len(self.vectors) else None

    def len(self) -> int:
        return len(self.vectors)

    def __len__(self) -> int:
        return len(self.vectors)

    def is_empty(self) -> bool:
        return not self.vectors

    def get_config(self) -> BinaryQuantizationConfig:
        return self.config

    def validate_vector(self, vector: BinaryVector) -> None:  # 333-347
        if vector.dimension == 0:
            raise InvalidVectorDimension("binary vector of dimension 0")

    def memory_usage(self) -> int:  # 350-353: code bytes + id bytes (UTF-8 length of a Rust String)
        return sum(v.byte_size() for v in self.vectors) + sum(len(m.encode()) for m in self.metadata)

    def multi_stage_search(self, query_binary: BinaryVector, original_query: Sequence[float],
                           original_candidates) -> List[Tuple[int, float]]:
        """BinaryQuantizer::multi_stage_search over this store's codes (GPU)."""
        return BinaryQuantizer(self.config).multi_stage_search(query_binary, self.vectors, original_query,
                                                               original_candidates)


# ---------------------------------------------------------------------------
# VectorIndex (index.rs:35-62)
# ---------------------------------------------------------------------------
@dataclass
class IndexStats:
    """index.rs:83-88."""
    vector_count: int
    dimension: int
    index_type: str
    memory_usage: int
    device_bytes: int = 0


@dataclass
class SearchParams:
    """Explicit knobs of the GPU search (the reference hard-codes them)."""
    mode: int = _ffi.GVDB_SEARCH_BQ_RERANK
    metric: int = _ffi.GVDB_METRIC_COSINE
    rescore_count: int = 0          # R; 0 -> (len as f32 * rescore_ratio) as usize
    rescore_ratio: float = 0.1      # BinaryQuantizationConfig.rescore_ratio default

    def to_c(self) -> _ffi.gvdb_search_params:
        return _ffi.gvdb_search_params(self.mode, self.metric, self.rescore_count, self.rescore_ratio, 0)


class GpuVectorIndex:
    """MI355X drop-in for HnswVectorIndex (index.rs:91-310).

    ``search`` runs BQ Hamming stage 1 + exact rerank on the GPU
    (:class:`SearchParams`); scores follow ``params.metric`` (cosine by default,
    ``GVDB_METRIC_L2`` reproduces HnswVectorIndex's L2 distances).
    """

    index_type = "GPU-BQ"

    def __init__(self, dimension: int = 0, threshold: float = 0.0, device: int = 0, capacity_hint: int = 0,
                 params: Optional[SearchParams] = None):
        self._lib = lib()
        h = C.c_void_p()
        p = _ffi.gvdb_params(dimension, threshold, device, 0, capacity_hint)
        check(self._lib.gvdb_index_create(C.byref(p), C.byref(h)))
        self._h = h
        self.device = device
        self._threshold = threshold
        self.params = params or SearchParams()
        self._id_of: dict = {}       # str -> u64
        self._str_of: List[str] = []  # u64 -> str

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.gvdb_index_destroy(h)
            self._h = None

    # -- id table -----------------------------------------------------------
    def _u64(self, sid: str) -> int:
        u = self._id_of.get(sid)
        if u is None:
            u = len(self._str_of)
            self._id_of[sid] = u
            self._str_of.append(sid)
        return u

    # -- trait methods ------------------------------------------------------
    def add_vector(self, id: str, vector: Sequence[float]) -> None:
        self.add_vectors([(id, vector)])

    def add_vectors(self, vectors: Iterable[Tuple[str, Sequence[float]]]) -> None:
        """index.rs:187-210: rows before a dimension mismatch are kept."""
        items = list(vectors)
        i = 0
        while i < len(items):
            D = len(items[i][1])
            j = i
            while j < len(items) and len(items[j][1]) == D:
                j += 1
            rows = np.stack([_f32(v).reshape(-1) for _, v in items[i:j]]) if D else np.zeros((j - i, 0), np.float32)
            ids = np.array([self._u64(s) for s, _ in items[i:j]], np.uint64)
            self.add_batch(ids, rows)
            i = j

    def add_batch(self, ids: np.ndarray, rows: np.ndarray) -> None:
        rows = _f32(rows)
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        check(self._lib.gvdb_index_add(self._h, ptr(rows), rows.shape[0], rows.shape[1] if rows.ndim == 2 else 0,
                                       ptr(ids)))

    def add_device(self, rows, ids, stream: Optional[int] = None) -> None:
        """rows: torch cuda float32 [n, D]; ids: torch cuda int64/uint64 [n] (copied into the index)."""
        check(self._lib.gvdb_index_add_device(self._h, rows.data_ptr(), rows.shape[0], rows.shape[1],
                                              ids.data_ptr(), _stream(stream)))

    def search(self, query: Sequence[float], k: int) -> List[Tuple[str, float]]:
        q = _f32(query).reshape(1, -1)
        ids, scores, n = self.search_batch(q, k)
        return [(self._str_of[int(ids[0, i])] if int(ids[0, i]) < len(self._str_of) else str(int(ids[0, i])),
                 float(scores[0, i])) for i in range(int(n[0]))]

    def search_batch(self, queries: np.ndarray, k: int, params: Optional[SearchParams] = None):
        q = _f32(queries)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        B, D = q.shape
        sp = (params or self.params).to_c()
        ids = np.zeros((B, max(k, 1)), np.uint64)
        sc = np.zeros((B, max(k, 1)), np.float32)
        n = np.zeros(B, np.uint32)
        check(self._lib.gvdb_index_search(self._h, ptr(q), B, D, k, C.byref(sp), ptr(ids), ptr(sc), ptr(n)))
        return ids[:, :k], sc[:, :k], n

    def search_batch_filtered(self, queries: np.ndarray, k: int, allowed: Iterable[str],
                              params: Optional[SearchParams] = None):
        """Vector search restricted to the ids a FilterEngine::execute_filter
        (filtering.rs:374) returned; ids the index does not hold are ignored.
        ``params.mode`` BQ: multi_stage_search over those rows (R from their
        count); FLAT: exact scan of those rows (metric of ``params``).  Without
        ``params`` the search is the exact scan (an approximate BQ pass over a
        small allowed set would keep only R = 0.1 M candidates)."""
        q = _f32(queries)
        if q.ndim == 1:
            q = q.reshape(1, -1)
        B, D = q.shape
        if params is None:
            params = SearchParams(mode=_ffi.GVDB_SEARCH_FLAT, metric=self.params.metric)
        sp = params.to_c()
        al = np.array([self._id_of[s] for s in allowed if s in self._id_of], np.uint64)
        ids = np.zeros((B, max(k, 1)), np.uint64)
        sc = np.zeros((B, max(k, 1)), np.float32)
        n = np.zeros(B, np.uint32)
        check(self._lib.gvdb_index_search_filtered(self._h, ptr(q), B, D, k, C.byref(sp), ptr(al) if al.size else None,
                                                   al.size, ptr(ids), ptr(sc), ptr(n)))
        return ids[:, :k], sc[:, :k], n

    def search_filtered(self, query: Sequence[float], k: int, allowed: Iterable[str],
                        params: Optional[SearchParams] = None) -> List[Tuple[str, float]]:
        ids, sc, n = self.search_batch_filtered(_f32(query).reshape(1, -1), k, allowed, params)
        return [(self._str_of[int(ids[0, i])], float(sc[0, i])) for i in range(int(n[0]))]

    def search_device(self, queries, k: int, out_ids, out_scores, out_n=None, params: Optional[SearchParams] = None,
                      stream: Optional[int] = None) -> None:
        sp = (params or self.params).to_c()
        check(self._lib.gvdb_index_search_device(self._h, queries.data_ptr(), queries.shape[0], queries.shape[1], k,
                                                 C.byref(sp), out_ids.data_ptr(), out_scores.data_ptr(),
                                                 out_n.data_ptr() if out_n is not None else None, _stream(stream)))

    def bq_topr_device(self, queries, R: int, out_rows, out_dist, stream: Optional[int] = None) -> None:
        check(self._lib.gvdb_index_bq_topr_device(self._h, queries.data_ptr(), queries.shape[0], queries.shape[1], R,
                                                  out_rows.data_ptr(), out_dist.data_ptr(), _stream(stream)))

    def remove_vector(self, id: str) -> bool:
        u = self._id_of.get(id)
        if u is None:
            return False
        r = C.c_int32()
        check(self._lib.gvdb_index_remove(self._h, u, C.byref(r)))
        return bool(r.value)

    def remove_vector_id(self, u: int) -> bool:
        """remove_vector by the u64 id of add_batch."""
        r = C.c_int32()
        check(self._lib.gvdb_index_remove(self._h, int(u), C.byref(r)))
        return bool(r.value)

    def len(self) -> int:
        return int(self._lib.gvdb_index_len(self._h))

    def __len__(self) -> int:
        return self.len()

    def is_empty(self) -> bool:
        return bool(self._lib.gvdb_index_is_empty(self._h))

    def optimize(self) -> None:
        check(self._lib.gvdb_index_optimize(self._h))

    def build_index(self) -> None:
        check(self._lib.gvdb_index_build(self._h))

    def clear(self) -> None:
        self._lib.gvdb_index_clear(self._h)

    def get_stats(self) -> IndexStats:
        s = _ffi.gvdb_index_stats()
        check(self._lib.gvdb_index_get_stats(self._h, C.byref(s)))
        return IndexStats(int(s.vector_count), int(s.dimension), self.index_type, int(s.memory_usage),
                          int(s.device_bytes))


    # -- persistence (QueryEngine::save_index / load_index, query.rs:282-409) --
    def get_all_vectors(self) -> List[Tuple[str, np.ndarray]]:
        """index.rs:120-135: every live (id, vector), sorted by id."""
        ids, rows = self._export()
        out = [(self._str_of[int(u)], rows[i]) for i, u in enumerate(ids)]
        out.sort(key=lambda t: t[0])
        return out

    def _export(self):
        """(u64 ids, rows) of the live rows, device -> host."""
        cap = self.len()
        D = self.get_stats().dimension
        rows = np.empty((cap, D), np.float32)
        ids = np.empty(cap, np.uint64)
        n = C.c_uint64()
        if cap:
            check(self._lib.gvdb_index_export(self._h, ptr(rows), ptr(ids), cap, C.byref(n)))
        return ids[: n.value], rows[: n.value]

    def save_index(self, path: str, config: Optional["HnswConfig"] = None, created_at: Optional[str] = None,
                   level: int = -1, batch: int = 1 << 16) -> None:
        """Write the reference's index file (gzip(postcard(IndexPersistenceData)),
        query.rs:16-28, 282-330): metadata {dimension, total_points, created_at,
        HnswConfig} then every live (id, vector) sorted by id."""
        import os

        cfg = config or HnswConfig()
        ids, rows = self._export()
        names = [self._str_of[int(u)] for u in ids]
        order = sorted(range(len(names)), key=names.__getitem__)
        D = rows.shape[1] if rows.ndim == 2 else 0
        m = _ffi.gvdb_persist_meta(D or self.get_stats().dimension, len(order), cfg.m, cfg.ef_construction,
                                   cfg.ef_search, cfg.max_layers, (created_at or utc_now_rfc3339()).encode())
        parent = os.path.dirname(os.path.abspath(path))
        os.makedirs(parent, exist_ok=True)  # query.rs:286-290 creates the directory
        w = C.c_void_p()
        check(self._lib.gvdb_persist_create(path.encode(), C.byref(m), len(order), level, C.byref(w)))
        try:
            for b0 in range(0, len(order), batch):
                sel = order[b0:b0 + batch]
                enc = [names[i].encode() for i in sel]
                offs = np.zeros(len(enc) + 1, np.uint64)
                offs[1:] = np.cumsum([len(e) for e in enc])
                blob = b"".join(enc) or b"\0"
                r = np.ascontiguousarray(rows[sel])
                check(self._lib.gvdb_persist_append(w, ptr(r), len(sel), D, blob, ptr(offs)))
        except BaseException:
            self._lib.gvdb_persist_close(w)
            raise
        check(self._lib.gvdb_persist_close(w))

    def load_index(self, path: str, batch: int = 1 << 16) -> "PersistMetadata":
        """query.rs:335-409: read the file, check its dimension against this
        index's (DimensionMismatch), then replace the contents with its
        vectors in file order.  Returns the stored metadata.  The file is
        decoded into a staging index first and swapped in only after its last
        entry and the gzip trailer are read, so a truncated or corrupt file
        leaves this index as it was (the reference decodes the whole file
        before touching the index, query.rs:355-373)."""
        m = _ffi.gvdb_persist_meta()
        cnt = C.c_uint64()
        r = C.c_void_p()
        check(self._lib.gvdb_persist_open(path.encode(), C.byref(m), C.byref(cnt), C.byref(r)))
        try:
            D = int(m.dimension)
            mine = self.get_stats().dimension
            if mine and mine != D:
                raise DimensionMismatch(f"Dimension mismatch: expected {mine}, actual {D}", mine, D)
            stage = GpuVectorIndex(dimension=0, threshold=self._threshold, device=self.device,
                                   capacity_hint=int(cnt.value), params=self.params)
            rows = np.empty((batch, D), np.float32)
            offs = np.empty(batch + 1, np.uint64)
            cap = batch * 64
            blob = C.create_string_buffer(cap)
            got = C.c_uint64()
            while True:
                check(self._lib.gvdb_persist_next(r, ptr(rows), D, batch, blob, cap, ptr(offs), C.byref(got)))
                n = got.value
                if n == 0:
                    break
                raw = blob.raw
                names = [raw[int(offs[i]):int(offs[i + 1])].decode() for i in range(n)]
                stage.add_batch(np.array([stage._u64(x) for x in names], np.uint64), rows[:n])
        finally:
            self._lib.gvdb_persist_free(r)
        # swap: this object takes the staged index, the staging object the old one
        self._h, stage._h = stage._h, self._h
        self._id_of, stage._id_of = stage._id_of, self._id_of
        self._str_of, stage._str_of = stage._str_of, self._str_of
        del stage
        return PersistMetadata(int(m.dimension), int(m.total_points), m.created_at.decode(),
                               HnswConfig(int(m.m), int(m.ef_construction), int(m.ef_search), int(m.max_layers)))


class RequestCoalescer:
    """Concurrent batch-1 searches over one index (gvdb_coalescer_*): callers on
    any number of threads each ask for ONE query's top-k, as the reference's
    concurrent readers of Arc<RwLock<dyn VectorIndex>> do (src/lib.rs:238,
    index.rs:212-231); queries that arrive while a batch runs are searched
    together in the next one, and every caller gets exactly its own
    gvdb_index_search result.  ctypes releases the GIL around the call, so
    Python threads really wait in parallel."""

    def __init__(self, index: "GpuVectorIndex", dim: int, k: int, params: Optional[SearchParams] = None,
                 max_batch: int = 256, max_inflight: int = 1):
        self._lib = lib()
        self.index, self.dim, self.k = index, dim, k
        self._sp = (params or index.params).to_c()
        h = C.c_void_p()
        check(self._lib.gvdb_coalescer_create(index._h, dim, k, C.byref(self._sp), max_batch, max_inflight,
                                              C.byref(h)))
        self._h = h

    def search(self, query) -> Tuple[np.ndarray, np.ndarray, int]:
        q = _f32(query).reshape(-1)
        if q.size != self.dim:
            raise DimensionMismatch(f"query has {q.size} dims, coalescer {self.dim}", self.dim, q.size)
        ids = np.zeros(self.k, np.uint64)
        sc = np.zeros(self.k, np.float32)
        n = C.c_uint32(0)
        check(self._lib.gvdb_coalescer_search(self._h, ptr(q), ptr(ids), ptr(sc), C.byref(n)))
        return ids, sc, int(n.value)

    def stats(self) -> Tuple[int, int, int]:
        """(batches run, queries served, largest batch)."""
        b, q, m = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(self._lib.gvdb_coalescer_stats(self._h, C.byref(b), C.byref(q), C.byref(m)))
        return b.value, q.value, m.value

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._lib.gvdb_coalescer_destroy(h)
            self._h = None

    def __del__(self):
        self.close()


@dataclass
class HnswConfig:
    """config.rs:196-209 (defaults config.rs:413-422)."""
    m: int = 16
    ef_construction: int = 200
    ef_search: int = 100
    max_layers: int = 16


@dataclass
class PersistMetadata:
    """IndexMetadata (query.rs:23-28)."""
    dimension: int
    total_points: int
    created_at: str
    config: HnswConfig


def utc_now_rfc3339() -> str:
    """chrono's serde form of Utc::now() (RFC 3339, SecondsFormat::AutoSi, 'Z')."""
    import time

    ns = time.time_ns()
    sec, frac = divmod(ns, 1_000_000_000)
    base = time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(sec))
    if frac == 0:
        return base + "Z"
    if frac % 1_000_000 == 0:
        return f"{base}.{frac // 1_000_000:03d}Z"
    if frac % 1000 == 0:
        return f"{base}.{frac // 1000:06d}Z"
    return f"{base}.{frac:09d}Z"


HnswVectorIndex = GpuVectorIndex


@dataclass
class QueryEngineConfig:
    """query_engine.rs:9-32 (defaults 24-32)."""
    default_limit: int = 10
    default_threshold: float = 0.7
    text_weight: float = 0.3
    enable_cache: bool = True
    cache_size: int = 1000


class QueryEngine:
    """query_engine.rs:117-147 ``vector_search``: limit defaults to 10 and the
    threshold to 0.7, then the store's exact cosine search keeps scores >=
    threshold, descending, truncated to limit (storage.rs:296-339).  Here the
    store is a GPU index searched exactly (GVDB_SEARCH_FLAT, cosine): its top
    ``limit`` filtered by the threshold is the same list, since scores that
    pass form a prefix of the descending order.  Results are cached per
    (query bits, limit, threshold) like the reference's cache (query_engine.rs:126-145)."""

    def __init__(self, index: GpuVectorIndex, config: Optional[QueryEngineConfig] = None):
        self.index = index
        self.config = config or QueryEngineConfig()
        self._cache: "dict" = {}

    def vector_search(self, query_vector: Sequence[float], limit: Optional[int] = None,
                      threshold: Optional[float] = None) -> List[Tuple[str, float]]:
        limit = self.config.default_limit if limit is None else int(limit)
        thr = np.float32(self.config.default_threshold if threshold is None else threshold)
        q = _f32(query_vector).reshape(1, -1)
        key = (q.tobytes(), limit, float(thr))
        if self.config.enable_cache and key in self._cache:
            return list(self._cache[key])
        if limit == 0:
            out: List[Tuple[str, float]] = []
        else:
            ids, sc, n = self.index.search_batch(q, limit, SearchParams(mode=_ffi.GVDB_SEARCH_FLAT,
                                                                        metric=_ffi.GVDB_METRIC_COSINE))
            out = [(self.index._str_of[int(ids[0, i])], float(sc[0, i])) for i in range(int(n[0]))
                   if np.float32(sc[0, i]) >= thr]
        if self.config.enable_cache:
            if len(self._cache) >= self.config.cache_size:
                self._cache.pop(next(iter(self._cache)))
            self._cache[key] = list(out)
        return out

    def clear_cache(self) -> None:
        self._cache.clear()


# ---------------------------------------------------------------------------
# flat scan and shard merge
# ---------------------------------------------------------------------------
def flat_search(queries, rows, limit: int, metric: int = _ffi.GVDB_METRIC_COSINE, threshold: Optional[float] = None):
    """storage.rs:296-339 (cosine, optional threshold) / index.rs:620-640
    (cosine distance) / exact L2, for a batch of queries over host rows."""
    q = _f32(queries)
    if q.ndim == 1:
        q = q.reshape(1, -1)
    x = _f32(rows)
    B, D = q.shape
    N = x.shape[0]
    idx = np.zeros((B, max(limit, 1)), np.uint64)
    sc = np.zeros((B, max(limit, 1)), np.float32)
    n = np.zeros(B, np.uint32)
    check(lib().gvdb_flat_search(ptr(q), B, ptr(x), N, D, limit, metric, int(threshold is not None),
                                 float(threshold or 0.0), ptr(idx), ptr(sc), ptr(n)))
    return idx[:, :limit], sc[:, :limit], n


def topk_merge(ids: np.ndarray, scores: np.ndarray, counts: np.ndarray, limit: int, descending: bool = True):
    """shard.rs:776-784.  ids/scores: [n_shards, B, stride]; counts [n_shards, B]."""
    ids = np.ascontiguousarray(ids, np.uint64)
    scores = np.ascontiguousarray(scores, np.float32)
    counts = np.ascontiguousarray(counts, np.uint32)
    S, B, stride = ids.shape
    oi = np.zeros((B, max(limit, 1)), np.uint64)
    os_ = np.zeros((B, max(limit, 1)), np.float32)
    on = np.zeros(B, np.uint32)
    check(lib().gvdb_topk_merge(ptr(ids), ptr(scores), ptr(counts), S, B, stride, limit, int(descending), ptr(oi),
                                ptr(os_), ptr(on)))
    return oi[:, :limit], os_[:, :limit], on
