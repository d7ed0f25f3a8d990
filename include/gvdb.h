/*
 * gvdb.h — C ABI of the MI355X-native ANN search path for grape-vector-db.
 *
 * Drop-in boundary for the reference's vector hot path (reference snapshot
 * 2025-08-24, Rust):
 *   - trait VectorIndex                      src/index.rs:35-62
 *   - HnswVectorIndex (search via HNSW)      src/index.rs:91-310
 *   - BinaryQuantizer::{quantize, hamming_distance, similarity,
 *                       multi_stage_search} src/quantization.rs:86-193
 *   - VectorStore::vector_search (flat)      src/storage.rs:296-339
 *   - FaissVectorIndex::search (Flat)        src/index.rs:620-640
 *   - ShardManager::search_vectors merge     src/distributed/shard.rs:776-784
 *
 * Rules of the boundary:
 *   - plain pointers and sizes only; no exceptions cross it;
 *   - caller-owned output buffers;
 *   - string ids never enter the library: the host keeps a String <-> u64
 *     table (see grape-vector-db_amd/host/gvdb.hpp and INTEGRATION.md);
 *   - gvdb_index_search* are reentrant for concurrent readers (each call
 *     takes its own stream + workspace from a pool); add/build/remove/clear
 *     need the caller's exclusive lock, mirroring Arc<RwLock<dyn VectorIndex>>
 *     (src/lib.rs:238);
 *   - errors: gvdb_status codes 1:1 with VectorDbError (src/types.rs:859-920)
 *     plus GVDB_ERR_DEVICE; details via gvdb_last_error() (thread-local).
 *   - functions suffixed _device take DEVICE pointers (HBM-resident inputs
 *     and outputs) and the hipStream_t (as void*) the caller produced them on
 *     and wants the work ordered on; NULL = the legacy default stream.  They
 *     are the zero-copy form used when the caller keeps data on the GPU.
 */
#ifndef GVDB_H_
#define GVDB_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GVDB_ABI_VERSION 3

/* out_n[q] of a _device search whose query hit a NaN score (the reference's
 * partial_cmp().unwrap() sort would panic): that query has no results.  The
 * host-buffer forms return GVDB_ERR_QUANTIZATION instead. */
#define GVDB_N_POISONED 0xFFFFFFFFu

typedef enum gvdb_status {
    GVDB_OK = 0,
    GVDB_ERR_INDEX_NOT_BUILT = 1,          /* VectorDbError::IndexNotBuilt               */
    GVDB_ERR_DIMENSION_MISMATCH = 2,       /* VectorDbError::DimensionMismatch{exp,act}  */
    GVDB_ERR_INVALID_VECTOR_DIMENSION = 3, /* VectorDbError::InvalidVectorDimension      */
    GVDB_ERR_QUANTIZATION = 4,             /* VectorDbError::QuantizationError(String)   */
    GVDB_ERR_INDEX = 5,                    /* VectorDbError::IndexError(String)          */
    GVDB_ERR_INVALID_ARGUMENT = 6,         /* null pointer / bad size at the ABI          */
    GVDB_ERR_DEVICE = 7,                   /* HIP runtime / kernel failure                */
    GVDB_ERR_OUT_OF_MEMORY = 8,            /* device allocation failed                    */
    GVDB_ERR_STORAGE = 9                   /* VectorDbError::Storage(String): index file IO */
} gvdb_status;

/* Scores reported by gvdb_index_search*. */
typedef enum gvdb_metric {
    /* cosine similarity, descending: multi_stage_search stage 2
     * (quantization.rs:181-190) and storage.rs:296-339 */
    GVDB_METRIC_COSINE = 0,
    /* Euclidean distance, ascending: VectorPoint::distance (index.rs:69-78),
     * the score HnswVectorIndex::search returns (index.rs:212-231) */
    GVDB_METRIC_L2 = 1,
    /* 1 - cosine, ascending: cosine_distance (index.rs:686-700), the score
     * FaissVectorIndex::search returns */
    GVDB_METRIC_COSINE_DISTANCE = 2
} gvdb_metric;

typedef enum gvdb_search_mode {
    /* BQ Hamming top-R prefilter then exact rerank of the R candidates
     * (multi_stage_search semantics, quantization.rs:151-193) */
    GVDB_SEARCH_BQ_RERANK = 0,
    /* exact scan of every live row (storage.rs:296-339 / index.rs:620-640) */
    GVDB_SEARCH_FLAT = 1
} gvdb_search_mode;

typedef struct gvdb_params {
    uint32_t dimension;       /* 0: fixed by the first add (index.rs:160-170) */
    float bq_threshold;       /* BinaryQuantizationConfig.threshold, default 0.0 (quantization.rs:25) */
    int32_t device;           /* HIP device ordinal                                     */
    uint32_t reserved;
    uint64_t capacity_hint;   /* rows to pre-reserve in HBM (0 = grow on demand)         */
} gvdb_params;

typedef struct gvdb_search_params {
    uint32_t mode;            /* gvdb_search_mode                                        */
    uint32_t metric;          /* gvdb_metric                                             */
    uint64_t rescore_count;   /* R; 0 => R = (len as f32 * rescore_ratio) as usize       */
    float rescore_ratio;      /* BinaryQuantizationConfig.rescore_ratio, default 0.1     */
    uint32_t reserved;
} gvdb_search_params;

typedef struct gvdb_index_stats {  /* IndexStats, index.rs:83-88 */
    uint64_t vector_count;
    uint64_t dimension;
    uint64_t memory_usage;    /* bytes of f32 rows, as the reference reports             */
    uint64_t device_bytes;    /* total HBM held by the index (rows + codes + norms + ids)*/
} gvdb_index_stats;

typedef struct gvdb_index gvdb_index;

/* ---- library ------------------------------------------------------------ */
uint32_t gvdb_abi_version(void);
const char* gvdb_last_error(void);                  /* thread-local, never NULL */
const char* gvdb_status_string(gvdb_status s);
/* Detail of the last GVDB_ERR_DIMENSION_MISMATCH on this thread. */
void gvdb_last_dimension_mismatch(uint64_t* expected, uint64_t* actual);
int32_t gvdb_device_count(void);
/* Kernel timing with HIP events recorded around the launches on the stream
 * they run on (read after each batch's own stream sync).  Slots:
 * 0 = stage-1 sample histogram + threshold, 1 = k_scan (the BQ Hamming hot
 * loop), 2 = stage-1 select, 3 = stage 2 (rerank + final sort), 5 = flat
 * search bf16-MFMA candidate pass (k_flat_mx), 6 = whole bf16 flat MFMA search
 * per 256-query group, 7 / 8 = the same for the i8-MFMA tier. */
void gvdb_timing_enable(int32_t on);
void gvdb_timing_reset(void);
gvdb_status gvdb_timing_read(uint32_t which, double* total_ms, uint64_t* launches);
/* Diagnostics: flat searches (GVDB_SEARCH_FLAT) whose bf16-MFMA candidate pass
 * could not be certified exact and were answered by the exact full scan, and
 * those whose i8-MFMA candidate pass (the first tier) could not be certified
 * and were retried on bf16. */
uint64_t gvdb_flat_fallback_count(void);
uint64_t gvdb_flat_i8_fallback_count(void);

/* ---- persistence: QueryEngine::save_index / load_index (query.rs:282-409) --
 * File = gzip(postcard(IndexPersistenceData)) exactly as the reference writes
 * it (query.rs:16-28): IndexMetadata {dimension, total_points, created_at
 * (RFC 3339 string), HnswConfig {m, ef_construction, ef_search, max_layers}}
 * then Vec<(String id, Vec<f32>)>.  Streaming: create declares the vector
 * count, append adds batches (ids as a byte blob + n+1 offsets), close checks
 * the count; open returns the metadata and count, next returns batches.
 * Host-only (no device work): rows come from gvdb_index_export and go back
 * through gvdb_index_add.  IO / format errors are GVDB_ERR_STORAGE. */
typedef struct gvdb_persist_meta {
    uint64_t dimension;
    uint64_t total_points;
    uint64_t m, ef_construction, ef_search, max_layers; /* HnswConfig (config.rs:196-209) */
    char created_at[64];                                 /* NUL-terminated RFC 3339 */
} gvdb_persist_meta;
typedef struct gvdb_persist_writer gvdb_persist_writer;
typedef struct gvdb_persist_reader gvdb_persist_reader;
/* level: gzip level 0-9, < 0 = flate2's Compression::default() (6) */
gvdb_status gvdb_persist_create(const char* path, const gvdb_persist_meta* meta, uint64_t n_vectors, int32_t level,
                                gvdb_persist_writer** out);
gvdb_status gvdb_persist_append(gvdb_persist_writer* w, const float* rows, uint64_t n, uint32_t dim,
                                const char* id_blob, const uint64_t* id_offs);
gvdb_status gvdb_persist_close(gvdb_persist_writer* w);
gvdb_status gvdb_persist_open(const char* path, gvdb_persist_meta* meta, uint64_t* n_vectors,
                              gvdb_persist_reader** out);
/* Up to max_n entries whose ids fit in blob_cap bytes; a stored vector whose
 * length differs from dim is GVDB_ERR_DIMENSION_MISMATCH (index.rs:187-210). */
gvdb_status gvdb_persist_next(gvdb_persist_reader* r, float* rows, uint32_t dim, uint64_t max_n, char* id_blob,
                              uint64_t blob_cap, uint64_t* id_offs, uint64_t* n_out);
void gvdb_persist_free(gvdb_persist_reader* r);

/* ---- VectorIndex (index.rs:35-62) --------------------------------------- */
/* HnswVectorIndex::new / with_config (index.rs:100-117) */
gvdb_status gvdb_index_create(const gvdb_params* params, gvdb_index** out);
void gvdb_index_destroy(gvdb_index* index);
/* add_vectors (index.rs:187-210): n rows of `dim` f32, row-major, host memory.
 * Dimension check per row order; on mismatch nothing after the failing row
 * is added (rows before it stay, as in the reference loop).  The index
 * becomes searchable at once (the reference rebuilds after every add). */
gvdb_status gvdb_index_add(gvdb_index* index, const float* rows, uint64_t n, uint32_t dim,
                           const uint64_t* ids);
/* Same, rows already in HBM on the index's device (copied into the index). */
gvdb_status gvdb_index_add_device(gvdb_index* index, const float* d_rows, uint64_t n, uint32_t dim,
                                  const uint64_t* d_ids, void* stream);
/* build_index / optimize (index.rs:140-154, 299-302): re-derives codes and
 * norms; a no-op when they are current. */
gvdb_status gvdb_index_build(gvdb_index* index);
/* search (index.rs:212-231) for a batch of B queries (B x dim, host memory).
 * Per query q, up to k results: out_ids[q*k + i], out_scores[q*k + i],
 * count out_n[q]; slots i >= out_n[q] are zero-filled.  IndexNotBuilt when
 * the index is empty (index.rs:213).  Synchronous: returns when the results
 * are in the caller's buffers.  Reentrant (many concurrent readers, the
 * reference's Arc<RwLock<dyn VectorIndex>>, lib.rs:238): concurrent B = 1
 * calls are coalesced inside the library -- whenever no coalesced batch is
 * executing, the waiting calls with the same k and params run as ONE batched
 * search (up to 256 queries) and each caller gets exactly the results its own
 * call would have returned (every mode is exact); a lone caller runs at once.
 * GVDB_B1_COALESCE=0 disables it.  A query with a NaN score fails only its
 * own call (GVDB_ERR_QUANTIZATION). */
gvdb_status gvdb_index_search(const gvdb_index* index, const float* queries, uint64_t B, uint32_t dim,
                              uint64_t k, const gvdb_search_params* sp, uint64_t* out_ids,
                              float* out_scores, uint32_t* out_n);
/* Same with queries and outputs in HBM.  out_n may be NULL.  The work is
 * ENQUEUED on `stream` and the call returns without any host synchronisation
 * in every mode: results are ready once the caller synchronises that stream
 * (or waits on an event recorded on it after the call).  Modes with tiers
 * decide them on the device: FLAT runs its MFMA candidate tier (i8, or bf16
 * while the index skips i8) and then the exact scan GATED by that tier's
 * certificate word (the scan's kernels exit at once when the tier certified);
 * BQ at the reference's default depth (R > 8192 with R >= N / 64, cosine,
 * k <= 32, N >= 65536, no orphan rows) answers from a certified exact cosine
 * top-32/64 list filtered by the stage-1 membership rule and enqueues the
 * B x R rerank behind it gated by the certificate.  Either way the results are
 * exact.  Tier outcomes are copied to pinned host words behind the search and
 * polled by later calls (they drive the adaptive i8 skip and the counters
 * gvdb_flat_fallback_count / gvdb_flat_i8_fallback_count); nothing waits for
 * them.  A query whose top-R holds a NaN score (the reference's
 * partial_cmp().unwrap() sort would panic) is reported ONLY through
 * out_n[q] = GVDB_N_POISONED: callers that need the reference's failure must
 * pass out_n and check it after the stream (with out_n == NULL such a query's
 * order is unspecified).  Argument and allocation errors are returned by the
 * call itself, before anything is enqueued. */
gvdb_status gvdb_index_search_device(const gvdb_index* index, const float* d_queries, uint64_t B,
                                     uint32_t dim, uint64_t k, const gvdb_search_params* sp,
                                     uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n,
                                     void* stream);
/* Stage-1 only (BQ top-R, quantization.rs:165-179) into device buffers:
 * out_rows[q*R + i] = row index (ascending Hamming, ascending row on ties),
 * out_dist[q*R + i] = Hamming distance.  For sharded search / tests. */
gvdb_status gvdb_index_bq_topr_device(const gvdb_index* index, const float* d_queries, uint64_t B,
                                      uint32_t dim, uint64_t R, uint64_t* d_out_rows,
                                      uint32_t* d_out_dist, void* stream);
/* Sharded-search building block: stage 1 (local top-R) + exact cosine of
 * every candidate, in stage-1 order (Hamming asc, row asc), no final sort.
 * out_ids[q*R + i] = ids[row] (callers use global row numbers as ids),
 * out_dist = Hamming distance, out_scores = cosine (quantization.rs:181-187). */
gvdb_status gvdb_index_bq_candidates_device(const gvdb_index* index, const float* d_queries, uint64_t B,
                                            uint32_t dim, uint64_t R, uint64_t* d_out_ids,
                                            uint32_t* d_out_dist, float* d_out_scores, void* stream);
/* remove_vector (index.rs:233-285): order-preserving compaction. *removed=1
 * if the id was present. */
/* Filtered search: the pre-mask of FilterEngine::execute_filter
 * (filtering.rs:374, whose Vec<String> result maps to u64 ids through the host
 * table) applied to the vector search over the live rows whose id is in
 * allowed[0..n_allowed); unknown ids are ignored, repeats count once, equal
 * scores keep row order.  sp->mode BQ_RERANK: multi_stage_search
 * (quantization.rs:151-193) over those rows, R = rescore_count or
 * (M as f32 * rescore_ratio) as usize for M allowed rows (the allowed rows'
 * codes are compacted on the device: O(M) extra memory); FLAT: the exact scan
 * of those rows; sp == NULL: FLAT, cosine.  Host buffers. */
gvdb_status gvdb_index_search_filtered(const gvdb_index* index, const float* queries, uint64_t B, uint32_t dim,
                                       uint64_t k, const gvdb_search_params* sp, const uint64_t* allowed,
                                       uint64_t n_allowed, uint64_t* out_ids, float* out_scores, uint32_t* out_n);
/* ---- batch-1 request coalescing (concurrent readers) ----------------------
 * Replaces the reference's concurrent single-query readers of
 * Arc<RwLock<dyn VectorIndex>> (src/lib.rs:238), each running
 * HnswVectorIndex::search(q, k) (src/index.rs:212-231).  A coalescer holds one
 * (index, dim, k, search params) triple; gvdb_coalescer_search is one query
 * from any thread: concurrent callers' queries are run together as one
 * gvdb_index_search (the first caller to find no batch executing takes up to
 * max_batch pending queries; requests that arrive meanwhile form the next
 * batch), so the code array is read once per batch instead of once per query.
 * A caller's results are exactly those of its own gvdb_index_search call.
 * max_batch 0 = 256; max_inflight 0 = 1 batch executing at a time.  The index
 * must not be mutated while the coalescer is in use (the reader lock). */
typedef struct gvdb_coalescer gvdb_coalescer;
gvdb_status gvdb_coalescer_create(const gvdb_index* index, uint32_t dim, uint64_t k, const gvdb_search_params* sp,
                                  uint32_t max_batch, uint32_t max_inflight, gvdb_coalescer** out);
/* query: dim floats; out_ids / out_scores: k entries; out_n may be NULL (host buffers) */
gvdb_status gvdb_coalescer_search(gvdb_coalescer* c, const float* query, uint64_t* out_ids, float* out_scores,
                                  uint32_t* out_n);
gvdb_status gvdb_coalescer_stats(gvdb_coalescer* c, uint64_t* batches, uint64_t* queries, uint64_t* max_batch);
void gvdb_coalescer_destroy(gvdb_coalescer* c);

gvdb_status gvdb_index_remove(gvdb_index* index, uint64_t id, int32_t* removed);
uint64_t gvdb_index_len(const gvdb_index* index);
int32_t gvdb_index_is_empty(const gvdb_index* index);
gvdb_status gvdb_index_optimize(gvdb_index* index);
void gvdb_index_clear(gvdb_index* index);
gvdb_status gvdb_index_get_stats(const gvdb_index* index, gvdb_index_stats* out);
/* Device pointers of the resident corpus, for sharded drivers and tests. */
const float* gvdb_index_device_rows(const gvdb_index* index);
/* Live rows and their u64 ids, device -> host, in row order (the source of
 * HnswVectorIndex::get_all_vectors, index.rs:120-135).  cap < live count:
 * GVDB_ERR_INVALID_ARGUMENT with *n_out = the live count. */
gvdb_status gvdb_index_export(const gvdb_index* index, float* rows, uint64_t* ids, uint64_t cap, uint64_t* n_out);

/* ---- BinaryQuantizer (quantization.rs:67-216) --------------------------- */
/* quantize / quantize_batch (86-127): n rows of D f32 -> n rows of
 * ceil(D/8) bytes, BitVec<u8, Msb0> packing, bit = x > threshold. */
gvdb_status gvdb_bq_quantize(const float* rows, uint64_t n, uint32_t D, float threshold, uint8_t* out);
gvdb_status gvdb_bq_quantize_device(const float* d_rows, uint64_t n, uint32_t D, float threshold,
                                    uint8_t* d_out, void* stream);
/* hamming_distance (130-141) for n pairs (a[i], b[i]) of ceil(D/8) bytes. */
gvdb_status gvdb_bq_hamming(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t D, uint32_t* out);
/* multi_stage_search (151-193).  q_bits: ceil(qdim/8) bytes; c_bits: N rows
 * of ceil(cdim/8) bytes; q: qlen f32; cands: N rows of clen f32.
 * Writes min(R, N) entries (R = (N as f32 * rescore_ratio) as usize) to
 * out_idx/out_cos, sorted like the reference; *out_n = that count.
 * Capacity of out_idx/out_cos must be >= min(R, N). */
gvdb_status gvdb_bq_multi_stage_search(const uint8_t* q_bits, uint32_t qdim, const uint8_t* c_bits,
                                       uint32_t cdim, uint64_t N, const float* q, uint64_t qlen,
                                       const float* cands, uint64_t clen, float rescore_ratio,
                                       uint64_t* out_idx, float* out_cos, uint64_t* out_n);

/* ---- flat scan (storage.rs:296-339, index.rs:620-640) ------------------- */
/* Exact scan over N rows (host memory) for B queries: metric COSINE keeps
 * scores >= threshold when has_threshold (storage.rs:313-317), descending;
 * COSINE_DISTANCE ascending; L2 ascending. limit results per query. */
gvdb_status gvdb_flat_search(const float* queries, uint64_t B, const float* rows, uint64_t N, uint32_t D,
                             uint64_t limit, uint32_t metric, int32_t has_threshold, float threshold,
                             uint64_t* out_idx, float* out_scores, uint32_t* out_n);

/* ---- shard merge (shard.rs:776-784) ------------------------------------- */
/* Per query: concat n_shards lists (stride entries each, counts[s*B + q]
 * valid), stable sort by score (descending if `descending`), truncate to
 * limit.  Layout: ids[(s*B + q)*stride + i].  Host memory. */
gvdb_status gvdb_topk_merge(const uint64_t* ids, const float* scores, const uint32_t* counts,
                            uint64_t n_shards, uint64_t B, uint64_t stride, uint64_t limit,
                            int32_t descending, uint64_t* out_ids, float* out_scores, uint32_t* out_n);
/* Same on device buffers (all-gathered shard results stay in HBM). */
gvdb_status gvdb_topk_merge_device(const uint64_t* d_ids, const float* d_scores, const uint32_t* d_counts,
                                   uint64_t n_shards, uint64_t B, uint64_t stride, uint64_t limit,
                                   int32_t descending, uint64_t* d_out_ids, float* d_out_scores,
                                   uint32_t* d_out_n, void* stream);

/* ---- exact sharded multi-stage merge (shard.rs:776-784 + quantization.rs:
 * 165-190 over the concatenated shards) ------------------------------------ */
/* Inputs gathered from G shards, layout [(g*B + q)*stride + i], counts[g*B+q]
 * valid entries each, as produced by gvdb_index_bq_candidates_device with
 * global ids.  Per query: union sorted by (dist asc, gid asc) -> first R ->
 * sorted by (cosine desc, that rank asc) -> first k.  Identical to one
 * multi_stage_search over all shards.  Device form needs G*stride <= 4096. */
gvdb_status gvdb_bq_shard_merge(const uint64_t* gids, const uint32_t* dist, const float* cos,
                                const uint32_t* counts, uint64_t G, uint64_t B, uint64_t stride, uint64_t R,
                                uint64_t k, uint64_t* out_ids, float* out_scores, uint32_t* out_n);
gvdb_status gvdb_bq_shard_merge_device(const uint64_t* d_gids, const uint32_t* d_dist, const float* d_cos,
                                       const uint32_t* d_counts, uint64_t G, uint64_t B, uint64_t stride,
                                       uint64_t R, uint64_t k, uint64_t* d_out_ids, float* d_out_scores,
                                       uint32_t* d_out_n, void* stream);
/* The same merge over the buffer ONE all-gather produces when every rank
 * lets gvdb_index_bq_candidates_device write straight into its send block:
 * rank g's block starts at word g*4*B*R of d_gathered and holds ids (u64
 * [B][R]), then dist (u32 [B][R]), then cosine (f32 [B][R]).  No packing or
 * unpacking copies around the collective.  Needs G*R <= 4096. */
gvdb_status gvdb_bq_shard_merge_packed_device(const uint32_t* d_gathered, const uint32_t* d_counts, uint64_t G,
                                              uint64_t B, uint64_t R, uint64_t k, uint64_t* d_out_ids,
                                              float* d_out_scores, uint32_t* d_out_n, void* stream);

/* ---- sharded search over RCCL (ShardManager::search_vectors, shard.rs:760-786,
 * inside one node: one process per GPU, corpus split into contiguous row
 * ranges whose ids are global row numbers) ---------------------------------- */
#define GVDB_COMM_ID_BYTES 128   /* = sizeof(ncclUniqueId) */
typedef struct gvdb_comm gvdb_comm;
/* Rank 0 creates the id and hands it to the other ranks out of band (the
 * host's own transport: torch.distributed, MPI, a file, ...).  RCCL is loaded
 * on first use (dlopen "librccl.so.1"); GVDB_ERR_DEVICE when it is absent. */
gvdb_status gvdb_comm_get_unique_id(uint8_t id[GVDB_COMM_ID_BYTES]);
/* Collective: every rank of the group calls it (ncclCommInitRank). */
gvdb_status gvdb_comm_create(const uint8_t id[GVDB_COMM_ID_BYTES], int32_t world, int32_t rank, int32_t device,
                             gvdb_comm** out);
void gvdb_comm_destroy(gvdb_comm* comm);
gvdb_status gvdb_comm_info(const gvdb_comm* comm, int32_t* world, int32_t* rank);
/* Exact sharded search (collective; every rank passes the same queries and its
 * own shard = a contiguous row range of the corpus, ranks in corpus order).
 * sp->mode BQ_RERANK (cosine), the two-exchange protocol of gvdb_shard_*:
 * local stage-1 top-R keys -> ncclAllGather (B*R*8 B per rank) -> every rank
 * takes the global top-R by (Hamming, corpus row), reranks only the rows it
 * owns (~R/world per query) and keeps its local top-k -> ncclAllGather
 * (B*k*16 B per rank) -> merged top-k.  sp->mode FLAT: the rank's exact top-k
 * -> ncclAllGather -> merge by (score, corpus row).  Bit-identical to one
 * search over the concatenated shards.  R = max(sp->rescore_count, k) (> 0;
 * the global rescore_ratio form needs the global row count: pass the count),
 * world * k <= 8192, dim <= 8192; R > 8192 (the reference's default ratio at
 * scale) runs the deep form of the protocol (exchange 1 = Hamming histograms,
 * below) with R <= 2^20, dim < 4096, k <= 1024.  Results land on every rank, on
 * `stream`, with no host sync in either mode: the deep form's certified phase 2
 * and every fallback tier (the owned-row rerank, FLAT's exact scan) are chosen on
 * the device by the failing tier's flag.  An empty shard contributes nothing; a
 * rank whose local part fails still joins both collectives (no deadlock),
 * returns its error, and poisons every query of the merge (out_n =
 * GVDB_N_POISONED on every rank), as does a NaN score.  Calls on one comm are
 * serialised; a call on a different stream than the previous one waits for
 * it on the device. */
gvdb_status gvdb_index_search_sharded_device(const gvdb_index* shard, gvdb_comm* comm, const float* d_queries,
                                             uint64_t B, uint32_t dim, uint64_t k, const gvdb_search_params* sp,
                                             uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n,
                                             void* stream);

/* ---- the two-exchange protocol as phases (for hosts with their own transport:
 * MPI, torch.distributed, a CPU fabric).  Block layouts in u32 words:
 *   exchange 1 (per rank, words1), R <= 8192: keys u64 [B][R] (Hamming << 32 |
 *     local row, sorted) | counts u32 [B] | err u32 | pad;
 *   exchange 1, deep form (R > 8192): hist u32 [B][dim+1] (Hamming histogram
 *     of the rank's local top-min(R, rows)) | counts u32 [B] | err u32 | pad
 *     -- B*(dim+1)*4 bytes per rank whatever R is;
 *   exchange 2 (per rank, words2): [B][k] x {cosine bits, order key, id lo,
 *     id hi} | meta u32 [B] (count | NaN << 31) | reff [B] | err | pad; the
 *     order key is the entry's global stage-1 position (key form) or its
 *     Hamming distance (deep form): the merge orders by (cosine desc, order
 *     key, rank, list index), in both forms the stable order of the global
 *     top-R.
 * Gathered buffers hold rank g's block at word g * words. ------------------- */
void gvdb_shard_sizes(uint64_t B, uint64_t R, uint64_t k, uint32_t dim, uint64_t* words1, uint64_t* words2,
                      uint64_t* scratch_bytes);
uint64_t gvdb_shard_flat_words(uint64_t B, uint64_t k);
/* Phase 1: this rank's exchange-1 block (an empty shard: count 0).  d_scratch
 * (scratch_bytes of device memory, NULL allowed when R <= 8192) keeps the deep
 * form's local membership for phase 2: pass the same scratch to both. */
gvdb_status gvdb_shard_stage1_device(const gvdb_index* shard, const float* d_queries, uint64_t B, uint32_t dim,
                                     uint64_t R, uint32_t* d_block1, void* d_scratch, void* stream);
/* Phase 2: from the gathered exchange-1 blocks, this rank's exchange-2 block
 * (global top-R, exact cosine of the owned rows, local top-k).  d_scratch:
 * scratch_bytes of device memory (deep form: the scratch phase 1 filled; phase
 * 2 only reads its member lists, so it may run again on them).  Deep form on a
 * shard of >= 65536 rows without orphan rows, k <= 32: the rank's local top-k
 * comes from its certified exact cosine top-32 / 64 filtered by its owned-row
 * rule (no rerank of the ~R / G owned rows); the owned-row rerank is enqueued
 * behind it, gated on the device by the certificate word, for a list that
 * cannot certify.  No host synchronisation in either form. */
gvdb_status gvdb_shard_rerank_device(const gvdb_index* shard, const float* d_queries, uint64_t B, uint32_t dim,
                                     uint64_t R, uint64_t k, const uint32_t* d_gathered1, uint64_t G, uint64_t rank,
                                     void* d_scratch, uint32_t* d_block2, void* stream);
/* Phase 3: the merged top-k from the gathered exchange-2 blocks. */
gvdb_status gvdb_shard_final_device(const uint32_t* d_gathered2, uint64_t G, uint64_t B, uint64_t k,
                                    uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n, void* stream);
/* Sharded FLAT: rank g's block (gvdb_shard_flat_words u32 words) holds its
 * exact top-k as gvdb_index_search_device writes it: ids u64 [B][k] at word 0,
 * scores f32 [B][k] at word 2*B*k, out_n u32 [B] at word 3*B*k, then an err
 * word (nonzero poisons every query); the merge orders by
 * (score per `metric`, rank, list position) = (score, corpus row). */
gvdb_status gvdb_shard_flat_final_device(const uint32_t* d_gathered, uint64_t G, uint64_t B, uint64_t k,
                                         uint32_t metric, uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n,
                                         void* stream);
/* Host forms of the merges (host memory, same layouts): phase 2's merge gives
 * this rank's owned rows / global positions [B][R], their count and the global
 * list length per query; local_topk builds the exchange-2 block from the owned
 * entries' cosines and ids (in own_pos order); final = phase 3. */
gvdb_status gvdb_shard_merge_host(const uint32_t* gathered1, uint64_t G, uint64_t rank, uint64_t B, uint64_t R,
                                  uint32_t* own_rows, uint32_t* own_pos, uint32_t* own_cnt, uint32_t* reff);
/* Deep form of phase 2's merge: this rank's members (m_rows / m_dist [B][R],
 * the first min(its count, R) valid, any order) -> its owned entries sorted by
 * (Hamming, row) in own_rows / own_dist [B][R]; pass own_dist as local_topk's
 * own_pos. */
gvdb_status gvdb_shard_deep_own_host(const uint32_t* gathered1, uint64_t G, uint64_t rank, uint64_t B, uint64_t R,
                                     uint32_t dim, const uint32_t* m_rows, const uint32_t* m_dist,
                                     uint32_t* own_rows, uint32_t* own_dist, uint32_t* own_cnt, uint32_t* reff);
gvdb_status gvdb_shard_local_topk_host(const float* scores, const uint32_t* own_pos, const uint64_t* own_ids,
                                       const uint32_t* own_cnt, const uint32_t* reff, uint64_t B, uint64_t R,
                                       uint64_t k, uint32_t err, uint32_t* block2);
gvdb_status gvdb_shard_final_host(const uint32_t* gathered2, uint64_t G, uint64_t B, uint64_t k, uint64_t* out_ids,
                                  float* out_scores, uint32_t* out_n);

/* ---- BM25 sparse index (src/sparse.rs:29-222) ---------------------------- */
/* SparseIndex: documents are (term id, term frequency) lists with a
 * document_length, exactly what DocumentSparseRepresentation carries
 * (types.rs:93-102).  The host keeps the document-major entries; the device
 * holds them as a blocked inverted index (per 64-document chunk, entries by
 * term), rebuilt lazily after a mutation.  Search is term-at-a-time per
 * chunk (gvdb_sparse.hip). */
typedef struct gvdb_bm25_params {  /* BM25Parameters, sparse.rs:42-53 */
    float k1;                       /* default 1.2 */
    float b;                        /* default 0.75 */
    int32_t device;                 /* HIP device ordinal */
    uint32_t reserved;
} gvdb_bm25_params;

typedef struct gvdb_bm25_stats {   /* BM25Stats, types.rs:104-115 */
    uint64_t total_documents;
    float average_document_length;  /* sum of EVERY posting entry's length / N (sparse.rs:96-104) */
    uint32_t reserved;
    uint64_t vocabulary_size;       /* terms with a document frequency */
    uint64_t total_entries;         /* posting entries held */
    uint64_t dense_fallbacks;       /* diagnostics: queries answered by the dense-key fallback */
} gvdb_bm25_stats;

typedef struct gvdb_sparse gvdb_sparse;

/* SparseIndex::new (sparse.rs:57-69); params NULL = defaults */
gvdb_status gvdb_sparse_create(const gvdb_bm25_params* params, gvdb_sparse** out);
void gvdb_sparse_destroy(gvdb_sparse* index);
/* add_document (sparse.rs:71-107): n distinct terms with their tf; a second
 * add of the same id adds a second entry per term (as the reference's
 * posting lists do).  Duplicate terms in one call: GVDB_ERR_INVALID_ARGUMENT. */
gvdb_status gvdb_sparse_add_document(gvdb_sparse* index, uint64_t doc_id, const uint32_t* terms, const float* tfs,
                                     uint64_t n, float document_length);
/* Bulk add: document d's terms are terms[doc_ptr[d] .. doc_ptr[d+1]). */
gvdb_status gvdb_sparse_add_documents(gvdb_sparse* index, const uint64_t* doc_ids, const uint64_t* doc_ptr,
                                      const uint32_t* terms, const float* tfs, const float* document_lengths,
                                      uint64_t n_docs);
/* remove_document (sparse.rs:109-149): *removed = 1 if any entry went. */
gvdb_status gvdb_sparse_remove_document(gvdb_sparse* index, uint64_t doc_id, int32_t* removed);
gvdb_status gvdb_sparse_get_stats(const gvdb_sparse* index, gvdb_bm25_stats* out);
void gvdb_sparse_clear(gvdb_sparse* index);
/* search_bm25 (sparse.rs:151-198) for B queries given as CSR: query q's
 * SparseVector indices / values are q_terms / q_values[q_ptr[q] ..
 * q_ptr[q+1]).  Per query up to `limit` (id, score) pairs, score descending,
 * out_ids[q*limit + i], count out_n[q].  Equal scores: ascending document slot
 * (first add); the reference leaves them in HashMap order. */
gvdb_status gvdb_sparse_search_bm25(gvdb_sparse* index, const uint64_t* q_ptr, const uint32_t* q_terms,
                                    const float* q_values, uint64_t B, uint64_t limit, uint64_t* out_ids,
                                    float* out_scores, uint32_t* out_n);

/* ---- reciprocal-rank fusion (HybridSearchEngine::rrf_fusion, hybrid.rs:422-488) */
/* Per query three ranked id lists (dense, sparse, text; NULL counts = empty
 * list), list l of query q at ids_l[q*stride_l + r], r < n_l[q], with its raw
 * score.  Fused score = sum of 1/(k + rank+1) (a repeated dense id replaces,
 * sparse / text repeats add), descending, ties by first appearance; the first
 * `limit` per query go to out_ids / out_scores [q*limit + i] and, when
 * out_breakdown is non-NULL, the raw dense / sparse / text score of each
 * result to out_breakdown[(q*limit + i)*3 + l] (NaN = absent, ScoreBreakdown).
 * At most 4096 items per query: the three list strides (of the lists passed)
 * may sum to 4096, more is GVDB_ERR_INVALID_ARGUMENT.  The _device form takes
 * device pointers. */
gvdb_status gvdb_rrf_fuse(const uint64_t* dense_ids, const float* dense_scores, const uint32_t* dense_n,
                          uint32_t dense_stride, const uint64_t* sparse_ids, const float* sparse_scores,
                          const uint32_t* sparse_n, uint32_t sparse_stride, const uint64_t* text_ids,
                          const float* text_scores, const uint32_t* text_n, uint32_t text_stride, uint64_t B, float k,
                          uint64_t limit, uint64_t* out_ids, float* out_scores, float* out_breakdown, uint32_t* out_n);
gvdb_status gvdb_rrf_fuse_device(const uint64_t* d_dense_ids, const float* d_dense_scores, const uint32_t* d_dense_n,
                                 uint32_t dense_stride, const uint64_t* d_sparse_ids, const float* d_sparse_scores,
                                 const uint32_t* d_sparse_n, uint32_t sparse_stride, const uint64_t* d_text_ids,
                                 const float* d_text_scores, const uint32_t* d_text_n, uint32_t text_stride, uint64_t B,
                                 float k, uint64_t limit, uint64_t* d_out_ids, float* d_out_scores,
                                 float* d_out_breakdown, uint32_t* d_out_n, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GVDB_H_ */
