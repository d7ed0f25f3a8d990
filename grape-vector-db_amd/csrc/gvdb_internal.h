// gvdb_internal.h — internal launch interface between the C ABI layer
// (gvdb_capi.hip) and the gfx950 kernels (gvdb_kernels.hip).
//
// HBM layout of one index shard:
//   rows  : float [cap][D]            row-major f32 corpus (rerank gathers rows)
//   codes : uint4 [W4][cap]           BQ codes, word-major SoA: plane w4 holds
//                                     code words 4*w4 .. 4*w4+3 of every row;
//                                     word w = little-endian u32 of Msb0 bytes
//                                     4w..4w+3 (quantization.rs:97-101 packing),
//                                     pad bytes 0.  Lane n reads row n: every
//                                     wave-load is 1 KiB contiguous.
//   norms : float [cap]               sqrt(sequential sum x*x) per row
//   ids   : uint64 [cap]              caller ids; GVDB_ORPHAN = shadowed row
#pragma once
#include "../../include/gvdb.h"
#include <string>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gvdb {

constexpr uint64_t kOrphan = ~0ull;       // row whose id was re-added (index.rs:175-176)
constexpr uint32_t kSelectLdsCap = 8192;  // stage-1 select: keys sorted in LDS
constexpr uint32_t kSortLdsCap = 4096;    // stage-2 sort: keys sorted in LDS

__host__ __device__ inline uint32_t code_words(uint32_t D) { return (((D + 7u) / 8u) + 3u) / 4u; }  // u32 words
// uint4 planes per row, rounded up to a width the scan kernel is instantiated
// for (pad planes hold zero bits in query and rows alike: no distance change).
__host__ __device__ inline uint32_t code_w4(uint32_t D) {
    const uint32_t raw = (code_words(D) + 3u) / 4u;
    const uint32_t set[10] = {1, 2, 3, 4, 6, 8, 12, 16, 24, 32};
    for (int i = 0; i < 10; ++i)
        if (raw <= set[i]) return set[i];
    return raw;
}

enum PackLayout : int {
    kPackBytesAoS = 0,  // Msb0 bytes, row stride ceil(D/8)           (BinaryVector::to_bytes)
    kPackWordsAoS = 1,  // u32 words, row stride 4*W4 words           (query codes)
    kPackSoA = 2,       // uint4 planes [W4][cap] (index codes)
};

enum ScoreKind : int { kScoreCosine = 0, kScoreL2 = 1, kScoreCosineDistance = 2 };

// ---- K1 pack ----------------------------------------------------------------
hipError_t launch_pack(const float* rows, uint64_t n, uint32_t D, float thr, void* out, int layout,
                       uint64_t cap, uint64_t row0, hipStream_t s);
hipError_t launch_bytes_to_soa(const uint8_t* bytes, uint64_t n, uint32_t D, uint4* codes, uint64_t cap,
                               uint64_t row0, hipStream_t s);
hipError_t launch_bytes_to_words(const uint8_t* bytes, uint64_t n, uint32_t D, uint32_t* words, hipStream_t s);
hipError_t launch_hamming_pairs(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t D, uint32_t* out,
                                hipStream_t s);

// ---- exact sequential norms (bit-identical to the reference's fold) -----------
// gate (optional): a device-side tier gate (gvdb_device.h gate_closed): the launch does
// nothing while *gate == 0 -- the host-sync-free fallback tiers take one everywhere below
hipError_t launch_row_norms(const float* rows, uint64_t n, uint32_t D, float* out, hipStream_t s,
                            const uint32_t* gate = nullptr);

// ---- K2 stage 1: BQ Hamming top-R -----------------------------------------------
struct Stage1Args {
    const uint4* codes;      // [W4][cap]
    uint64_t cap;
    uint32_t N;              // rows scanned
    uint32_t D;              // dimension (bits)
    const uint4* qcodes;     // [B][W4]
    uint32_t B;
    uint32_t R;
    // sampling for the threshold estimate
    uint32_t sample_chunks;  // number of contiguous 4096-row chunks
    uint32_t sample_stride;  // rows between chunk starts
    uint32_t target;         // sample count that defines the threshold
    // workspace
    uint32_t* hist;          // [B][D+1]
    uint32_t* thr;           // [B]
    uint32_t* counts;        // [B]
    uint64_t* buf;           // [B][bufcap]
    uint32_t bufcap;
    uint32_t* fail;          // [B]  (1 = fast path could not certify the top-R)
    uint32_t* any_fail;      // [1]  OR of fail[]
    uint32_t* s1_rows;       // [B][R]
    uint32_t* s1_dist;       // [B][R]
    hipEvent_t* ev;          // optional [4]: before hist, before scan, after scan, after select
    int use_mfma;            // large batches: 0 popcount only, 1 FP4 MFMA scan, 2 i8 MFMA scan
    int force_rescan;        // tests: every query takes k_select's exact all-rows rescan (GVDB_FORCE_RESCAN)
    // FP4-MFMA paths (stage1_plan): query fragments built once per batch by k_qfrag
    int sample_mode;         // kSampleValu / kSampleMxHist / kSampleDense
    bool mfma_scan;          // k_scan_mx5 runs (needs qfrag / qpc)
    uint4* qfrag;            // [ceil(B/256)][8 * 2*W4 * 64] FP4 query fragments
    uint32_t* qpc;           // [ceil(B/256) * 256] |q|
    uint16_t* smp;           // kSampleDense: [B][sample rows] sampled distances
    uint64_t* keys_out;      // optional [B][keys_stride]: the sorted top-R keys (d << 32 | row) (sharded
                             // search), followed by u32 counts [B] (= R)
    uint32_t keys_stride;
    uint32_t* zero;          // mfma_scan: words k_qfrag zeroes before stage 1 (else the caller memsets)
    uint32_t nzero;
    int big_select;          // R > kSelectLdsCap: k_select_big (unordered exact top-R membership)
    int dense_sel;           // big_select at density R/N >= 1/64 with an FP4 scan width: every distance is
                             // written (k_scan_mx7<DENSE>, f16 dots) and k_select_dense picks the members
    uint16_t* dense;         // dense_sel: [min(B, 256)][dense_np] f16 dots of one 256-query group
    uint32_t dense_np;       //   row stride (N rounded up to 32)
    const float* qf32;       // mfma_scan: the f32 queries [B][D] -- k_qprep packs qcodes itself
    float qthr;              //   (packing threshold)
    uint32_t* tcut;          // optional, dense_sel: [B][4] the membership rule (T, cut, need, 0) instead of
                             // the lists
    uint32_t* mhist;         // optional, dense_sel: [B][H = D+1] the members' Hamming histogram (deep sharded
    uint32_t* mcount;        //   exchange-1 block) and [B] their count, written by k_select_dense
    const uint32_t* gate;    // optional tier gate (dense_sel + FP4 scan only): the stage runs iff *gate != 0
    uint32_t* seg_hist;      // optional, dense_sel + tcut: [B][seg_n][D+1] per-segment Hamming histograms (the
    uint32_t seg_n;          //   parallel rule form: k_dense_seg_hist + k_dense_rule); seg_n segments of
    uint32_t seg_len;        //   seg_len rows (dense_segments)
    int dense_keep;          // dense_sel: `dense` holds every query's row ([B][dense_np], caller memory) instead
                             // of one 256-query group's
    uint32_t* pc_out;        // optional, the parallel rule form: |q| per query [B] (kept for a later call)
    int dense8;              // the parallel rule form only (tcut + seg_hist, no mhist / dense_keep): one byte
    uint32_t* qwin;          //   per pair, clamp(d - base, 0, 255); qwin [2][B]: base[B] then hi[B], from
                             //   k_dense_base (hi: the largest distance the histograms count); `dense` holds bytes
};
constexpr uint32_t kDenseSegs = 64;  // row segments of the parallel dense rule
// S segments of L rows (L % 256 == 0) covering N rows, S <= min(smax, kDenseSegs)
void dense_segments(uint32_t N, uint32_t smax, uint32_t* S, uint32_t* L);
// the deep sharded fallback without member lists: this rank's owned rows under tcut's rule (T, -, quota)
// -- every row with d < T, then the first `quota` rows with d == T in row order -- compacted in row
// order from the dense block into o_rows / o_dist [B][ostride]
hipError_t launch_dense_own(const uint16_t* dense, uint32_t np, uint32_t N, const uint32_t* tcut, const uint32_t* qpc,
                            uint32_t B, uint32_t* o_rows, uint32_t* o_dist, uint32_t ostride, const uint32_t* gate,
                            hipStream_t s);
// ---- large rescore depth (gvdb_bigr.hip): R up to 2^20, D < 4096, k <= 1024 --------
constexpr uint32_t kBigRMax = 1u << 20;
hipError_t launch_select_big(const Stage1Args& a, hipStream_t s);
// dense_sel: the members of queries [g0, g0 + bg) from their dense f16 dots (gvdb_bigr.hip)
hipError_t launch_select_dense(const Stage1Args& a, uint32_t g0, uint32_t bg, hipStream_t s);
// dense8: every query's byte window (base, hi) into a.qwin from a strided sample (gvdb_bigr.hip)
hipError_t launch_dense_base(const Stage1Args& a, hipStream_t s);
// certified default-depth search (gvdb_bigr.hip): the first min(k, R) members of the exact top-K2 cosine
// list (rows + scores, (cos desc, row) order, fn[q] entries) under the membership rule tcut; fail[0] |= 1
// for a query the list cannot certify
constexpr uint32_t kDeepK2 = 64;  // exact cosine list length (one lane per entry)
// (kcnt: per-query member counts instead of R; block2 / reff: write the exchange-2 block of the deep sharded
// form -- {cos bits, Hamming, id lo, id hi} [B][k] + meta -- instead of out_ids / out_scores / out_n)
hipError_t launch_deep_certify(const uint64_t* frow, const float* fsc, const uint32_t* fn, uint32_t K2,
                               const uint32_t* tcut, const uint4* codes, uint64_t cap, uint32_t W4,
                               const uint4* qcodes, uint32_t B, uint32_t k, uint32_t R, const uint64_t* ids,
                               uint64_t* out_ids, float* out_scores, uint32_t* out_n, uint32_t* fail, hipStream_t s,
                               const uint32_t* kcnt = nullptr, uint32_t* block2 = nullptr,
                               const uint32_t* reff = nullptr, const uint32_t* m_rows = nullptr,
                               const uint32_t* m_dist = nullptr, uint32_t mlen = 0,
                               const uint32_t* list_fail = nullptr,  // != 0: the list is not certified
                                                                     // (every query fails)
                               const uint32_t* seg_hist = nullptr, uint32_t seg_n = 0, uint32_t seg_len = 0,
                               uint32_t seg_h = 0, const uint16_t* dense = nullptr, uint32_t dense_np = 0);  // mode 3 from the
                                                                     // dense block instead of m_rows / m_dist
constexpr uint32_t kMfmaMinB = 96;  // batch size from which k_scan_mfma replaces k_scan
enum SampleMode : int { kSampleValu = 0, kSampleMxHist = 1, kSampleDense = 2, kSampleWide = 3 };
// Decide sample_mode / mfma_scan for a prepared Stage1Args (use_mfma, B, D, N,
// sample_chunks, target set) and return the workspace bytes of qfrag + qpc +
// smp it needs (0 = none).
size_t stage1_plan(Stage1Args& a);
// code widths with an MFMA scan instantiation (D <= 768; wider codes would
// not fit the query fragments + prefetch in 256 VGPRs at 2 waves/SIMD)
__host__ __device__ inline bool mfma_scan_supported(uint32_t W4) { return W4 == 2 || W4 == 3 || W4 == 4 || W4 == 6; }
// k_scan_mx4 (wide codes, D = 1024 / 1536 / 2048 / 3072 / 4096 bits)
__host__ __device__ inline bool mx4_scan_supported(uint32_t W4) {
    return W4 == 8 || W4 == 12 || W4 == 16 || W4 == 24 || W4 == 32;
}
// hist/counts/fail must be zeroed by the caller on stream s.
hipError_t launch_stage1_fast(const Stage1Args& a, hipStream_t s);
// Batch-1 fast path (gvdb_kernels.hip: k_b1_sample -> k_b1_scan -> k_b1_tail):
// sample histogram + threshold, scan, exact select + rerank + final sort, with
// no host round trip.  D <= 1024, R <= kSortLdsCap.  hist / counts / ticket
// must be zero before the first call; the path leaves them zero.
struct B1Args {
    const uint4* codes;
    uint64_t cap;
    uint32_t N, D, R, kout;
    const float* q;          // [qlen] f32 query (packed in-kernel with thr)
    uint64_t qlen;
    float thr;
    const float* rows;
    uint64_t clen;
    const float* norms;
    const uint64_t* ids;
    uint64_t row_offset;
    int kind, descending, force_rescan;
    uint32_t sample_chunks, sample_stride, target, bufcap;
    uint32_t* hist;          // [D+1]
    uint32_t* counts;        // [1]
    uint32_t* ticket;        // [1]
    uint32_t* rescans;       // [1] diagnostics
    uint32_t* qwords;        // [4*W4]
    float* scores;           // [bufcap] exact scores of the buffered candidates
    float* rscores;          // [R] exact scores of a rescan's rows
    uint64_t* topr;          // [R] sorted top-R keys published by the select block
    uint64_t* buf;           // [bufcap]
    uint64_t* out_ids;
    float* out_scores;
    uint32_t* out_n;         // or nullptr
    hipEvent_t* ev;          // optional [4]
    unsigned long long* clk; // timing study only: phase wall clocks of k_b1_tail
};
constexpr uint32_t kB1ChunkRows = 1024;  // rows per k_b1_sample chunk
constexpr uint32_t kB1MaxD = 1024;
constexpr uint32_t kB1RerankBlocks = 128;  // k_b1_tail blocks re-scoring candidates (16 each per round)
constexpr uint32_t kB1MaxBufcap = 1u << 20;  // buffer index fits the 21-bit key field
hipError_t launch_b1_search(const B1Args& b, hipStream_t s);

// Exact slow path for ONE query: all N distances + stable radix sort.
// tmp buffers sized by stage1_slow_bytes().
size_t stage1_slow_bytes(uint32_t N);
hipError_t launch_stage1_slow(const uint4* codes, uint64_t cap, uint32_t N, uint32_t D, const uint4* qcode,
                              uint32_t R, uint32_t* out_rows, uint32_t* out_dist, void* tmp, size_t tmp_bytes,
                              hipStream_t s);
// Stage 1 when the query dimension differs from the candidates' (every
// similarity is 0.0, quantization.rs:168): rows 0..R-1 in order.
hipError_t launch_iota_rows(uint32_t* rows, uint32_t B, uint32_t R, hipStream_t s);

// ---- K3 stage 2: exact rerank of the stage-1 list ------------------------------
struct RerankArgs {
    const float* rows;       // [*][clen]
    uint64_t clen;
    const float* norms;      // [*]
    const float* q;          // [B][qlen]   (query norms are folded in-kernel)
    uint64_t qlen;
    const uint32_t* s1_rows; // [B][R]
    uint32_t B, R;
    int kind;                // ScoreKind
    float* scores;           // [B][R]
    const uint32_t* counts;  // optional [B]: only the first counts[q] entries are valid
    int short_lists;         // counts are mostly <= 16 (sharded owned rows): k_rerank_small
    const uint32_t* gate;    // optional tier gate: the rerank runs iff *gate != 0
};
hipError_t launch_rerank(const RerankArgs& a, hipStream_t s);

// Final ordering of each query's R scores (stable: ties keep stage-1 rank),
// truncated to kout; rows -> ids (ids==nullptr: emit row numbers); orphans
// dropped after truncation.  R <= kSortLdsCap: one workgroup per query.
struct FinalArgs {
    const float* scores;     // [B][R]
    const uint32_t* s1_rows; // [B][R]
    uint32_t B, R, kout;
    int descending;
    const uint64_t* ids;     // row -> id, or nullptr
    uint64_t row_offset;     // added to emitted row numbers when ids == nullptr
    uint64_t* out_ids;       // [B][kout]
    float* out_scores;       // [B][kout]
    uint32_t* out_n;         // [B] or nullptr
    uint32_t* nan_flag;      // [0] set to 1 if a NaN score would make the reference panic;
                             // [1] per-query scratch of the global sort (zero on entry)
    const uint32_t* gate;    // optional tier gate (launch_topk_big only): runs iff *gate != 0
};
hipError_t launch_final_sort(const FinalArgs& a, hipStream_t s);
size_t final_sort_global_bytes(uint32_t R);
hipError_t launch_final_sort_global(const FinalArgs& a, void* tmp, size_t tmp_bytes, hipStream_t s);
// the first kout (<= 1024) of the stable order of an UNORDERED stage-1 list
// (k_select_big's): keys (score order, Hamming, row) (gvdb_bigr.hip)
hipError_t launch_topk_big(const FinalArgs& a, const uint32_t* s1_dist, hipStream_t s);

// ---- flat exact scan (storage.rs:296-339, index.rs:620-640) --------------------
// list (optional, [N]): scan the shard rows list[0..N) instead of rows 0..N-1
// (filtered search); scores stay indexed by scan position.
hipError_t launch_flat_scores(const float* q, uint32_t B, const float* qnorm, const float* rows, uint32_t N,
                              uint32_t D, const float* norms, int kind, const uint32_t* list,
                              float* scores /*[B][N]*/, hipStream_t s, const uint32_t* gate = nullptr);
size_t flat_select_bytes(uint32_t N);
// per query: keep score >= threshold when has_threshold (cosine), stable sort,
// first `limit`.
// ids: row -> id with orphans skipped (nullptr: emit row numbers).
hipError_t launch_flat_select(const float* scores, uint32_t B, uint32_t N, uint32_t limit, int descending,
                              int has_threshold, float threshold, const uint64_t* ids, uint64_t* out_idx,
                              float* out_scores, uint32_t* out_n, void* tmp, size_t tmp_bytes, uint32_t* nan_flag,
                              hipStream_t s, const uint32_t* gate = nullptr);  // gated: limit <= 1024

// ---- K4 flat exact search on bf16 MFMA (gvdb_flat.hip) ---------------------------
// Candidate pass on bf16 MFMA + exact rerank + per-query certificate; see
// gvdb_flat.hip.  rowsb: bf16 fragment-major mirror (fx_frag), KC = fx_kc(D).
constexpr uint32_t kFxRows = 256;      // rows per tile
constexpr uint32_t kFxQ = 256;         // query slots per launch group
constexpr uint32_t kFxCandCap = 8192;  // candidates per query (LDS sort capacity)
constexpr uint32_t kFxMinN = 65536;    // smaller shards use the exact full scan
constexpr uint32_t kFxSampleEvery = 64;  // sample pass: every 64th row tile
constexpr uint32_t kFxProbeParts = 16;   // probe selection: blocks per query (partial top-16 lists)
__host__ __device__ inline uint32_t fx_kc(uint32_t D) { return (D + 63u) / 64u; }        // bf16 chunks
__host__ __device__ inline uint32_t fx_kc_i8(uint32_t D) { return (D + 127u) / 128u; }  // i8 chunks
// Fragment-major flat mirror: per 256-row tile and 128-B chunk, 8 groups of
// 32 rows, each [k-step s 0..3][lane 0..63][16 B] = 4 KiB, so one wave reads
// the MFMA operand fragment of its 32 rows for one k-step as 1 KiB contiguous
// (lane = 32 h + r holds bytes [32 s + 16 h, +16) of row r's chunk).  Byte
// offset of 16-B piece pc (0..7) of chunk c of `row`; queries use the same
// layout with the slot as the row (one tile).
__host__ __device__ inline uint64_t fx_frag(uint64_t row, uint32_t c, uint32_t KC, uint32_t pc) {
    return (((((row >> 8) * KC + c) * 8 + ((row >> 5) & 7u)) * 4 + (pc >> 1)) * 64 + (pc & 1u) * 32 + (row & 31u)) * 16;
}
__host__ __device__ inline uint64_t fx_mirror_bytes(uint64_t cap, uint32_t KC) {
    return ((cap + 255u) >> 8) * KC * 256u * 128u;
}
struct FlatMxArgs {
    int i8;                  // element kind: 1 = int8 (k_flat_mx<., true>), 0 = bf16
    const void* rowsx;       // fragment-major mirror (fx_frag): bf16 x64 or int8 x128 per chunk row
    uint64_t cap;
    uint32_t N, KC;
    const void* qx;          // fragment-major (fx_frag), one 256-slot tile
    const float* qinv;       // [kFxQ]  bf16: 1/|q|; i8: s_q/|q|
    const float* rnorm;      // [N] exact row norms (bf16)
    const float* rscale;     // [N] s_x/|x| (i8)
    const float* rrho;       // [N] relative quantisation error rho_x (i8)
    const float* qa;         // [kFxQ] pair-bound terms (see k_flat_mx's epilogue)
    const float* qd;         // [kFxQ]
    uint32_t B;              // live query slots (<= kFxQ)
    uint32_t every;          // sample pass: tile stride
    float* smp;              // sample pass: [B][S] MFMA scores of the sampled rows
    uint32_t S;              // sample pass: sampled rows (= sampled tiles * kFxRows)
    const float* thr;        // emit pass: [B]
    uint32_t* counts;        // emit pass: [B] (zeroed by the caller)
    uint32_t* cand;          // emit pass: [B][candcap] candidate rows
    float* cscore;           // emit pass: [B][candcap] their approx scores (null: not stored)
    uint32_t candcap;
    uint32_t* overflow;      // emit pass: set to 1 if a wave's LDS staging slice overflowed
};
float flat_eps(uint32_t D);
hipError_t launch_rows_to_bf16(const float* rows, uint64_t n, uint32_t D, uint16_t* rowsb, uint64_t cap,
                               uint32_t* nan_flag, hipStream_t s);
hipError_t launch_queries_to_bf16(const float* q, uint32_t B, uint32_t D, const float* qnorm, uint16_t* qb,
                                  float* qinv, float* qd, hipStream_t s);
// rows -> int8 [KC_i8][cap][128], rscale = s_x/|x|, rrho = relative
// quantisation error, *bad = non-finite rows
hipError_t launch_rows_to_i8(const float* rows, const float* norms, uint64_t n, uint32_t D, int8_t* rowsq, uint64_t cap,
                             float* rscale, float* rrho, uint32_t* bad_flag, hipStream_t s);
hipError_t launch_queries_to_i8(const float* q, uint32_t B, uint32_t D, const float* qnorm, int8_t* qq, float* qinv,
                                float* qa, float* qd, hipStream_t s);
hipError_t launch_flat_mx_sample(const FlatMxArgs& a, hipStream_t s);
hipError_t launch_flat_mx_emit(const FlatMxArgs& a, hipStream_t s);
// Drops the candidates that cannot reach a query's top k (upper bound below the
// k-th largest lower bound of the live candidates) and orphaned rows; counts[q]
// becomes the survivors.  qa / rrho null for bf16 (bound = qd).
hipError_t launch_flat_prune(uint32_t* counts, uint32_t* cand, const float* cscore, uint32_t candcap, uint32_t B,
                             uint32_t k, const float* qa, const float* qd, const float* rrho, const uint64_t* ids,
                             hipStream_t s);
// probes[q][16] = rows of the 16 largest sampled MFMA scores, pcount[q] valid
hipError_t launch_flat_probes(const float* smp, uint32_t B, uint32_t S, uint32_t every, uint32_t N, const uint64_t* ids,
                              uint32_t* probes, uint32_t* pcount, uint64_t* part, hipStream_t s);  // part: [B][16][16]
// thr[q] = (mk-th largest exact probe score) - qd[q] (mk <= 16); +inf for q >= B.
// distance: pscores hold 1 - cos (the index metric's rerank output).
hipError_t launch_flat_tau(const float* pscores, const uint32_t* pcount, uint32_t B, uint32_t mk, int distance,
                           const float* qd, float* thr, hipStream_t s);
// sort reranked candidates by (exact score, row), emit first k live rows,
// OR 1 into *fail for a query whose list is not certified exact
hipError_t launch_flat_final(const uint32_t* counts, const uint32_t* cand, uint32_t candcap, const float* scores,
                             const float* thr, const float* qd, uint32_t B, uint32_t k, int descending,
                             const uint64_t* ids, uint64_t* out_ids, float* out_scores, uint32_t* out_n, uint32_t* fail,
                             hipStream_t s);

// ---- shard merge (shard.rs:776-784) --------------------------------------------
hipError_t launch_topk_merge(const uint64_t* ids, const float* scores, const uint32_t* counts, uint32_t n_shards,
                             uint32_t B, uint32_t stride, uint32_t limit, int descending, uint64_t* out_ids,
                             float* out_scores, uint32_t* out_n, hipStream_t s);

hipError_t launch_widen(const uint32_t* a, uint64_t* b, uint64_t n, hipStream_t s);

hipError_t launch_emit_candidates(const uint32_t* s1_rows, const uint32_t* s1_dist, const float* scores, uint32_t B,
                                  uint32_t R, const uint64_t* ids, uint64_t* out_ids, uint32_t* out_dist,
                                  float* out_scores, hipStream_t s, uint64_t out_stride = 0);  // 0 = R
// Exact sharded multi-stage merge (one exchange): see gvdb_kernels.hip.
// G*stride <= kSortLdsCap.
hipError_t launch_bq_shard_merge(const uint64_t* gids, const uint32_t* dist, const float* cosv, const uint32_t* counts,
                                 uint32_t G, uint32_t B, uint32_t stride, uint32_t R, uint32_t kout, uint64_t* out_ids,
                                 float* out_scores, uint32_t* out_n, uint32_t* nan_flag, hipStream_t s,
                                 uint64_t gs_id = 0, uint64_t gs_w = 0,  // rank strides (0 = dense [G][B][stride])
                                 uint64_t gs_c = 0,                      // count stride per rank (0 = B)
                                 int mark_nan = 0);                      // poisoned query -> out_n = GVDB_N_POISONED

// ---- index maintenance -----------------------------------------------------------
// Order-preserving gather of rows/codes/norms/ids: new row r <- old row map[r]
// (remove_vector compaction, index.rs:245-266).
// filtered BQ: compact the allowed rows' code planes (cap = m); map stage-1 rows back
hipError_t launch_gather_code_rows(const uint4* codes, uint64_t cap, const uint32_t* rows, uint32_t m, uint32_t D,
                                   uint4* ncodes, hipStream_t s);
hipError_t launch_map_rows(uint32_t* s1_rows, uint64_t n, const uint32_t* rows, hipStream_t s);
hipError_t launch_gather(const float* rows, float* nrows, const uint4* codes, uint4* ncodes, const float* norms,
                         float* nnorms, const uint64_t* ids, uint64_t* nids, const uint64_t* map, uint64_t m,
                         uint64_t cap, uint32_t D, hipStream_t s);

// ---- sharded search (gvdb_shard.hip, gvdb_comm.hip) -------------------------------
int index_device(const gvdb_index* ix);
struct ShardInfo {
    const float* rows;
    const float* norms;
    const uint64_t* ids;
    uint64_t n;
    uint32_t dim;
    int device;
};
ShardInfo index_shard_info(const gvdb_index* ix);
// a _device call read ix on stream s (mutations wait for it; gvdb_capi.hip)
void index_track_use(const gvdb_index* ix, hipStream_t s);
// this shard's exact stage-1 top-min(R, rows) as sorted keys (d << 32 | row) at
// keys[q*R + i] (gvdb_capi.hip); nothing for an empty shard
gvdb_status shard_stage1_keys(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, uint64_t R,
                              uint64_t* keys, hipStream_t s);
// Two-exchange block layouts (u32 words; even, so u64 fields stay aligned):
//   block 1 (rank -> all): keys u64 [B][R] | counts u32 [B] | err u32 | pad
//   block 2 (rank -> all): entries [B][k] x {cos bits, global stage-1 position,
//                          id lo, id hi} | meta u32 [B] (count | nan << 31) |
//                          reff u32 [B] | err u32 | pad
inline uint64_t shard_words1(uint64_t B, uint64_t R) { return (2 * B * R + B + 1 + 1) & ~1ull; }
inline uint64_t shard_words2(uint64_t B, uint64_t k) { return (4 * B * k + 2 * B + 1 + 1) & ~1ull; }
// gathered exchange-1 blocks -> this rank's exchange-2 block: global top-R, exact
// cosine of the owned rows, local top-k (one kernel per query; gvdb_shard.hip).
// rows / norms / ids may be null for a shard that owns nothing; opos / orow / ocos:
// [B][R] scratch (used when R exceeds the kernel's LDS arrays)
hipError_t launch_shard_phase2(const uint32_t* gathered1, uint64_t words1, uint32_t G, uint32_t me, uint32_t B,
                               uint32_t R, uint32_t D, const float* rows, const float* norms, const uint64_t* ids,
                               const float* queries, uint32_t k, uint32_t err, uint32_t* block2, uint32_t* opos,
                               uint32_t* orow, float* ocos, hipStream_t s);
// Deep two-exchange (R > kSelectLdsCap; gvdb_shard.hip):
//   block 1 deep: hist u32 [B][dim+1] (Hamming histogram of the local top-min(R, n)
//                 membership) | counts u32 [B] | err u32 | pad
//   scratch deep: member rows u32 [B][R] | member dist u32 [B][R] | owned rows u32 [B][R] |
//                 owned dist u32 [B][R] | cosines f32 [B][R] | own count u32 [B] | reff u32 [B] |
//                 certify word u32 (the certified phase 2's gate)
//                 (lists dense with stride Rl = min(R, n); phase 2 reads the members only)
inline bool shard_deep(uint64_t R) { return R > kSelectLdsCap; }
inline uint64_t shard_words1_deep(uint64_t B, uint32_t dim) { return (B * (dim + 1ull) + B + 1 + 1) & ~1ull; }
gvdb_status shard_stage1_members(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, uint64_t R,
                                 uint32_t* m_rows, uint32_t* m_dist, uint32_t* block1, hipStream_t s);
hipError_t launch_shard_member_hist(const uint32_t* m_dist, uint32_t B, uint32_t Rl, uint32_t H, uint32_t* block1,
                                    hipStream_t s);
hipError_t launch_shard_deep_own(const uint32_t* gathered1, uint64_t words1, uint32_t G, uint32_t me, uint32_t B,
                                 uint32_t R, uint32_t Rl, uint32_t H, const uint32_t* m_rows, const uint32_t* m_dist,
                                 uint32_t* o_rows, uint32_t* o_dist, uint32_t* own_cnt, uint32_t* reff,
                                 hipStream_t s, uint32_t* tcut = nullptr, const uint32_t* gate = nullptr);
// the certified deep phase 2 (gvdb_capi.hip): this rank's local top-k of its owned rows (rule tcut [B][4],
// counts own_cnt) from its exact cosine top-K2 list, into the exchange-2 block, with no host sync; *dfail
// (a device word that outlives the call) becomes non-zero when the batch is not certified: it gates the
// caller's rerank of the owned lists on the device.  *enqueued = false: not eligible, nothing enqueued
bool shard_certified_eligible(const gvdb_index* ix, uint32_t dim, uint64_t k);
// (dl: the dense-block form below -- the tied rows are counted from its segment histograms, not the lists)
struct ShardDenseLayout;
gvdb_status shard_certified_phase2(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, uint64_t k,
                                   const uint32_t* tcut, const uint32_t* own_cnt, const uint32_t* reff,
                                   const uint32_t* m_rows, const uint32_t* m_dist, uint32_t Rl, uint32_t* block2,
                                   uint32_t* dfail, void* early_list, hipStream_t s, bool* enqueued,
                                   const ShardDenseLayout* dl = nullptr);
// The deep form without member lists (round 5): when the shard's stage 1 is the dense FP4
// scan and its dense block fits the scratch's member-list regions, stage 1 keeps the block
// there ([B][np] f16 dots over m_rows | m_dist) and writes, in the m_cos region (words from
// m_cos): [4B, 8B) its own rule, [8B, 9B) |q|, [12B, ...) the segment histograms [B][S][dim+1]
// -- the exchange-1 histograms come from the same pass.  Phase 2 certifies from them and its
// fallback compacts the owned rows from the block (k_dense_own).  Both calls derive the
// layout from (shard, B, R, dim) alone.
struct ShardDenseLayout {
    uint32_t S = 0, L = 0, np = 0, n = 0;
    uint16_t* dense = nullptr;
    uint32_t* rule = nullptr;
    uint32_t* qpc = nullptr;
    uint32_t* seg = nullptr;
};
bool shard_dense_layout(const gvdb_index* ix, uint64_t B, uint64_t R, uint32_t dim, void* scratch,
                        ShardDenseLayout* dl);
// the certified phase 2's exact cosine list, enqueued EARLY by the stage-1 call on a second
// stream (concurrent with stage 1 and the exchange) into `list` (shard_early_list_bytes(B) bytes
// of the caller's scratch); phase 2 joins it by the list's address.  Not eligible: nothing.
size_t shard_early_list_bytes(uint64_t B);
gvdb_status shard_deep_flat_early(const gvdb_index* ix, const float* d_q, uint64_t B, uint32_t dim, void* list,
                                  hipStream_t s);
// gvdb_bigr.hip: the owned entries' local top-k (k <= 1024) -> the exchange-2 block
hipError_t launch_shard_deep_topk(const float* m_cos, const uint32_t* m_rows, const uint32_t* m_dist,
                                  const uint32_t* own_cnt, const uint32_t* reff, uint32_t B, uint32_t Rl, uint32_t k,
                                  const uint64_t* ids, uint32_t err, uint32_t* block2, hipStream_t s,
                                  const uint32_t* gate = nullptr);
// sharded FLAT: gathered blocks of the ranks' exact top-k -> merged top-k
//   block F (sharded FLAT): ids u64 [B][k] | scores f32 [B][k] | counts [B] | err | pad
inline uint64_t shard_words_flat(uint64_t B, uint64_t k) { return (3 * B * k + B + 1 + 1) & ~1ull; }
hipError_t launch_shard_flat_final(const uint32_t* gathered, uint64_t words, uint32_t G, uint32_t B, uint32_t k,
                                   int descending, uint64_t* out_ids, float* out_scores, uint32_t* out_n,
                                   hipStream_t s);
// gathered exchange-2 blocks -> top-k on every rank
hipError_t launch_shard_final(const uint32_t* gathered2, uint64_t words2, uint32_t G, uint32_t B, uint32_t k,
                              uint64_t* out_ids, float* out_scores, uint32_t* out_n, hipStream_t s);

// ---- error reporting shared by the C-ABI translation units ---------------------
// sets the thread-local gvdb_last_error() text and returns s
gvdb_status report_status(gvdb_status s, const std::string& msg);

}  // namespace gvdb
