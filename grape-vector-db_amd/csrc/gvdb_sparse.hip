// gvdb_sparse.hip — BM25 sparse search and reciprocal-rank fusion on gfx950.
//
// Replaces the CPU paths of (reference snapshot 2025-08-24, Rust):
//   * SparseIndex (src/sparse.rs:29-222): add_document 71-107,
//     remove_document 109-149, search_bm25 151-198, idf / bm25 200-222,
//     BM25Parameters k1 = 1.2, b = 0.75 (49-53);
//   * HybridSearchEngine::rrf_fusion (src/hybrid.rs:422-488).
//
// Layout in HBM.  The host keeps the authoritative document-major CSR over
// document SLOTS (slot = first add of a document id; a slot's entries sorted
// by (term, add order)), mirrored to the device as ptr / term / tf / dl.  From
// it the device builds, whenever the index changed, the term-major INVERTED
// index the reference searches (sparse.rs:167-190): per term one posting run
// of (slot u32, tf f32, dl f32) in SoA arrays, slots ascending (a re-added id's
// entries adjacent, in add order).  A stable radix sort of the entries by
// term gives exactly that order.
//
// Search = term-at-a-time, as the reference, over document CHUNKS of 128
// slots.  Per launch group (<= 64 queries, <= 512 distinct terms):
//   k_ta_dir     one pass over the group's posting runs records, per (chunk,
//                term), the first and last posting inside the chunk;
//   k_bm25_taat  per chunk: stage the chunk's postings of every group term in
//                LDS (tf_component evaluated once per posting), then round r
//                adds each query's r-th term into per-(query, slot) LDS
//                accumulators.  Query q's rounds all run in wave q % 8, so a
//                document's f32 sum folds its contributions in query-term
//                order and, per term, in posting order: the reference's
//                `*scores.entry(id).or_insert(0.0) += s`, bit for bit
//                (no FMA: -ffp-contract=off; idf from the host's logf, the
//                function Rust's f32::ln calls);
//   selection    a sample pass (every `every`-th chunk) gives, per query, a
//                lower bound tau of the limit-th best key (score, then slot
//                ascending); the emit pass keeps keys >= tau, an LDS sort
//                orders them.  Exact for every input: a query whose
//                candidates overflow the buffer is answered from a dense key
//                array + radix sort.
//
// Deterministic choices where the reference uses HashMap order (its results
// vary run to run there): equal scores order by slot; avgdl's f32 fold runs
// in slot order (each slot's entries in add order); NaN scores (possible only
// once remove_document left df > total_documents) sort last.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/gvdb.h"
#include "gvdb_device.h"
#include "gvdb_internal.h"

using namespace gvdb;

namespace {

constexpr uint32_t kTaCh = 64;                  // document slots per chunk: one per lane
constexpr uint32_t kTaThreads = 1024;           // one block per CU: 16 waves; wave w owns queries w, w + 16, ...
constexpr uint32_t kTaWaves = kTaThreads / 64;
constexpr uint32_t kTaQW = 4;                   // queries per wave
constexpr uint32_t kTaQ = kTaWaves * kTaQW;     // queries per launch group
constexpr uint32_t kTaStage = 4096;             // entries per chunk staged through registers (more: from HBM)
constexpr uint32_t kTaGrp = 8;                  // sample pass: one max key per 8 slots
constexpr uint32_t kTaCptrLds = 512;            // chunks per block (their ranges cached in LDS)
constexpr uint32_t kSpQT = 1024;                // query terms per launch group (LDS)
constexpr uint32_t kSpU = 511;                  // distinct terms per launch group (map row kSpU stays empty)
constexpr uint32_t kSpCand = 4096;              // candidates per query (LDS sort)
constexpr uint32_t kSpTopLocal = 2;             // per-thread keys kept by the tau pass
static_assert(kSpU < kTaThreads, "one thread per group term in the directory row");
static_assert(kTaCh == 64, "a chunk slot is a lane");

// total order of a BM25 score (NaN lowest: 0), then slot ascending
__device__ __forceinline__ uint64_t sp_key(float s, uint32_t slot) {
    const uint32_t o = s != s ? 0u : f32_order(s);
    return ((uint64_t)o << 32) | (uint32_t)(~slot);
}
__device__ __forceinline__ float sp_score(uint64_t key) {
    const uint32_t o = (uint32_t)(key >> 32);
    if (o == 0) return __builtin_nanf("");
    const uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    return __uint_as_float(u);
}
__device__ __forceinline__ uint32_t sp_slot(uint64_t key) { return ~(uint32_t)key; }

// ---------------------------------------------------------------------------
// Blocked inverted index: the entries of each 64-slot chunk sorted by (term,
// slot, add order) -- the inverted index restricted to the chunk's documents
// -- by one stable radix sort of (chunk, term) keys over the slot-ordered
// forward entries.  A chunk's entries stay the forward range
// [ptr[64c], ptr[64c + 64]).  Terms are stored as their rank in the index's
// sorted vocabulary (dense ids, same order), so a search group's terms are
// found through a direct-mapped table instead of a hash.
// ---------------------------------------------------------------------------
__global__ void k_blk_keys(const uint64_t* __restrict__ ptr, uint32_t N, const uint32_t* __restrict__ term,
                           uint64_t* __restrict__ keys, uint32_t* __restrict__ iota, uint32_t* __restrict__ eslot) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= N) return;
    for (uint64_t e = ptr[s], e1 = ptr[s + 1]; e < e1; ++e) {
        keys[e] = ((uint64_t)(s / kTaCh) << 32) | term[e];
        iota[e] = (uint32_t)e;
        eslot[e] = s;
    }
}

__global__ void k_blk_gather(const uint32_t* __restrict__ order, const uint64_t* __restrict__ keys,
                             const uint32_t* __restrict__ eslot, const float* __restrict__ tf,
                             const float* __restrict__ dl, uint64_t E, const uint32_t* __restrict__ vocab,
                             uint32_t V, uint32_t* __restrict__ cterm, uint8_t* __restrict__ cslot,
                             float* __restrict__ ctf, float* __restrict__ cdl, uint32_t* __restrict__ runs) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t e = order[i], s = eslot[e], t = (uint32_t)keys[i];
        uint32_t lo = 0, hi = V;  // lower_bound(vocab, t)
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (vocab[mid] < t) lo = mid + 1; else hi = mid;
        }
        if (lo >= V || vocab[lo] != t) *runs |= 2u;  // a term missing from the vocabulary
        cterm[i] = lo;
        cslot[i] = (uint8_t)(s % (2 * kTaCh));  // slot within the search's 128-document chunk
        ctf[i] = tf[e];
        cdl[i] = dl[e];
        if (i > 0 && keys[i] == keys[i - 1] && eslot[order[i - 1]] == s) *runs |= 1u;  // same term, same document
    }
}

// tf_component of every entry for the index's current avgdl (calculate_bm25_score,
// sparse.rs:215-218: (tf * (k1 + 1)) / (tf + k1 * (1 - b + b * (dl / avgdl))))
__global__ void k_blk_tfc(const float* __restrict__ ctf, const float* __restrict__ cdl, uint64_t E, float k1, float b,
                          float avgdl, float* __restrict__ ctfc) {
    const float k1p1 = k1 + 1.0f, omb = 1.0f - b;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < E; i += (uint64_t)gridDim.x * blockDim.x) {
        const float t = ctf[i];
        const float c = (t * k1p1) / (t + k1 * (omb + b * (cdl[i] / avgdl)));
        // +0.0 is kept as -0.0 (the search's map reads +0.0 as "no posting"): q_tf * c * idf is then
        // +-0.0 or the same NaN either way, and acc + +-0.0 == acc (acc never holds -0.0)
        ctfc[i] = __float_as_uint(c) == 0u ? -0.0f : c;
    }
}

// A search group's direct-mapped term table: gmap[dense term] = (epoch << 9) | group
// term index; entries of earlier epochs read as "not in the group".
constexpr uint32_t kGmapShift = 9;
// (and zeroes the group's candidate counters)
__global__ void k_gmap_set(uint32_t* __restrict__ gmap, const uint32_t* __restrict__ ut, uint32_t nu, uint32_t epoch,
                           uint32_t* __restrict__ counts, uint32_t B) {
    for (uint32_t i = threadIdx.x; i < nu; i += blockDim.x) gmap[ut[i]] = (epoch << kGmapShift) | i;
    for (uint32_t i = threadIdx.x; i < B; i += blockDim.x) counts[i] = 0u;
}

struct TaArgs {
    const uint64_t* cptr;   // [nchunks+1] entry range of each blocked-index chunk (= forward ptr every 64 slots)
    const uint32_t* cterm;  // blocked entries: term, slot within the chunk, tf_component
    const uint8_t* cslot;
    const float* ctfc;
    uint32_t N;             // slots
    uint32_t nchunks;       // blocked-index (64-slot) chunks
    uint64_t n_entries;     // > 0
    const uint32_t* ut;     // [nu] the group's distinct live terms (dense ids, sorted)
    uint32_t nu;
    const uint32_t* gmap;   // [vocabulary] (epoch << 9) | group term index
    uint32_t epoch;
    const uint64_t* qmask;  // [nu] the group's queries (bit = index in the group) holding each term
    uint64_t qsel;          // queries with a non-finite q_tf or idf (bit = index in the group)
    const uint32_t* qp;     // [B+1] offsets into qrec
    const uint32_t* perm;   // [B] query of each wave slot (w + 16 m)
    const uint4* qrec;      // [nqt+4] per query term: (group term, q_tf bits, idf bits, map row bytes), each
                            // query's padded with empty records (empty row, 0, 0) to a multiple of 4; [nqt, nqt+4) empty
    uint32_t nqt;
    uint32_t B;
    uint32_t every;         // sample pass: chunk stride
    uint64_t* smp;          // sample: [B][S] keys (0 = unmatched)
    uint32_t S;
    const uint64_t* tau;    // emit: [B]
    uint32_t* counts;       // emit: [B]
    uint64_t* cand;         // emit: [B][kSpCand]
    uint64_t* dense;        // dense mode: [N] keys of query `dense_q`
    uint32_t dense_q;
    uint32_t runs;          // the index holds a (term, document) run longer than one entry (a re-added id)
    uint32_t abl;           // timing probe only (GVDB_BM25_ABL): 1 skip rounds (results invalid), 8 phase clocks
    uint64_t* prof;         // [gridDim][8] cycles per phase (wave 0), with abl & 8
};

// MODE 0: sample (every `every`-th chunk -> per 8 slots the max key -> smp),
// 1: emit (key >= tau -> cand), 2: dense keys of query `dense_q`.
//
// One block per CU walks a contiguous range of chunks of 128 documents (two
// blocked-index chunks; lane = 2 slots).  Per chunk:
//   1. its blocked entries (all terms, ~30 per document) stream in; the
//      group's direct-mapped term table (gmap, read a chunk ahead) keeps those
//      of the batch: their tf_components are compacted into an LDS stage
//      (per wave: ballot + one counter add) and an LDS (group term x slot) map
//      of u16 stage offsets (0 = no posting; the first entry of a re-added
//      document's run) points at them -- 512 rows x 128 slots in 128 KB, so
//      one group holds up to 511 distinct terms.  (Which documents each query
//      matches comes from the rounds' own map reads: no per-posting LDS hit mask
//      -- round 6: the 64-bit LDS atomic OR per posting was ~2 of the build's 5
//      LDS operations);
//   2. rounds: wave w owns 4 queries (host-balanced), accumulators in
//      registers.  Query q's terms in order: a map read, two stage reads,
//      acc = acc + q_tf * tfc * idf -- per document exactly the reference's
//      fold (sparse.rs:167-190; acc starts at 0.0 = or_insert).  No posting
//      reads stage[0] = +0.0 (the index keeps a posting's +0.0 tfc as -0.0):
//      when q_tf and idf are finite its product is +-0.0 and acc + +-0.0 ==
//      acc (acc never holds -0.0), so the fold needs no select; queries with a
//      non-finite q_tf or idf (host flag) select per term.  A run of several
//      entries (rare: the index records whether any exists) or a stage
//      overflow is folded from HBM in order;
//   3. selection by the mode.
// Software pipeline: a chunk's entries are loaded three chunks ahead, their
// group words two chunks ahead; emitted candidates pool in LDS.
constexpr uint32_t kTaSpl = 2;              // slots per lane
constexpr uint32_t kTaRows = 512;           // map rows: group terms + the empty row
constexpr uint32_t kTaStaged = 4096;        // staged tf_components per chunk (index 0: +0.0)
constexpr uint16_t kTaUnstaged = 0xffffu;   // a posting past the stage (odd: never a stage offset)
constexpr uint32_t kTaPool = 448;           // emit: candidates pooled in LDS per block (more: direct)
static_assert(kSpU < kTaRows, "the empty row");
static_assert(kTaStaged * 4 <= 0xffffu, "u16 byte offsets");
template <int MODE>
__global__ __launch_bounds__(kTaThreads, 1) void k_bm25_taat(TaArgs a) {
    constexpr uint32_t SPL = kTaSpl, kCh = kTaCh * SPL, kRows = kTaRows, kEmpty = kRows - 1;
    __shared__ __attribute__((aligned(16))) uint16_t s_tmap[kRows * kCh];  // stage byte offset per (term, slot)
    __shared__ __attribute__((aligned(16))) float s_tfc[kTaStaged];
    __shared__ __attribute__((aligned(4))) uint8_t s_present[kRows];  // group terms with a posting in the chunk
    __shared__ uint32_t s_cptr[(SPL + 1) * (kTaCptrLds + 1)];  // the block's chunk (sub-)ranges, from cbase
    __shared__ uint32_t s_slow, s_nst, s_npool;
    __shared__ uint64_t s_pkey[kTaPool];  // emit: the block's candidates (key, query), flushed at the end
    __shared__ uint8_t s_pq[kTaPool];
    typedef const uint32_t __attribute__((address_space(4)))* cu32;
    const cu32 qp = (cu32)(uintptr_t)a.qp;  // read-only query tables: scalar loads
    const cu32 qr32 = (cu32)(uintptr_t)a.qrec;
    auto qrec_at = [&](uint32_t p) {
        return make_uint4(qr32[4 * p], qr32[4 * p + 1], qr32[4 * p + 2], qr32[4 * p + 3]);
    };
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t nu = a.nu;  // < kRows (host)
    for (uint32_t i = tid; i < kRows * kCh / 2; i += kTaThreads) ((uint32_t*)s_tmap)[i] = 0u;
    if (tid == 0) {
        s_tfc[0] = 0.0f;
        s_npool = 0;
    }
    auto tfc_at = [&](uint32_t off) { return *(const float*)((const char*)s_tfc + off); };
    // group term index of a gmap word, kEmpty for a term outside the group
    auto group_of = [&](uint32_t gv) { return (gv >> kGmapShift) == a.epoch ? gv & ((1u << kGmapShift) - 1) : kEmpty; };
    // this wave's queries (uniform): wave slot w + 16 m holds query perm[w + 16 m]
    // (the host balances the slots' total terms across waves)
    const cu32 perm = (cu32)(uintptr_t)a.perm;
    uint32_t qid[kTaQW], qp0[kTaQW], ql[kTaQW], rmax = 0;
#pragma unroll
    for (uint32_t m = 0; m < kTaQW; ++m) {
        qid[m] = perm[wave + kTaWaves * m];  // 0xffffffff: an empty slot
        const bool live = qid[m] != 0xffffffffu && (MODE != 2 || qid[m] == a.dense_q);
        qp0[m] = live ? qp[qid[m]] : 0u;
        ql[m] = live ? qp[qid[m] + 1] - qp0[m] : 0u;
        rmax = max(rmax, ql[m]);
    }
    bool wave_sel = false;  // a query of the wave has a non-finite q_tf or idf: select per term
#pragma unroll
    for (uint32_t m = 0; m < kTaQW; ++m) wave_sel |= qid[m] != 0xffffffffu && ((a.qsel >> qid[m]) & 1ull);
    uint64_t tau[kTaQW];
#pragma unroll
    for (uint32_t m = 0; m < kTaQW; ++m) tau[m] = MODE == 1 && qid[m] != 0xffffffffu ? a.tau[qid[m]] : 0ull;
    // the wave's query terms, lane-resident: lane 16 m + r holds query m's r-th (padded) term
    // record: map row bytes, q_tf, idf (the empty record past the query's end)
    uint32_t lr_row, lr_v, lr_idf, lr_g;
    {
        const uint32_t m = lane >> 4, r = lane & 15u;
        const uint4 rec = qrec_at(r < ql[m & 3] ? qp0[m & 3] + r : a.nqt);
        lr_row = rec.w;
        lr_g = rec.x;
        lr_v = rec.y;
        lr_idf = rec.z;
    }
    // emit: a score below tau's cannot pass (acc is never -0.0; a NaN tau score passes every hit)
    float thr[kTaQW];
    bool loose[kTaQW];
#pragma unroll
    for (uint32_t m = 0; m < kTaQW; ++m) {
        loose[m] = (tau[m] >> 32) == 0;
        thr[m] = loose[m] ? 0.0f : sp_score(tau[m]);
    }
    const uint32_t every = MODE == 0 ? a.every : 1u;
    const uint32_t nchunks = (a.nchunks + SPL - 1) / SPL;  // in chunks of kCh slots
    const uint32_t nj = (nchunks + every - 1) / every;
    // contiguous chunk range per block (the host sizes the grid: je - jb <= kTaCptrLds)
    const uint32_t jb = (uint32_t)((uint64_t)nj * blockIdx.x / gridDim.x);
    const uint32_t je = (uint32_t)((uint64_t)nj * (blockIdx.x + 1) / gridDim.x);
    const uint64_t cbase = a.cptr[min((uint64_t)jb * every * SPL, (uint64_t)a.nchunks)];
    for (uint32_t i = tid; i < je - jb; i += kTaThreads) {
        const uint64_t c = (uint64_t)(jb + i) * every * SPL;  // in blocked-index chunks
#pragma unroll
        for (uint32_t h = 0; h <= SPL; ++h)
            s_cptr[(SPL + 1) * i + h] = (uint32_t)(a.cptr[min(c + h, (uint64_t)a.nchunks)] - cbase);
    }
    __syncthreads();
    uint64_t ph[5] = {0, 0, 0, 0, 0}, tprev = 0;
    auto mark = [&](int k) {
        if (a.abl & 8) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            if (k >= 0) ph[k] += t - tprev;
            tprev = t;
        }
    };
    // ---- a chunk's entries through registers, three chunks ahead (triple buffer)
    constexpr uint32_t kPer = kTaStage / kTaThreads;
    struct Stage {
        uint32_t t[kPer], s[kPer];  // dense term, slot within the blocked-index chunk
        float f[kPer];              // tf_component
        uint32_t g[kPer];           // gmap word of the term (loaded a chunk ahead of the build)
    };
    Stage st0, st1, st2;
    uint32_t cell[kPer];  // map cells this thread wrote for the current chunk (unwritten after its rounds)
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) cell[k] = 0xffffffffu;
    const uint64_t last = a.n_entries - 1;
    auto load_entries = [&](Stage& sg, uint32_t jx) {
        // unconditional loads (an index past the range reads a valid entry that the
        // build skips): no use and no register write before the chunk's turn
        const uint64_t e0 = jx < je ? cbase + s_cptr[(SPL + 1) * (jx - jb)] : 0ull;
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) sg.t[k] = a.cterm[min(e0 + tid + k * kTaThreads, last)];
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint64_t i = min(e0 + tid + k * kTaThreads, last);
            sg.s[k] = a.cslot[i];
            sg.f[k] = a.ctfc[i];
        }
    };
    // the group table words of a stage's terms, two chunks before its build
    auto lookup = [&](Stage& sg) {
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) sg.g[k] = a.gmap[sg.t[k]];
    };
    bool prev_overflow = false;
    auto chunk = [&](Stage& sg, Stage& nx2, uint32_t jj) {
        const uint32_t c0 = jj * every * kCh;
        const uint32_t* cr = &s_cptr[(SPL + 1) * (jj - jb)];
        const uint64_t ce0 = cbase + cr[0], ce1 = cbase + cr[SPL];
        const uint32_t cn = cr[SPL] - cr[0];  // the chunk's entries
        __syncthreads();  // (1) the previous chunk's rounds are done
        mark(-1);
        if (prev_overflow) {  // cells written past the register stage are not tracked: clear the rows
            for (uint32_t i = tid; i < nu * kCh / 2; i += kTaThreads) ((uint32_t*)s_tmap)[i] = 0u;
        } else {
#pragma unroll
            for (uint32_t k = 0; k < kPer; ++k)
                if (cell[k] != 0xffffffffu) s_tmap[cell[k]] = 0;
        }
        if (tid < kRows / 4) ((uint32_t*)s_present)[tid] = 0u;
        if (tid == 0) {
            s_slow = 0;
            s_nst = 1;
        }
        __syncthreads();  // (2) the map is clean
        mark(0);
        {
            bool slow = false;
            bool take[kPer];
            uint32_t gk[kPer], pre[kPer], tot = 0;
            uint64_t bal[kPer];
#pragma unroll
            for (uint32_t k = 0; k < kPer; ++k) {
                const uint64_t i = ce0 + tid + k * kTaThreads;
                gk[k] = group_of(sg.g[k]);
                take[k] = tid + k * kTaThreads < cn && gk[k] != kEmpty;
                if (take[k] && a.runs) {  // a re-added document: only the first entry of its run enters the map
                    if (i + 1 < ce1 && a.cterm[i + 1] == sg.t[k] && a.cslot[i + 1] == sg.s[k]) slow = true;
                    if (i > ce0 && a.cterm[i - 1] == sg.t[k] && a.cslot[i - 1] == sg.s[k]) take[k] = false;
                }
                bal[k] = __ballot(take[k]);
                pre[k] = tot;
                tot += (uint32_t)__popcll(bal[k]);
            }
            // stage positions: the wave's takers in (k, lane) order after one counter add
            uint32_t base = 0;
            if (lane == 0 && tot) base = atomicAdd(&s_nst, tot);
            base = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
            for (uint32_t k = 0; k < kPer; ++k) {
                cell[k] = 0xffffffffu;
                if (!take[k]) continue;
                const uint32_t g = gk[k];
                const uint32_t pos = base + pre[k] +
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u));
                const uint32_t sl = sg.s[k];
                cell[k] = g * kCh + sl;
                if (pos < kTaStaged) {
                    s_tfc[pos] = sg.f[k];
                    s_tmap[cell[k]] = (uint16_t)(pos * 4);
                } else {
                    s_tmap[cell[k]] = kTaUnstaged;
                    slow = true;
                }
                s_present[g] = 1;
            }
            for (uint64_t i = ce0 + kTaStage + tid; i < ce1; i += kTaThreads) {  // past the register stage
                const uint32_t g = group_of(a.gmap[a.cterm[i]]);
                if (g == kEmpty) continue;
                const uint32_t s = a.cslot[i];
                if (i > ce0 && a.cterm[i - 1] == a.cterm[i] && a.cslot[i - 1] == s) {
                    slow = true;
                    continue;
                }
                const uint32_t sl = s;
                const uint32_t pos = atomicAdd(&s_nst, 1u);
                if (pos < kTaStaged) {
                    s_tfc[pos] = a.ctfc[i];
                    s_tmap[g * kCh + sl] = (uint16_t)(pos * 4);
                } else {
                    s_tmap[g * kCh + sl] = kTaUnstaged;
                    slow = true;
                }
                s_present[g] = 1;
                slow = slow || (i + 1 < ce1 && a.cterm[i + 1] == a.cterm[i] && a.cslot[i + 1] == s);
            }
            if (slow) s_slow = 1u;
        }
        __syncthreads();  // (3) the chunk's map is built
        mark(1);
        prev_overflow = cn > kTaStage;
        load_entries(sg, jj + 3);  // in flight during the next two chunks
        mark(4);
        // 2. rounds, per query m in its term order; lane holds slots SPL*lane + h
        float acc[kTaQW][SPL];
        // the documents each query matches (a posting of one of its terms: the reference's
        // scores.entry(id)), from the map reads themselves -- OR of the 16-bit offsets per
        // (query, slot half); no LDS hit mask built per posting
        uint32_t orv[kTaQW];
#pragma unroll
        for (uint32_t m = 0; m < kTaQW; ++m) {
            orv[m] = 0u;
#pragma unroll
            for (uint32_t h = 0; h < SPL; ++h) acc[m][h] = 0.0f;
        }
        // Only the query terms with a posting in the chunk (a term without one adds +-0.0, or is
        // skipped by the select: either way acc is unchanged), in term order, N <= 4 at a time:
        // the map reads issued together, then the stage reads, then the folds in order.
        // calculate_bm25_score: query_tf * tf_component * idf; `or_insert(0.0) += s`
        auto fast_rounds = [&](auto sel_c) {
            constexpr bool kSel = decltype(sel_c)::value;
            const uint64_t pm = __ballot(s_present[lr_g] != 0);  // lane 16 m + r: query m's term r
            auto batch = [&](auto n_c, uint32_t m, uint32_t& bits) {
                constexpr uint32_t N = decltype(n_c)::value;
                uint32_t ln[N], off[N];
#pragma unroll
                for (uint32_t k = 0; k < N; ++k) {
                    const uint32_t b = (uint32_t)__builtin_ctz(bits);
                    bits &= bits - 1;
                    ln[k] = __builtin_amdgcn_readfirstlane(m * 16 + b);
                    const uint32_t rowb = __builtin_amdgcn_readlane(lr_row, ln[k]);
                    off[k] = *(const uint32_t*)((const char*)s_tmap + rowb + 4 * lane);
                }
                float tf[N][SPL];
#pragma unroll
                for (uint32_t k = 0; k < N; ++k) {
                    tf[k][0] = tfc_at(off[k] & 0xffffu);
                    tf[k][1] = tfc_at(off[k] >> 16);
                    orv[m] |= off[k];
                }
#pragma unroll
                for (uint32_t k = 0; k < N; ++k) {
                    const float v = __uint_as_float(__builtin_amdgcn_readlane(lr_v, ln[k]));
                    const float idf = __uint_as_float(__builtin_amdgcn_readlane(lr_idf, ln[k]));
#pragma unroll
                    for (uint32_t h = 0; h < SPL; ++h) {
                        const float sc = v * tf[k][h] * idf;
                        if constexpr (kSel)
                            acc[m][h] = acc[m][h] + (((off[k] >> (16 * h)) & 0xffffu) != 0u ? sc : 0.0f);
                        else
                            acc[m][h] = acc[m][h] + sc;  // no posting in this slot: +-0.0
                    }
                }
            };
#pragma unroll
            for (uint32_t m = 0; m < kTaQW; ++m) {
                uint32_t bits = __builtin_amdgcn_readfirstlane((uint32_t)(pm >> (16 * m)) & 0xffffu);
                while (__builtin_popcount(bits) >= 4) batch(std::integral_constant<uint32_t, 4>{}, m, bits);
                const uint32_t rest = __builtin_popcount(bits);
                if (rest == 3) batch(std::integral_constant<uint32_t, 3>{}, m, bits);
                else if (rest == 2) batch(std::integral_constant<uint32_t, 2>{}, m, bits);
                else if (rest == 1) batch(std::integral_constant<uint32_t, 1>{}, m, bits);
            }
        };
        if (a.abl & 1) {
        } else if (!s_slow && rmax <= 16) {
            if (wave_sel) fast_rounds(std::true_type{});
            else fast_rounds(std::false_type{});
        } else {
            // a re-added document's run (every entry of (term, document) in order, from HBM), a stage
            // overflow, or a query with more than 16 live terms
#pragma unroll
            for (uint32_t m = 0; m < kTaQW; ++m) {
                for (uint32_t r = 0; r < ql[m]; ++r) {
                    const uint4 rec = qrec_at(qp0[m] + r);
                    const float v = __uint_as_float(rec.y), idf = __uint_as_float(rec.z);
#pragma unroll
                    for (uint32_t h = 0; h < SPL; ++h) {
                        const uint32_t sl = SPL * lane + h;  // slot within the chunk
                        const uint32_t off = s_tmap[rec.x * kCh + sl];
                        if (off == 0u) continue;  // no posting
                        orv[m] |= 1u << (16 * h);
                        if (!s_slow) {
                            acc[m][h] = acc[m][h] + v * tfc_at(off) * idf;
                            continue;
                        }
                        // the sub-chunk's entries are sorted by (term, slot): lower_bound((term, slot))
                        const uint32_t term = a.ut[rec.x], sub = sl / kTaCh, ss = sl;
                        const uint64_t r0 = cbase + cr[sub], r1 = cbase + cr[sub + 1];
                        uint64_t lo = r0, hi = r1;
                        while (lo < hi) {
                            const uint64_t mid = (lo + hi) >> 1;
                            const uint32_t mt = a.cterm[mid];
                            if (mt < term || (mt == term && a.cslot[mid] < ss)) lo = mid + 1; else hi = mid;
                        }
                        for (uint64_t i = lo; i < r1 && a.cterm[i] == term && a.cslot[i] == ss; ++i)
                            acc[m][h] = acc[m][h] + v * a.ctfc[i] * idf;
                    }
                }
            }
        }
        mark(2);
        // 3. selection: (query qid[m], slot c0 + SPL lane + h)
#pragma unroll
        for (uint32_t m = 0; m < kTaQW; ++m) {
            const uint32_t q = qid[m];
            if (q == 0xffffffffu) continue;
            bool hb[SPL];
#pragma unroll
            for (uint32_t h = 0; h < SPL; ++h) hb[h] = ((orv[m] >> (16 * h)) & 0xffffu) != 0u;
            if constexpr (MODE == 1) {
                bool pass[SPL], any = false;
#pragma unroll
                for (uint32_t h = 0; h < SPL; ++h) {
                    pass[h] = hb[h] && (loose[m] || acc[m][h] >= thr[m]);
                    any |= pass[h];
                }
                if (__ballot(any) == 0ull) continue;  // usual: no document of the chunk reaches tau
#pragma unroll
                for (uint32_t h = 0; h < SPL; ++h) {
                    const uint64_t key = pass[h] ? sp_key(acc[m][h], c0 + SPL * lane + h) : 0ull;
                    if (key != 0ull && key >= tau[m]) {
                        const uint32_t pp = atomicAdd(&s_npool, 1u);
                        if (pp < kTaPool) {
                            s_pkey[pp] = key;
                            s_pq[pp] = (uint8_t)q;
                        } else {
                            const uint32_t pos = atomicAdd(&a.counts[q], 1u);
                            if (pos < kSpCand) a.cand[(uint64_t)q * kSpCand + pos] = key;
                        }
                    }
                }
                continue;
            }
            uint64_t key[SPL];
#pragma unroll
            for (uint32_t h = 0; h < SPL; ++h) key[h] = hb[h] ? sp_key(acc[m][h], c0 + SPL * lane + h) : 0ull;
            if constexpr (MODE == 0) {
                uint64_t best = key[0];
#pragma unroll
                for (uint32_t h = 1; h < SPL; ++h) best = max(best, key[h]);
                constexpr uint32_t kLanes = kTaGrp / SPL;  // lanes per group of 8 slots
#pragma unroll
                for (uint32_t o = 1; o < kLanes; o <<= 1) {
                    const uint32_t lo32 = __shfl_xor((uint32_t)best, o), hi32 = __shfl_xor((uint32_t)(best >> 32), o);
                    best = max(best, ((uint64_t)hi32 << 32) | lo32);
                }
                if ((lane & (kLanes - 1)) == 0)
                    a.smp[(uint64_t)q * a.S + (uint64_t)jj * (kCh / kTaGrp) + lane / kLanes] = best;
            } else {
#pragma unroll
                for (uint32_t h = 0; h < SPL; ++h) {
                    const uint32_t slot = c0 + SPL * lane + h;
                    if (q == a.dense_q && slot < a.N) a.dense[slot] = key[h];
                }
            }
        }
        mark(3);
        lookup(nx2);  // the group words of chunk jj + 2 (its entries were issued a chunk ago)
    };
    load_entries(st0, jb);
    load_entries(st1, jb + 1);
    load_entries(st2, jb + 2);
    lookup(st0);
    lookup(st1);
    for (uint32_t jj = jb; jj < je; jj += 3) {
        chunk(st0, st2, jj);
        if (jj + 1 < je) chunk(st1, st0, jj + 1);
        if (jj + 2 < je) chunk(st2, st1, jj + 2);
    }
    if constexpr (MODE == 1) {  // the pooled candidates
        __syncthreads();
        const uint32_t n = min(s_npool, kTaPool);
        for (uint32_t i = tid; i < n; i += kTaThreads) {
            const uint32_t q = s_pq[i];
            const uint32_t pos = atomicAdd(&a.counts[q], 1u);
            if (pos < kSpCand) a.cand[(uint64_t)q * kSpCand + pos] = s_pkey[i];
        }
    }
    if ((a.abl & 8) && tid == 0)
        for (int k = 0; k < 5; ++k) a.prof[blockIdx.x * 8 + k] = ph[k];
}

// tau[q] = the kk-th largest sampled key (0 when fewer than kk matched): each
// of 1024 threads keeps its top kSpTopLocal keys, an LDS sort of all of them
// follows.  Any kk keys it keeps are real documents, so tau never exceeds the
// true kk-th best key; dropped keys only lower it (more candidates, still exact).
constexpr uint32_t kTauThreads = 1024;
__global__ __launch_bounds__(kTauThreads) void k_bm25_tau(const uint64_t* __restrict__ smp, uint32_t S, uint32_t kk,
                                                          uint64_t* __restrict__ tau) {
    __shared__ uint64_t keys[kTauThreads * kSpTopLocal];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    uint64_t top[kSpTopLocal];
#pragma unroll
    for (uint32_t i = 0; i < kSpTopLocal; ++i) top[i] = 0;
    const uint64_t* src = smp + (uint64_t)q * S;
    constexpr uint32_t kIn = 8;  // loads in flight per thread
    for (uint32_t i0 = tid; i0 < S; i0 += kTauThreads * kIn) {
        uint64_t kv[kIn];
#pragma unroll
        for (uint32_t u = 0; u < kIn; ++u) kv[u] = i0 + u * kTauThreads < S ? src[i0 + u * kTauThreads] : 0ull;
#pragma unroll
        for (uint32_t u = 0; u < kIn; ++u) {
            uint64_t k = kv[u];
#pragma unroll
            for (uint32_t j = 0; j < kSpTopLocal; ++j) {
                const uint64_t hi = k > top[j] ? k : top[j], lo = k > top[j] ? top[j] : k;
                top[j] = hi;
                k = lo;
            }
        }
    }
#pragma unroll
    for (uint32_t i = 0; i < kSpTopLocal; ++i) keys[tid * kSpTopLocal + i] = ~top[i];
    __syncthreads();
    bitonic_sort_lds(keys, kTauThreads * kSpTopLocal);
    if (tid == 0) tau[q] = kk >= 1 && kk <= kTauThreads * kSpTopLocal ? ~keys[kk - 1] : 0ull;
}

// Per query: sort the candidates (descending key) and emit the first `limit`.
__global__ __launch_bounds__(256) void k_bm25_final(const uint64_t* __restrict__ cand, const uint32_t* __restrict__ counts,
                                                    uint32_t limit, const uint64_t* __restrict__ slot_ids,
                                                    uint64_t* __restrict__ out_ids, float* __restrict__ out_scores,
                                                    uint32_t* __restrict__ out_n, uint32_t* __restrict__ fail) {
    __shared__ uint64_t keys[kSpCand];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const uint32_t c = counts[q];
    if (c > kSpCand) {
        if (tid == 0) {
            fail[q] = 1u;
            out_n[q] = 0;
        }
        return;
    }
    const uint32_t P = next_pow2(c < 2u ? 2u : c);
    for (uint32_t i = tid; i < P; i += 256u) keys[i] = i < c ? ~cand[(uint64_t)q * kSpCand + i] : ~0ull;
    __syncthreads();
    bitonic_sort_lds(keys, P);
    const uint32_t n = min(limit, c);
    for (uint32_t i = tid; i < n; i += 256u) {
        const uint64_t k = ~keys[i];
        out_ids[(uint64_t)q * limit + i] = slot_ids[sp_slot(k)];
        out_scores[(uint64_t)q * limit + i] = sp_score(k);
    }
    if (tid == 0) {
        out_n[q] = n;
        fail[q] = 0u;
    }
}

// dense fallback: the first `limit` nonzero keys of a descending-sorted array
__global__ void k_bm25_emit_dense(const uint64_t* __restrict__ sorted, uint32_t N, uint32_t limit,
                                  const uint64_t* __restrict__ slot_ids, uint64_t* __restrict__ out_ids,
                                  float* __restrict__ out_scores, uint32_t* __restrict__ out_n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < limit && i < N && sorted[i] != 0) {
        out_ids[i] = slot_ids[sp_slot(sorted[i])];
        out_scores[i] = sp_score(sorted[i]);
    }
    if (i == 0) {  // nonzero keys form a prefix
        uint32_t lo = 0, hi = min(limit, N);
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sorted[mid] != 0) lo = mid + 1; else hi = mid;
        }
        *out_n = lo;
    }
}

// ---------------------------------------------------------------------------
// RRF (hybrid.rs:422-488), one block per query.  Items = the three lists
// concatenated (dense, sparse, text).  An LDS sort of (id, item index) makes
// every id's occurrences one run in list order; the run's first item owns the
// document: score = the LAST dense occurrence's 1/(k + rank + 1) (HashMap::
// insert replaces) or else the first other occurrence's, then += every later
// sparse / text occurrence in order; ties by first appearance.
// ---------------------------------------------------------------------------
constexpr uint32_t kRrfMax = 4096;  // items per query (dynamic LDS: 24 B per item)

__device__ void bitonic_pairs_lds(uint64_t* id, uint16_t* ix, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t p = threadIdx.x; p < P / 2; p += blockDim.x) {
                const uint32_t lo = ((p & ~(j - 1)) << 1) | (p & (j - 1));
                const uint32_t hi = lo | j;
                const uint64_t a = id[lo], b = id[hi];
                const uint16_t ia = ix[lo], ib = ix[hi];
                const bool gt = a > b || (a == b && ia > ib);
                if (gt == ((lo & k) == 0)) {
                    id[lo] = b;
                    id[hi] = a;
                    ix[lo] = ib;
                    ix[hi] = ia;
                }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(256) void k_rrf(const uint64_t* __restrict__ ids0, const float* __restrict__ sc0,
                                             const uint32_t* __restrict__ n0, uint32_t st0,
                                             const uint64_t* __restrict__ ids1, const float* __restrict__ sc1,
                                             const uint32_t* __restrict__ n1, uint32_t st1,
                                             const uint64_t* __restrict__ ids2, const float* __restrict__ sc2,
                                             const uint32_t* __restrict__ n2, uint32_t st2, float k, uint32_t limit,
                                             uint32_t pmax, uint64_t* __restrict__ out_ids,
                                             float* __restrict__ out_scores, float* __restrict__ out_raw,
                                             uint32_t* __restrict__ out_n) {
    extern __shared__ __attribute__((aligned(16))) uint64_t rrf_lds[];
    uint64_t* s_id = rrf_lds;                     // [pmax] item ids, sorted with their item index
    uint64_t* s_key = s_id + pmax;                // [pmax] (score desc, owner item) per document
    float* s_sc = (float*)(s_key + pmax);         // [pmax] fused score, at the owner item
    uint16_t* s_ix = (uint16_t*)(s_sc + pmax);    // [pmax] item index of s_id
    uint16_t* s_run = s_ix + pmax;                // [pmax] owner item -> its run in s_id
    __shared__ uint32_t s_cnt;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const uint32_t a = n0 ? min(n0[q], st0) : 0u, b = n1 ? min(n1[q], st1) : 0u, c = n2 ? min(n2[q], st2) : 0u;
    const uint32_t n = a + b + c;  // <= pmax (host: sum of strides)
    auto list_of = [&](uint32_t i) { return i < a ? 0u : i < a + b ? 1u : 2u; };
    auto rank_of = [&](uint32_t i) { return i < a ? i : i < a + b ? i - a : i - a - b; };
    auto raw_of = [&](uint32_t i) {
        const uint32_t l = list_of(i), r = rank_of(i);
        return l == 0 ? sc0[(uint64_t)q * st0 + r] : l == 1 ? sc1[(uint64_t)q * st1 + r] : sc2[(uint64_t)q * st2 + r];
    };
    auto rrf = [&](uint32_t i) { return 1.0f / (k + (float)(rank_of(i) + 1u)); };  // 1.0 / (k + (rank + 1) as f32)
    const uint32_t P = next_pow2(n < 2u ? 2u : n);
    for (uint32_t i = tid; i < P; i += 256u) {
        uint64_t id = ~0ull;
        if (i < n) {
            const uint32_t l = list_of(i), r = rank_of(i);
            id = l == 0 ? ids0[(uint64_t)q * st0 + r] : l == 1 ? ids1[(uint64_t)q * st1 + r] : ids2[(uint64_t)q * st2 + r];
        }
        s_id[i] = id;
        s_ix[i] = i < n ? (uint16_t)i : (uint16_t)0xffffu;
    }
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    bitonic_pairs_lds(s_id, s_ix, P);
    for (uint32_t p = tid; p < n; p += 256u) {
        const uint64_t id = s_id[p];
        if (p > 0 && s_id[p - 1] == id) continue;  // not the first occurrence
        uint32_t t = p;
        int32_t last_dense = -1;  // dense: HashMap::insert replaces (hybrid.rs:432-445)
        for (; t < n && s_id[t] == id && s_ix[t] < a; ++t) last_dense = s_ix[t];
        float score = 0.0f;
        bool have = false;
        if (last_dense >= 0) {
            score = rrf((uint32_t)last_dense);
            have = true;
        }
        for (; t < n && s_id[t] == id; ++t) {  // sparse, then text: insert or += (447-478)
            const float r = rrf(s_ix[t]);
            score = have ? score + r : r;
            have = true;
        }
        const uint32_t owner = s_ix[p];
        s_run[owner] = (uint16_t)p;
        s_sc[owner] = score;
        const uint32_t pos = atomicAdd(&s_cnt, 1u);
        s_key[pos] = ((uint64_t)(~f32_order(score)) << 32) | owner;  // score desc, first appearance asc
    }
    __syncthreads();
    const uint32_t m = s_cnt;
    const uint32_t P2 = next_pow2(m < 2u ? 2u : m);
    for (uint32_t i = m + tid; i < P2; i += 256u) s_key[i] = ~0ull;
    __syncthreads();
    bitonic_sort_lds(s_key, P2);
    const uint32_t take = min(limit, m);
    for (uint32_t t = tid; t < take; t += 256u) {
        const uint32_t owner = (uint32_t)s_key[t];
        const uint32_t p = s_run[owner];
        const uint64_t o = (uint64_t)q * limit + t;
        const uint64_t id = s_id[p];
        out_ids[o] = id;
        out_scores[o] = s_sc[owner];
        if (out_raw) {  // ScoreBreakdown: the last occurrence per list
            float bd[3] = {__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
            for (uint32_t u = p; u < n && s_id[u] == id; ++u) bd[list_of(s_ix[u])] = raw_of(s_ix[u]);
            for (int l = 0; l < 3; ++l) out_raw[o * 3 + l] = bd[l];
        }
    }
    if (tid == 0) out_n[q] = take;
}

}  // namespace

// ============================================================================
// host object
// ============================================================================
struct gvdb_sparse {
    int device = 0;
    float k1 = 1.2f, b = 0.75f;
    std::mutex mu;  // mutations are exclusive (caller's RwLock); searches serialize on the stream
    // host state (authoritative)
    std::unordered_map<uint64_t, uint32_t> slot_of;
    std::vector<uint64_t> slot_id;
    std::vector<uint64_t> ptr{0};
    std::vector<uint32_t> term;
    std::vector<float> tf, dl;
    std::unordered_map<uint32_t, uint64_t> df, plen;  // document frequency, posting-list length
    uint64_t total_documents = 0;
    float total_length = 0.0f, avgdl = 0.0f;
    // device mirror
    hipStream_t stream = nullptr;
    uint64_t* d_ptr = nullptr;
    uint32_t* d_term = nullptr;
    float *d_tf = nullptr, *d_dl = nullptr;
    uint64_t* d_ids = nullptr;
    uint64_t cap_ptr = 0, cap_ids = 0, cap_term = 0, cap_tf = 0, cap_dl = 0;
    uint64_t up_slots = 0, up_ent = 0;  // uploaded prefix (append-only adds)
    bool dirty = true;                  // full re-upload needed
    // blocked inverted index (device), rebuilt from the mirror after a change:
    // per 64-slot chunk its entries by (term, slot, add order)
    uint64_t* d_cptr = nullptr;
    uint32_t* d_cterm = nullptr;
    uint8_t* d_cslot = nullptr;
    float *d_ctf = nullptr, *d_cdl = nullptr, *d_ctfc = nullptr;
    uint64_t cap_cptr = 0, cap_cterm = 0, cap_cslot = 0, cap_ctf = 0, cap_cdl = 0, cap_ctfc = 0;
    // the blocked index's vocabulary (sorted distinct terms; d_cterm holds ranks in it) and
    // the search groups' direct-mapped term table over it (epoch-tagged words)
    std::vector<uint32_t> vocab;
    uint32_t* d_vocab = nullptr;
    uint32_t* d_gmap = nullptr;
    uint64_t cap_vocab = 0, cap_gmap = 0;
    uint32_t epoch = 0;
    uint64_t version = 0, inv_version = ~0ull, tfc_version = ~0ull;
    uint32_t tfc_avgdl = 0;  // the avgdl bits d_ctfc was computed with
    bool runs = false;       // some (term, document) has more than one entry (re-added ids)
    // search scratch
    void* scratch = nullptr;
    size_t scratch_n = 0;
    char* h_io = nullptr;  // pinned staging of a launch group's inputs and outputs
    size_t h_io_n = 0;
    uint64_t dense_fallbacks = 0;

    // avgdl's fold order: storage order = slot order, each slot's entries by
    // (term, add order); a new slot appends, so adds of new ids fold
    // incrementally and only re-adds / removes refold
    void recompute_length() {
        float t = 0.0f;
        for (float x : dl) t = t + x;
        total_length = t;
    }
};

namespace {

gvdb_status sp_dev(hipError_t e, const char* where) {
    return report_status(e == hipErrorOutOfMemory ? GVDB_ERR_OUT_OF_MEMORY : GVDB_ERR_DEVICE,
                         std::string(where) + ": " + hipGetErrorString(e));
}
#define SP_TRY(expr, where)                             \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return sp_dev(e_, where); \
    } while (0)

template <class T>
hipError_t grow(T*& p, uint64_t& cap, uint64_t need, uint64_t keep) {
    if (need <= cap && p) return hipSuccess;
    const uint64_t nc = std::max<uint64_t>(need, cap + cap / 2 + 1024);
    T* np = nullptr;
    hipError_t e = hipMalloc((void**)&np, nc * sizeof(T));
    if (e != hipSuccess) return e;
    if (p && keep) e = hipMemcpy(np, p, keep * sizeof(T), hipMemcpyDeviceToDevice);
    if (p) (void)hipFree(p);
    p = np;
    cap = nc;
    return e;
}

// Device mirror of the host CSR: appended slots upload their tail only; a
// re-add or remove (dirty) re-uploads everything.
gvdb_status upload(gvdb_sparse* sp) {
    const uint64_t N = sp->slot_id.size(), E = sp->term.size();
    if (!sp->dirty && sp->up_slots == N && sp->up_ent == E) return GVDB_OK;
    const uint64_t s0 = sp->dirty ? 0 : sp->up_slots, e0 = sp->dirty ? 0 : sp->up_ent;
    SP_TRY(grow(sp->d_ptr, sp->cap_ptr, N + 1, s0 ? s0 + 1 : 0), "alloc doc ptr");
    SP_TRY(grow(sp->d_ids, sp->cap_ids, N + 1, s0), "alloc doc ids");
    SP_TRY(grow(sp->d_term, sp->cap_term, E + 1, e0), "alloc terms");
    SP_TRY(grow(sp->d_tf, sp->cap_tf, E + 1, e0), "alloc tf");
    SP_TRY(grow(sp->d_dl, sp->cap_dl, E + 1, e0), "alloc dl");
    SP_TRY(hipMemcpy(sp->d_ptr + s0, sp->ptr.data() + s0, (N + 1 - s0) * 8, hipMemcpyHostToDevice), "upload ptr");
    if (N > s0) SP_TRY(hipMemcpy(sp->d_ids + s0, sp->slot_id.data() + s0, (N - s0) * 8, hipMemcpyHostToDevice), "ids");
    if (E > e0) {
        SP_TRY(hipMemcpy(sp->d_term + e0, sp->term.data() + e0, (E - e0) * 4, hipMemcpyHostToDevice), "upload terms");
        SP_TRY(hipMemcpy(sp->d_tf + e0, sp->tf.data() + e0, (E - e0) * 4, hipMemcpyHostToDevice), "upload tf");
        SP_TRY(hipMemcpy(sp->d_dl + e0, sp->dl.data() + e0, (E - e0) * 4, hipMemcpyHostToDevice), "upload dl");
    }
    sp->up_slots = N;
    sp->up_ent = E;
    sp->dirty = false;
    return GVDB_OK;
}

__global__ void k_blk_cptr(const uint64_t* __restrict__ ptr, uint32_t N, uint32_t nchunks, uint64_t* __restrict__ cptr) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c <= nchunks) cptr[c] = ptr[min((uint64_t)c * kTaCh, (uint64_t)N)];
}

// The blocked inverted index from the forward mirror (one stable radix sort
// of (chunk, term) keys; the forward entries are slot-ordered, each slot's by
// (term, add order)), and tf_component of every entry for the current avgdl.
gvdb_status build_blocked(gvdb_sparse* sp, hipStream_t s) {
    const uint64_t N = sp->slot_id.size(), E = sp->term.size();
    const uint32_t nchunks = (uint32_t)((N + kTaCh - 1) / kTaCh);
    if (sp->inv_version != sp->version) {
        if (E > 0x7fffffffull) return report_status(GVDB_ERR_INVALID_ARGUMENT, "more than 2^31 - 1 posting entries");
        SP_TRY(grow(sp->d_cptr, sp->cap_cptr, (uint64_t)nchunks + 1, 0), "alloc chunk ptr");
        hipLaunchKernelGGL(k_blk_cptr, dim3(nchunks / 256 + 1), dim3(256), 0, s, sp->d_ptr, (uint32_t)N, nchunks,
                           sp->d_cptr);
        SP_TRY(hipGetLastError(), "chunk ptr");
        uint32_t h_runs = 0;
        sp->vocab.clear();
        for (const auto& x : sp->plen)
            if (x.second) sp->vocab.push_back(x.first);
        std::sort(sp->vocab.begin(), sp->vocab.end());
        const uint64_t V = sp->vocab.size();
        SP_TRY(grow(sp->d_vocab, sp->cap_vocab, V + 1, 0), "alloc vocabulary");
        SP_TRY(grow(sp->d_gmap, sp->cap_gmap, V + 1, 0), "alloc group table");
        if (V) SP_TRY(hipMemcpyAsync(sp->d_vocab, sp->vocab.data(), V * 4, hipMemcpyHostToDevice, s), "vocabulary");
        SP_TRY(hipMemsetAsync(sp->d_gmap, 0, (V + 1) * 4, s), "group table");
        sp->epoch = 0;
        if (E > 0) {
            int end_bit = 32;
            while (end_bit < 64 && ((uint64_t)nchunks >> (end_bit - 32))) ++end_bit;
            size_t cub_bytes = 0;
            SP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, cub_bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                      (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)E, 0, end_bit,
                                                      s),
                   "blocked sort size");
            SP_TRY(grow(sp->d_cterm, sp->cap_cterm, E, 0), "alloc blocked terms");
            SP_TRY(grow(sp->d_cslot, sp->cap_cslot, E, 0), "alloc blocked slots");
            SP_TRY(grow(sp->d_ctf, sp->cap_ctf, E, 0), "alloc blocked tf");
            SP_TRY(grow(sp->d_cdl, sp->cap_cdl, E, 0), "alloc blocked dl");
            SP_TRY(grow(sp->d_ctfc, sp->cap_ctfc, E, 0), "alloc blocked tfc");
            const size_t a8 = ((size_t)E * 8 + 255) & ~(size_t)255, a4 = ((size_t)E * 4 + 255) & ~(size_t)255;
            char* tmp = nullptr;
            SP_TRY(hipMalloc((void**)&tmp, 2 * a8 + 3 * a4 + cub_bytes + 256), "alloc blocked build");
            uint64_t* keys = (uint64_t*)tmp;
            uint64_t* skeys = (uint64_t*)(tmp + a8);
            uint32_t* iota = (uint32_t*)(tmp + 2 * a8);
            uint32_t* order = (uint32_t*)(tmp + 2 * a8 + a4);
            uint32_t* eslot = (uint32_t*)(tmp + 2 * a8 + 2 * a4);
            uint32_t* d_runs = (uint32_t*)(tmp + 2 * a8 + 3 * a4);
            void* ct = tmp + 2 * a8 + 3 * a4 + 256;
            hipLaunchKernelGGL(k_blk_keys, dim3((uint32_t)((N + 255) / 256)), dim3(256), 0, s, sp->d_ptr, (uint32_t)N,
                               sp->d_term, keys, iota, eslot);
            hipError_t e = hipGetLastError();
            if (e == hipSuccess)
                e = hipcub::DeviceRadixSort::SortPairs(ct, cub_bytes, keys, skeys, iota, order, (int)E, 0, end_bit, s);
            if (e == hipSuccess) e = hipMemsetAsync(d_runs, 0, 4, s);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_blk_gather, dim3(2048), dim3(256), 0, s, order, skeys, eslot, sp->d_tf, sp->d_dl,
                                   E, sp->d_vocab, (uint32_t)V, sp->d_cterm, sp->d_cslot, sp->d_ctf, sp->d_cdl,
                                   d_runs);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipMemcpyAsync(&h_runs, d_runs, 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            (void)hipFree(tmp);
            if (e != hipSuccess) return sp_dev(e, "build blocked index");
            if (h_runs & 2u) return report_status(GVDB_ERR_INDEX, "posting term missing from the vocabulary");
        }
        sp->runs = (h_runs & 1u) != 0;
        sp->inv_version = sp->version;
    }
    uint32_t avg_bits;
    std::memcpy(&avg_bits, &sp->avgdl, 4);
    if (E > 0 && (sp->tfc_version != sp->version || sp->tfc_avgdl != avg_bits)) {
        hipLaunchKernelGGL(k_blk_tfc, dim3(2048), dim3(256), 0, s, sp->d_ctf, sp->d_cdl, E, sp->k1, sp->b, sp->avgdl,
                           sp->d_ctfc);
        SP_TRY(hipGetLastError(), "blocked tf_component");
        sp->tfc_version = sp->version;
        sp->tfc_avgdl = avg_bits;
    }
    return GVDB_OK;
}

// k_bm25_taat: one resident block per CU (its LDS map), each a contiguous range of
// at most kTaCptrLds chunks (more blocks than CUs for very large indexes)
uint32_t sp_grid(uint32_t tiles) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t need = (tiles + kTaCptrLds - 1) / kTaCptrLds;
    return std::max<uint32_t>(1, std::max(need, std::min<uint32_t>(tiles, (uint32_t)cus)));
}

// items per query bounded by the list strides: dynamic LDS for the next power of two
gvdb_status rrf_capacity(const uint32_t* n0, uint32_t st0, const uint32_t* n1, uint32_t st1, const uint32_t* n2,
                         uint32_t st2, uint32_t* pmax) {
    const uint64_t cap = (n0 ? (uint64_t)st0 : 0) + (n1 ? (uint64_t)st1 : 0) + (n2 ? (uint64_t)st2 : 0);
    if (cap > kRrfMax)
        return report_status(GVDB_ERR_INVALID_ARGUMENT,
                             "rrf: the three list strides sum to " + std::to_string(cap) + " items, more than 4096");
    uint32_t p = 2;
    while (p < cap) p <<= 1;
    *pmax = p;
    return GVDB_OK;
}

// gvdb_rrf_fuse's staging: one HBM buffer and stream per device, reused
struct RrfPool {
    std::mutex mu;
    hipStream_t stream = nullptr;
    char* buf = nullptr;
    size_t cap = 0;
};
RrfPool& rrf_pool(int dev) {
    static std::mutex m;
    static std::map<int, RrfPool*> pools;  // process lifetime
    std::lock_guard<std::mutex> g(m);
    RrfPool*& p = pools[dev];
    if (!p) p = new RrfPool();
    return *p;
}
}  // namespace

extern "C" {

gvdb_status gvdb_sparse_create(const gvdb_bm25_params* p, gvdb_sparse** out) {
    if (!out) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null out");
    auto* sp = new gvdb_sparse();
    if (p) {
        sp->k1 = p->k1;
        sp->b = p->b;
        sp->device = p->device;
    }
    hipError_t e = hipSetDevice(sp->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&sp->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete sp;
        return sp_dev(e, "gvdb_sparse_create");
    }
    *out = sp;
    return GVDB_OK;
}

void gvdb_sparse_destroy(gvdb_sparse* sp) {
    if (!sp) return;
    (void)hipSetDevice(sp->device);
    for (void* p : {(void*)sp->d_ptr, (void*)sp->d_term, (void*)sp->d_tf, (void*)sp->d_dl, (void*)sp->d_ids,
                    (void*)sp->d_cptr, (void*)sp->d_cterm, (void*)sp->d_cslot, (void*)sp->d_ctf, (void*)sp->d_cdl,
                    (void*)sp->d_ctfc, (void*)sp->d_vocab, (void*)sp->d_gmap, sp->scratch})
        if (p) (void)hipFree(p);
    if (sp->h_io) (void)hipHostFree(sp->h_io);
    if (sp->stream) (void)hipStreamDestroy(sp->stream);
    delete sp;
}

// SparseIndex::add_document (sparse.rs:71-107)
gvdb_status gvdb_sparse_add_document(gvdb_sparse* sp, uint64_t doc_id, const uint32_t* terms, const float* tfs,
                                     uint64_t n, float doc_length) {
    if (!sp || (n && (!terms || !tfs))) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    std::lock_guard<std::mutex> g(sp->mu);
    std::vector<std::pair<uint32_t, float>> e(n);
    for (uint64_t i = 0; i < n; ++i) e[i] = {terms[i], tfs[i]};
    std::stable_sort(e.begin(), e.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
    for (uint64_t i = 1; i < n; ++i)
        if (e[i].first == e[i - 1].first)
            return report_status(GVDB_ERR_INVALID_ARGUMENT, "duplicate term in one document (term_frequencies is a map)");
    auto it = sp->slot_of.find(doc_id);
    if (it == sp->slot_of.end()) {  // new slot: append (the fast, upload-the-tail path)
        const uint32_t slot = (uint32_t)sp->slot_id.size();
        sp->slot_of[doc_id] = slot;
        sp->slot_id.push_back(doc_id);
        for (const auto& x : e) {
            sp->term.push_back(x.first);
            sp->tf.push_back(x.second);
            sp->dl.push_back(doc_length);
            sp->total_length = sp->total_length + doc_length;  // slot order: this slot is last
        }
        sp->ptr.push_back(sp->term.size());
    } else {  // re-add: merge into the slot (stable: earlier adds first per term)
        const uint32_t slot = it->second;
        const uint64_t lo = sp->ptr[slot], hi = sp->ptr[slot + 1];
        std::vector<uint32_t> mt;
        std::vector<float> mtf, mdl;
        uint64_t i = lo;
        size_t j = 0;
        while (i < hi || j < e.size()) {
            if (j == e.size() || (i < hi && sp->term[i] <= e[j].first)) {
                mt.push_back(sp->term[i]);
                mtf.push_back(sp->tf[i]);
                mdl.push_back(sp->dl[i]);
                ++i;
            } else {
                mt.push_back(e[j].first);
                mtf.push_back(e[j].second);
                mdl.push_back(doc_length);
                ++j;
            }
        }
        sp->term.erase(sp->term.begin() + lo, sp->term.begin() + hi);
        sp->tf.erase(sp->tf.begin() + lo, sp->tf.begin() + hi);
        sp->dl.erase(sp->dl.begin() + lo, sp->dl.begin() + hi);
        sp->term.insert(sp->term.begin() + lo, mt.begin(), mt.end());
        sp->tf.insert(sp->tf.begin() + lo, mtf.begin(), mtf.end());
        sp->dl.insert(sp->dl.begin() + lo, mdl.begin(), mdl.end());
        for (size_t s = slot + 1; s < sp->ptr.size(); ++s) sp->ptr[s] += n;
        sp->recompute_length();
        sp->dirty = true;
    }
    for (const auto& x : e) {
        sp->df[x.first] += 1;
        sp->plen[x.first] += 1;
    }
    sp->total_documents += 1;
    sp->avgdl = sp->total_length / (float)sp->total_documents;  // sparse.rs:102-104
    ++sp->version;
    return GVDB_OK;
}

// Bulk form: n_docs documents in CSR (doc_ptr[n_docs+1] into terms/tfs).
gvdb_status gvdb_sparse_add_documents(gvdb_sparse* sp, const uint64_t* doc_ids, const uint64_t* doc_ptr,
                                      const uint32_t* terms, const float* tfs, const float* doc_lengths,
                                      uint64_t n_docs) {
    if (!sp || (n_docs && (!doc_ids || !doc_ptr || !doc_lengths)))
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    {
        // fast path: every id new and distinct -> append whole documents to the
        // CSR in one pass (same state as n_docs single adds)
        std::lock_guard<std::mutex> g(sp->mu);
        bool fresh = true;
        std::unordered_map<uint64_t, uint32_t> batch;
        batch.reserve(n_docs);
        for (uint64_t d = 0; d < n_docs && fresh; ++d)
            fresh = sp->slot_of.find(doc_ids[d]) == sp->slot_of.end() && batch.emplace(doc_ids[d], 0).second;
        if (fresh) {
            const uint64_t E0 = sp->term.size();
            const uint64_t add = doc_ptr[n_docs] - doc_ptr[0];
            sp->term.reserve(E0 + add);
            sp->tf.reserve(E0 + add);
            sp->dl.reserve(E0 + add);
            sp->ptr.reserve(sp->ptr.size() + n_docs);
            sp->slot_id.reserve(sp->slot_id.size() + n_docs);
            std::vector<std::pair<uint32_t, float>> e;
            for (uint64_t d = 0; d < n_docs; ++d) {
                const uint64_t a = doc_ptr[d], b = doc_ptr[d + 1];
                e.resize(b - a);
                bool sorted = true;
                for (uint64_t i = a; i < b; ++i) {
                    e[i - a] = {terms[i], tfs[i]};
                    if (i > a && terms[i] <= terms[i - 1]) sorted = false;
                }
                if (!sorted) {
                    std::stable_sort(e.begin(), e.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
                    for (size_t i = 1; i < e.size(); ++i)
                        if (e[i].first == e[i - 1].first) {
                            // roll back this batch: nothing of it was committed to the maps yet
                            sp->term.resize(E0);
                            sp->tf.resize(E0);
                            sp->dl.resize(E0);
                            sp->ptr.resize(sp->slot_id.size() + 1);
                            return report_status(GVDB_ERR_INVALID_ARGUMENT,
                                                 "duplicate term in one document (term_frequencies is a map)");
                        }
                }
                for (const auto& x : e) {
                    sp->term.push_back(x.first);
                    sp->tf.push_back(x.second);
                    sp->dl.push_back(doc_lengths[d]);
                }
                sp->ptr.push_back(sp->term.size());
            }
            for (uint64_t d = 0; d < n_docs; ++d) {
                sp->slot_of[doc_ids[d]] = (uint32_t)sp->slot_id.size();
                sp->slot_id.push_back(doc_ids[d]);
            }
            for (uint64_t i = E0; i < sp->term.size(); ++i) {
                sp->df[sp->term[i]] += 1;
                sp->plen[sp->term[i]] += 1;
                sp->total_length = sp->total_length + sp->dl[i];  // slot order: appended slots fold last
            }
            sp->total_documents += n_docs;
            if (sp->total_documents) sp->avgdl = sp->total_length / (float)sp->total_documents;
            ++sp->version;
            return GVDB_OK;
        }
    }
    for (uint64_t d = 0; d < n_docs; ++d) {
        const uint64_t a = doc_ptr[d], b = doc_ptr[d + 1];
        gvdb_status st = gvdb_sparse_add_document(sp, doc_ids[d], terms + a, tfs + a, b - a, doc_lengths[d]);
        if (st != GVDB_OK) return st;
    }
    return GVDB_OK;
}

// SparseIndex::remove_document (sparse.rs:109-149)
gvdb_status gvdb_sparse_remove_document(gvdb_sparse* sp, uint64_t doc_id, int32_t* removed) {
    if (!sp) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null index");
    std::lock_guard<std::mutex> g(sp->mu);
    if (removed) *removed = 0;
    auto it = sp->slot_of.find(doc_id);
    if (it == sp->slot_of.end()) return GVDB_OK;
    const uint32_t slot = it->second;
    const uint64_t lo = sp->ptr[slot], hi = sp->ptr[slot + 1];
    if (lo == hi) return GVDB_OK;
    // the first entry of every term group goes (the first posting occurrence)
    std::vector<uint32_t> mt;
    std::vector<float> mtf, mdl;
    uint64_t dropped = 0;
    for (uint64_t i = lo; i < hi; ++i) {
        if (i == lo || sp->term[i] != sp->term[i - 1]) {
            const uint32_t t = sp->term[i];
            auto pl = sp->plen.find(t);
            if (pl != sp->plen.end() && --pl->second == 0) {
                sp->plen.erase(pl);
                sp->df.erase(t);  // sparse.rs:128-133
            }
            ++dropped;
            continue;
        }
        mt.push_back(sp->term[i]);
        mtf.push_back(sp->tf[i]);
        mdl.push_back(sp->dl[i]);
    }
    sp->term.erase(sp->term.begin() + lo, sp->term.begin() + hi);
    sp->tf.erase(sp->tf.begin() + lo, sp->tf.begin() + hi);
    sp->dl.erase(sp->dl.begin() + lo, sp->dl.begin() + hi);
    sp->term.insert(sp->term.begin() + lo, mt.begin(), mt.end());
    sp->tf.insert(sp->tf.begin() + lo, mtf.begin(), mtf.end());
    sp->dl.insert(sp->dl.begin() + lo, mdl.begin(), mdl.end());
    for (size_t s = slot + 1; s < sp->ptr.size(); ++s) sp->ptr[s] -= dropped;
    sp->dirty = true;
    sp->total_documents = sp->total_documents > 0 ? sp->total_documents - 1 : 0;
    sp->recompute_length();
    sp->avgdl = sp->total_documents > 0 ? sp->total_length / (float)sp->total_documents : 0.0f;
    ++sp->version;
    if (removed) *removed = 1;
    return GVDB_OK;
}

gvdb_status gvdb_sparse_get_stats(const gvdb_sparse* sp, gvdb_bm25_stats* out) {
    if (!sp || !out) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    out->total_documents = sp->total_documents;
    out->average_document_length = sp->avgdl;
    out->vocabulary_size = sp->df.size();
    out->total_entries = sp->term.size();
    out->dense_fallbacks = sp->dense_fallbacks;
    return GVDB_OK;
}

void gvdb_sparse_clear(gvdb_sparse* sp) {
    if (!sp) return;
    std::lock_guard<std::mutex> g(sp->mu);
    sp->slot_of.clear();
    sp->slot_id.clear();
    sp->ptr.assign(1, 0);
    sp->term.clear();
    sp->tf.clear();
    sp->dl.clear();
    sp->df.clear();
    sp->plen.clear();
    sp->total_documents = 0;
    sp->total_length = 0.0f;
    sp->avgdl = 0.0f;
    sp->dirty = true;
    ++sp->version;
}

// SparseIndex::search_bm25 (sparse.rs:151-198) for B queries in CSR
// (q_ptr[B+1] into q_terms / q_values = SparseVector.indices / .values).
gvdb_status gvdb_sparse_search_bm25(gvdb_sparse* sp, const uint64_t* q_ptr, const uint32_t* q_terms,
                                    const float* q_values, uint64_t B, uint64_t limit, uint64_t* out_ids,
                                    float* out_scores, uint32_t* out_n) {
    if (!sp || (B && (!q_ptr || !out_n)) || (B && limit && (!out_ids || !out_scores)))
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (limit > 0xffffffffull) return report_status(GVDB_ERR_INVALID_ARGUMENT, "limit too large");
    std::lock_guard<std::mutex> g(sp->mu);
    for (uint64_t q = 0; q < B; ++q) out_n[q] = 0;
    // no entries: no document matches any term (the reference's map stays empty)
    if (B == 0 || limit == 0 || sp->total_documents == 0 || sp->slot_id.empty() || sp->term.empty()) return GVDB_OK;
    SP_TRY(hipSetDevice(sp->device), "hipSetDevice");
    gvdb_status st = upload(sp);
    if (st == GVDB_OK) st = build_blocked(sp, sp->stream);
    if (st != GVDB_OK) return st;
    const uint32_t N = (uint32_t)sp->slot_id.size();
    const uint32_t L = (uint32_t)limit;
    const uint32_t nblk = (N + kTaCh - 1) / kTaCh;  // blocked-index chunks
    hipStream_t s = sp->stream;
    uint64_t q0 = 0;
    std::vector<uint32_t> h_qp;
    std::vector<uint32_t> h_qt;
    std::vector<float> h_qv, h_qidf;
    while (q0 < B) {
        // launch group: <= kTaQ queries, <= kSpQT live query terms, <= kSpU distinct terms
        h_qp.assign(1, 0);
        h_qt.clear();
        h_qv.clear();
        h_qidf.clear();
        std::vector<uint32_t> group_terms;  // distinct live terms of the group
        uint64_t q1 = q0;
        while (q1 < B && q1 - q0 < kTaQ) {
            std::vector<uint32_t> t;
            std::vector<float> v, idf;
            for (uint64_t p = q_ptr[q1]; p < q_ptr[q1 + 1]; ++p) {
                const uint32_t term = q_terms[p];
                auto pl = sp->plen.find(term);
                if (pl == sp->plen.end() || pl->second == 0) continue;  // no posting list: no contribution
                auto d = sp->df.find(term);
                const uint64_t dfv = d == sp->df.end() ? 1 : d->second;  // unwrap_or(1)
                // calculate_idf (sparse.rs:200-203): f32 ln, as Rust's f32::ln (libm logf)
                const float x = ((float)sp->total_documents - (float)dfv + 0.5f) / ((float)dfv + 0.5f);
                t.push_back(term);
                v.push_back(q_values[p]);
                idf.push_back(std::log(x));
            }
            if (t.size() > kSpQT) return report_status(GVDB_ERR_INVALID_ARGUMENT, "query has more than 1024 terms");
            if (h_qt.size() + t.size() > kSpQT) break;
            {
                std::vector<uint32_t> u(group_terms);
                u.insert(u.end(), t.begin(), t.end());
                std::sort(u.begin(), u.end());
                u.erase(std::unique(u.begin(), u.end()), u.end());
                if (u.size() > kSpU) {
                    if (q1 == q0)
                        return report_status(GVDB_ERR_INVALID_ARGUMENT, "query has more than 511 distinct terms");
                    break;
                }
                group_terms.swap(u);
            }
            h_qt.insert(h_qt.end(), t.begin(), t.end());
            h_qv.insert(h_qv.end(), v.begin(), v.end());
            h_qidf.insert(h_qidf.end(), idf.begin(), idf.end());
            h_qp.push_back((uint32_t)h_qt.size());
            ++q1;
        }
        const uint32_t Bg = (uint32_t)(q1 - q0);
        const uint32_t nu = (uint32_t)group_terms.size();
        const uint32_t nchunks = (nblk + kTaSpl - 1) / kTaSpl;  // 128-document chunks
        // sample stride: expected candidates ~ limit * every, kept well under kSpCand
        uint32_t every = std::max<uint32_t>(1u, std::min<uint32_t>(32u, kSpCand / std::max<uint32_t>(1u, 4u * L)));
        if (nchunks <= 8u * every) every = 1;  // small index: the sample is the whole index
        const uint32_t nsamp = (nchunks + every - 1) / every;
        const uint32_t S = nsamp * (kTaCh * kTaSpl / kTaGrp);
        auto launch_taat = [&](int mode, uint32_t grid, const TaArgs& ta) {
            if (mode == 0) hipLaunchKernelGGL((k_bm25_taat<0>), dim3(grid), dim3(kTaThreads), 0, s, ta);
            if (mode == 1) hipLaunchKernelGGL((k_bm25_taat<1>), dim3(grid), dim3(kTaThreads), 0, s, ta);
            if (mode == 2) hipLaunchKernelGGL((k_bm25_taat<2>), dim3(grid), dim3(kTaThreads), 0, s, ta);
        };
        // per query its term records (group term, q_tf, idf, map row bytes), padded with empty
        // records (the empty row, never written; q_tf = idf = 0) to a multiple of 4 -- the
        // kernel's batches -- plus one more; per group term the queries holding it; the
        // queries whose q_tf or idf is not finite
        std::vector<uint32_t> h_pqp(1, 0u), h_qrec;
        std::vector<uint64_t> h_qmask(nu + 1, 0ull);
        uint64_t qsel = 0;
        auto push_rec = [&](uint32_t g, float v, float idf) {
            uint32_t r[4] = {g, 0u, 0u, g * kTaCh * kTaSpl * 2};
            std::memcpy(&r[1], &v, 4);
            std::memcpy(&r[2], &idf, 4);
            h_qrec.insert(h_qrec.end(), r, r + 4);
        };
        for (uint32_t q = 0; q < Bg; ++q) {
            for (uint32_t i = h_qp[q]; i < h_qp[q + 1]; ++i) {
                const uint32_t g =
                    (uint32_t)(std::lower_bound(group_terms.begin(), group_terms.end(), h_qt[i]) - group_terms.begin());
                push_rec(g, h_qv[i], h_qidf[i]);
                h_qmask[g] |= 1ull << q;
                if (!std::isfinite(h_qv[i]) || !std::isfinite(h_qidf[i])) qsel |= 1ull << q;
            }
            while ((h_qrec.size() / 4) % 4) push_rec(kTaRows - 1, 0.0f, 0.0f);
            h_pqp.push_back((uint32_t)(h_qrec.size() / 4));
        }
        const uint32_t nrec = (uint32_t)(h_qrec.size() / 4);
        for (int k = 0; k < 4; ++k) push_rec(kTaRows - 1, 0.0f, 0.0f);  // [nrec, nrec + 4): a whole empty batch
        // wave slots w + 16 m: longest-processing-time assignment of the queries to the
        // 16 waves (each wave's rounds cost about the sum of its queries' term counts)
        std::vector<uint32_t> h_perm(kTaQ, 0xffffffffu);
        {
            std::vector<uint32_t> order(Bg);
            for (uint32_t q = 0; q < Bg; ++q) order[q] = q;
            std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
                return h_qp[x + 1] - h_qp[x] > h_qp[y + 1] - h_qp[y];
            });
            const uint32_t nw = std::min<uint32_t>(kTaWaves, Bg);
            std::vector<uint32_t> load(nw, 0), cnt(nw, 0);
            for (uint32_t q : order) {
                uint32_t best = 0xffffffffu;
                for (uint32_t w = 0; w < nw; ++w)
                    if (cnt[w] < kTaQW && (best == 0xffffffffu || load[w] < load[best])) best = w;
                h_perm[best + kTaWaves * cnt[best]] = q;
                load[best] += h_qp[q + 1] - h_qp[q];
                ++cnt[best];
            }
        }
        // scratch: [qp | perm | qrec | ut | qmask] (one upload) | tau | counts | smp | cand |
        // [fail | out_n | out ids | out scores] (one download)
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t o_qp = 0, o_perm = o_qp + al((Bg + 1) * 4), o_qrec = o_perm + al(kTaQ * 4),
                     o_ut = o_qrec + al((nrec + 4) * 16), o_qm = o_ut + al(nu * 4 + 4),
                     o_tau = o_qm + al(nu * 8 + 8), o_cnt = o_tau + al(Bg * 8), o_smp = o_cnt + al(Bg * 4),
                     o_cand = o_smp + al((size_t)Bg * S * 8), o_fail = o_cand + al((size_t)Bg * kSpCand * 8),
                     o_n = o_fail + al(Bg * 4), o_oi = o_n + al(Bg * 4), o_os = o_oi + al((size_t)Bg * L * 8),
                     total = o_os + al((size_t)Bg * L * 4);
        const size_t in_bytes = o_tau, out_bytes = total - o_fail;
        if (total > sp->scratch_n) {
            if (sp->scratch) (void)hipFree(sp->scratch);
            sp->scratch = nullptr;
            sp->scratch_n = 0;
            SP_TRY(hipMalloc(&sp->scratch, total), "alloc bm25 scratch");
            sp->scratch_n = total;
        }
        const size_t io_need = std::max(in_bytes, out_bytes);
        if (io_need > sp->h_io_n) {
            if (sp->h_io) (void)hipHostFree(sp->h_io);
            sp->h_io = nullptr;
            sp->h_io_n = 0;
            SP_TRY(hipHostMalloc((void**)&sp->h_io, io_need, hipHostMallocDefault), "alloc bm25 staging");
            sp->h_io_n = io_need;
        }
        char* base = (char*)sp->scratch;
        char* hio = sp->h_io;
        SP_TRY(hipStreamSynchronize(s), "sync");  // the staging buffer's previous download was consumed
        for (auto& t : group_terms)  // dense ids (the vocabulary holds every live term; same order)
            t = (uint32_t)(std::lower_bound(sp->vocab.begin(), sp->vocab.end(), t) - sp->vocab.begin());
        std::memcpy(hio + o_qp, h_pqp.data(), (Bg + 1) * 4);
        std::memcpy(hio + o_perm, h_perm.data(), kTaQ * 4);
        std::memcpy(hio + o_qrec, h_qrec.data(), (nrec + 4) * 16);
        if (nu) std::memcpy(hio + o_ut, group_terms.data(), nu * 4);
        if (nu) std::memcpy(hio + o_qm, h_qmask.data(), nu * 8);
        SP_TRY(hipMemcpyAsync(base, hio, in_bytes, hipMemcpyHostToDevice, s), "bm25 inputs");
        if (++sp->epoch >> (32 - kGmapShift)) {  // epoch tag wrapped: clear the table
            SP_TRY(hipMemsetAsync(sp->d_gmap, 0, (sp->vocab.size() + 1) * 4, s), "group table");
            sp->epoch = 1;
        }
        hipLaunchKernelGGL(k_gmap_set, dim3(1), dim3(512), 0, s, sp->d_gmap, (const uint32_t*)(base + o_ut), nu,
                           sp->epoch, (uint32_t*)(base + o_cnt), Bg);
        SP_TRY(hipGetLastError(), "bm25 group table");
        TaArgs a{};
        a.cptr = sp->d_cptr;
        a.cterm = sp->d_cterm;
        a.cslot = sp->d_cslot;
        a.ctfc = sp->d_ctfc;
        a.N = N;
        a.nchunks = nblk;
        a.n_entries = sp->term.size();
        a.ut = (const uint32_t*)(base + o_ut);
        a.nu = nu;
        a.gmap = sp->d_gmap;
        a.epoch = sp->epoch;
        a.qmask = (const uint64_t*)(base + o_qm);
        a.qsel = qsel;
        a.qp = (const uint32_t*)(base + o_qp);
        a.qrec = (const uint4*)(base + o_qrec);
        a.perm = (const uint32_t*)(base + o_perm);
        a.nqt = nrec;
        a.runs = sp->runs ? 1u : 0u;
        a.B = Bg;
        a.every = every;
        a.smp = (uint64_t*)(base + o_smp);
        a.S = S;
        a.tau = (const uint64_t*)(base + o_tau);
        a.counts = (uint32_t*)(base + o_cnt);
        a.cand = (uint64_t*)(base + o_cand);
        {
            static const uint32_t abl = [] {
                const char* e = getenv("GVDB_BM25_ABL");
                return e ? (uint32_t)atoi(e) : 0u;
            }();
            a.abl = abl;
        }
        std::vector<uint64_t> h_prof;
        uint64_t* d_prof = nullptr;
        if (a.abl & 8) {
            SP_TRY(hipMalloc((void**)&d_prof, 1024 * 8 * 8), "prof");
            SP_TRY(hipMemsetAsync(d_prof, 0, 1024 * 8 * 8, s), "prof");
            a.prof = d_prof;
        }
        launch_taat(0, sp_grid(nsamp), a);
        SP_TRY(hipGetLastError(), "bm25 sample");
        hipLaunchKernelGGL(k_bm25_tau, dim3(Bg), dim3(kTauThreads), 0, s, a.smp, S, L, (uint64_t*)(base + o_tau));
        SP_TRY(hipGetLastError(), "bm25 tau");
        launch_taat(1, sp_grid(nchunks), a);
        SP_TRY(hipGetLastError(), "bm25 emit");
        if (d_prof) {
            h_prof.resize(1024 * 8);
            SP_TRY(hipMemcpyAsync(h_prof.data(), d_prof, 1024 * 8 * 8, hipMemcpyDeviceToHost, s), "prof");
            SP_TRY(hipStreamSynchronize(s), "prof");
            double acc[5] = {0, 0, 0, 0, 0};
            const uint32_t G = sp_grid(nchunks);
            for (uint32_t g = 0; g < G; ++g)
                for (int k = 0; k < 5; ++k) acc[k] += (double)h_prof[g * 8 + k];
            fprintf(stderr,
                    "[bm25 prof] per block, shader clock cycles: dir %.0f stage %.0f rounds %.0f select %.0f "
                    "issue %.0f\n",
                    acc[0] / G, acc[1] / G, acc[2] / G, acc[3] / G, acc[4] / G);
            (void)hipFree(d_prof);
        }
        uint64_t* d_oi = (uint64_t*)(base + o_oi);
        float* d_os = (float*)(base + o_os);
        uint32_t* d_n = (uint32_t*)(base + o_n);
        uint32_t* d_fail = (uint32_t*)(base + o_fail);
        hipLaunchKernelGGL(k_bm25_final, dim3(Bg), dim3(256), 0, s, a.cand, a.counts, L, sp->d_ids, d_oi, d_os, d_n,
                           d_fail);
        SP_TRY(hipGetLastError(), "bm25 final");
        SP_TRY(hipMemcpyAsync(hio, base + o_fail, out_bytes, hipMemcpyDeviceToHost, s), "bm25 outputs");
        SP_TRY(hipStreamSynchronize(s), "sync");
        const uint32_t* h_failv = (const uint32_t*)hio;
        bool any_fail = false;
        // exact fallback for overflowing queries: dense keys + radix sort
        for (uint32_t q = 0; q < Bg; ++q) {
            if (!h_failv[q]) continue;
            any_fail = true;
            ++sp->dense_fallbacks;
            size_t cub_bytes = 0;
            hipcub::DoubleBuffer<uint64_t> kb(nullptr, nullptr);
            SP_TRY(hipcub::DeviceRadixSort::SortKeysDescending(nullptr, cub_bytes, kb, (int)N, 0, 64, s), "cub size");
            void* tmp = nullptr;
            SP_TRY(hipMalloc(&tmp, (size_t)N * 16 + cub_bytes + 512), "alloc dense fallback");
            uint64_t* k0 = (uint64_t*)tmp;
            uint64_t* k1 = k0 + N;
            void* ct = (char*)tmp + (size_t)N * 16 + 256;
            a.dense = k0;
            a.dense_q = q;
            launch_taat(2, sp_grid(nchunks), a);
            hipError_t e = hipGetLastError();
            hipcub::DoubleBuffer<uint64_t> db(k0, k1);
            if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortKeysDescending(ct, cub_bytes, db, (int)N, 0, 64, s);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_bm25_emit_dense, dim3((L + 255) / 256), dim3(256), 0, s, db.Current(), N, L,
                                   sp->d_ids, d_oi + (size_t)q * L, d_os + (size_t)q * L, d_n + q);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            (void)hipFree(tmp);
            if (e != hipSuccess) return sp_dev(e, "bm25 dense fallback");
        }
        if (any_fail) {  // the fallback rewrote some outputs
            SP_TRY(hipMemcpyAsync(hio, base + o_fail, out_bytes, hipMemcpyDeviceToHost, s), "bm25 outputs");
            SP_TRY(hipStreamSynchronize(s), "sync");
        }
        std::memcpy(out_ids + q0 * L, hio + (o_oi - o_fail), (size_t)Bg * L * 8);
        std::memcpy(out_scores + q0 * L, hio + (o_os - o_fail), (size_t)Bg * L * 4);
        std::memcpy(out_n + q0, hio + (o_n - o_fail), (size_t)Bg * 4);
        q0 = q1;
    }
    return GVDB_OK;
}

gvdb_status gvdb_rrf_fuse_device(const uint64_t* d_dense_ids, const float* d_dense_scores, const uint32_t* d_dense_n,
                                 uint32_t dense_stride, const uint64_t* d_sparse_ids, const float* d_sparse_scores,
                                 const uint32_t* d_sparse_n, uint32_t sparse_stride, const uint64_t* d_text_ids,
                                 const float* d_text_scores, const uint32_t* d_text_n, uint32_t text_stride, uint64_t B,
                                 float k, uint64_t limit, uint64_t* d_out_ids, float* d_out_scores,
                                 float* d_out_breakdown, uint32_t* d_out_n, void* stream) {
    if (B == 0) return GVDB_OK;
    if (!d_out_n || (limit && (!d_out_ids || !d_out_scores)) || limit > 0xffffffffull || B > 0x7fffffffull)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "bad output arguments");
    uint32_t pmax = 0;
    gvdb_status st = rrf_capacity(d_dense_n, dense_stride, d_sparse_n, sparse_stride, d_text_n, text_stride, &pmax);
    if (st != GVDB_OK) return st;
    hipLaunchKernelGGL(k_rrf, dim3((uint32_t)B), dim3(256), (size_t)pmax * 24, (hipStream_t)stream, d_dense_ids,
                       d_dense_scores, d_dense_n, dense_stride, d_sparse_ids, d_sparse_scores, d_sparse_n,
                       sparse_stride, d_text_ids, d_text_scores, d_text_n, text_stride, k, (uint32_t)limit, pmax,
                       d_out_ids, d_out_scores, d_out_breakdown, d_out_n);
    SP_TRY(hipGetLastError(), "rrf");
    return GVDB_OK;
}


// Host-pointer form: stages the lists through a per-device pooled HBM buffer
// on a pooled stream (no allocation per call once the buffer is large enough).
gvdb_status gvdb_rrf_fuse(const uint64_t* dense_ids, const float* dense_scores, const uint32_t* dense_n,
                          uint32_t dense_stride, const uint64_t* sparse_ids, const float* sparse_scores,
                          const uint32_t* sparse_n, uint32_t sparse_stride, const uint64_t* text_ids,
                          const float* text_scores, const uint32_t* text_n, uint32_t text_stride, uint64_t B, float k,
                          uint64_t limit, uint64_t* out_ids, float* out_scores, float* out_breakdown,
                          uint32_t* out_n) {
    if (B == 0) return GVDB_OK;
    if (!out_n || (limit && (!out_ids || !out_scores))) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null output");
    uint32_t pmax = 0;
    gvdb_status st = rrf_capacity(dense_n, dense_stride, sparse_n, sparse_stride, text_n, text_stride, &pmax);
    if (st != GVDB_OK) return st;
    struct L {
        const uint64_t* ids;
        const float* sc;
        const uint32_t* n;
        uint32_t st;
    } lists[3] = {{dense_ids, dense_scores, dense_n, dense_stride},
                  {sparse_ids, sparse_scores, sparse_n, sparse_stride},
                  {text_ids, text_scores, text_n, text_stride}};
    auto al = [](size_t n) { return (n + 255) & ~(size_t)255; };
    size_t bytes = 0;
    for (const L& l : lists)
        if (l.n) bytes += al(B * 4) + al((size_t)B * l.st * 8) + al((size_t)B * l.st * 4);
    bytes += al((size_t)B * limit * 8) + al((size_t)B * limit * 4) + al((size_t)B * limit * 12) + al(B * 4);
    int dev = 0;
    SP_TRY(hipGetDevice(&dev), "hipGetDevice");
    RrfPool& pool = rrf_pool(dev);
    std::lock_guard<std::mutex> g(pool.mu);
    if (!pool.stream) SP_TRY(hipStreamCreateWithFlags(&pool.stream, hipStreamNonBlocking), "rrf stream");
    if (bytes > pool.cap) {
        if (pool.buf) (void)hipFree(pool.buf);
        pool.buf = nullptr;
        pool.cap = 0;
        const size_t want = std::max(bytes, (size_t)1 << 20);
        SP_TRY(hipMalloc((void**)&pool.buf, want), "alloc rrf");
        pool.cap = want;
    }
    hipStream_t s = pool.stream;
    char* p = pool.buf;
    auto take = [&](size_t n) {
        char* r = p;
        p += al(n);
        return r;
    };
    const uint64_t* dl_ids[3] = {nullptr, nullptr, nullptr};
    const float* dl_sc[3] = {nullptr, nullptr, nullptr};
    const uint32_t* dl_n[3] = {nullptr, nullptr, nullptr};
    hipError_t e = hipSuccess;
    for (int i = 0; i < 3 && e == hipSuccess; ++i) {
        const L& l = lists[i];
        if (!l.n) continue;
        uint32_t* n = (uint32_t*)take(B * 4);
        uint64_t* ids = (uint64_t*)take((size_t)B * l.st * 8);
        float* sc = (float*)take((size_t)B * l.st * 4);
        e = hipMemcpyAsync(n, l.n, B * 4, hipMemcpyHostToDevice, s);
        if (e == hipSuccess && l.st) e = hipMemcpyAsync(ids, l.ids, (size_t)B * l.st * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess && l.st) e = hipMemcpyAsync(sc, l.sc, (size_t)B * l.st * 4, hipMemcpyHostToDevice, s);
        dl_ids[i] = ids;
        dl_sc[i] = sc;
        dl_n[i] = n;
    }
    uint64_t* oi = (uint64_t*)take((size_t)B * limit * 8);
    float* os = (float*)take((size_t)B * limit * 4);
    float* ob = (float*)take((size_t)B * limit * 12);
    uint32_t* on = (uint32_t*)take(B * 4);
    if (!out_breakdown) ob = nullptr;
    if (e == hipSuccess)
        st = gvdb_rrf_fuse_device(dl_ids[0], dl_sc[0], dl_n[0], dense_stride, dl_ids[1], dl_sc[1], dl_n[1], sparse_stride,
                                  dl_ids[2], dl_sc[2], dl_n[2], text_stride, B, k, limit, oi, os, ob, on, s);
    if (e == hipSuccess && st == GVDB_OK) {
        if (limit) e = hipMemcpyAsync(out_ids, oi, (size_t)B * limit * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && limit) e = hipMemcpyAsync(out_scores, os, (size_t)B * limit * 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && ob) e = hipMemcpyAsync(out_breakdown, ob, (size_t)B * limit * 12, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(out_n, on, B * 4, hipMemcpyDeviceToHost, s);
    }
    // the pooled buffer is reused by the next call: drain the stream whatever happened
    const hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    if (e != hipSuccess) return sp_dev(e, "rrf");
    return st;
}

}  // extern "C"
