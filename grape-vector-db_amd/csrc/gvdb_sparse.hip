// gvdb_sparse.hip — BM25 sparse search and reciprocal-rank fusion on gfx950.
//
// Replaces the CPU paths of (reference snapshot 2025-08-24, Rust):
//   * SparseIndex (src/sparse.rs:29-222): add_document 71-107,
//     remove_document 109-149, search_bm25 151-198, idf / bm25 200-222,
//     BM25Parameters k1 = 1.2, b = 0.75 (49-53);
//   * HybridSearchEngine::rrf_fusion (src/hybrid.rs:422-488).
//
// Layout in HBM: a document-major forward index (CSR over document SLOTS,
// slot = first add of a document id): ptr[u64 N+1], term[u32 nnz], tf[f32],
// dl[f32] (dl per entry: a re-added id carries each add's document_length).
// A slot's entries are sorted by (term, add order), so the k-th entry of a
// term in a slot is the slot's k-th occurrence in that term's posting list.
//
// Search = document-at-a-time over the forward index for a batch of queries
// (the reference walks postings term-at-a-time into a HashMap; per document
// the contributions are added in query-term order either way, so the sums are
// bit-identical):  for every (document, query) pair a lane binary-searches
// each query term among the document's terms (staged in LDS per 64-document
// tile) and folds  acc = acc + (q_tf * tfc) * idf  in query order, exactly the
// reference's f32 expression (no FMA: -ffp-contract=off).  idf is computed on
// the host per (query, term) with the same logf the Rust f32::ln calls.
// Selection: a sample pass scores every `every`-th tile and the k-th largest
// sampled key (score, then slot ascending) is a lower bound tau of the k-th
// best key (k documents reach it); the emit pass keeps documents with
// key >= tau (~k * every of them), an LDS sort orders them.  Exact for every
// input: a query whose candidates overflow the buffer is answered by a dense
// key array + radix sort.
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
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/gvdb.h"
#include "gvdb_device.h"
#include "gvdb_internal.h"

using namespace gvdb;

namespace {

constexpr uint32_t kSpTile = 64;        // documents per tile (one per lane of a wave)
constexpr uint32_t kSpThreads = 512;    // 8 query groups x 64 documents: 16 waves per CU at 2 blocks (the loop is latency-bound)
constexpr uint32_t kSpEnt = 4096;       // staged term entries per tile (else read from HBM)
constexpr uint32_t kSpQT = 1024;        // query terms per launch group (LDS)
constexpr uint32_t kSpU = 512;          // distinct terms per launch group (LDS match map)
constexpr uint32_t kSpMaxB = 256;       // queries per launch group
constexpr uint32_t kSpCand = 4096;      // candidates per query (LDS sort)
constexpr uint32_t kSpTopLocal = 8;     // per-thread keys kept by the tau pass

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

struct SpArgs {
    const uint64_t* ptr;   // [N+1]
    const uint32_t* term;  // [nnz]
    const float* tf;
    const float* dl;
    uint32_t N;            // slots
    const uint32_t* qp;    // [B+1] offsets into qb/qv/qidf
    const uint16_t* qb;    // index of each query term in ut
    const uint32_t* ut;    // the group's distinct live terms, ascending
    uint32_t nu;
    const float* qv;
    const float* qidf;
    uint32_t B;
    float k1, b, avgdl;
    uint32_t every;        // sample pass: tile stride
    uint64_t* smp;         // sample: [B][S] keys (0 = unmatched)
    uint32_t S;
    const uint64_t* tau;   // emit: [B]
    uint32_t* counts;      // emit: [B]
    uint64_t* cand;        // emit: [B][kSpCand]
    uint64_t* dense;       // dense mode: [N] keys of query `dense_q`
    uint32_t dense_q;
};

// MODE 0: sample (every `every`-th tile -> smp), 1: emit (key >= tau ->
// cand), 2: dense keys of one query.
// Per 64-document tile: the documents' term lists are staged in LDS, then a
// (document x batch-term) match map is built -- each entry looks its term up
// once among the batch's distinct terms `ut` (sorted, <= kSpU) and records its
// position (first entry of a run; 255 = "search", for documents past 254
// entries).  Scoring a (document, query) pair is then one LDS byte per query
// term instead of a binary search.
template <int MODE>
__global__ __launch_bounds__(kSpThreads, 2) void k_bm25(SpArgs a) {
    __shared__ uint32_t s_qp[kSpMaxB + 1];
    __shared__ uint64_t s_tau[MODE == 1 ? kSpMaxB : 1];  // emit thresholds, staged once
    __shared__ uint16_t s_qb[kSpQT];
    __shared__ float s_qv[kSpQT], s_qidf[kSpQT];
    __shared__ uint32_t s_ut[kSpU];
    __shared__ uint32_t s_ent[kSpEnt];
    __shared__ float s_tfc[kSpEnt];  // tf_component of each staged entry (query-independent)
    __shared__ uint32_t s_dp[kSpTile + 1];
    __shared__ __attribute__((aligned(16))) uint8_t s_map[kSpTile * kSpU];
    const uint32_t tid = threadIdx.x, doc = tid & (kSpTile - 1), qg = tid / kSpTile;
    const uint32_t B = a.B, nu = a.nu;
    for (uint32_t i = tid; i <= B; i += kSpThreads) s_qp[i] = a.qp[i];
    if constexpr (MODE == 1)
        for (uint32_t i = tid; i < B; i += kSpThreads) s_tau[i] = a.tau[i];
    for (uint32_t i = tid; i < nu; i += kSpThreads) s_ut[i] = a.ut[i];
    __syncthreads();
    const uint32_t nqt = s_qp[B];
    for (uint32_t i = tid; i < nqt; i += kSpThreads) {
        s_qb[i] = a.qb[i];
        s_qv[i] = a.qv[i];
        s_qidf[i] = a.qidf[i];
    }
    const float k1 = a.k1, b = a.b, avgdl = a.avgdl;
    const float k1p1 = k1 + 1.0f, omb = 1.0f - b;  // (k1 + 1.0), (1.0 - b) as the reference evaluates them
    const uint32_t ntiles_all = (a.N + kSpTile - 1) / kSpTile;
    const uint32_t every = MODE == 0 ? a.every : 1u;
    const uint32_t ntiles = (ntiles_all + every - 1) / every;
    const uint32_t map_words = (kSpTile * nu + 3) / 4;
    for (uint32_t j = blockIdx.x; j < ntiles; j += gridDim.x) {
        const uint32_t d0 = j * every * kSpTile;
        const uint32_t nd = min(kSpTile, a.N - d0);
        __syncthreads();  // previous tile's LDS readers are done
        if (tid <= nd) s_dp[tid] = (uint32_t)(a.ptr[d0 + tid] - a.ptr[d0]);
        for (uint32_t i = tid; i < map_words; i += kSpThreads) ((uint32_t*)s_map)[i] = 0u;
        __syncthreads();
        const uint64_t base = a.ptr[d0];
        const uint32_t E = s_dp[nd];
        const bool staged = E <= kSpEnt;
        // calculate_bm25_score's tf_component (sparse.rs:215-218) depends on the
        // entry only: evaluated once per staged entry
        auto tfc_of = [&](uint64_t g) {
            const float tfv = a.tf[g], dlv = a.dl[g];
            return (tfv * k1p1) / (tfv + k1 * (omb + b * (dlv / avgdl)));
        };
        if (staged) {
            // all loads first (up to kSpEnt / kSpThreads per thread in flight),
            // then the arithmetic: a load-compute-store loop would serialise
            // one HBM latency per entry
            constexpr uint32_t kPer = kSpEnt / kSpThreads;
            uint32_t tv[kPer];
            float fv[kPer], dv[kPer];
#pragma unroll
            for (uint32_t k = 0; k < kPer; ++k) {
                const uint32_t i = tid + k * kSpThreads;
                if (i < E) {
                    tv[k] = a.term[base + i];
                    fv[k] = a.tf[base + i];
                    dv[k] = a.dl[base + i];
                }
            }
#pragma unroll
            for (uint32_t k = 0; k < kPer; ++k) {
                const uint32_t i = tid + k * kSpThreads;
                if (i < E) {
                    s_ent[i] = tv[k];
                    s_tfc[i] = (fv[k] * k1p1) / (fv[k] + k1 * (omb + b * (dv[k] / avgdl)));
                }
            }
        }
        __syncthreads();
        auto term_at = [&](uint32_t e) { return staged ? s_ent[e] : a.term[base + e]; };
        const bool live = doc < nd;
        const uint32_t lo0 = live ? s_dp[doc] : 0u, hi0 = live ? s_dp[doc + 1] : 0u;
        // match map: 8 threads per document walk its entries
#ifndef BM_ABL
#define BM_ABL 0
#endif
        for (uint32_t e = lo0 + qg; e < hi0 && !(BM_ABL & 1); e += kSpThreads / kSpTile) {
            const uint32_t t = term_at(e);
            if (e > lo0 && term_at(e - 1) == t) continue;  // not the first of a run (re-added id)
            uint32_t lo = 0, hi = nu;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_ut[mid] < t) lo = mid + 1; else hi = mid;
            }
            if (lo < nu && s_ut[lo] == t) s_map[lo * kSpTile + doc] = (uint8_t)min(e - lo0 + 1u, 255u);
        }
        __syncthreads();
        const uint32_t slot = d0 + doc;
        const uint32_t qbeg = MODE == 2 ? a.dense_q : qg, qstep = MODE == 2 ? B + 1 : kSpThreads / kSpTile;
        for (uint32_t q = qbeg; q < B && !(BM_ABL & 2); q += qstep) {
            if (MODE == 2 && qg != 0) break;
            float acc = 0.0f;
            bool hit = false;
            const uint32_t p0 = s_qp[q], p1 = s_qp[q + 1];
            for (uint32_t pc = p0; pc < p1; pc += 8) {
                // 8 map lookups in flight, then the contributions in query-term order
                uint32_t vv[8];
#pragma unroll
                for (uint32_t i = 0; i < 8; ++i) {
                    const bool in = pc + i < p1;
                    const uint32_t ub = in ? s_qb[pc + i] : 0u;
                    vv[i] = in && live ? ((uint32_t)s_map[ub * kSpTile + doc] | (ub << 8)) : 0u;
                }
                // fast path, all reads independent: a staged document whose
                // entry for the term is the whole run (v < 255 and the next
                // entry holds another term) contributes tf_component[e] once
                float tf8[8];
                bool one8[8];
#pragma unroll
                for (uint32_t i = 0; i < 8; ++i) {
                    const uint32_t v = vv[i] & 255u;
                    const uint32_t e = lo0 + (v ? v - 1 : 0);
                    const bool cand = staged && v != 0 && v != 255;
                    tf8[i] = cand ? s_tfc[e] : 0.0f;
                    one8[i] = cand && (e + 1 >= hi0 || s_ent[e + 1] != s_ut[vv[i] >> 8]);
                }
#pragma unroll
                for (uint32_t i = 0; i < 8; ++i) {
                    const uint32_t v = vv[i] & 255u;
                    if (v == 0) continue;
                    const uint32_t p = pc + i;
                    if (one8[i]) {
                        const float sc = s_qv[p] * tf8[i] * s_qidf[p];
                        acc = hit ? acc + sc : 0.0f + sc;
                        hit = true;
                        continue;
                    }
                    const uint32_t t = s_ut[vv[i] >> 8];
                    uint32_t e = lo0 + v - 1;
                    if (v == 255) {  // long document: lower_bound(t)
                        uint32_t lo = lo0, hi = hi0;
                        while (lo < hi) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (term_at(mid) < t) lo = mid + 1; else hi = mid;
                        }
                        e = lo;
                    }
                    for (; e < hi0 && term_at(e) == t; ++e) {
                        const float tfc = staged ? s_tfc[e] : tfc_of(base + e);
                        // calculate_bm25_score (sparse.rs:206-222): query_tf * tf_component * idf
                        const float sc = s_qv[p] * tfc * s_qidf[p];
                        acc = hit ? acc + sc : 0.0f + sc;  // or_insert(0.0) += s
                        hit = true;
                    }
                }
            }
            const uint64_t key = hit && live ? sp_key(acc, slot) : 0ull;
            if (MODE == 0) {
                a.smp[(uint64_t)q * a.S + (uint64_t)j * kSpTile + doc] = key;
            } else if (MODE == 1) {
                if (key != 0 && key >= s_tau[q]) {
                    const uint32_t pos = atomicAdd(&a.counts[q], 1u);
                    if (pos < kSpCand) a.cand[(uint64_t)q * kSpCand + pos] = key;
                }
            } else {
                if (live) a.dense[slot] = key;
            }
        }
    }
}

// tau[q] = the kk-th largest sampled key (0 when fewer than kk matched): each
// thread keeps its top kSpTopLocal keys, an LDS sort of all of them follows.
// Any kk keys it keeps are real documents, so tau never exceeds the true
// kk-th best key; dropped keys only lower it (more candidates, still exact).
__global__ __launch_bounds__(256) void k_bm25_tau(const uint64_t* __restrict__ smp, uint32_t S, uint32_t kk,
                                                  uint64_t* __restrict__ tau) {
    __shared__ uint64_t keys[256 * kSpTopLocal];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    uint64_t top[kSpTopLocal];
#pragma unroll
    for (uint32_t i = 0; i < kSpTopLocal; ++i) top[i] = 0;
    const uint64_t* src = smp + (uint64_t)q * S;
    for (uint32_t i = tid; i < S; i += 256u) {
        uint64_t k = src[i];
        if (k <= top[kSpTopLocal - 1]) continue;
#pragma unroll
        for (uint32_t j = 0; j < kSpTopLocal; ++j) {
            const uint64_t hi = k > top[j] ? k : top[j], lo = k > top[j] ? top[j] : k;
            top[j] = hi;
            k = lo;
        }
    }
#pragma unroll
    for (uint32_t i = 0; i < kSpTopLocal; ++i) keys[tid * kSpTopLocal + i] = ~top[i];
    __syncthreads();
    bitonic_sort_lds(keys, 256 * kSpTopLocal);
    if (tid == 0) tau[q] = kk >= 1 && kk <= 256 * kSpTopLocal ? ~keys[kk - 1] : 0ull;
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
// concatenated (dense, sparse, text); the first occurrence of an id owns it.
// score: the LAST dense occurrence (HashMap::insert replaces) or else the
// first other occurrence, then += every later sparse / text occurrence in
// order; ties by first appearance.
// ---------------------------------------------------------------------------
constexpr uint32_t kRrfMax = 1024;  // items per query (LDS)

__global__ __launch_bounds__(256) void k_rrf(const uint64_t* __restrict__ ids0, const float* __restrict__ sc0,
                                             const uint32_t* __restrict__ n0, uint32_t st0,
                                             const uint64_t* __restrict__ ids1, const float* __restrict__ sc1,
                                             const uint32_t* __restrict__ n1, uint32_t st1,
                                             const uint64_t* __restrict__ ids2, const float* __restrict__ sc2,
                                             const uint32_t* __restrict__ n2, uint32_t st2, float k, uint32_t limit,
                                             uint64_t* __restrict__ out_ids, float* __restrict__ out_scores,
                                             float* __restrict__ out_raw, uint32_t* __restrict__ out_n) {
    __shared__ uint64_t s_id[kRrfMax];
    __shared__ float s_raw[kRrfMax];
    __shared__ float s_score[kRrfMax];
    __shared__ float s_bd[3][kRrfMax];
    __shared__ uint64_t s_key[kRrfMax];
    __shared__ uint32_t s_cnt;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const uint32_t a = n0 ? min(n0[q], st0) : 0u, b = n1 ? min(n1[q], st1) : 0u, c = n2 ? min(n2[q], st2) : 0u;
    const uint32_t n = min(a + b + c, kRrfMax);
    for (uint32_t i = tid; i < n; i += 256u) {
        const uint32_t l = i < a ? 0u : i < a + b ? 1u : 2u;
        const uint32_t r = l == 0 ? i : l == 1 ? i - a : i - a - b;
        s_id[i] = l == 0 ? ids0[(uint64_t)q * st0 + r] : l == 1 ? ids1[(uint64_t)q * st1 + r] : ids2[(uint64_t)q * st2 + r];
        s_raw[i] = l == 0 ? sc0[(uint64_t)q * st0 + r] : l == 1 ? sc1[(uint64_t)q * st1 + r] : sc2[(uint64_t)q * st2 + r];
    }
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    auto rrf = [&](uint32_t i) {  // 1.0 / (k + (rank + 1) as f32)
        const uint32_t r = i < a ? i : i < a + b ? i - a : i - a - b;
        return 1.0f / (k + (float)(r + 1u));
    };
    for (uint32_t i = tid; i < n; i += 256u) {
        bool owner = true;
        for (uint32_t j = 0; j < i && owner; ++j) owner = s_id[j] != s_id[i];
        if (!owner) continue;
        const uint64_t id = s_id[i];
        int32_t last_dense = -1;  // dense: HashMap::insert replaces (hybrid.rs:432-445)
        for (uint32_t j = 0; j < a; ++j)
            if (s_id[j] == id) last_dense = (int32_t)j;
        float score = 0.0f;
        bool have = false;
        float bd[3] = {__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
        if (last_dense >= 0) {
            score = rrf((uint32_t)last_dense);
            bd[0] = s_raw[last_dense];
            have = true;
        }
        for (uint32_t j = a; j < n; ++j) {  // sparse, then text: insert or += (447-478)
            if (s_id[j] != id) continue;
            const float r = rrf(j);
            score = have ? score + r : r;
            have = true;
            bd[j < a + b ? 1 : 2] = s_raw[j];
        }
        s_score[i] = score;
        s_bd[0][i] = bd[0];
        s_bd[1][i] = bd[1];
        s_bd[2][i] = bd[2];
        const uint32_t pos = atomicAdd(&s_cnt, 1u);
        s_key[pos] = ((uint64_t)(~f32_order(score)) << 32) | i;  // score desc, first appearance asc
    }
    __syncthreads();
    const uint32_t m = s_cnt;
    const uint32_t P = next_pow2(m < 2u ? 2u : m);
    for (uint32_t i = m + tid; i < P; i += 256u) s_key[i] = ~0ull;
    __syncthreads();
    bitonic_sort_lds(s_key, P);
    const uint32_t take = min(limit, m);
    for (uint32_t t = tid; t < take; t += 256u) {
        const uint32_t i = (uint32_t)s_key[t];
        const uint64_t o = (uint64_t)q * limit + t;
        out_ids[o] = s_id[i];
        out_scores[o] = s_score[i];
        if (out_raw)
            for (int l = 0; l < 3; ++l) out_raw[o * 3 + l] = s_bd[l][i];
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
    // search scratch
    void* scratch = nullptr;
    size_t scratch_n = 0;
    uint32_t* h_fail = nullptr;
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

uint32_t sp_grid(uint32_t tiles) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return std::max<uint32_t>(1, std::min<uint32_t>(tiles, 2u * (uint32_t)cus));
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
    if (e == hipSuccess) e = hipHostMalloc((void**)&sp->h_fail, kSpMaxB * 4, hipHostMallocDefault);
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
                    sp->scratch})
        if (p) (void)hipFree(p);
    if (sp->h_fail) (void)hipHostFree(sp->h_fail);
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
    if (B == 0 || limit == 0 || sp->total_documents == 0 || sp->slot_id.empty()) return GVDB_OK;
    SP_TRY(hipSetDevice(sp->device), "hipSetDevice");
    gvdb_status st = upload(sp);
    if (st != GVDB_OK) return st;
    const uint32_t N = (uint32_t)sp->slot_id.size();
    const uint32_t L = (uint32_t)limit;
    const uint32_t ntiles = (N + kSpTile - 1) / kSpTile;
    // sample stride: expected candidates ~ limit * every, kept well under kSpCand
    uint32_t every = std::max<uint32_t>(1u, std::min<uint32_t>(32u, kSpCand / std::max<uint32_t>(1u, 4u * L)));
    if (ntiles <= 8u * every) every = 1;  // small index: the sample is the whole index
    const uint32_t S = ((ntiles + every - 1) / every) * kSpTile;
    hipStream_t s = sp->stream;
    uint64_t q0 = 0;
    std::vector<uint32_t> h_qp;
    std::vector<uint32_t> h_qt;
    std::vector<float> h_qv, h_qidf;
    while (q0 < B) {
        // launch group: <= kSpMaxB queries and <= kSpQT live query terms
        h_qp.assign(1, 0);
        h_qt.clear();
        h_qv.clear();
        h_qidf.clear();
        std::vector<uint32_t> group_terms;  // distinct live terms of the group
        uint64_t q1 = q0;
        while (q1 < B && q1 - q0 < kSpMaxB) {
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
                        return report_status(GVDB_ERR_INVALID_ARGUMENT, "query has more than 512 distinct terms");
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
        const uint32_t nqt = (uint32_t)h_qt.size();
        const uint32_t nu = (uint32_t)group_terms.size();
        std::vector<uint16_t> h_qb(nqt);
        for (uint32_t i = 0; i < nqt; ++i)
            h_qb[i] = (uint16_t)(std::lower_bound(group_terms.begin(), group_terms.end(), h_qt[i]) - group_terms.begin());
        // scratch: qp | qt | qv | qidf | tau | counts | fail | out_n | smp | cand | out ids | out scores
        auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
        const size_t o_qp = 0, o_ut = o_qp + al((Bg + 1) * 4), o_qt = o_ut + al(nu * 4 + 4), o_qv = o_qt + al(nqt * 4 + 4),
                     o_qidf = o_qv + al(nqt * 4 + 4), o_tau = o_qidf + al(nqt * 4 + 4), o_cnt = o_tau + al(Bg * 8),
                     o_fail = o_cnt + al(Bg * 4), o_n = o_fail + al(Bg * 4), o_smp = o_n + al(Bg * 4),
                     o_cand = o_smp + al((size_t)Bg * S * 8), o_oi = o_cand + al((size_t)Bg * kSpCand * 8),
                     o_os = o_oi + al((size_t)Bg * L * 8), total = o_os + al((size_t)Bg * L * 4);
        if (total > sp->scratch_n) {
            if (sp->scratch) (void)hipFree(sp->scratch);
            sp->scratch = nullptr;
            sp->scratch_n = 0;
            SP_TRY(hipMalloc(&sp->scratch, total), "alloc bm25 scratch");
            sp->scratch_n = total;
        }
        char* base = (char*)sp->scratch;
        SP_TRY(hipMemcpyAsync(base + o_qp, h_qp.data(), (Bg + 1) * 4, hipMemcpyHostToDevice, s), "qp");
        if (nqt) {
            SP_TRY(hipMemcpyAsync(base + o_qt, h_qb.data(), nqt * 2, hipMemcpyHostToDevice, s), "qb");
            SP_TRY(hipMemcpyAsync(base + o_ut, group_terms.data(), nu * 4, hipMemcpyHostToDevice, s), "ut");
            SP_TRY(hipMemcpyAsync(base + o_qv, h_qv.data(), nqt * 4, hipMemcpyHostToDevice, s), "qv");
            SP_TRY(hipMemcpyAsync(base + o_qidf, h_qidf.data(), nqt * 4, hipMemcpyHostToDevice, s), "qidf");
        }
        SP_TRY(hipMemsetAsync(base + o_cnt, 0, Bg * 4, s), "counts");
        SpArgs a{};
        a.ptr = sp->d_ptr;
        a.term = sp->d_term;
        a.tf = sp->d_tf;
        a.dl = sp->d_dl;
        a.N = N;
        a.qp = (const uint32_t*)(base + o_qp);
        a.qb = (const uint16_t*)(base + o_qt);
        a.ut = (const uint32_t*)(base + o_ut);
        a.nu = nu;
        a.qv = (const float*)(base + o_qv);
        a.qidf = (const float*)(base + o_qidf);
        a.B = Bg;
        a.k1 = sp->k1;
        a.b = sp->b;
        a.avgdl = sp->avgdl;
        a.every = every;
        a.smp = (uint64_t*)(base + o_smp);
        a.S = S;
        a.tau = (const uint64_t*)(base + o_tau);
        a.counts = (uint32_t*)(base + o_cnt);
        a.cand = (uint64_t*)(base + o_cand);
        const uint32_t stiles = (ntiles + every - 1) / every;
        hipLaunchKernelGGL(k_bm25<0>, dim3(sp_grid(stiles)), dim3(kSpThreads), 0, s, a);
        SP_TRY(hipGetLastError(), "bm25 sample");
        hipLaunchKernelGGL(k_bm25_tau, dim3(Bg), dim3(256), 0, s, a.smp, S, L, (uint64_t*)(base + o_tau));
        SP_TRY(hipGetLastError(), "bm25 tau");
        hipLaunchKernelGGL(k_bm25<1>, dim3(sp_grid(ntiles)), dim3(kSpThreads), 0, s, a);
        SP_TRY(hipGetLastError(), "bm25 emit");
        uint64_t* d_oi = (uint64_t*)(base + o_oi);
        float* d_os = (float*)(base + o_os);
        uint32_t* d_n = (uint32_t*)(base + o_n);
        uint32_t* d_fail = (uint32_t*)(base + o_fail);
        hipLaunchKernelGGL(k_bm25_final, dim3(Bg), dim3(256), 0, s, a.cand, a.counts, L, sp->d_ids, d_oi, d_os, d_n,
                           d_fail);
        SP_TRY(hipGetLastError(), "bm25 final");
        SP_TRY(hipMemcpyAsync(sp->h_fail, d_fail, Bg * 4, hipMemcpyDeviceToHost, s), "fail flags");
        SP_TRY(hipStreamSynchronize(s), "sync");
        // exact fallback for overflowing queries: dense keys + radix sort
        for (uint32_t q = 0; q < Bg; ++q) {
            if (!sp->h_fail[q]) continue;
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
            hipLaunchKernelGGL(k_bm25<2>, dim3(sp_grid(ntiles)), dim3(kSpThreads), 0, s, a);
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
        SP_TRY(hipMemcpyAsync(out_ids + q0 * L, d_oi, (size_t)Bg * L * 8, hipMemcpyDeviceToHost, s), "out ids");
        SP_TRY(hipMemcpyAsync(out_scores + q0 * L, d_os, (size_t)Bg * L * 4, hipMemcpyDeviceToHost, s), "out scores");
        SP_TRY(hipMemcpyAsync(out_n + q0, d_n, (size_t)Bg * 4, hipMemcpyDeviceToHost, s), "out n");
        SP_TRY(hipStreamSynchronize(s), "sync");
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
    if (!d_out_n || (limit && (!d_out_ids || !d_out_scores)) || limit > 0xffffffffull)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "bad output arguments");
    hipLaunchKernelGGL(k_rrf, dim3((uint32_t)B), dim3(256), 0, (hipStream_t)stream, d_dense_ids, d_dense_scores,
                       d_dense_n, dense_stride, d_sparse_ids, d_sparse_scores, d_sparse_n, sparse_stride, d_text_ids,
                       d_text_scores, d_text_n, text_stride, k, (uint32_t)limit, d_out_ids, d_out_scores,
                       d_out_breakdown, d_out_n);
    SP_TRY(hipGetLastError(), "rrf");
    return GVDB_OK;
}

// Host-pointer form: stages the lists through HBM on a private stream.
gvdb_status gvdb_rrf_fuse(const uint64_t* dense_ids, const float* dense_scores, const uint32_t* dense_n,
                          uint32_t dense_stride, const uint64_t* sparse_ids, const float* sparse_scores,
                          const uint32_t* sparse_n, uint32_t sparse_stride, const uint64_t* text_ids,
                          const float* text_scores, const uint32_t* text_n, uint32_t text_stride, uint64_t B, float k,
                          uint64_t limit, uint64_t* out_ids, float* out_scores, float* out_breakdown,
                          uint32_t* out_n) {
    if (B == 0) return GVDB_OK;
    if (!out_n || (limit && (!out_ids || !out_scores))) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null output");
    struct L {
        const uint64_t* ids;
        const float* sc;
        const uint32_t* n;
        uint32_t st;
    } lists[3] = {{dense_ids, dense_scores, dense_n, dense_stride},
                  {sparse_ids, sparse_scores, sparse_n, sparse_stride},
                  {text_ids, text_scores, text_n, text_stride}};
    size_t bytes = 0;
    for (const L& l : lists)
        if (l.n) bytes += B * 4 + (size_t)B * l.st * 12 + 768;
    bytes += (size_t)B * limit * (8 + 4 + 12) + B * 4 + 1024;
    char* d = nullptr;
    hipStream_t s = nullptr;
    SP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "rrf stream");
    hipError_t e = hipMalloc((void**)&d, bytes);
    if (e != hipSuccess) {
        (void)hipStreamDestroy(s);
        return sp_dev(e, "alloc rrf");
    }
    char* p = d;
    auto take = [&](size_t n) {
        char* r = p;
        p += (n + 255) & ~(size_t)255;
        return r;
    };
    const uint64_t* dl_ids[3] = {nullptr, nullptr, nullptr};
    const float* dl_sc[3] = {nullptr, nullptr, nullptr};
    const uint32_t* dl_n[3] = {nullptr, nullptr, nullptr};
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
    float* ob = out_breakdown ? (float*)take((size_t)B * limit * 12) : nullptr;
    uint32_t* on = (uint32_t*)take(B * 4);
    gvdb_status st = GVDB_OK;
    if (e == hipSuccess)
        st = gvdb_rrf_fuse_device(dl_ids[0], dl_sc[0], dl_n[0], dense_stride, dl_ids[1], dl_sc[1], dl_n[1], sparse_stride,
                                  dl_ids[2], dl_sc[2], dl_n[2], text_stride, B, k, limit, oi, os, ob, on, s);
    if (e == hipSuccess && st == GVDB_OK) {
        if (limit) e = hipMemcpyAsync(out_ids, oi, (size_t)B * limit * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && limit) e = hipMemcpyAsync(out_scores, os, (size_t)B * limit * 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && ob) e = hipMemcpyAsync(out_breakdown, ob, (size_t)B * limit * 12, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(out_n, on, B * 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
    }
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
    if (e != hipSuccess) return sp_dev(e, "rrf");
    return st;
}

}  // extern "C"
