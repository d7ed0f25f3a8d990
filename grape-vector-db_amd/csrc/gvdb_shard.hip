// gvdb_shard.hip — the exact two-exchange sharded BQ search:
// kernels, their launchers, host forms of the two merges, and the phase-level
// C ABI (include/gvdb.h) that gvdb_index_search_sharded_device composes with
// RCCL and that a host with its own transport can drive directly.
//
// Replaces ShardManager::search_vectors (src/distributed/shard.rs:760-786:
// scatter, concat, sort, truncate) over BinaryQuantizer::multi_stage_search
// (src/quantization.rs:151-193) inside one node.  Rank g holds the contiguous
// rows [off_g, off_g + n_g) of the corpus; the concatenation in rank order is
// "the corpus" whose multi_stage_search the protocol reproduces bit for bit:
//
//   1. rank g: exact local stage-1 top-min(R, n_g) by (Hamming, row) as keys
//      (d << 32 | row)                                   -> exchange-1 block
//   2. all-gather of the exchange-1 blocks (B*R*8 B per rank)
//   3. every rank: the global top-R by (d, rank, row) -- the reference's
//      stable order by candidate index over the concatenated corpus -- and its
//      OWN entries among them (~R/G per query) with their global positions;
//      exact cosine of those rows only (k_rerank), then its local top-k by
//      (cosine desc, position asc)                       -> exchange-2 block
//   4. all-gather of the exchange-2 blocks (B*k*16 B per rank)
//   5. every rank: merge of the G local top-k lists = the first k of the
//      stable cosine sort of the global top-R (every entry of the global top-k
//      is in its owner's local top-k); take(k) then drop orphan rows, as the
//      single-index search does.
//
// The rerank per rank shrinks with G (R/G rows instead of R) and the second
// exchange carries k entries per query instead of R.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/gvdb.h"
#include "gvdb_device.h"
#include "gvdb_internal.h"

namespace gvdb {

constexpr uint32_t kShardMaxG = 1024;   // ranks (the merge key holds 16 bits of rank)
constexpr uint32_t kShardMaxD = 8192;   // distance histogram of the merge in LDS (key field: 16 bits)

// ---- step 3: one kernel per query -- global top-R, rerank of the owned rows, local top-k
// Every list is sorted by (d, row).  (i) A histogram of the distances of all
// G lists gives the R-th smallest distance T of the union; list g contributes
// its a_g entries with d < T and then, in rank order, ties at T until R are
// taken -- exactly the first R of the union in (d, rank, row) order, and a
// PREFIX of every list.  (ii) This rank's owned entries are the prefix of its
// own list; the global position of each is its index plus, for every other
// list, the count of its selected keys below it (binary searches in LDS).
// (iii) Exact cosine of the owned rows, 16 at a time: the rows stream through
// LDS in 256-dimension chunks, lane r < 16 folds row r in the reference's
// order (acc = acc + q_j * x_j from -0.0), lane 16 folds q_j * q_j.  (iv) The
// owned entries sorted by (cosine desc, position) -> the first k go to the
// exchange-2 block.
// LDS (dynamic): hist [(D+4)&~3] | lg, eg, bg, cg [G] | sel u64 [R] | tile; the owned
// positions / rows go to global scratch (opos, orow [B][R]).
constexpr uint32_t kP2Threads = 256;
constexpr uint32_t kP2Rows = 16;    // rows re-scored together
constexpr uint32_t kP2Ch = 256;     // dimensions per LDS chunk
constexpr uint32_t kP2Ld = kP2Ch + 4;
constexpr uint32_t kP2AllCap = 4096;  // keys of all lists staged in LDS up to this many
__global__ __launch_bounds__(kP2Threads) void k_shard_phase2(const uint32_t* __restrict__ gathered, uint64_t words1,
                                                             uint32_t G, uint32_t me, uint32_t B, uint32_t R,
                                                             uint32_t D, const float* __restrict__ rows,
                                                             const float* __restrict__ norms,
                                                             const uint64_t* __restrict__ ids,
                                                             const float* __restrict__ queries, uint32_t k,
                                                             uint32_t err, uint32_t* __restrict__ block2,
                                                             uint32_t* __restrict__ opos_g,
                                                             uint32_t* __restrict__ orow_g) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* hist = lds;
    uint32_t* lg = hist + ((D + 4u) & ~3u);
    uint32_t* eg = lg + G;
    uint32_t* bg = eg + G;
    uint32_t* cg = bg + G;
    uint64_t* sel = (uint64_t*)(((uintptr_t)(cg + G) + 15) & ~(uintptr_t)15);
    float* tile = (float*)(((uintptr_t)(sel + R) + 15) & ~(uintptr_t)15);  // [kP2Rows][kP2Ld]
    float* qs = tile + kP2Rows * kP2Ld;                                       // [kP2Ch]
    uint64_t* allk = (uint64_t*)(qs + kP2Ch);  // [G*R] every list's keys, when G*R <= kP2AllCap
    const bool staged = G * R <= kP2AllCap;
    __shared__ uint32_t s_total, s_T, s_lt, s_nan, s_rows[kP2Rows];
    __shared__ float s_cos[kP2Rows], s_qq;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    uint32_t* opos = opos_g + (uint64_t)q * R;
    uint32_t* orow = orow_g + (uint64_t)q * R;
    auto glist = [&](uint32_t g) { return (const uint64_t*)(gathered + (uint64_t)g * words1) + (uint64_t)q * R; };
    auto key_at = [&](uint32_t g, uint32_t i) { return staged ? allk[g * R + i] : glist(g)[i]; };
    for (uint32_t i = tid; i <= D; i += kP2Threads) hist[i] = 0u;
    if (tid == 0) {
        s_total = 0u;
        s_nan = 0u;
    }
    __syncthreads();
    for (uint32_t g = tid; g < G; g += kP2Threads) {
        const uint32_t c = min(gathered[(uint64_t)g * words1 + 2ull * B * R + q], R);
        cg[g] = c;
        lg[g] = 0u;
        eg[g] = 0u;
        atomicAdd(&s_total, c);
    }
    __syncthreads();
    // (i) histogram of every list's distances: one flat pass (all loads in flight),
    //     the keys staged in LDS for the passes below
    for (uint32_t x = tid; x < G * R; x += kP2Threads) {
        const uint32_t g = x / R, i = x - g * R;
        if (i < cg[g]) {
            const uint64_t key = glist(g)[i];
            if (staged) allk[x] = key;
            atomicAdd(&hist[min((uint32_t)(key >> 32), D)], 1u);
        }
    }
    __syncthreads();
    const uint32_t Re = min(R, s_total);
    uint32_t* meta = block2 + 4ull * B * k;
    if (Re == 0) {
        if (tid == 0) {
            meta[q] = 0u;
            meta[B + q] = 0u;
            if (q == 0) meta[2 * B] = err;
        }
        return;
    }
    if (tid < 64) {
        const uint32_t t = wave_find_cum(hist, D + 1u, Re);
        const uint32_t lt = wave_sum_below(hist, t);
        if (tid == 0) {
            s_T = t;
            s_lt = lt;
        }
    }
    __syncthreads();
    const uint32_t T = s_T;
    for (uint32_t x = tid; x < G * R; x += kP2Threads) {
        const uint32_t g = x / R, i = x - g * R;
        if (i < cg[g]) {
            const uint32_t d = (uint32_t)(key_at(g, i) >> 32);
            if (d < T) atomicAdd(&lg[g], 1u);
            else if (d == T) atomicAdd(&eg[g], 1u);
        }
    }
    __syncthreads();
    if (tid == 0) {  // ties at T go to the lowest ranks first (rank order = corpus order)
        uint32_t need = Re - s_lt, base = 0;
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t t = min(eg[g], need);
            need -= t;
            eg[g] = lg[g] + t;  // the selected prefix of list g
            bg[g] = base;
            base += eg[g];
        }
    }
    __syncthreads();
    for (uint32_t x = tid; x < G * R; x += kP2Threads) {
        const uint32_t g = x / R, i = x - g * R;
        if (i < eg[g]) {
            const uint64_t key = key_at(g, i);
            sel[bg[g] + i] = ((key >> 32) << 48) | ((uint64_t)g << 32) | (key & 0xffffffffull);
        }
    }
    __syncthreads();
    // (ii) global positions of the owned entries (the prefix of this rank's list)
    const uint32_t c = eg[me];
    for (uint32_t i = tid; i < c; i += kP2Threads) {
        const uint64_t key = sel[bg[me] + i];
        uint32_t pos = i;
        for (uint32_t g = 0; g < G; ++g) {
            if (g == me) continue;
            uint32_t lo = 0, hi = eg[g];
            const uint64_t* L = sel + bg[g];
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (L[mid] < key) lo = mid + 1; else hi = mid;
            }
            pos += lo;
        }
        opos[i] = pos;
        orow[i] = (uint32_t)key;
    }
    __syncthreads();
    // (iii) exact cosine of the owned rows, kP2Rows at a time (scores into the sel area)
    float* cosv = (float*)sel;
    const float* qv = queries + (uint64_t)q * D;
    const uint32_t nch = (D + kP2Ch - 1) / kP2Ch;
    constexpr uint32_t kPer = kP2Rows * kP2Ch / kP2Threads;  // floats per thread per chunk (16)
    for (uint32_t r0 = 0; r0 < c; r0 += kP2Rows) {
        const uint32_t nr = min(kP2Rows, c - r0);
        float acc = -0.0f;
        float x[kPer];
        if (tid < kP2Rows) s_rows[tid] = tid < nr ? (uint32_t)sel[bg[me] + r0 + tid] : 0u;
        __syncthreads();
        auto load = [&](uint32_t ch) {
#pragma unroll
            for (uint32_t e = 0; e < kPer; ++e) {
                const uint32_t f = tid + e * kP2Threads, r = f / kP2Ch, j = ch * kP2Ch + (f % kP2Ch);
                x[e] = (r < nr && j < D) ? rows[(uint64_t)s_rows[r] * D + j] : 0.0f;
            }
        };
        load(0);
        for (uint32_t ch = 0; ch < nch; ++ch) {
#pragma unroll
            for (uint32_t e = 0; e < kPer; ++e) {
                const uint32_t f = tid + e * kP2Threads;
                tile[(f / kP2Ch) * kP2Ld + (f % kP2Ch)] = x[e];
            }
            qs[tid] = ch * kP2Ch + tid < D ? qv[ch * kP2Ch + tid] : 0.0f;  // kP2Threads == kP2Ch
            __syncthreads();
            if (ch + 1 < nch) load(ch + 1);  // next chunk in flight during the folds
            const uint32_t m = min(kP2Ch, D - ch * kP2Ch);
            // lanes < 16 fold their row, lane 16 the query norm (group 0): the
            // reference's left-to-right order; float4 LDS reads, 8 in flight
            const bool fold_q = tid == kP2Rows && r0 == 0;
            if (tid < nr || fold_q) {
                const float* tr = fold_q ? qs : tile + tid * kP2Ld;
                float a2 = fold_q ? (ch == 0 ? -0.0f : s_qq) : acc;
                uint32_t j = 0;
                if (m == kP2Ch) {
#pragma unroll 8
                    for (; j < kP2Ch; j += 4) {
                        const float4 x4 = *(const float4*)(tr + j);
                        const float4 w4 = *(const float4*)(qs + j);
                        a2 = a2 + w4.x * x4.x;
                        a2 = a2 + w4.y * x4.y;
                        a2 = a2 + w4.z * x4.z;
                        a2 = a2 + w4.w * x4.w;
                    }
                }
                for (; j < m; ++j) a2 = a2 + qs[j] * tr[j];
                if (fold_q) s_qq = a2; else acc = a2;
            }
            __syncthreads();
        }
        if (tid < nr) {
            const float na = sqrtf(s_qq), nb = norms[orow[r0 + tid]];
            const float sc = (na == 0.0f || nb == 0.0f) ? 0.0f : acc / (na * nb);
            s_cos[tid] = sc;
        }
        __syncthreads();
        if (tid < nr) {
            cosv[r0 + tid] = s_cos[tid];  // bytes below every sel entry a later group reads
            if (s_cos[tid] != s_cos[tid]) s_nan = 1u;
        }
        __syncthreads();
    }
    // (iv) local top-k by (cosine desc, global position): keys (~order(cos), pos, owned
    //      index) sorted in the tile area (up to 2080 keys; more owned entries: scans)
    const uint32_t P = next_pow2(max(c, 1u));
    const uint32_t* rows_keep = orow;
    uint64_t* keys = (uint64_t*)tile;
    const bool keys_fit = P <= kP2Rows * kP2Ld / 2;
    if (keys_fit) {
        for (uint32_t i = tid; i < P; i += kP2Threads)
            keys[i] = i < c ? ((uint64_t)~f32_order(cosv[i]) << 32) | ((uint64_t)opos[i] << 13) | i : ~0ull;
        __syncthreads();
        if (c > 1) bitonic_sort_lds(keys, P);
    }
    const uint32_t take = min(k, c);
    uint32_t* ent = block2 + (uint64_t)q * k * 4u;
    if (keys_fit) {
        for (uint32_t t = tid; t < take; t += kP2Threads) {
            const uint32_t j = (uint32_t)keys[t] & 0x1fffu;
            const uint32_t row = rows_keep[j];
            const uint64_t id = ids ? ids[row] : (uint64_t)row;
            ent[4 * t + 0] = __float_as_uint(cosv[j]);
            ent[4 * t + 1] = opos[j];
            ent[4 * t + 2] = (uint32_t)id;
            ent[4 * t + 3] = (uint32_t)(id >> 32);
        }
    } else if (tid == 0) {
        // many owned entries (a skewed shard): selection of the k best by repeated scans
        uint64_t prev = 0;
        for (uint32_t t = 0; t < take; ++t) {
            uint64_t best = ~0ull;
            for (uint32_t i = 0; i < c; ++i) {
                const uint64_t key = ((uint64_t)~f32_order(cosv[i]) << 32) | ((uint64_t)opos[i] << 13) | i;
                if ((t == 0 || key > prev) && key < best) best = key;
            }
            prev = best;
            const uint32_t j = (uint32_t)best & 0x1fffu;
            const uint32_t row = rows_keep[j];
            const uint64_t id = ids ? ids[row] : (uint64_t)row;
            ent[4 * t + 0] = __float_as_uint(cosv[j]);
            ent[4 * t + 1] = opos[j];
            ent[4 * t + 2] = (uint32_t)id;
            ent[4 * t + 3] = (uint32_t)(id >> 32);
        }
    }
    if (tid == 0) {
        meta[q] = take | ((s_nan && Re >= 2u) ? 0x80000000u : 0u);
        meta[B + q] = Re;
        if (q == 0) meta[2 * B] = err;
    }
}

size_t shard_phase2_lds(uint32_t G, uint32_t R, uint32_t D) {
    return (size_t)((D + 4u) & ~3u) * 4u + 4u * (size_t)G * 4u + 16u + (size_t)R * 8u + 16u +
           (size_t)(kP2Rows * kP2Ld + kP2Ch) * 4u + (G * R <= kP2AllCap ? (size_t)G * R * 8u : 0u);
}

hipError_t launch_shard_phase2(const uint32_t* gathered1, uint64_t words1, uint32_t G, uint32_t me, uint32_t B,
                               uint32_t R, uint32_t D, const float* rows, const float* norms, const uint64_t* ids,
                               const float* queries, uint32_t k, uint32_t err, uint32_t* block2, uint32_t* opos,
                               uint32_t* orow, hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_shard_phase2, dim3(B), dim3(kP2Threads), shard_phase2_lds(G, R, D), s, gathered1, words1, G,
                       me, B, R, D, rows, norms, ids, queries, k, err, block2, opos, orow);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ---- step 5: merge of the gathered exchange-2 blocks ---------------------------
// Per query the G local top-k lists; keys (~order(cos) << 32 | pos << 18 | idx)
// with idx = g * k + i (< 2^18), sorted, first k, orphans dropped after the
// truncation.  Poisoned (out_n = GVDB_N_POISONED) if a rank saw a NaN or
// reported a local failure.
__global__ __launch_bounds__(256) void k_shard_final(const uint32_t* __restrict__ gathered, uint64_t words2,
                                                     uint32_t G, uint32_t B, uint32_t k, uint64_t* __restrict__ out_ids,
                                                     float* __restrict__ out_scores, uint32_t* __restrict__ out_n) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];  // [next_pow2(G * k)]
    __shared__ uint32_t s_bad;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) s_bad = 0u;
    __syncthreads();
    for (uint32_t g = tid; g < G; g += 256) {
        const uint32_t* meta = gathered + (uint64_t)g * words2 + 4ull * B * k;
        if ((meta[q] >> 31) || meta[2 * B]) atomicOr(&s_bad, 1u);
    }
    const uint32_t n = G * k;
    for (uint32_t x = tid; x < n; x += 256) {
        const uint32_t g = x / k, i = x % k;
        const uint32_t* blk = gathered + (uint64_t)g * words2;
        const uint32_t cnt = blk[4ull * B * k + q] & 0x7fffffffu;
        uint64_t key = ~0ull;
        if (i < cnt) {
            const uint32_t* e = blk + ((uint64_t)q * k + i) * 4u;
            key = ((uint64_t)~f32_order(__uint_as_float(e[0])) << 32) | ((uint64_t)e[1] << 18) | x;
        }
        sk[x] = key;
    }
    const uint32_t P = next_pow2(max(n, 1u));
    for (uint32_t i = n + tid; i < P; i += 256) sk[i] = ~0ull;
    __syncthreads();
    bitonic_sort_lds(sk, P);
    if (tid < 64) {  // take(k), then drop orphans (order-preserving ballot compaction)
        uint32_t o = 0;
        for (uint32_t i0 = 0; i0 < k; i0 += 64) {
            const uint32_t i = i0 + tid;
            const uint64_t key = i < k ? sk[i] : ~0ull;
            uint64_t id = kOrphan;
            float sc = 0.0f;
            if (key != ~0ull) {
                const uint32_t x = (uint32_t)key & 0x3ffffu, g = x / k, j = x % k;
                const uint32_t* e = gathered + (uint64_t)g * words2 + ((uint64_t)q * k + j) * 4u;
                id = (uint64_t)e[2] | ((uint64_t)e[3] << 32);
                sc = __uint_as_float(e[0]);
            }
            const bool keep = id != kOrphan;
            const uint64_t m = __ballot(keep);
            const uint32_t before = __popcll(m & ((1ull << tid) - 1ull));
            if (keep) {
                out_ids[(uint64_t)q * k + o + before] = id;
                out_scores[(uint64_t)q * k + o + before] = sc;
            }
            o += __popcll(m);
        }
        if (tid == 0 && out_n) out_n[q] = s_bad ? GVDB_N_POISONED : o;
    }
}

hipError_t launch_shard_final(const uint32_t* gathered2, uint64_t words2, uint32_t G, uint32_t B, uint32_t k,
                              uint64_t* out_ids, float* out_scores, uint32_t* out_n, hipStream_t s) {
    if (B == 0) return hipSuccess;
    const size_t lds = (size_t)next_pow2(std::max<uint32_t>(G * k, 1u)) * 8u;
    hipLaunchKernelGGL(k_shard_final, dim3(B), dim3(256), lds, s, gathered2, words2, G, B, k, out_ids, out_scores,
                       out_n);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ---- sharded FLAT: merge of the G local exact top-k lists ----------------------
// Block F (u32 words): ids u64 [B][k] | scores f32 [B][k] | counts u32 [B] | err | pad.
// Each rank's list is its exact top-k by (score, row); the merge orders by
// (score, rank, list index) = (score, corpus row), the single-index order over
// the concatenated corpus (storage.rs:331-336 stable sort, shard.rs:776-784
// concat + sort + truncate).

__global__ __launch_bounds__(256) void k_shard_flat_final(const uint32_t* __restrict__ gathered, uint64_t words,
                                                          uint32_t G, uint32_t B, uint32_t k, int descending,
                                                          uint64_t* __restrict__ out_ids,
                                                          float* __restrict__ out_scores, uint32_t* __restrict__ out_n) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];
    __shared__ uint32_t s_bad;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) s_bad = 0u;
    __syncthreads();
    const uint32_t n = G * k;
    for (uint32_t x = tid; x < n; x += 256) {
        const uint32_t g = x / k, i = x % k;
        const uint32_t* blk = gathered + (uint64_t)g * words;
        const uint32_t raw = blk[3ull * B * k + q];
        if (i == 0 && (blk[3ull * B * k + B] || raw == GVDB_N_POISONED)) atomicOr(&s_bad, 1u);
        const uint32_t cnt = raw == GVDB_N_POISONED ? 0u : min(raw, k);
        uint64_t key = ~0ull;
        if (i < cnt) {
            uint32_t o = f32_order(__uint_as_float(blk[2ull * B * k + (uint64_t)q * k + i]));
            if (descending) o = ~o;
            key = ((uint64_t)o << 32) | x;  // x = g*k + i: rank, then list order
        }
        sk[x] = key;
    }
    const uint32_t P = next_pow2(max(n, 1u));
    for (uint32_t i = n + tid; i < P; i += 256) sk[i] = ~0ull;
    __syncthreads();
    bitonic_sort_lds(sk, P);
    uint32_t o = 0;
    for (uint32_t i = tid; i < k; i += 256) {
        const uint64_t key = sk[i];
        if (key == ~0ull) continue;
        const uint32_t x = (uint32_t)key, g = x / k, j = x % k;
        const uint32_t* blk = gathered + (uint64_t)g * words;
        out_ids[(uint64_t)q * k + i] = ((const uint64_t*)blk)[(uint64_t)q * k + j];
        out_scores[(uint64_t)q * k + i] = __uint_as_float(blk[2ull * B * k + (uint64_t)q * k + j]);
    }
    if (tid == 0 && out_n) {
        for (uint32_t i = 0; i < k && sk[i] != ~0ull; ++i) ++o;
        out_n[q] = s_bad ? GVDB_N_POISONED : o;
    }
}

hipError_t launch_shard_flat_final(const uint32_t* gathered, uint64_t words, uint32_t G, uint32_t B, uint32_t k,
                                   int descending, uint64_t* out_ids, float* out_scores, uint32_t* out_n,
                                   hipStream_t s) {
    if (B == 0) return hipSuccess;
    const size_t lds = (size_t)next_pow2(std::max<uint32_t>(G * k, 1u)) * 8u;
    hipLaunchKernelGGL(k_shard_flat_final, dim3(B), dim3(256), lds, s, gathered, words, G, B, k, descending, out_ids,
                       out_scores, out_n);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ---- host forms of the merges (same block layouts; CPU transports and tests) -----
namespace {
inline uint32_t f32_order_h(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if (u == 0x80000000u) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
}  // namespace

}  // namespace gvdb

using namespace gvdb;

extern "C" {

void gvdb_shard_sizes(uint64_t B, uint64_t R, uint64_t k, uint64_t* words1, uint64_t* words2,
                      uint64_t* scratch_bytes) {
    if (words1) *words1 = shard_words1(B, R);
    if (words2) *words2 = shard_words2(B, k);
    // the owned positions and rows [B][R] of phase 2
    if (scratch_bytes) *scratch_bytes = 8 * B * R + 256;
}

uint64_t gvdb_shard_flat_words(uint64_t B, uint64_t k) { return shard_words_flat(B, k); }

gvdb_status gvdb_shard_stage1_device(const gvdb_index* shard, const float* d_queries, uint64_t B, uint32_t dim,
                                     uint64_t R, uint32_t* d_block1, void* stream) {
    if (!shard || !d_block1 || (B && !d_queries)) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (B == 0) return GVDB_OK;
    if (R == 0 || R > kSelectLdsCap) return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: 1 <= R <= 8192");
    hipStream_t s = (hipStream_t)stream;
    const ShardInfo si = index_shard_info(shard);
    if (hipSetDevice(si.device) != hipSuccess) return report_status(GVDB_ERR_DEVICE, "hipSetDevice");
    const uint64_t BR = B * R;
    uint32_t* counts = d_block1 + 2 * BR;
    gvdb_status st = GVDB_OK;
    if (si.n > 0 && dim > kShardMaxD) st = report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: dim > 8192");
    if (st == GVDB_OK) st = shard_stage1_keys(shard, d_queries, B, dim, R, reinterpret_cast<uint64_t*>(d_block1), s);
    // every rank joins the exchange: a failed or empty shard contributes no
    // entries (and a failure flag that poisons every query of the merge)
    // (k_select writes the counts of a searched shard; err is informational: a
    // failure is propagated through the exchange-2 block)
    if (st != GVDB_OK || si.n == 0) {
        if (hipMemsetD32Async(counts, 0, B, s) != hipSuccess ||
            hipMemsetD32Async(counts + B, st == GVDB_OK ? 0 : 1, 1, s) != hipSuccess)
            return report_status(GVDB_ERR_DEVICE, "sharded stage 1: counts");
    }
    return st;
}

gvdb_status gvdb_shard_rerank_device(const gvdb_index* shard, const float* d_queries, uint64_t B, uint32_t dim,
                                     uint64_t R, uint64_t k, const uint32_t* d_gathered1, uint64_t G, uint64_t rank,
                                     void* d_scratch, uint32_t* d_block2, void* stream) {
    if (!shard || !d_gathered1 || !d_scratch || !d_block2 || (B && !d_queries))
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (B == 0) return GVDB_OK;
    if (R == 0 || R > kSelectLdsCap || k == 0 || G == 0 || G > kShardMaxG || rank >= G || G * k > kSelectLdsCap ||
        B > 0xFFFFFFFFull || dim == 0 || dim > kShardMaxD)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: bad R / k / G / rank / dim");
    hipStream_t s = (hipStream_t)stream;
    const ShardInfo si = index_shard_info(shard);
    if (hipSetDevice(si.device) != hipSuccess) return report_status(GVDB_ERR_DEVICE, "hipSetDevice");
    const uint64_t BR = B * R;
    uint32_t* opos = (uint32_t*)d_scratch;
    uint32_t* orow = opos + BR;
    // a shard that cannot rerank (empty, or a dimension mismatch already reported by
    // phase 1) sent no entries, so it owns none: its rows are never read
    const bool usable = si.n > 0 && si.dim == dim;
    const hipError_t e = launch_shard_phase2(d_gathered1, shard_words1(B, R), (uint32_t)G, (uint32_t)rank, (uint32_t)B,
                                             (uint32_t)R, dim, usable ? si.rows : nullptr,
                                             usable ? si.norms : nullptr, usable ? si.ids : nullptr, d_queries,
                                             (uint32_t)k, 0u, d_block2, opos, orow, s);
    if (e != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("shard phase 2: ") + hipGetErrorString(e));
    if (usable) index_track_use(shard, s);
    return GVDB_OK;
}

gvdb_status gvdb_shard_final_device(const uint32_t* d_gathered2, uint64_t G, uint64_t B, uint64_t k,
                                    uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n, void* stream) {
    if (B == 0) return GVDB_OK;
    if (!d_gathered2 || !d_out_ids || !d_out_scores) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (k == 0 || G == 0 || G * k > kSelectLdsCap) return report_status(GVDB_ERR_INVALID_ARGUMENT, "bad G / k");
    hipError_t e = launch_shard_final(d_gathered2, shard_words2(B, k), (uint32_t)G, (uint32_t)B, (uint32_t)k, d_out_ids,
                                      d_out_scores, d_out_n, (hipStream_t)stream);
    if (e != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("shard final: ") + hipGetErrorString(e));
    return GVDB_OK;
}

gvdb_status gvdb_shard_flat_final_device(const uint32_t* d_gathered, uint64_t G, uint64_t B, uint64_t k,
                                         uint32_t metric, uint64_t* d_out_ids, float* d_out_scores, uint32_t* d_out_n,
                                         void* stream) {
    if (B == 0) return GVDB_OK;
    if (!d_gathered || !d_out_ids || !d_out_scores) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (k == 0 || G == 0 || G * k > kSelectLdsCap) return report_status(GVDB_ERR_INVALID_ARGUMENT, "bad G / k");
    hipError_t e = launch_shard_flat_final(d_gathered, shard_words_flat(B, k), (uint32_t)G, (uint32_t)B, (uint32_t)k,
                                           metric == GVDB_METRIC_COSINE, d_out_ids, d_out_scores, d_out_n,
                                           (hipStream_t)stream);
    if (e != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("shard flat merge: ") + hipGetErrorString(e));
    return GVDB_OK;
}

// Host form of k_shard_merge: this rank's owned entries of the global top-R.
gvdb_status gvdb_shard_merge_host(const uint32_t* gathered1, uint64_t G, uint64_t rank, uint64_t B, uint64_t R,
                                  uint32_t* own_rows, uint32_t* own_pos, uint32_t* own_cnt, uint32_t* reff) {
    if (!gathered1 || !own_rows || !own_pos || !own_cnt || !reff) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    const uint64_t w1 = shard_words1(B, R);
    std::vector<std::pair<uint64_t, uint32_t>> all;  // ((d, rank, row) key, -)
    for (uint64_t q = 0; q < B; ++q) {
        all.clear();
        for (uint64_t g = 0; g < G; ++g) {
            const uint32_t* blk = gathered1 + g * w1;
            const uint64_t c = std::min<uint64_t>(blk[2 * B * R + q], R);
            const uint64_t* L = (const uint64_t*)blk + q * R;
            for (uint64_t i = 0; i < c; ++i)
                all.push_back({((L[i] >> 32) << 48) | (g << 32) | (L[i] & 0xffffffffull), 0u});
        }
        std::sort(all.begin(), all.end());
        const uint64_t re = std::min<uint64_t>(R, all.size());
        uint32_t c = 0;
        for (uint64_t p = 0; p < re; ++p) {
            if (((all[p].first >> 32) & 0xffffu) == rank) {
                own_rows[q * R + c] = (uint32_t)all[p].first;
                own_pos[q * R + c] = (uint32_t)p;
                ++c;
            }
        }
        own_cnt[q] = c;
        reff[q] = (uint32_t)re;
    }
    return GVDB_OK;
}

// Host form of k_shard_local_topk: scores / ids of the owned entries (in
// own_pos order) -> this rank's exchange-2 block.
gvdb_status gvdb_shard_local_topk_host(const float* scores, const uint32_t* own_pos, const uint64_t* own_ids,
                                       const uint32_t* own_cnt, const uint32_t* reff, uint64_t B, uint64_t R,
                                       uint64_t k, uint32_t err, uint32_t* block2) {
    if (!scores || !own_pos || !own_ids || !own_cnt || !reff || !block2)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    uint32_t* meta = block2 + 4 * B * k;
    std::vector<std::pair<uint64_t, uint32_t>> v;
    for (uint64_t q = 0; q < B; ++q) {
        const uint64_t c = std::min<uint64_t>(own_cnt[q], R);
        v.clear();
        bool nan = false;
        for (uint64_t i = 0; i < c; ++i) {
            const float f = scores[q * R + i];
            nan |= f != f;
            v.push_back({((uint64_t)~f32_order_h(f) << 32) | own_pos[q * R + i], (uint32_t)i});
        }
        std::sort(v.begin(), v.end());
        const uint64_t take = std::min<uint64_t>(k, c);
        for (uint64_t i = 0; i < take; ++i) {
            const uint32_t j = v[i].second;
            uint32_t* e = block2 + (q * k + i) * 4;
            std::memcpy(&e[0], &scores[q * R + j], 4);
            e[1] = own_pos[q * R + j];
            e[2] = (uint32_t)own_ids[q * R + j];
            e[3] = (uint32_t)(own_ids[q * R + j] >> 32);
        }
        meta[q] = (uint32_t)take | ((nan && reff[q] >= 2) ? 0x80000000u : 0u);
        meta[B + q] = reff[q];
    }
    meta[2 * B] = err;
    return GVDB_OK;
}

// Host form of k_shard_final.
gvdb_status gvdb_shard_final_host(const uint32_t* gathered2, uint64_t G, uint64_t B, uint64_t k, uint64_t* out_ids,
                                  float* out_scores, uint32_t* out_n) {
    if (!gathered2 || !out_ids || !out_scores || !out_n) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    const uint64_t w2 = shard_words2(B, k);
    std::vector<std::pair<uint64_t, uint64_t>> v;  // (order key, (g, i))
    for (uint64_t q = 0; q < B; ++q) {
        v.clear();
        bool bad = false;
        for (uint64_t g = 0; g < G; ++g) {
            const uint32_t* blk = gathered2 + g * w2;
            const uint32_t* meta = blk + 4 * B * k;
            bad |= (meta[q] >> 31) || meta[2 * B];
            const uint64_t c = meta[q] & 0x7fffffffu;
            for (uint64_t i = 0; i < c && i < k; ++i) {
                const uint32_t* e = blk + (q * k + i) * 4;
                float f;
                std::memcpy(&f, &e[0], 4);
                v.push_back({((uint64_t)~f32_order_h(f) << 32) | e[1], g * k + i});
            }
        }
        std::sort(v.begin(), v.end());
        uint32_t o = 0;
        for (uint64_t i = 0; i < k && i < v.size(); ++i) {
            const uint64_t g = v[i].second / k, j = v[i].second % k;
            const uint32_t* e = gathered2 + g * w2 + (q * k + j) * 4;
            const uint64_t id = (uint64_t)e[2] | ((uint64_t)e[3] << 32);
            if (id == kOrphan) continue;
            out_ids[q * k + o] = id;
            std::memcpy(&out_scores[q * k + o], &e[0], 4);
            ++o;
        }
        out_n[q] = bad ? GVDB_N_POISONED : o;
    }
    return GVDB_OK;
}

}  // extern "C"
