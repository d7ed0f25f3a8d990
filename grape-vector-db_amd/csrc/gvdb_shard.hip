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

// ---- step 3a: merge of the gathered exchange-1 blocks ---------------------------
// One block per query.  Every list is sorted by (d, row), so after the R-th
// smallest distance T of the union is known (LDS histogram), list g contributes
// its a_g entries with d < T and then, in rank order, ties at T until R
// entries are taken -- exactly the first R of the union in (d, rank, row)
// order.  Those R keys (d << 48 | rank << 32 | row) are sorted in LDS to get
// each one's global position.  LDS: keys [8192] u64, hist [D + 1], per-list
// [3 * G].
__global__ __launch_bounds__(256) void k_shard_merge(const uint32_t* __restrict__ gathered, uint64_t words1,
                                                     uint32_t G, uint32_t me, uint32_t B, uint32_t R, uint32_t D,
                                                     uint32_t* __restrict__ own_rows, uint32_t* __restrict__ own_pos,
                                                     uint32_t* __restrict__ own_cnt, uint32_t* __restrict__ reff) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];  // [kSelectLdsCap]
    uint32_t* hist = (uint32_t*)(sk + kSelectLdsCap);               // [D + 1]
    uint32_t* lg = hist + ((D + 4u) & ~3u);                          // [G] count of d < T
    uint32_t* eg = lg + G;                                           // [G] count of d == T
    uint32_t* bg = eg + G;                                           // [G] first slot in sk
    __shared__ uint32_t s_total, s_own, s_T, s_lt;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    auto list = [&](uint32_t g) { return (const uint64_t*)(gathered + (uint64_t)g * words1) + (uint64_t)q * R; };
    auto count = [&](uint32_t g) { return min(gathered[(uint64_t)g * words1 + 2ull * B * R + q], R); };
    for (uint32_t i = tid; i <= D; i += 256) hist[i] = 0u;
    if (tid == 0) {
        s_total = 0u;
        s_own = 0u;
    }
    __syncthreads();
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t c = count(g);
        const uint64_t* L = list(g);
        for (uint32_t i = tid; i < c; i += 256) atomicAdd(&hist[min((uint32_t)(L[i] >> 32), D)], 1u);
        if (tid == 0) s_total += c;
    }
    __syncthreads();
    const uint32_t Re = min(R, s_total);
    if (Re == 0) {
        if (tid == 0) {
            own_cnt[q] = 0u;
            reff[q] = 0u;
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
    // per list: entries below T and tied at T (binary searches on the sorted d field)
    for (uint32_t g = tid; g < G; g += 256) {
        const uint32_t c = count(g);
        const uint64_t* L = list(g);
        uint32_t lo = 0, hi = c;  // first index with d >= T
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint32_t)(L[mid] >> 32) < T) lo = mid + 1; else hi = mid;
        }
        const uint32_t a = lo;
        hi = c;  // first index with d > T
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint32_t)(L[mid] >> 32) <= T) lo = mid + 1; else hi = mid;
        }
        lg[g] = a;
        eg[g] = lo - a;
    }
    __syncthreads();
    if (tid == 0) {  // ties at T go to the lowest ranks first (rank order = corpus order)
        uint32_t need = Re - s_lt, base = 0;
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t t = min(eg[g], need);
            need -= t;
            bg[g] = base;
            eg[g] = lg[g] + t;  // entries taken from list g
            base += eg[g];
        }
    }
    __syncthreads();
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t take = eg[g], b0 = bg[g];
        const uint64_t* L = list(g);
        for (uint32_t i = tid; i < take; i += 256) {
            const uint64_t k = L[i];
            sk[b0 + i] = ((k >> 32) << 48) | ((uint64_t)g << 32) | (k & 0xffffffffull);
        }
    }
    const uint32_t P = next_pow2(Re);
    for (uint32_t i = Re + tid; i < P; i += 256) sk[i] = ~0ull;
    __syncthreads();
    bitonic_sort_lds(sk, P);
    for (uint32_t p = tid; p < Re; p += 256) {
        const uint64_t k = sk[p];
        if (((uint32_t)(k >> 32) & 0xffffu) == me) {
            const uint32_t c = atomicAdd(&s_own, 1u);
            own_rows[(uint64_t)q * R + c] = (uint32_t)k;
            own_pos[(uint64_t)q * R + c] = p;
        }
    }
    __syncthreads();
    if (tid == 0) {
        own_cnt[q] = s_own;
        reff[q] = Re;
    }
}

hipError_t launch_shard_merge(const uint32_t* gathered1, uint64_t words1, uint32_t G, uint32_t me, uint32_t B,
                              uint32_t R, uint32_t D, uint32_t* own_rows, uint32_t* own_pos, uint32_t* own_cnt,
                              uint32_t* reff, hipStream_t s) {
    if (B == 0) return hipSuccess;
    const size_t lds = (size_t)kSelectLdsCap * 8u + (size_t)((D + 4u) & ~3u) * 4u + 3u * (size_t)G * 4u;
    hipLaunchKernelGGL(k_shard_merge, dim3(B), dim3(256), lds, s, gathered1, words1, G, me, B, R, D, own_rows, own_pos,
                       own_cnt, reff);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ---- step 3b: this rank's local top-k of its owned entries --------------------
// Keys (~order(cos) << 32 | position): cosine descending, ties by global
// stage-1 position (the reference's stable sort).  A NaN among the owned
// scores poisons the query when the global list has >= 2 entries (the
// reference's partial_cmp().unwrap() sort panics).
__global__ __launch_bounds__(256) void k_shard_local_topk(const float* __restrict__ scores,
                                                          const uint32_t* __restrict__ own_rows,
                                                          const uint32_t* __restrict__ own_pos,
                                                          const uint32_t* __restrict__ own_cnt,
                                                          const uint32_t* __restrict__ reff, uint32_t B, uint32_t R,
                                                          uint32_t k, const uint64_t* __restrict__ ids, uint32_t err,
                                                          uint32_t* __restrict__ block2) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];  // [next_pow2(R)]
    __shared__ uint32_t s_nan;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const uint32_t c = min(own_cnt[q], R);
    if (tid == 0) s_nan = 0u;
    __syncthreads();
    for (uint32_t i = tid; i < c; i += 256) {
        const float f = scores[(uint64_t)q * R + i];
        if (f != f) s_nan = 1u;
        // (position, owned index) in the low bits: positions are distinct (< 2^13)
        sk[i] = ((uint64_t)~f32_order(f) << 32) | ((uint64_t)own_pos[(uint64_t)q * R + i] << 13) | i;
    }
    const uint32_t P = next_pow2(max(c, 1u));
    for (uint32_t i = c + tid; i < P; i += 256) sk[i] = ~0ull;
    __syncthreads();
    if (c > 1) bitonic_sort_lds(sk, P);
    const uint32_t take = min(k, c);
    uint32_t* ent = block2 + (uint64_t)q * k * 4u;
    for (uint32_t i = tid; i < take; i += 256) {
        const uint64_t key = sk[i];
        const uint32_t pos = ((uint32_t)key >> 13) & 0x1fffu, j = (uint32_t)key & 0x1fffu;
        const uint32_t row = own_rows[(uint64_t)q * R + j];
        const uint64_t id = ids ? ids[row] : (uint64_t)row;
        ent[4 * i + 0] = __float_as_uint(scores[(uint64_t)q * R + j]);
        ent[4 * i + 1] = pos;
        ent[4 * i + 2] = (uint32_t)id;
        ent[4 * i + 3] = (uint32_t)(id >> 32);
    }
    if (tid == 0) {
        uint32_t* meta = block2 + 4ull * B * k;
        meta[q] = take | ((s_nan && reff[q] >= 2u) ? 0x80000000u : 0u);
        meta[B + q] = reff[q];
        if (q == 0) meta[2 * B] = err;
    }
}

hipError_t launch_shard_local_topk(const float* scores, const uint32_t* own_rows, const uint32_t* own_pos,
                                   const uint32_t* own_cnt, const uint32_t* reff, uint32_t B, uint32_t R, uint32_t k,
                                   const uint64_t* ids, uint32_t err, uint32_t* block2, hipStream_t s) {
    if (B == 0) return hipSuccess;
    const size_t lds = (size_t)next_pow2(std::max<uint32_t>(R, 1u)) * 8u;
    hipLaunchKernelGGL(k_shard_local_topk, dim3(B), dim3(256), lds, s, scores, own_rows, own_pos, own_cnt, reff, B, R,
                       k, ids, err, block2);
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
    // own_rows | own_pos | scores [B][R] + own_cnt | reff [B]
    if (scratch_bytes) *scratch_bytes = 12 * B * R + 8 * B + 256;
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
        B > 0xFFFFFFFFull)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: bad R / k / G / rank");
    hipStream_t s = (hipStream_t)stream;
    const ShardInfo si = index_shard_info(shard);
    if (hipSetDevice(si.device) != hipSuccess) return report_status(GVDB_ERR_DEVICE, "hipSetDevice");
    const uint64_t BR = B * R;
    uint32_t* own_rows = (uint32_t*)d_scratch;
    uint32_t* own_pos = own_rows + BR;
    float* scores = (float*)(own_pos + BR);
    uint32_t* own_cnt = (uint32_t*)(scores + BR);
    uint32_t* reff = own_cnt + B;
    // the distance histogram spans [0, D]: use the widest distance any rank can send
    const uint32_t D = std::max<uint32_t>(dim, 1u);
    hipError_t e = launch_shard_merge(d_gathered1, shard_words1(B, R), (uint32_t)G, (uint32_t)rank, (uint32_t)B,
                                      (uint32_t)R, std::min<uint32_t>(D, kShardMaxD), own_rows, own_pos, own_cnt, reff,
                                      s);
    if (e != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("shard merge: ") + hipGetErrorString(e));
    const bool usable = si.n > 0 && si.dim == dim;
    if (usable) {
        RerankArgs rr{};
        rr.rows = si.rows;
        rr.clen = dim;
        rr.norms = si.norms;
        rr.q = d_queries;
        rr.qlen = dim;
        rr.s1_rows = own_rows;
        rr.B = (uint32_t)B;
        rr.R = (uint32_t)R;
        rr.kind = kScoreCosine;
        rr.scores = scores;
        rr.counts = own_cnt;
        rr.short_lists = R <= 64u * G;  // ~R/G owned rows per query: 16-row blocks, loads all in flight
        e = launch_rerank(rr, s);
        if (e != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("shard rerank: ") + hipGetErrorString(e));
    } else if (hipMemsetAsync(own_cnt, 0, B * 4, s) != hipSuccess) {
        return report_status(GVDB_ERR_DEVICE, "shard rerank: memset");
    }
    e = launch_shard_local_topk(scores, own_rows, own_pos, own_cnt, reff, (uint32_t)B, (uint32_t)R, (uint32_t)k,
                                si.ids, 0u, d_block2, s);
    if (usable) index_track_use(shard, s);
    if (e != hipSuccess) return report_status(GVDB_ERR_DEVICE, std::string("shard top-k: ") + hipGetErrorString(e));
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
