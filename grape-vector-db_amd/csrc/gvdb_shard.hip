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
// Every list is sorted by (d, row), and the global order is (d, rank, row)
// (the reference's stable order by candidate index over the concatenated
// corpus).  (i) The global position of this rank's i-th entry is
//     i + sum_{g < me} #{list g: d <= d_i} + sum_{g > me} #{list g: d < d_i}
// (binary searches over the other lists' distances, staged in LDS); the
// entry is in the global top-R iff that position is < Re = min(R, total), so
// the owned entries are a prefix of the own list and their positions are
// exactly their ranks in the global top-R.  (ii) Exact cosine of the owned
// rows, kP2Rows at a time: the rows of the first group are loaded
// speculatively (the first kP2Rows own-list entries) while (i) runs, through
// LDS in chunks of kP2Ch dimensions, multiplied by the query as they are
// staged (every product q_j * x_j rounded once, by all threads); lane r <
// kP2Rows of wave 0 then folds row r's products in the reference's order
// (acc = acc + p_j from -0.0: the same sums as acc + q_j * x_j without
// contraction), wave 1's lane 0 folds the staged q_j * q_j.  The serial
// chains carry one add and a quarter of a ds_read_b128 per dimension.  (iii) The owned entries ranked by (cosine desc, position)
// (rank counting; a bitonic sort beyond kP2RankMax) -> the first k go to the
// exchange-2 block.
// LDS (dynamic): qv [D] | qsq [D] | cg [G] | dist [G*R] when G*R <= kP2DistLds |
// own pos / row / cos [R] when R <= kP2OwnLds (else the global scratch) | tile.
constexpr uint32_t kP2Threads = 256;
constexpr uint32_t kP2Rows = 24;    // rows re-scored together (one lane each)
constexpr uint32_t kP2Ch = 768;     // dimensions per LDS chunk
constexpr uint32_t kP2Ld = kP2Ch + 4;  // padded row stride: conflict-free ds_read_b128 across lanes
constexpr uint32_t kP2F4 = kP2Rows * (kP2Ch / 4) / kP2Threads;  // float4 per thread per chunk (18)
constexpr uint32_t kP2DistLds = 4096;  // other lists' distances staged in LDS up to this many
constexpr uint32_t kP2OwnLds = 2048;   // own-entry arrays in LDS up to this R
constexpr uint32_t kP2RankMax = 1024;  // rank counting up to this many owned entries
static_assert(kP2Rows * (kP2Ch / 4) % kP2Threads == 0, "chunk tiling");
static_assert(kP2Rows <= 64, "one wave folds the group");

__device__ __forceinline__ uint32_t p2_count(const uint32_t* dl, uint32_t n, uint32_t d, bool le) {
    // #{j < n: dl[j] <= d} (le) or < d; dl ascending
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (le ? dl[mid] <= d : dl[mid] < d) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// OWN_LDS: the own-entry arrays in LDS (R <= kP2OwnLds) -- a compile-time choice, so
// every access is a plain LDS op (a runtime LDS-or-global pointer makes them FLAT ops,
// whose vmcnt waits stall the ranking behind the in-flight row loads)
template <bool OWN_LDS, bool VEC, bool DSTAGED>
__global__ __launch_bounds__(kP2Threads) void k_shard_phase2(const uint32_t* __restrict__ gathered, uint64_t words1,
                                                             uint32_t G, uint32_t me, uint32_t B, uint32_t R,
                                                             uint32_t D, const float* __restrict__ rows,
                                                             const float* __restrict__ norms,
                                                             const uint64_t* __restrict__ ids,
                                                             const float* __restrict__ queries, uint32_t k,
                                                             uint32_t err, uint32_t* __restrict__ block2,
                                                             uint32_t* __restrict__ opos_g,
                                                             uint32_t* __restrict__ orow_g,
                                                             float* __restrict__ ocos_g,
                                                             unsigned long long* __restrict__ clk) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    // GVDB_P2_CLK timing study: thread 0's shader clock at each phase boundary
    const unsigned long long c0 = clk ? __builtin_amdgcn_s_memrealtime() : 0ull;
    auto mark = [&](int i) {
        if (clk && threadIdx.x == 0) clk[blockIdx.x * 8u + i] = __builtin_amdgcn_s_memrealtime() - c0;
    };
    // a barrier for LDS traffic only, while the speculative row loads are in flight
    // (__syncthreads' fence would wait for them: vmcnt(0)); the global-scratch form
    // (OWN_LDS false) shares global words across the block and keeps the fence
    auto sync_lds = [&]() __attribute__((always_inline)) {
        if constexpr (OWN_LDS)
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
            __syncthreads();
    };
    // DSTAGED: the other lists' distances fit LDS (G*R <= kP2DistLds); compile-time, so
    // the LDS search loop carries no merged global-load waits that would drain the
    // speculative row loads
    constexpr bool dstaged = DSTAGED;
    constexpr bool own_lds = OWN_LDS;
    float* qv = (float*)lds;                                   // [D]
    float* qsq = qv + ((D + 3u) & ~3u);                        // [D]: q_j * q_j
    uint32_t* cg = lds + 2u * ((D + 3u) & ~3u);                // [G]
    uint32_t* dist = cg + ((G + 3u) & ~3u);                    // [G*R] (dstaged)
    uint32_t* own = dist + (dstaged ? ((G * R + 3u) & ~3u) : 0u);
    float* tile = (float*)(own + (own_lds ? ((3u * R + 3u) & ~3u) : 0u));  // [kP2Rows][kP2Ld]
    __shared__ uint32_t s_total, s_c, s_nan;
    __shared__ float s_qq;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    uint32_t* opos;
    uint32_t* orow;
    float* ocos;
    if constexpr (OWN_LDS) {
        opos = own;
        orow = own + R;
        ocos = (float*)(own + 2 * R);
    } else {
        opos = opos_g + (uint64_t)q * R;
        orow = orow_g + (uint64_t)q * R;
        ocos = ocos_g + (uint64_t)q * R;
    }
    auto glist = [&](uint32_t g) { return (const uint64_t*)(gathered + (uint64_t)g * words1) + (uint64_t)q * R; };
    const uint64_t* mine = glist(me);
    // round A: every read that depends on nothing else, issued together -- the
    // counts, this rank's keys (d parked in opos), the other lists' distances,
    // the query row.  The first kP2Threads / 4 kP2Threads items of each go to
    // registers before any LDS store, so their latencies overlap (a load-then-store
    // loop waits out each load); the loops past them only run for large G / R / D
    const uint32_t GR = G * R;
    constexpr uint32_t kA = 4u;
    // unpredicated loads (clamped indices, always in bounds; the unused values are masked
    // at the stores): a predicated load sits in its own branch and the stores' waits
    // interleave with the remaining loads
    const uint32_t cg0 = gathered[(uint64_t)min(tid, G - 1u) * words1 + 2ull * B * R + q];
    const uint64_t key0 = mine[min(tid, R - 1u)];
    uint32_t dv[kA];
    float qx[kA];
    const float* qg = queries + (uint64_t)q * D;
#pragma unroll
    for (uint32_t u = 0; u < kA; ++u) {
        const uint32_t x = min(tid + u * kP2Threads, GR - 1u), g = x / R;
        // the distance is the key's high word
        if constexpr (DSTAGED) dv[u] = gathered[(uint64_t)g * words1 + 2ull * ((uint64_t)q * R + (x - g * R)) + 1u];
        qx[u] = qg[min(tid + u * kP2Threads, D - 1u)];
    }
    if (tid == 0) {
        s_total = 0u;
        s_c = 0u;
        s_nan = 0u;
    }
    __syncthreads();
    auto put_cg = [&](uint32_t g, uint32_t c) __attribute__((always_inline)) {
        c = min(c, R);
        cg[g] = g == me && !rows ? 0u : c;  // a shard that cannot rerank sent nothing
        atomicAdd(&s_total, c);
    };
    auto put_key = [&](uint32_t i, uint64_t key) __attribute__((always_inline)) {  // R key slots per query
        opos[i] = (uint32_t)(key >> 32);
        orow[i] = (uint32_t)key;
    };
    if (tid < G) put_cg(tid, cg0);
    if (tid < R) put_key(tid, key0);
    for (uint32_t g = tid + kP2Threads; g < G; g += kP2Threads) put_cg(g, gathered[(uint64_t)g * words1 + 2ull * B * R + q]);
    for (uint32_t i = tid + kP2Threads; i < R; i += kP2Threads) put_key(i, mine[i]);
    if constexpr (DSTAGED) {
#pragma unroll
        for (uint32_t u = 0; u < kA; ++u) {
            const uint32_t x = tid + u * kP2Threads;
            if (x < GR && x / R != me) dist[x] = dv[u];
        }
        for (uint32_t x = tid + kA * kP2Threads; x < GR; x += kP2Threads) {
            const uint32_t g = x / R, i = x - g * R;
            if (g != me) dist[x] = (uint32_t)(glist(g)[i] >> 32);
        }
    }
#pragma unroll
    for (uint32_t u = 0; u < kA; ++u) {
        const uint32_t j = tid + u * kP2Threads;
        if (j < D) {
            qv[j] = qx[u];
            qsq[j] = qx[u] * qx[u];
        }
    }
    for (uint32_t j = tid + kA * kP2Threads; j < D; j += kP2Threads) {
        const float v = qg[j];
        qv[j] = v;
        qsq[j] = v * v;
    }
    __syncthreads();
    mark(0);
    const uint32_t cnt_me = cg[me];
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
    // round B: the first kP2Rows own-list rows (speculative: the owned entries are a
    // prefix of the list), their norms and ids, in flight during the ranking
    float4 xr[kP2F4];
    constexpr bool vec = VEC;  // D % 4 == 0: 16-B row loads and LDS folds (a compile-time choice: clean loads)
    auto load = [&](uint32_t r0, uint32_t nr, uint32_t ch) __attribute__((always_inline)) {
        if constexpr (VEC) {
            // unpredicated: rows past nr re-read row nr - 1 and dimensions past D the last
            // float4 (no fold reads those slots), so every orow read and every row load is
            // issued back to back instead of one branch (and one LDS wait) per load
            if (nr == 0u) return;
            uint32_t rr[kP2F4];
#pragma unroll
            for (uint32_t e = 0; e < kP2F4; ++e) rr[e] = orow[r0 + min((tid + e * kP2Threads) / (kP2Ch / 4), nr - 1u)];
#pragma unroll
            for (uint32_t e = 0; e < kP2F4; ++e) {
                const uint32_t L = tid + e * kP2Threads, j = min(ch * kP2Ch + 4u * (L % (kP2Ch / 4)), D - 4u);
                xr[e] = *(const float4*)(rows + (uint64_t)rr[e] * D + j);
            }
        } else {
#pragma unroll
            for (uint32_t e = 0; e < kP2F4; ++e) {
                const uint32_t L = tid + e * kP2Threads, r = L / (kP2Ch / 4), j = ch * kP2Ch + 4u * (L % (kP2Ch / 4));
                float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (r < nr && j < D) {
                    const float* src = rows + (uint64_t)orow[r0 + r] * D + j;
                    v.x = src[0];
                    if (j + 1 < D) v.y = src[1];
                    if (j + 2 < D) v.z = src[2];
                    if (j + 3 < D) v.w = src[3];
                }
                xr[e] = v;
            }
        }
    };
    const uint32_t nr0 = min(cnt_me, kP2Rows);
    load(0, nr0, 0);
    const float nb0 = tid < nr0 ? norms[orow[tid]] : 0.0f;
    const uint64_t id0 = tid < nr0 ? (ids ? ids[orow[tid]] : (uint64_t)orow[tid]) : 0ull;
    // (i) global positions of the own entries: pos_i = i + the other lists' counts
    //     below d_i, one (entry, list) pair per thread (binary searches over the
    //     staged distances), summed into posacc (the cosine slots, free until (ii))
    uint32_t* posacc = (uint32_t*)ocos;
    for (uint32_t i = tid; i < cnt_me; i += kP2Threads) posacc[i] = i;
    sync_lds();
    for (uint32_t x = tid; x < cnt_me * G; x += kP2Threads) {
        const uint32_t i = x / G, g = x - i * G;
        if (g == me) continue;
        const uint32_t d = opos[i];
        uint32_t cnt;
        if constexpr (DSTAGED) {
            cnt = p2_count(dist + g * R, cg[g], d, g < me);
        } else {  // large G * R: the same search over the gathered keys
            const uint64_t* L = glist(g);
            uint32_t lo = 0, hi = cg[g];
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1, dm = (uint32_t)(L[mid] >> 32);
                if (g < me ? dm <= d : dm < d) lo = mid + 1; else hi = mid;
            }
            cnt = lo;
        }
        if (cnt) atomicAdd(&posacc[i], cnt);
    }
    sync_lds();
    // the owned entries are those below Re (a prefix of the own list)
    for (uint32_t i = tid; i < cnt_me; i += kP2Threads) {
        const uint32_t pos = posacc[i];
        opos[i] = pos;
        if (pos < Re) atomicAdd(&s_c, 1u);
    }
    sync_lds();
    mark(1);
    const uint32_t c = s_c;  // the owned entries: own-list prefix [0, c)
    // (ii) exact cosine of the owned rows, kP2Rows at a time
    const uint32_t nch = (D + kP2Ch - 1) / kP2Ch;
    for (uint32_t r0 = 0; r0 < c; r0 += kP2Rows) {
        const uint32_t nr = min(kP2Rows, c - r0);
        if (r0 > 0) load(r0, nr, 0);  // groups past the speculative one (> kP2Rows owned)
        float acc = -0.0f;
        const bool fold_q = r0 == 0 && tid == 64;
        float qq = -0.0f;
        const float nb = r0 == 0 ? nb0 : tid < nr ? norms[orow[r0 + tid]] : 0.0f;
        for (uint32_t ch = 0; ch < nch; ++ch) {
#pragma unroll
            for (uint32_t e = 0; e < kP2F4; ++e) {  // staged as the products q_j * x_j
                const uint32_t L = tid + e * kP2Threads, c4 = 4u * (L % (kP2Ch / 4)), j = ch * kP2Ch + c4;
                float4 v = xr[e];
                if (j + 3u < D) {
                    const float4 w = *(const float4*)(qv + j);
                    v.x = w.x * v.x;
                    v.y = w.y * v.y;
                    v.z = w.z * v.z;
                    v.w = w.w * v.w;
                } else {  // the row's last dimensions (D % 4 != 0); past D unused by the fold
                    v.x = j < D ? qv[j] * v.x : 0.0f;
                    v.y = j + 1u < D ? qv[j + 1u] * v.y : 0.0f;
                    v.z = j + 2u < D ? qv[j + 2u] * v.z : 0.0f;
                    v.w = 0.0f;
                }
                *(float4*)(tile + (L / (kP2Ch / 4)) * kP2Ld + c4) = v;
            }
            __syncthreads();
            if (ch + 1 < nch) load(r0, nr, ch + 1);  // next chunk in flight during the folds
            const uint32_t j0 = ch * kP2Ch, m = min(kP2Ch, D - j0);
            if (tid < nr || fold_q) {
                const float* tr = fold_q ? qsq + j0 : tile + tid * kP2Ld;  // products
                float a2 = fold_q ? qq : acc;
                uint32_t j = 0;
                if (vec) {
#pragma unroll 8
                    for (; j + 4 <= m; j += 4) {
                        const float4 p4 = *(const float4*)(tr + j);
                        a2 = a2 + p4.x;
                        a2 = a2 + p4.y;
                        a2 = a2 + p4.z;
                        a2 = a2 + p4.w;
                    }
                }
                for (; j < m; ++j) a2 = a2 + tr[j];
                if (fold_q) qq = a2; else acc = a2;
            }
            if (fold_q && ch + 1 == nch) s_qq = qq;
            __syncthreads();
        }
        if (tid < nr) {
            const float na = sqrtf(s_qq);
            const float sc = (na == 0.0f || nb == 0.0f) ? 0.0f : acc / (na * nb);
            ocos[r0 + tid] = sc;
            if (sc != sc) s_nan = 1u;
        }
    }
    __syncthreads();
    mark(2);
    // (iii) local top-k by (cosine desc, global position): key (~order(cos), pos)
    const uint32_t take = min(k, c);
    uint32_t* ent = block2 + (uint64_t)q * k * 4u;
    uint64_t* keys = (uint64_t*)tile;
    auto emit = [&](uint32_t t, uint32_t j) {  // j == tid for the rank-counted entries
        const uint32_t row = orow[j];
        const uint64_t id = j == tid && j < nr0 ? id0 : ids ? ids[row] : (uint64_t)row;
        ent[4 * t + 0] = __float_as_uint(ocos[j]);
        ent[4 * t + 1] = opos[j];
        ent[4 * t + 2] = (uint32_t)id;
        ent[4 * t + 3] = (uint32_t)(id >> 32);
    };
    if (c <= kP2RankMax) {
        for (uint32_t i = tid; i < c; i += kP2Threads)
            keys[i] = ((uint64_t)~f32_order(ocos[i]) << 32) | opos[i];
        __syncthreads();
        for (uint32_t i = tid; i < c; i += kP2Threads) {
            const uint64_t ki = keys[i];
            uint32_t rk = 0;
            for (uint32_t j = 0; j < c; ++j) rk += keys[j] < ki;  // positions are distinct
            if (rk < take) emit(rk, i);
        }
    } else {  // P <= next_pow2(8192) keys of 8 B fit the tile (148 KiB)
        const uint32_t P = next_pow2(c);
        for (uint32_t i = tid; i < P; i += kP2Threads)
            keys[i] = i < c ? ((uint64_t)~f32_order(ocos[i]) << 32) | ((uint64_t)opos[i] << 13) | i : ~0ull;
        __syncthreads();
        bitonic_sort_lds(keys, P);
        for (uint32_t t = tid; t < take; t += kP2Threads) emit(t, (uint32_t)keys[t] & 0x1fffu);
    }
    if (tid == 0) {
        meta[q] = take | ((s_nan && Re >= 2u) ? 0x80000000u : 0u);
        meta[B + q] = Re;
        if (q == 0) meta[2 * B] = err;
    }
    mark(3);
}

size_t shard_phase2_lds(uint32_t G, uint32_t R, uint32_t D) {
    const size_t dist = G * R <= kP2DistLds ? (size_t)((G * R + 3u) & ~3u) * 4u : 0u;
    const size_t own = R <= kP2OwnLds ? (size_t)((3u * R + 3u) & ~3u) * 4u : 0u;
    const size_t tile = std::max<size_t>((size_t)kP2Rows * kP2Ld * 4u,
                                         R > kP2RankMax ? (size_t)next_pow2(R) * 8u : 0u);
    return (size_t)((D + 3u) & ~3u) * 8u + (size_t)((G + 3u) & ~3u) * 4u + dist + own + tile;
}

struct ShardClk {
    unsigned long long* p;
    uint32_t B;
};
static ShardClk& shard_clk() {
    static ShardClk c{nullptr, 0};
    return c;
}

hipError_t launch_shard_phase2(const uint32_t* gathered1, uint64_t words1, uint32_t G, uint32_t me, uint32_t B,
                               uint32_t R, uint32_t D, const float* rows, const float* norms, const uint64_t* ids,
                               const float* queries, uint32_t k, uint32_t err, uint32_t* block2, uint32_t* opos,
                               uint32_t* orow, float* ocos, hipStream_t s) {
    if (B == 0) return hipSuccess;
    const size_t lds = shard_phase2_lds(G, R, D);
    if (lds > 160u * 1024u) return hipErrorInvalidValue;
    unsigned long long* clk = nullptr;
    if (getenv("GVDB_P2_CLK")) {  // timing study (gvdb_debug_shard_clock)
        static unsigned long long* buf = nullptr;
        static uint32_t cap = 0;
        if (cap < B) {
            if (buf) (void)hipFree(buf);
            if (hipMalloc((void**)&buf, (size_t)B * 64) != hipSuccess) buf = nullptr;
            cap = buf ? B : 0;
        }
        clk = buf;
        shard_clk() = {buf, B};
    }
    const bool own = R <= kP2OwnLds, vec = (D & 3u) == 0, dst = G * R <= kP2DistLds;
    auto kern = own ? (vec ? (dst ? k_shard_phase2<true, true, true> : k_shard_phase2<true, true, false>)
                           : (dst ? k_shard_phase2<true, false, true> : k_shard_phase2<true, false, false>))
                    : (vec ? (dst ? k_shard_phase2<false, true, true> : k_shard_phase2<false, true, false>)
                           : (dst ? k_shard_phase2<false, false, true> : k_shard_phase2<false, false, false>));
    hipLaunchKernelGGL(kern, dim3(B), dim3(kP2Threads), lds, s, gathered1, words1, G, me, B, R, D, rows, norms, ids,
                       queries, k, err, block2, opos, orow, ocos, clk);
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
    const bool by_rank = n <= kP2RankMax;  // rank counting (sk[n..n+k): the k smallest keys), else a sort
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
        if (by_rank && x < k) sk[n + x] = ~0ull;
    }
    if (by_rank) {
        __syncthreads();
        for (uint32_t x = tid; x < n; x += 256) {
            const uint64_t kx = sk[x];
            if (kx == ~0ull) continue;
            uint32_t rk = 0;
            for (uint32_t j = 0; j < n; ++j) rk += sk[j] < kx;  // keys are distinct (x)
            if (rk < k) sk[n + rk] = kx;
        }
    } else {
        const uint32_t P = next_pow2(max(n, 1u));
        for (uint32_t i = n + tid; i < P; i += 256) sk[i] = ~0ull;
        __syncthreads();
        bitonic_sort_lds(sk, P);
    }
    __syncthreads();
    const uint64_t* top = by_rank ? sk + n : sk;
    if (tid < 64) {  // take(k), then drop orphans (order-preserving ballot compaction)
        uint32_t o = 0;
        for (uint32_t i0 = 0; i0 < k; i0 += 64) {
            const uint32_t i = i0 + tid;
            const uint64_t key = i < k ? top[i] : ~0ull;
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
    const uint32_t n = std::max<uint32_t>(G * k, 1u);
    const size_t lds = (size_t)std::max<uint32_t>(next_pow2(n), n <= kP2RankMax ? n + k : 0u) * 8u;
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

// ---- deep two-exchange (R > kSelectLdsCap: the reference's default ratio) -------
// Exchange 1 carries, per query, the Hamming histogram of the rank's local
// top-min(R, n_g) membership instead of its keys (B*(dim+1)*4 bytes per rank,
// independent of R).  Every rank then knows the global top-R by (d, rank, row)
// exactly: its threshold T = the smallest t with sum_g #{list g: d <= t} >= Re,
// the ties at T taken in rank order (ranks before this one first), and within
// this rank the first `quota` tied rows by row.  Its owned entries are its own
// members below T plus those tied rows.  The local top-k then orders by
// (cosine desc, Hamming, row) and exchange 2 carries the Hamming distance in
// the entry's order-key word: the merge's (cosine, Hamming, rank, list index)
// order is the global stable order (cosine, d, rank, row).

// block 1 (deep): per query the histogram of the member distances, counts = Rl
__global__ __launch_bounds__(256) void k_shard_member_hist(const uint32_t* __restrict__ m_dist, uint32_t B,
                                                           uint32_t Rl, uint32_t H, uint32_t* __restrict__ block1) {
    extern __shared__ uint32_t h[];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    for (uint32_t t = tid; t < H; t += 256) h[t] = 0u;
    __syncthreads();
    const uint32_t* d = m_dist + (uint64_t)q * Rl;
    for (uint32_t i = tid; i < Rl; i += 256) atomicAdd(&h[min(d[i], H - 1u)], 1u);
    __syncthreads();
    uint32_t* out = block1 + (uint64_t)q * H;
    for (uint32_t t = tid; t < H; t += 256) out[t] = h[t];
    if (tid == 0) block1[(uint64_t)B * H + q] = Rl;
}

hipError_t launch_shard_member_hist(const uint32_t* m_dist, uint32_t B, uint32_t Rl, uint32_t H, uint32_t* block1,
                                    hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_shard_member_hist, dim3(B), dim3(256), (size_t)H * 4u, s, m_dist, B, Rl, H, block1);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// step 3 (i) deep: this rank's owned entries of the global top-R, compacted
// (order kept) into o_rows / o_dist; own_cnt / reff [B].  The member lists are
// only read: phase 2 can run again on the same phase-1 scratch.
constexpr uint32_t kDeepThreads = 1024;
__global__ __launch_bounds__(kDeepThreads) void k_shard_deep_own(const uint32_t* __restrict__ gathered,
                                                                 uint64_t words1, uint32_t G, uint32_t me, uint32_t B,
                                                                 uint32_t R, uint32_t Rl, uint32_t H,
                                                                 const uint32_t* __restrict__ m_rows,
                                                                 const uint32_t* __restrict__ m_dist,
                                                                 uint32_t* __restrict__ o_rows,
                                                                 uint32_t* __restrict__ o_dist,
                                                                 uint32_t* __restrict__ own_cnt,
                                                                 uint32_t* __restrict__ reff,
                                                                 uint32_t* __restrict__ tcut,
                                                                 const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t tot[];  // [H] global histogram, then bins [2048]
    uint32_t* bins = tot + ((H + 3u) & ~3u);
    __shared__ uint32_t s_S, s_T, s_lt, s_tb, s_cut, s_below, wcnt[kDeepThreads / 64];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    auto hist = [&](uint32_t g) { return gathered + (uint64_t)g * words1 + (uint64_t)q * H; };
    auto count = [&](uint32_t g) { return min(gathered[(uint64_t)g * words1 + (uint64_t)B * H + q], R); };
    if (tid == 0) s_S = 0u;
    __syncthreads();
    for (uint32_t t = tid; t < H; t += nt) {
        uint32_t s = 0;
        for (uint32_t g = 0; g < G; ++g) s += hist(g)[t];
        tot[t] = s;
    }
    for (uint32_t g = tid; g < G; g += nt) atomicAdd(&s_S, count(g));
    __syncthreads();
    const uint32_t Re = min(R, s_S);
    const uint32_t n = Rl ? min(count(me), Rl) : 0u;  // this rank's members
    if (Re == 0 || n == 0) {
        if (tid == 0) {
            own_cnt[q] = 0u;
            reff[q] = Re;
            if (tcut) {  // no owned row
                tcut[4u * q] = 0u;
                tcut[4u * q + 1u] = 0u;
                tcut[4u * q + 2u] = 0u;
                tcut[4u * q + 3u] = 2u;
            }
        }
        return;
    }
    if (tid < 64) {
        const uint32_t t = wave_find_cum(tot, H, Re);
        const uint32_t lt = wave_sum_below(tot, t);
        if (tid == 0) {
            s_T = t;
            s_lt = lt;
            uint32_t tb = 0;
            for (uint32_t g = 0; g < me; ++g) tb += hist(g)[t];  // ties at T of the ranks before this one
            s_tb = tb;
        }
    }
    __syncthreads();
    const uint32_t T = s_T, need = Re - s_lt, tb = s_tb, mine = hist(me)[T];
    const uint32_t quota = need > tb ? min(need - tb, mine) : 0u;  // this rank's tied rows in the top-R
    if (tcut) {
        // the certified phase 2 only needs the rule: member iff d < T, or d == T and fewer than
        // `quota` of the member list's rows tied at T lie below it (the list holds the shard's first
        // tied rows by row; k_deep_certify counts, for the few listed rows it asks about) -- no radix
        // select, no compaction (own_cnt = the owned count)
        if (tid < 64) {
            uint32_t below = 0u;  // members with d < T: the prefix of this rank's histogram
            const uint32_t* hm = hist(me);
            for (uint32_t t = tid; t < T; t += 64) below += hm[t];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) below += (uint32_t)__shfl_xor((int)below, off);
            if (tid == 0) own_cnt[q] = min(below + quota, n);
        }
        if (tid == 0) {
            reff[q] = Re;
            tcut[4u * q] = T;
            tcut[4u * q + 1u] = 0u;
            tcut[4u * q + 2u] = quota;
            tcut[4u * q + 3u] = quota ? 3u : 2u;
        }
        return;
    }
    // the quota-th smallest row among this rank's members at d == T: 11 + 11 + 10 bits
    uint32_t cut = 0u;
    const bool all_ties = quota == mine, no_ties = quota == 0u;
    if (!all_ties && !no_ties) {
        uint32_t left = quota, prefix = 0u, pmask = 0u;
        const uint32_t* rw = m_rows + (uint64_t)q * Rl;
        const uint32_t* dd = m_dist + (uint64_t)q * Rl;
        for (int pass = 0; pass < 3; ++pass) {
            const int shift = pass == 0 ? 21 : pass == 1 ? 10 : 0;
            const uint32_t nb = pass == 2 ? 1024u : 2048u, dm = nb - 1u;
            for (uint32_t i = tid; i < nb; i += nt) bins[i] = 0u;
            __syncthreads();
            for (uint32_t i = tid; i < n; i += nt) {
                const uint32_t row = rw[i];
                if (dd[i] == T && (row & pmask) == prefix) atomicAdd(&bins[(row >> shift) & dm], 1u);
            }
            __syncthreads();
            if (tid < 64) {
                const uint32_t bin = wave_find_cum(bins, nb, left);
                const uint32_t below = wave_sum_below(bins, bin);
                if (tid == 0) {
                    s_cut = bin;
                    s_below = below;
                }
            }
            __syncthreads();
            left -= s_below;
            prefix |= s_cut << shift;
            pmask |= dm << shift;
            __syncthreads();
        }
        cut = prefix;
    }
    // order-preserving compaction into the owned lists
    const uint32_t* rw = m_rows + (uint64_t)q * Rl;
    const uint32_t* dd = m_dist + (uint64_t)q * Rl;
    uint32_t* orw = o_rows + (uint64_t)q * Rl;
    uint32_t* odd = o_dist + (uint64_t)q * Rl;
    uint32_t o = 0;
    for (uint32_t base = 0; base < n; base += nt) {
        const uint32_t i = base + tid;
        uint32_t row = 0u, d = ~0u;
        if (i < n) {
            row = rw[i];
            d = dd[i];
        }
        const bool keep = i < n && (d < T || (d == T && (all_ties || (!no_ties && row <= cut))));
        uint32_t total;
        const uint32_t pos = o + big_prefix(keep, wcnt, &total);
        if (keep) {
            orw[pos] = row;
            odd[pos] = d;
        }
        o += total;
    }
    if (tid == 0) {
        own_cnt[q] = o;
        reff[q] = Re;
    }
}

hipError_t launch_shard_deep_own(const uint32_t* gathered1, uint64_t words1, uint32_t G, uint32_t me, uint32_t B,
                                 uint32_t R, uint32_t Rl, uint32_t H, const uint32_t* m_rows, const uint32_t* m_dist,
                                 uint32_t* o_rows, uint32_t* o_dist, uint32_t* own_cnt, uint32_t* reff,
                                 hipStream_t s, uint32_t* tcut, const uint32_t* gate) {
    if (B == 0) return hipSuccess;
    const size_t lds = (size_t)((H + 3u) & ~3u) * 4u + 2048u * 4u;
    if (lds > 160u * 1024u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_shard_deep_own, dim3(B), dim3(kDeepThreads), lds, s, gathered1, words1, G, me, B, R, Rl, H,
                       m_rows, m_dist, o_rows, o_dist, own_cnt, reff, tcut, gate);
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

void gvdb_shard_sizes(uint64_t B, uint64_t R, uint64_t k, uint32_t dim, uint64_t* words1, uint64_t* words2,
                      uint64_t* scratch_bytes) {
    if (words1) *words1 = shard_deep(R) ? shard_words1_deep(B, dim) : shard_words1(B, R);
    if (words2) *words2 = shard_words2(B, k);
    // key form: the owned positions, rows and cosines [B][R] of phase 2 (used when R > 2048);
    // deep form: the member rows and distances, the owned rows and distances, their
    // cosines [B][R], own counts and reff [B]
    if (scratch_bytes) *scratch_bytes = (shard_deep(R) ? 20 : 12) * B * R + 8 * B + 256;
}

uint64_t gvdb_shard_flat_words(uint64_t B, uint64_t k) { return shard_words_flat(B, k); }

gvdb_status gvdb_shard_stage1_device(const gvdb_index* shard, const float* d_queries, uint64_t B, uint32_t dim,
                                     uint64_t R, uint32_t* d_block1, void* d_scratch, void* stream) {
    if (!shard || !d_block1 || (B && !d_queries)) return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (B == 0) return GVDB_OK;
    const bool deep = shard_deep(R);
    if (R == 0 || R > kBigRMax) return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: 1 <= R <= 2^20");
    if (deep && (!d_scratch || dim == 0 || dim >= 4096))
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "deep sharded search (R > 8192): scratch, 0 < dim < 4096");
    hipStream_t s = (hipStream_t)stream;
    const ShardInfo si = index_shard_info(shard);
    if (hipSetDevice(si.device) != hipSuccess) return report_status(GVDB_ERR_DEVICE, "hipSetDevice");
    const uint64_t BR = B * R;
    gvdb_status st = GVDB_OK;
    // every rank joins the exchange: a failed or empty shard contributes no
    // entries (and a failure flag that poisons every query of the merge)
    if (deep) {
        uint32_t* m_rows = (uint32_t*)d_scratch;
        const uint64_t hw = B * (dim + 1ull);  // histogram words before the counts
        // the certified phase 2's exact cosine list, beside stage 1 (into the owned-rows region,
        // which only the rerank fallback writes, after the certify pass has read the list)
        if (shard_early_list_bytes(B) <= B * R * 4) {  // (it checks the shard's eligibility itself)
            st = shard_deep_flat_early(shard, d_queries, B, dim, m_rows + 2 * BR, s);
            if (st != GVDB_OK) return st;
        }
        st = shard_stage1_members(shard, d_queries, B, dim, R, m_rows, m_rows + BR, d_block1, s);
        if (st != GVDB_OK || si.n == 0) {
            if (hipMemsetD32Async(d_block1, 0, hw + B, s) != hipSuccess ||
                hipMemsetD32Async(d_block1 + hw + B, st == GVDB_OK ? 0 : 1, 1, s) != hipSuccess)
                return report_status(GVDB_ERR_DEVICE, "sharded stage 1: counts");
        } else if (hipMemsetD32Async(d_block1 + hw + B, 0, 1, s) != hipSuccess) {
            return report_status(GVDB_ERR_DEVICE, "sharded stage 1: err word");
        }
        return st;
    }
    uint32_t* counts = d_block1 + 2 * BR;
    if (si.n > 0 && dim > kShardMaxD) st = report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: dim > 8192");
    if (st == GVDB_OK) st = shard_stage1_keys(shard, d_queries, B, dim, R, reinterpret_cast<uint64_t*>(d_block1), s);
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
    const bool deep = shard_deep(R);
    if (R == 0 || R > kBigRMax || k == 0 || G == 0 || G > kShardMaxG || rank >= G || G * k > kSelectLdsCap ||
        B > 0xFFFFFFFFull || dim == 0 || dim > kShardMaxD || (deep && (dim >= 4096 || k > 1024)))
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: bad R / k / G / rank / dim");
    hipStream_t s = (hipStream_t)stream;
    const ShardInfo si = index_shard_info(shard);
    if (hipSetDevice(si.device) != hipSuccess) return report_status(GVDB_ERR_DEVICE, "hipSetDevice");
    const uint64_t BR = B * R;
    // a shard that cannot rerank (empty, or a dimension mismatch already reported by
    // phase 1) sent no entries, so it owns none: its rows are never read
    const bool usable = si.n > 0 && si.dim == dim;
    if (deep) {
        uint32_t* m_rows = (uint32_t*)d_scratch;  // phase 1's members (read only here)
        uint32_t* m_dist = m_rows + BR;
        uint32_t* o_rows = m_dist + BR;            // the owned members
        uint32_t* o_dist = o_rows + BR;
        float* m_cos = (float*)(o_dist + BR);
        uint32_t* own_cnt = (uint32_t*)(m_cos + BR);
        uint32_t* reff = own_cnt + B;
        uint32_t* tcut = (uint32_t*)m_cos;  // the certified form's rule [B][4] (the cosines are not written then)
        const uint32_t Rl = usable ? (uint32_t)std::min<uint64_t>(R, si.n) : 0u;
        const bool try_cert = usable && Rl > 0 && B * 4 <= BR && shard_certified_eligible(shard, dim, k);
        hipError_t e = hipSuccess;
        ShardDenseLayout lay;
        if (usable && Rl > 0 && shard_dense_layout(shard, B, R, dim, d_scratch, &lay)) {
            // stage 1 kept the dense block: the rule (T, quota) from the exchange, then the certified
            // form, then -- gated by its failure word -- the owned rows compacted from the block
            uint32_t* dfail = reff + B;
            const uint32_t* gate = nullptr;
            e = launch_shard_deep_own(d_gathered1, shard_words1_deep(B, dim), (uint32_t)G, (uint32_t)rank,
                                      (uint32_t)B, (uint32_t)R, Rl, dim + 1u, m_rows, m_dist, o_rows, o_dist, own_cnt,
                                      reff, s, tcut);
            if (e == hipSuccess && try_cert) {
                bool enqueued = false;
                const gvdb_status st = shard_certified_phase2(shard, d_queries, B, dim, k, tcut, own_cnt, reff,
                                                              nullptr, nullptr, Rl, d_block2, dfail, o_rows, s,
                                                              &enqueued, &lay);
                if (st != GVDB_OK) return st;
                if (enqueued) gate = dfail;
            }
            if (e == hipSuccess)
                e = launch_dense_own(lay.dense, lay.np, lay.n, tcut, lay.qpc, (uint32_t)B, o_rows, o_dist, Rl, gate, s);
            if (e == hipSuccess) {
                RerankArgs rr{};
                rr.rows = si.rows;
                rr.clen = dim;
                rr.norms = si.norms;
                rr.q = d_queries;
                rr.qlen = dim;
                rr.s1_rows = o_rows;
                rr.B = (uint32_t)B;
                rr.R = Rl;
                rr.kind = kScoreCosine;
                rr.scores = m_cos;
                rr.counts = own_cnt;
                rr.gate = gate;
                e = launch_rerank(rr, s);
            }
            if (e == hipSuccess)
                e = launch_shard_deep_topk(m_cos, o_rows, o_dist, own_cnt, reff, (uint32_t)B, Rl, (uint32_t)k, si.ids,
                                           0u, d_block2, s, gate);
            if (e != hipSuccess)
                return report_status(GVDB_ERR_DEVICE, std::string("deep shard phase 2: ") + hipGetErrorString(e));
            index_track_use(shard, s);
            return GVDB_OK;
        }
        // the certified form: the rank's exact cosine top-32 / 64 filtered by its owned-row rule; the
        // rerank of the owned lists below is then gated on the device by its failure word (scratch)
        uint32_t* dfail = reff + B;
        const uint32_t* gate = nullptr;
        if (try_cert) {
            e = launch_shard_deep_own(d_gathered1, shard_words1_deep(B, dim), (uint32_t)G, (uint32_t)rank,
                                      (uint32_t)B, (uint32_t)R, Rl, dim + 1u, m_rows, m_dist, o_rows, o_dist, own_cnt,
                                      reff, s, tcut);
            bool enqueued = false;
            if (e == hipSuccess) {
                const gvdb_status st = shard_certified_phase2(shard, d_queries, B, dim, k, tcut, own_cnt, reff,
                                                              m_rows, m_dist, Rl, d_block2, dfail, o_rows, s,
                                                              &enqueued);
                if (st != GVDB_OK) return st;
            }
            if (enqueued) gate = dfail;
        }
        if (e == hipSuccess)
            e = launch_shard_deep_own(d_gathered1, shard_words1_deep(B, dim), (uint32_t)G, (uint32_t)rank,
                                      (uint32_t)B, (uint32_t)R, Rl, dim + 1u, m_rows, m_dist, o_rows, o_dist, own_cnt,
                                      reff, s, nullptr, gate);
        if (e == hipSuccess && Rl > 0) {
            RerankArgs rr{};
            rr.rows = si.rows;
            rr.clen = dim;
            rr.norms = si.norms;
            rr.q = d_queries;
            rr.qlen = dim;
            rr.s1_rows = o_rows;
            rr.B = (uint32_t)B;
            rr.R = Rl;
            rr.kind = kScoreCosine;
            rr.scores = m_cos;
            rr.counts = own_cnt;
            rr.gate = gate;
            e = launch_rerank(rr, s);
        }
        if (e == hipSuccess)
            e = launch_shard_deep_topk(m_cos, o_rows, o_dist, own_cnt, reff, (uint32_t)B, Rl, (uint32_t)k,
                                       usable ? si.ids : nullptr, 0u, d_block2, s, gate);
        if (e != hipSuccess)
            return report_status(GVDB_ERR_DEVICE, std::string("deep shard phase 2: ") + hipGetErrorString(e));
        if (usable) index_track_use(shard, s);
        return GVDB_OK;
    }
    if (R > kSelectLdsCap) return report_status(GVDB_ERR_INVALID_ARGUMENT, "sharded search: R");
    uint32_t* opos = (uint32_t*)d_scratch;
    uint32_t* orow = opos + BR;
    const hipError_t e = launch_shard_phase2(d_gathered1, shard_words1(B, R), (uint32_t)G, (uint32_t)rank, (uint32_t)B,
                                             (uint32_t)R, dim, usable ? si.rows : nullptr,
                                             usable ? si.norms : nullptr, usable ? si.ids : nullptr, d_queries,
                                             (uint32_t)k, 0u, d_block2, opos, orow, (float*)(orow + BR), s);
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

// GVDB_P2_CLK=1 timing study: average phase-boundary clocks (s_memrealtime, 100 MHz ticks, from
// the block start) of the last phase-2 launch: out[0..3] = round A, ranking, folds, end.
int gvdb_debug_shard_clock(double* out) {
    const ShardClk c = shard_clk();
    if (!c.p || !out) return -1;
    std::vector<unsigned long long> h((size_t)c.B * 8);
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(h.data(), c.p, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return -2;
    for (int i = 0; i < 4; ++i) {
        double s = 0;
        for (uint32_t q = 0; q < c.B; ++q) s += (double)h[(size_t)q * 8 + i];
        out[i] = s / c.B;
    }
    return 0;
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

// Host form of the deep step 3 (i) (k_shard_deep_own): from the gathered deep
// exchange-1 blocks and this rank's members (m_rows / m_dist [B][R], the
// first min(count, R) valid, any order), its owned entries sorted by
// (Hamming, row) -> own_rows / own_dist [B][R], own_cnt, reff.  Their
// Hamming distances are the order keys gvdb_shard_local_topk_host takes as
// own_pos (a list sorted by (d, row) breaks (cosine, d) ties by row).
gvdb_status gvdb_shard_deep_own_host(const uint32_t* gathered1, uint64_t G, uint64_t rank, uint64_t B, uint64_t R,
                                     uint32_t dim, const uint32_t* m_rows, const uint32_t* m_dist,
                                     uint32_t* own_rows, uint32_t* own_dist, uint32_t* own_cnt, uint32_t* reff) {
    if (!gathered1 || !m_rows || !m_dist || !own_rows || !own_dist || !own_cnt || !reff)
        return report_status(GVDB_ERR_INVALID_ARGUMENT, "null argument");
    if (rank >= G || dim == 0) return report_status(GVDB_ERR_INVALID_ARGUMENT, "bad rank / dim");
    const uint64_t H = dim + 1ull, w1 = shard_words1_deep(B, dim);
    std::vector<uint64_t> tot(H), mine;
    for (uint64_t q = 0; q < B; ++q) {
        std::fill(tot.begin(), tot.end(), 0ull);
        uint64_t S = 0;
        for (uint64_t g = 0; g < G; ++g) {
            const uint32_t* blk = gathered1 + g * w1;
            for (uint64_t t = 0; t < H; ++t) tot[t] += blk[q * H + t];
            S += std::min<uint64_t>(blk[B * H + q], R);
        }
        const uint64_t re = std::min<uint64_t>(R, S);
        reff[q] = (uint32_t)re;
        own_cnt[q] = 0;
        const uint64_t n = std::min<uint64_t>(gathered1[rank * w1 + B * H + q], R);
        if (re == 0 || n == 0) continue;
        uint64_t T = 0, cum = 0;
        while (T < H && cum + tot[T] < re) cum += tot[T++];  // cum = entries below T
        if (T == H) T = H - 1;
        uint64_t tb = 0;
        for (uint64_t g = 0; g < rank; ++g) tb += gathered1[g * w1 + q * H + T];
        const uint64_t need = re - cum, tied = gathered1[rank * w1 + q * H + T];
        const uint64_t quota = need > tb ? std::min(need - tb, tied) : 0;
        mine.clear();
        for (uint64_t i = 0; i < n; ++i) mine.push_back(((uint64_t)m_dist[q * R + i] << 32) | m_rows[q * R + i]);
        std::sort(mine.begin(), mine.end());
        uint32_t c = 0, ties = 0;
        for (const uint64_t key : mine) {
            const uint64_t d = key >> 32;
            if (d > T || (d == T && ties++ >= quota)) break;
            own_rows[q * R + c] = (uint32_t)key;
            own_dist[q * R + c] = (uint32_t)d;
            ++c;
        }
        own_cnt[q] = c;
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
