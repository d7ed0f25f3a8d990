// gvdb_bigr.hip — multi_stage_search at the reference's DEFAULT rescore depth.
//
// BinaryQuantizationConfig::default() sets rescore_ratio = 0.1
// (src/quantization.rs:27), so multi_stage_search reranks R = (N as f32 * 0.1)
// as usize candidates (quantization.rs:178-179): 100K per query at 1M rows,
// far beyond the LDS select (<= 8192 keys) of the regular stage 1.  Batched
// here, for every query of the batch at once:
//
//   stage 1   the regular sample -> threshold -> scan (k_scan_mx5 / k_scan)
//             into a candidate buffer sized for R, then k_select_big per
//             query: exact top-R MEMBERSHIP by (Hamming, row) -- histogram of
//             the buffered distances -> T_R, every key below T_R, and the
//             first R - count(< T_R) rows tied at T_R in row order (radix
//             select over the row index).  No sort: the order among the R is
//             restored exactly by the final step.  A query whose buffer cannot
//             certify (fewer than R keys passed the estimate, or overflow)
//             is recomputed by the same block over all rows.
//   stage 2   k_rerank over the R members (exact cosine, reference fold order)
//   final     k_topk_big per query: the first k of the reference's stable
//             cosine sort of the stage-1 list = the k smallest keys
//             (~order(cos), Hamming, row); radix select on the 32-bit cosine
//             order, ties resolved by (Hamming, row); take(k), then orphan rows
//             are dropped, as in k_final_sort.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "gvdb_device.h"
#include "gvdb_internal.h"

namespace gvdb {

constexpr int kBigThreads = 1024;

__device__ __forceinline__ uint32_t big_dist(const uint4* __restrict__ codes, uint64_t cap, uint32_t W4,
                                             const uint4* __restrict__ qc, uint64_t n) {
    uint32_t d = 0;
    for (uint32_t w = 0; w < W4; ++w) {
        const uint4 c = codes[(uint64_t)w * cap + n], q = qc[w];
        d += __popc(c.x ^ q.x) + __popc(c.y ^ q.y) + __popc(c.z ^ q.z) + __popc(c.w ^ q.w);
    }
    return d;
}

// Wave-aggregated append of (row, d) to the query's member list.
__device__ __forceinline__ void big_append(bool keep, uint32_t row, uint32_t d, uint32_t* s_n, uint32_t* rows,
                                           uint32_t* dist, uint32_t R) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t m = __ballot(keep);
    if (!m) return;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(s_n, (uint32_t)__popcll(m));
    base = __shfl(base, 0);
    const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (keep && pos < R) {
        rows[pos] = row;
        dist[pos] = d;
    }
}

// LDS: hist [(D + 4) & ~3] u32, then bins [2048] u32.
__global__ __launch_bounds__(kBigThreads) void k_select_big(const uint32_t* __restrict__ counts,
                                                            const uint64_t* __restrict__ buf, uint32_t bufcap,
                                                            uint32_t D, uint32_t R, const uint4* __restrict__ codes,
                                                            uint64_t cap, uint32_t N, uint32_t W4,
                                                            const uint4* __restrict__ qcodes,
                                                            uint32_t* __restrict__ fail, uint32_t* __restrict__ any_fail,
                                                            uint32_t* __restrict__ s1_rows,
                                                            uint32_t* __restrict__ s1_dist, int force_rescan) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    uint32_t* bins = hist + ((D + 4u) & ~3u);
    __shared__ uint32_t s_T, s_lt, s_n, s_cut, s_below, s_tie, wcnt[kBigThreads / 64];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
    const uint32_t cnt = counts[q];
    const uint64_t* b = buf + (uint64_t)q * bufcap;
    const uint4* qc = qcodes + (uint64_t)q * W4;
    uint32_t* orow = s1_rows + (uint64_t)q * R;
    uint32_t* odist = s1_dist + (uint64_t)q * R;
    const bool rescan = cnt < R || cnt > bufcap || force_rescan;
    for (uint32_t i = tid; i <= D; i += nt) hist[i] = 0u;
    if (tid == 0) s_n = 0u;
    __syncthreads();
    if (rescan) {
        for (uint64_t n = tid; n < N; n += nt) atomicAdd(&hist[big_dist(codes, cap, W4, qc, n)], 1u);
    } else {
        for (uint32_t i = tid; i < cnt; i += nt) atomicAdd(&hist[(uint32_t)(b[i] >> 32)], 1u);
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t t = wave_find_cum(hist, D + 1u, R);
        const uint32_t lt = wave_sum_below(hist, t);
        if (tid == 0) {
            s_T = t;
            s_lt = lt;
        }
    }
    __syncthreads();
    const uint32_t T = s_T, need = R - s_lt;
    if (rescan) {
        // every row in order: d < T, then the first `need` rows tied at T
        if (tid == 0) s_tie = 0u;
        __syncthreads();
        for (uint64_t base = 0; base < N; base += nt) {
            const uint64_t n = base + tid;
            const uint32_t d = n < N ? big_dist(codes, cap, W4, qc, n) : ~0u;
            uint32_t tot;
            const uint32_t rank = s_tie + big_prefix(d == T, wcnt, &tot);
            big_append(d < T || (d == T && rank < need), (uint32_t)n, d, &s_n, orow, odist, R);
            __syncthreads();
            if (tid == 0) s_tie += tot;
            __syncthreads();
        }
        if (tid == 0) {
            fail[q] = 1u;
            atomicOr(any_fail, 1u);
        }
        return;
    }
    uint32_t cut = ~0u;  // tied rows with row <= cut are kept
    if (hist[T] > need) {
        // the need-th smallest row among the keys with d == T: 11 + 11 + 10 bits
        uint32_t left = need, prefix = 0u, pmask = 0u;
        for (int pass = 0; pass < 3; ++pass) {
            const int shift = pass == 0 ? 21 : pass == 1 ? 10 : 0;
            const uint32_t nb = pass == 2 ? 1024u : 2048u, dm = nb - 1u;
            for (uint32_t i = tid; i < nb; i += nt) bins[i] = 0u;
            __syncthreads();
            for (uint32_t i = tid; i < cnt; i += nt) {
                const uint64_t key = b[i];
                const uint32_t row = (uint32_t)key;
                if ((uint32_t)(key >> 32) == T && (row & pmask) == prefix) atomicAdd(&bins[(row >> shift) & dm], 1u);
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
    for (uint32_t i0 = 0; i0 < cnt; i0 += nt) {
        const uint32_t i = i0 + tid;
        uint64_t key = ~0ull;
        if (i < cnt) key = b[i];
        const uint32_t d = (uint32_t)(key >> 32), row = (uint32_t)key;
        big_append(i < cnt && (d < T || (d == T && row <= cut)), row, d, &s_n, orow, odist, R);
    }
}

hipError_t launch_select_big(const Stage1Args& a, hipStream_t s) {
    const uint32_t W4 = code_w4(a.D);
    const size_t lds = (size_t)((a.D + 4u) & ~3u) * 4u + 2048u * 4u;
    hipLaunchKernelGGL(k_select_big, dim3(a.B), dim3(kBigThreads), lds, s, a.counts, a.buf, a.bufcap, a.D, a.R,
                       a.codes, a.cap, a.N, W4, a.qcodes, a.fail, a.any_fail, a.s1_rows, a.s1_dist, a.force_rescan);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ---- dense select (Stage1Args::dense_sel): one block per query over its row of
// f16 dots (k_scan_mx7<DENSE>): the Hamming distance of row n is |q| - dot; the
// members are every row with d < T plus the first R - count(< T) rows tied at
// T in row order -- k_select_big's rule, with every distance known (no
// candidate buffer, nothing to certify).  One pass: wave w histograms its own
// contiguous 1/16 of the rows (private LDS histogram: no atomics shared across
// waves), the sum gives T, and the per-segment counts at T locate the segment
// holding the cut, which alone is rescanned in row order (a block prefix of the
// tied rows) -- instead of three radix passes over every row.  With `tcut` set
// the block writes only the rule, tcut[q] = (T, cut, need, 0): row n is a member
// iff d_n < T or (d_n == T and n <= cut); `mhist` / `mcount`: the members'
// histogram (the deep sharded exchange-1 block).
__device__ __forceinline__ uint32_t dense_d(uint32_t h16, float pc) {
    return (uint32_t)(int)(pc - (float)__builtin_bit_cast(_Float16, (uint16_t)h16));
}

constexpr uint32_t kSdWaves = kBigThreads / 64;
__global__ __launch_bounds__(kBigThreads) void k_select_dense(const uint16_t* __restrict__ dense, uint32_t np,
                                                              uint32_t N, uint32_t D, uint32_t R,
                                                              const uint32_t* __restrict__ qpc,
                                                              uint32_t* __restrict__ s1_rows,
                                                              uint32_t* __restrict__ s1_dist,
                                                              uint32_t* __restrict__ tcut,
                                                              uint32_t* __restrict__ mhist,
                                                              uint32_t* __restrict__ mcount,
                                                              const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t H4 = (D + 4u) & ~3u;
    uint32_t* hist = lds;        // [H4] the query's histogram
    uint32_t* whist = lds + H4;  // [kSdWaves][H4] per wave: its row segment's
    __shared__ uint32_t s_T, s_lt, s_n, s_cut, s_seg, s_left, wsum[kSdWaves];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, nt = blockDim.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint4* dq = (const uint4*)(dense + (uint64_t)q * np);  // 8 rows per 16-B load (np % 32 == 0)
    const float pc = (float)qpc[q];
    const uint32_t nv = (N + 7u) / 8u;
    const uint32_t segv = (nv + kSdWaves - 1u) / kSdWaves;  // 16-B words per wave segment
    for (uint32_t i = tid; i < (kSdWaves + 1u) * H4; i += nt) lds[i] = 0u;
    if (tid == 0) s_n = 0u;
    __syncthreads();
    {
        constexpr uint32_t kU = 4;  // 16-B loads in flight per lane
        uint32_t* wh = whist + wv * H4;
        const uint32_t v1 = min(nv, (wv + 1u) * segv);
        for (uint32_t v = wv * segv + lane; v < v1; v += 64u * kU) {
            uint4 w[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u) w[u] = v + 64u * u < v1 ? dq[v + 64u * u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u) {
                const uint32_t vv = v + 64u * u;
                const uint32_t ws[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (vv < v1 && 8u * vv + (uint32_t)j < N)
                        atomicAdd(&wh[min(dense_d((ws[j >> 1] >> (16 * (j & 1))) & 0xffffu, pc), D)], 1u);
            }
        }
    }
    __syncthreads();
    for (uint32_t t = tid; t <= D; t += nt) {
        uint32_t c = 0u;
#pragma unroll
        for (uint32_t w = 0; w < kSdWaves; ++w) c += whist[w * H4 + t];
        hist[t] = c;
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t t = wave_find_cum(hist, D + 1u, R);
        const uint32_t lt = wave_sum_below(hist, t);
        if (tid == 0) {
            s_T = t;
            s_lt = lt;
        }
    }
    __syncthreads();
    const uint32_t T = s_T, need = R - s_lt;
    if (mhist) {  // the members' histogram: every bin below T, `need` at T (the exchange-1 block)
        uint32_t* out = mhist + (uint64_t)q * (D + 1u);
        for (uint32_t t = tid; t <= D; t += nt) out[t] = t < T ? hist[t] : t == T ? need : 0u;
        if (tid == 0) mcount[q] = R;
    }
    uint32_t cut = ~0u;  // tied rows with row <= cut are members
    if (hist[T] > need) {
        if (tid == 0) {  // the segment holding the need-th tied row, and its rank there
            uint32_t c = 0u, sg = 0u;
            for (; sg + 1u < kSdWaves; ++sg) {
                const uint32_t ws = whist[sg * H4 + T];
                if (c + ws >= need) break;
                c += ws;
            }
            s_seg = sg;
            s_left = need - c;
            s_cut = ~0u;
        }
        __syncthreads();
        const uint32_t sv0 = s_seg * segv, sv1 = min(nv, sv0 + segv), left = s_left;
        uint32_t base = 0u;  // tied rows of the segment before this round
        constexpr uint32_t kR = 4;  // 16-B words per thread per round: 32 consecutive rows
        for (uint32_t it = sv0; it < sv1; it += nt * kR) {  // block-uniform rounds, rows in order
            const uint32_t v = it + tid * kR;
            uint32_t tm = 0u;  // this thread's 32 rows tied at T (bit 8 u + j)
            uint4 w[kR];
#pragma unroll
            for (uint32_t u = 0; u < kR; ++u) w[u] = v + u < sv1 ? dq[v + u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (uint32_t u = 0; u < kR; ++u) {
                const uint32_t ws[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (v + u < sv1 && 8u * (v + u) + (uint32_t)j < N &&
                        dense_d((ws[j >> 1] >> (16 * (j & 1))) & 0xffffu, pc) == T)
                        tm |= 1u << (8u * u + (uint32_t)j);
            }
            const uint32_t cnt = (uint32_t)__popc(tm);
            uint32_t incl = cnt;  // wave-inclusive prefix
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
                if ((int)lane >= off) incl += y;
            }
            if (lane == 63u) wsum[wv] = incl;
            __syncthreads();
            uint32_t offs = 0u, total = 0u;
            for (uint32_t w = 0; w < kSdWaves; ++w) {
                const uint32_t c = wsum[w];
                if (w < wv) offs += c;
                total += c;
            }
            const uint32_t excl = base + offs + incl - cnt;
            if (cnt && excl < left && left <= excl + cnt) {  // the left-th tied row is one of this thread's
                uint32_t r = left - excl, bits = tm;
                while (--r) bits &= bits - 1u;
                s_cut = 8u * v + (uint32_t)__builtin_ctz(bits);
            }
            __syncthreads();
            base += total;
            if (base >= left) break;
        }
        cut = s_cut;
    }
    if (tcut) {
        if (tid == 0) {
            tcut[4u * q] = T;
            tcut[4u * q + 1u] = cut;
            tcut[4u * q + 2u] = need;
            tcut[4u * q + 3u] = 0u;
        }
        return;
    }
    // members (wave-aggregated appends: the list is unordered, as k_select_big's)
    for (uint32_t v0 = 0; v0 < nv; v0 += nt) {
        const uint32_t v = v0 + tid;
        uint4 w = make_uint4(0u, 0u, 0u, 0u);
        if (v < nv) w = dq[v];
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t n = 8u * v + (uint32_t)j;
            const uint32_t d = dense_d((ws[j >> 1] >> (16 * (j & 1))) & 0xffffu, pc);
            const bool keep = v < nv && n < N && (d < T || (d == T && n <= cut));
            big_append(keep, n, d, &s_n, s1_rows + (uint64_t)q * R, s1_dist + (uint64_t)q * R, R);
        }
    }
}

// ---- the rule form of the dense select in parallel (round 5): k_select_dense runs one
// block per query over its whole dense row (a batch of 64 at a 1.25M-row shard: 64
// blocks reading 2.5 MB each, 0.5 ms).  Here the rows are cut into S segments of L
// rows: k_dense_seg_hist (one block per (segment, query)) writes each segment's
// Hamming histogram, seg_hist[q][s][0..D]; k_dense_rule (one block per query) sums
// them, finds T and the tie quota, and rescans only the segment that holds the
// quota-th tied row.  The per-segment histograms stay in memory: the deep sharded
// phase 2 counts a row's tied predecessors from them (k_deep_certify) and k_dense_own
// compacts owned rows from the dense block without member lists.
constexpr uint32_t kSegThreads = 256;
__global__ __launch_bounds__(kSegThreads) void k_dense_seg_hist(const uint16_t* __restrict__ dense, uint32_t np,
                                                                uint32_t N, uint32_t D, const uint32_t* __restrict__ qpc,
                                                                uint32_t S, uint32_t L,
                                                                uint32_t* __restrict__ seg_hist,
                                                                const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t wh_all[];  // [4][H4] one histogram per wave
    const uint32_t sg = blockIdx.x, q = blockIdx.y, tid = threadIdx.x, H = D + 1u, H4 = (H + 3u) & ~3u;
    const uint32_t wv = tid >> 6;
    for (uint32_t i = tid; i < 4u * H4; i += kSegThreads) wh_all[i] = 0u;
    __syncthreads();
    const float pc = (float)qpc[q];
    const uint32_t r0 = sg * L, r1 = min(N, r0 + L);  // L % 8 == 0
    const uint4* dq = (const uint4*)(dense + (uint64_t)q * np);
    uint32_t* wh = wh_all + wv * H4;
    const uint32_t v0 = r0 / 8u, v1 = (r1 + 7u) / 8u;
    constexpr uint32_t kU = 4;  // 16-B loads in flight per thread
    for (uint32_t v = v0 + tid; v < v1; v += kSegThreads * kU) {
        uint4 w[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t vv = v + kSegThreads * u;
            w[u] = vv < v1 ? dq[vv] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t vv = v + kSegThreads * u;
            const uint32_t ws[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (vv < v1 && 8u * vv + (uint32_t)j < r1)
                    atomicAdd(&wh[min(dense_d((ws[j >> 1] >> (16 * (j & 1))) & 0xffffu, pc), D)], 1u);
        }
    }
    __syncthreads();
    uint32_t* out = seg_hist + ((uint64_t)q * S + sg) * H;
    for (uint32_t t = tid; t < H; t += kSegThreads) out[t] = wh_all[t] + wh_all[H4 + t] + wh_all[2 * H4 + t] + wh_all[3 * H4 + t];
}

// the rule of query q from its segment histograms: (T, cut, need, 0) into tcut; optional
// mhist / mcount (the deep exchange-1 block: members below T, `need` at T)
__global__ __launch_bounds__(kBigThreads) void k_dense_rule(const uint32_t* __restrict__ seg_hist, uint32_t S,
                                                            uint32_t L, const uint16_t* __restrict__ dense,
                                                            uint32_t np, uint32_t N, uint32_t D, uint32_t R,
                                                            const uint32_t* __restrict__ qpc,
                                                            uint32_t* __restrict__ tcut, uint32_t* __restrict__ mhist,
                                                            uint32_t* __restrict__ mcount,
                                                            uint32_t* __restrict__ pc_out,
                                                            const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];  // [H]
    __shared__ uint32_t s_T, s_lt, s_seg, s_left, s_cut, wsum[kBigThreads / 64];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, H = D + 1u;
    const uint32_t wv = tid >> 6, lane = tid & 63u;
    const uint32_t* sh = seg_hist + (uint64_t)q * S * H;
    for (uint32_t t = tid; t < H; t += kBigThreads) {
        uint32_t c = 0u;
        for (uint32_t sg = 0; sg < S; ++sg) c += sh[(uint64_t)sg * H + t];
        hist[t] = c;
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t t = wave_find_cum(hist, H, R);
        const uint32_t lt = wave_sum_below(hist, t);
        if (tid == 0) {
            s_T = t;
            s_lt = lt;
        }
    }
    __syncthreads();
    const uint32_t T = s_T, need = R - s_lt;
    if (mhist) {
        uint32_t* out = mhist + (uint64_t)q * H;
        for (uint32_t t = tid; t < H; t += kBigThreads) out[t] = t < T ? hist[t] : t == T ? need : 0u;
        if (tid == 0) mcount[q] = R;
    }
    uint32_t cut = ~0u;
    if (hist[T] > need) {  // block-uniform
        if (tid == 0) {  // the segment holding the need-th tied row, and its rank there
            uint32_t c = 0u, sg = 0u;
            for (; sg + 1u < S; ++sg) {
                const uint32_t w = sh[(uint64_t)sg * H + T];
                if (c + w >= need) break;
                c += w;
            }
            s_seg = sg;
            s_left = need - c;
            s_cut = ~0u;
        }
        __syncthreads();
        const float pc = (float)qpc[q];
        const uint4* dq = (const uint4*)(dense + (uint64_t)q * np);
        const uint32_t r0 = s_seg * L, r1 = min(N, r0 + L), left = s_left;
        const uint32_t sv0 = r0 / 8u, sv1 = (r1 + 7u) / 8u;
        uint32_t base = 0u;
        for (uint32_t it = sv0; it < sv1; it += kBigThreads) {  // block-uniform rounds, rows in order
            const uint32_t v = it + tid;
            uint32_t tm = 0u;  // this thread's 8 rows tied at T
            if (v < sv1) {
                const uint4 w = dq[v];
                const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (8u * v + (uint32_t)j < r1 && dense_d((ws[j >> 1] >> (16 * (j & 1))) & 0xffffu, pc) == T)
                        tm |= 1u << j;
            }
            uint32_t total;
            const uint32_t excl = base + block_scan_u32((uint32_t)__popc(tm), wsum, &total);
            const uint32_t cnt = (uint32_t)__popc(tm);
            if (cnt && excl < left && left <= excl + cnt) {
                uint32_t r = left - excl, bits = tm;
                while (--r) bits &= bits - 1u;
                s_cut = 8u * v + (uint32_t)__builtin_ctz(bits);
            }
            base += total;
            if (base >= left) break;
        }
        __syncthreads();
        cut = s_cut;
    }
    (void)wv;
    (void)lane;
    if (tid == 0) {
        if (pc_out) pc_out[q] = qpc[q];  // |q| for the deep sharded phase 2 (the stage-1 operands do not outlive it)
        tcut[4u * q] = T;
        tcut[4u * q + 1u] = cut;
        tcut[4u * q + 2u] = need;
        tcut[4u * q + 3u] = 0u;
    }
}

// segments of a dense row: S segments of L rows (L % 256 == 0), S <= smax
void dense_segments(uint32_t N, uint32_t smax, uint32_t* S, uint32_t* L) {
    const uint32_t s0 = std::max<uint32_t>(1u, std::min<uint32_t>(smax, kDenseSegs));
    uint32_t l = ((N + s0 - 1u) / s0 + 255u) & ~255u;
    if (l == 0) l = 256u;
    *L = l;
    *S = std::max<uint32_t>(1u, (N + l - 1u) / l);
}

// ---- the byte form of the parallel rule (round 6, Stage1Args::dense8) ----------
// The f16 dense block of the certified default depth (B x N x 2 B: 5.1 GB per batch of
// 256 at 10M rows) was written by the scan at ~2.5 TB/s and read back by the segment
// histograms: 3 of the 5.7 ms step.  The rule only needs the distances near T, so a
// pair is stored as one byte b = clamp(d - base, 0, 255) around a per-query window:
//   k_dense_base      one block per query: the Hamming histogram of an 8192-row sample (64
//                     spread chunks of 128 consecutive rows), its quantile at R / N -> t_est; base = t_est - 127 (>= 0),
//                     hi = the sample's quantile at target + 6 sqrt(target) + 16 (at least
//                     t_est + 2, at most base + 254): the histograms count d <= hi only;
//   k_dense_seg_hist8 the segment histograms over bytes <= hi - base (d-space bins
//                     [base, hi] of seg_hist; no other bin is written or read);
//   k_dense_rule8     T and the tie cut from them as k_dense_rule, or -- when T is not
//                     strictly inside the window (cum(hi) < R, or T == base > 0: rows
//                     below base share byte 0) -- rule mode 5: k_deep_certify then fails
//                     the batch and the exact fallback (gated bq_search) answers it.
// Exact whenever it certifies: inside the window every byte is d - base exactly.
constexpr uint32_t kBaseThreads = 1024;
constexpr uint32_t kBaseSample = 8192;  // 64 chunks of 128 consecutive rows (coalesced plane loads)
constexpr uint32_t kRuleInvalid = 5u;   // tcut mode: no rule (the window missed T)
template <int W4>
__global__ __launch_bounds__(kBaseThreads) void k_dense_base(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                             uint32_t D, uint32_t R, const uint4* __restrict__ qcodes,
                                                             uint32_t B, uint32_t* __restrict__ qwin, int shift,
                                                             const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    extern __shared__ uint32_t hist[];  // [D + 1]
    const uint32_t q = blockIdx.x, tid = threadIdx.x, H = D + 1u;
    for (uint32_t t = tid; t < H; t += kBaseThreads) hist[t] = 0u;
    uint4 qc[W4];
#pragma unroll
    for (int p = 0; p < W4; ++p) qc[p] = qcodes[(uint64_t)q * W4 + p];
    __syncthreads();
    const uint32_t S = min(N, kBaseSample);  // N <= S: every row (t_est = T)
    constexpr uint32_t kPer = kBaseSample / kBaseThreads;
    uint32_t dv[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {  // every load of the thread in flight together
        const uint32_t i = tid + k * kBaseThreads;
        const uint32_t n = N <= kBaseSample ? min(i, N - 1u)
                                            : (uint32_t)((uint64_t)(i >> 7) * (N - 128u) / 63u) + (i & 127u);
        uint4 c[W4];
#pragma unroll
        for (int p = 0; p < W4; ++p) c[p] = codes[(uint64_t)p * cap + n];
        uint32_t d = 0;
#pragma unroll
        for (int p = 0; p < W4; ++p)
            d += __popc(c[p].x ^ qc[p].x) + __popc(c[p].y ^ qc[p].y) + __popc(c[p].z ^ qc[p].z) +
                 __popc(c[p].w ^ qc[p].w);
        dv[k] = d;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
        if (tid + k * kBaseThreads < S) atomicAdd(&hist[min(dv[k], D)], 1u);
    __syncthreads();
    if (tid < 64u) {
        const uint32_t target = max(1u, (uint32_t)(((uint64_t)R * S + N - 1u) / N));
        // shift (tests, GVDB_DENSE8_SHIFT): a deliberately wrong estimate -- the rule must then fail
        const uint32_t t = (uint32_t)min(max((int)wave_find_cum(hist, H, target) + shift, 0), (int)D);
        const uint32_t tgt_hi = min(S, target + (uint32_t)(6.0f * sqrtf((float)target)) + 16u);
        const uint32_t th = (uint32_t)min(max((int)wave_find_cum(hist, H, tgt_hi) + shift, 0), (int)D);
        if (tid == 0) {
            const uint32_t base = t > 127u ? t - 127u : 0u;
            const uint32_t hi = min(min(max(th, t + 2u), base + 254u), D);
            qwin[q] = base;
            qwin[B + q] = hi;
        }
    }
}

// the blocked byte layout (k_scan_mx7<..., D8>): unit v = half v & 1 of sub-tile v / 2 of query q
// as one uint4; its byte j is row 32 (v / 2) + d8_row(v & 1, j)
__device__ __forceinline__ const uint4* d8_at(const uint8_t* dense, uint32_t bg, uint32_t q, uint32_t v) {
    return (const uint4*)(dense + ((uint64_t)(v >> 4) * bg + q) * 256u + 16u * (v & 15u));
}
__device__ __forceinline__ uint32_t d8_row(uint32_t h, uint32_t j) { return 8u * (j >> 2) + 4u * h + (j & 3u); }

__global__ __launch_bounds__(kSegThreads) void k_dense_seg_hist8(const uint8_t* __restrict__ dense, uint32_t bg,
                                                                 uint32_t N, uint32_t D,
                                                                 const uint32_t* __restrict__ qwin, uint32_t Bt,
                                                                 uint32_t S, uint32_t L,
                                                                 uint32_t* __restrict__ seg_hist,
                                                                 const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ uint32_t wh_all[4][256];  // one histogram of bytes per wave
    // grid (query, segment): consecutive blocks read neighbouring 256-B pieces of one region
    const uint32_t q = blockIdx.x, sg = blockIdx.y, tid = threadIdx.x, H = D + 1u;
    const uint32_t wv = tid >> 6;
    for (uint32_t i = tid; i < 4u * 256u; i += kSegThreads) (&wh_all[0][0])[i] = 0u;
    __syncthreads();
    const uint32_t base = qwin[q], hb = qwin[Bt + q] - base;  // bytes 0 .. hb are counted (hb <= 254)
    const uint32_t r0 = sg * L, r1 = min(N, r0 + L);  // L % 256 == 0
    uint32_t* wh = wh_all[wv];
    // 16-byte units of whole sub-tiles (a sub-tile's two units interleave its rows)
    const uint32_t v0 = r0 / 16u, v1 = 2u * ((r1 + 31u) / 32u);
    constexpr uint32_t kU = 4;  // 16-B loads in flight per thread
    for (uint32_t v = v0 + tid; v < v1; v += kSegThreads * kU) {
        uint4 w[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t vv = v + kSegThreads * u;
            w[u] = vv < v1 ? *d8_at(dense, bg, q, vv) : make_uint4(~0u, ~0u, ~0u, ~0u);  // 255: never counted
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t vv = v + kSegThreads * u;
            const uint32_t ws[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t b = (ws[j >> 2] >> (8 * (j & 3))) & 0xffu;
                if (b <= hb && 32u * (vv >> 1) + d8_row(vv & 1u, (uint32_t)j) < r1) atomicAdd(&wh[b], 1u);
            }
        }
    }
    __syncthreads();
    uint32_t* out = seg_hist + ((uint64_t)q * S + sg) * H + base;  // d-space bins base .. base + hb
    for (uint32_t t = tid; t <= hb; t += kSegThreads) out[t] = wh_all[0][t] + wh_all[1][t] + wh_all[2][t] + wh_all[3][t];
}

__global__ __launch_bounds__(kBigThreads) void k_dense_rule8(const uint32_t* __restrict__ seg_hist, uint32_t S,
                                                             uint32_t L, const uint8_t* __restrict__ dense,
                                                             uint32_t bg, uint32_t N, uint32_t D, uint32_t R,
                                                             const uint32_t* __restrict__ qwin, uint32_t Bt,
                                                             uint32_t* __restrict__ tcut,
                                                             const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ uint32_t hist[256];  // the window's bins (byte b = distance base + b)
    __shared__ uint32_t s_T, s_lt, s_seg, s_left, s_cut, wsum[kBigThreads / 64];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, H = D + 1u;
    const uint32_t base = qwin[q], hw = qwin[Bt + q] - base + 1u;  // bins 0 .. hw - 1
    const uint32_t* sh = seg_hist + (uint64_t)q * S * H + base;
    for (uint32_t t = tid; t < hw; t += kBigThreads) {
        uint32_t c = 0u;
        for (uint32_t sg = 0; sg < S; ++sg) c += sh[(uint64_t)sg * H + t];
        hist[t] = c;
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t t = wave_find_cum(hist, hw, R);
        const uint32_t lt = wave_sum_below(hist, t);
        if (tid == 0) {
            s_T = t;
            s_lt = lt;
        }
    }
    __syncthreads();
    const uint32_t tb = s_T, lt = s_lt;
    // T strictly inside the window: cum(hi) reaches R, and byte 0 (d <= base) is exact or below T
    if (lt + hist[tb] < R || (tb == 0u && base > 0u)) {
        if (tid == 0) {
            tcut[4u * q] = 0u;
            tcut[4u * q + 1u] = 0u;
            tcut[4u * q + 2u] = 0u;
            tcut[4u * q + 3u] = kRuleInvalid;
        }
        return;
    }
    const uint32_t need = R - lt;
    uint32_t cut = ~0u;
    if (hist[tb] > need) {  // block-uniform: the segment holding the need-th tied row, and its rank there
        if (tid == 0) {
            uint32_t c = 0u, sg = 0u;
            for (; sg + 1u < S; ++sg) {
                const uint32_t w = sh[(uint64_t)sg * H + tb];
                if (c + w >= need) break;
                c += w;
            }
            s_seg = sg;
            s_left = need - c;
            s_cut = ~0u;
        }
        __syncthreads();
        const uint32_t r0 = s_seg * L, r1 = min(N, r0 + L), left = s_left;
        const uint32_t st0 = r0 / 32u, st1 = (r1 + 31u) / 32u;  // sub-tiles: one per thread per round
        uint32_t done = 0u;
        for (uint32_t it = st0; it < st1; it += kBigThreads) {  // block-uniform rounds, rows in order
            const uint32_t t = it + tid;
            uint32_t tm = 0u;  // this thread's 32 rows tied at T, bit = row within the sub-tile
            if (t < st1) {
#pragma unroll
                for (uint32_t hh = 0; hh < 2; ++hh) {
                    const uint4 w = *d8_at(dense, bg, q, 2u * t + hh);
                    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        const uint32_t rr = d8_row(hh, (uint32_t)j);
                        if (32u * t + rr < r1 && ((ws[j >> 2] >> (8 * (j & 3))) & 0xffu) == tb) tm |= 1u << rr;
                    }
                }
            }
            uint32_t total;
            const uint32_t excl = done + block_scan_u32((uint32_t)__popc(tm), wsum, &total);
            const uint32_t cnt = (uint32_t)__popc(tm);
            if (cnt && excl < left && left <= excl + cnt) {
                uint32_t r = left - excl, bits = tm;
                while (--r) bits &= bits - 1u;
                s_cut = 32u * t + (uint32_t)__builtin_ctz(bits);
            }
            done += total;
            if (done >= left) break;
        }
        __syncthreads();
        cut = s_cut;
    }
    if (tid == 0) {
        tcut[4u * q] = base + tb;
        tcut[4u * q + 1u] = cut;
        tcut[4u * q + 2u] = need;
        tcut[4u * q + 3u] = 0u;
    }
}

hipError_t launch_dense_base(const Stage1Args& a, hipStream_t s) {
    if (a.B == 0) return hipSuccess;
    if (!a.qwin || !a.qcodes || a.D >= 4096u) return hipErrorInvalidValue;
    const char* sh = getenv("GVDB_DENSE8_SHIFT");
    const int shift = sh ? atoi(sh) : 0;
    const uint32_t W4 = code_w4(a.D);
    auto kern = W4 == 2 ? k_dense_base<2> : W4 == 3 ? k_dense_base<3> : W4 == 4 ? k_dense_base<4> : k_dense_base<6>;
    if (W4 != 2 && W4 != 3 && W4 != 4 && W4 != 6) return hipErrorInvalidValue;  // the FP4 scan's widths
    hipLaunchKernelGGL(kern, dim3(a.B), dim3(kBaseThreads), (size_t)(a.D + 1u) * 4u, s, a.codes, a.cap, a.N, a.D,
                       a.R, a.qcodes, a.B, a.qwin, shift, a.gate);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_select_dense(const Stage1Args& a, uint32_t g0, uint32_t bg, hipStream_t s) {
    if (bg == 0) return hipSuccess;
    if (a.R > a.N || !a.dense) return hipErrorInvalidValue;  // every list slot must be filled
    if (a.dense8) {  // the byte form (rule only)
        if (!a.seg_hist || !a.tcut || !a.qwin || a.mhist || a.dense_keep) return hipErrorInvalidValue;
        const uint32_t H = a.D + 1u;
        const uint8_t* dn = (const uint8_t*)a.dense;
        uint32_t* sh = a.seg_hist + (uint64_t)g0 * a.seg_n * H;
        if (a.seg_len % 256u) return hipErrorInvalidValue;  // segments of whole 256-row regions
        hipLaunchKernelGGL(k_dense_seg_hist8, dim3(bg, a.seg_n), dim3(kSegThreads), 0, s, dn, bg, a.N, a.D,
                           a.qwin + g0, a.B, a.seg_n, a.seg_len, sh, a.gate);
        GVDB_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_dense_rule8, dim3(bg), dim3(kBigThreads), 0, s, sh, a.seg_n, a.seg_len, dn, bg, a.N, a.D,
                           a.R, a.qwin + g0, a.B, a.tcut + 4ull * g0, a.gate);
        GVDB_LAUNCH_CHECK();
        return hipSuccess;
    }
    if (a.seg_hist && a.tcut) {  // the parallel rule form
        const uint32_t H = a.D + 1u;
        const uint16_t* dn = a.dense + (a.dense_keep ? (uint64_t)g0 * a.dense_np : 0ull);
        uint32_t* sh = a.seg_hist + (uint64_t)g0 * a.seg_n * H;
        hipLaunchKernelGGL(k_dense_seg_hist, dim3(a.seg_n, bg), dim3(kSegThreads), (size_t)4u * ((H + 3u) & ~3u) * 4u,
                           s, dn, a.dense_np, a.N, a.D, a.qpc + g0, a.seg_n, a.seg_len, sh, a.gate);
        GVDB_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_dense_rule, dim3(bg), dim3(kBigThreads), (size_t)H * 4u, s, sh, a.seg_n, a.seg_len, dn,
                           a.dense_np, a.N, a.D, a.R, a.qpc + g0, a.tcut + 4ull * g0,
                           a.mhist ? a.mhist + (uint64_t)g0 * H : nullptr, a.mcount ? a.mcount + g0 : nullptr,
                           a.pc_out ? a.pc_out + g0 : nullptr, a.gate);
        GVDB_LAUNCH_CHECK();
        return hipSuccess;
    }
    const size_t lds = (size_t)(kSdWaves + 1u) * ((a.D + 4u) & ~3u) * 4u;
    if (lds > 160u * 1024u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_select_dense, dim3(bg), dim3(kBigThreads), lds, s, a.dense, a.dense_np, a.N, a.D, a.R,
                       a.qpc + g0, a.tcut ? nullptr : a.s1_rows + (uint64_t)g0 * a.R,
                       a.tcut ? nullptr : a.s1_dist + (uint64_t)g0 * a.R, a.tcut ? a.tcut + 4ull * g0 : nullptr,
                       a.mhist ? a.mhist + (uint64_t)g0 * (a.D + 1u) : nullptr, a.mcount ? a.mcount + g0 : nullptr,
                       a.gate);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ---- certified default depth: multi_stage_search at R = 0.1 N without the
// rerank of R rows per query.  The exact cosine top-K2 list of the WHOLE shard
// (the flat path: i8 / bf16 candidates, exact rerank in the reference's fold,
// certified; entries in (cos desc, row) order) holds every row whose cosine
// exceeds its last entry's.  The stage-1 members among it (k_select_dense's
// rule (T, cut), Hamming recomputed from the codes), ordered by (cos desc,
// Hamming, row) -- the reference's stable cosine sort of its Hamming-ordered
// candidates (quantization.rs:165-190) -- are the query's result whenever the
// min(k, R)-th of them scores STRICTLY above the list's last entry: every
// member scoring that high is then in the list, ties included.  Otherwise the
// query fails and the caller reranks the batch the regular way.  The deep
// sharded phase 2 passes a rule without a cut (mode 3): a listed row tied at T
// is then resolved by counting the rank's member-list rows tied at T below it
// (member iff fewer than `need`), only for queries with such a row.  One block
// per query; wave 0 holds the list, one lane per entry (K2 <= 64).
constexpr uint32_t kCertThreads = 1024;
__global__ __launch_bounds__(kCertThreads) void k_deep_certify(
    const uint64_t* __restrict__ frow, const float* __restrict__ fsc, const uint32_t* __restrict__ fn, uint32_t K2,
    const uint32_t* __restrict__ tcut, const uint4* __restrict__ codes, uint64_t cap, uint32_t W4,
    const uint4* __restrict__ qcodes, uint32_t k, uint32_t R, const uint64_t* __restrict__ ids,
    uint64_t* __restrict__ out_ids, float* __restrict__ out_scores, uint32_t* __restrict__ out_n,
    uint32_t* __restrict__ fail, const uint32_t* __restrict__ kcnt, uint32_t* __restrict__ block2,
    const uint32_t* __restrict__ reff, const uint32_t* __restrict__ m_rows, const uint32_t* __restrict__ m_dist,
    uint32_t mlen, const uint32_t* __restrict__ list_fail, const uint32_t* __restrict__ seg_hist, uint32_t seg_n,
    uint32_t seg_len, uint32_t seg_h, const uint16_t* __restrict__ dense, uint32_t dense_np) {
    __shared__ uint32_t s_trow[64], s_cnt[64];
    __shared__ uint32_t s_nt;
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u;
    if (list_fail && *list_fail != 0u) {  // the exact list itself was not certified: nothing to certify
        if (tid == 0) atomicOr(fail, 1u);
        return;
    }
    const uint32_t n = min(fn[q], K2);
    const uint32_t T = tcut[4u * q], cut = tcut[4u * q + 1u], need = tcut[4u * q + 2u];
    // 0: cut, 2: no tied member, 3: the tie rank counted in the member list (deep sharded phase 2)
    const uint32_t mode = tcut[4u * q + 3u];
    if (mode == kRuleInvalid) {  // the byte form's window missed T: no rule, the batch takes the fallback
        if (tid == 0) atomicOr(fail, 1u);
        return;
    }
    const bool lazy = mode == 3u && (m_rows || seg_hist);
    bool mem = false, tied = false;
    uint32_t row = 0u, d = 0u, o = ~0u;  // o: ascending = cosine descending
    if (tid < 64u) {
        if (lane < n) {
            row = (uint32_t)frow[(uint64_t)q * K2 + lane];
            const float sc = fsc[(uint64_t)q * K2 + lane];
            d = big_dist(codes, cap, W4, qcodes + (uint64_t)q * W4, row);
            tied = d == T;
            mem = d < T || (tied && mode == 0u && row <= cut);
            o = ~f32_order(sc);
        }
        const uint64_t tm = __ballot(tied && lazy);
        if (tied && lazy) {
            const uint32_t i = (uint32_t)__popcll(tm & ((1ull << lane) - 1ull));
            s_trow[i] = row;
            s_cnt[i] = 0u;
        }
        if (lane == 0) s_nt = (uint32_t)__popcll(tm);
    }
    __syncthreads();
    const uint32_t nt = s_nt;
    if (nt && mode == 3u && seg_hist) {  // block-uniform: the shard's rows tied at T below each listed tied row,
        // from the segment histograms (whole segments) and the dense block (the row's own segment)
        uint32_t pcq = 0u;
        for (uint32_t w = 0; w < W4; ++w) {
            const uint4 c = qcodes[(uint64_t)q * W4 + w];
            pcq += (uint32_t)(__popc(c.x) + __popc(c.y) + __popc(c.z) + __popc(c.w));
        }
        const float pc = (float)pcq;
        const uint32_t* sh = seg_hist + (uint64_t)q * seg_n * seg_h;
        const uint4* dq = (const uint4*)(dense + (uint64_t)q * dense_np);
        for (uint32_t i = 0; i < nt; ++i) {
            const uint32_t r = s_trow[i], sg = r / seg_len;
            uint32_t c = 0u;
            for (uint32_t t = tid; t < sg; t += kCertThreads) c += sh[(uint64_t)t * seg_h + T];
            const uint32_t v0 = sg * seg_len / 8u, v1 = (r + 7u) / 8u;
            for (uint32_t v = v0 + tid; v < v1; v += kCertThreads) {
                const uint4 w = dq[v];
                const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    c += (8u * v + (uint32_t)j < r && dense_d((ws[j >> 1] >> (16 * (j & 1))) & 0xffffu, pc) == T) ? 1u
                                                                                                                 : 0u;
            }
            if (c) atomicAdd(&s_cnt[i], c);
        }
        __syncthreads();
    } else if (nt && mode == 3u) {  // block-uniform: the member list's rows tied at T below each listed tied row
        const uint32_t* mr = m_rows + (uint64_t)q * mlen;
        const uint32_t* md = m_dist + (uint64_t)q * mlen;
        constexpr uint32_t kU = 32;  // 4-B loads in flight per thread (a 1M-entry list: 32 rounds)
        for (uint32_t i0 = 0; i0 < mlen; i0 += kCertThreads * kU) {
            uint32_t dv[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u) {
                const uint32_t i = i0 + u * kCertThreads + tid;
                dv[u] = i < mlen ? md[i] : ~0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u) {
                if (dv[u] != T) continue;
                const uint32_t r = mr[i0 + u * kCertThreads + tid];
                for (uint32_t i = 0; i < nt; ++i)
                    if (r < s_trow[i]) atomicAdd(&s_cnt[i], 1u);
            }
        }
        __syncthreads();
    }
    if (tid >= 64u) return;
    if (nt) {
        const uint64_t tm = __ballot(tied && lazy);
        if (tied && lazy) mem = s_cnt[(uint32_t)__popcll(tm & ((1ull << lane) - 1ull))] < need;
    }
    uint32_t rank = 0u;  // among the members by (cos desc, Hamming, row)
    for (uint32_t j = 0; j < n; ++j) {
        const uint32_t oj = __shfl(o, j), dj = __shfl(d, j), rj = __shfl(row, j);
        const bool mj = __shfl((int)mem, j) != 0;
        if (mj && (oj < o || (oj == o && (dj < d || (dj == d && rj < row))))) ++rank;
    }
    const uint32_t m = (uint32_t)__popcll(__ballot(mem));
    const uint32_t kk = min(k, kcnt ? kcnt[q] : R);
    const uint32_t o_last = __shfl(o, n > 0u ? n - 1u : 0u);
    const uint64_t at_k = __ballot(mem && kk > 0u && rank == kk - 1u);
    const uint32_t o_k = __shfl(o, at_k ? (uint32_t)__builtin_ctzll(at_k) : 0u);
    const bool ok = kk == 0u || (n == K2 && m >= kk && o_k < o_last);
    if (!ok) {
        if (lane == 0) atomicOr(fail, 1u);
        return;
    }
    if (block2) {  // the deep sharded exchange-2 entry: {cos bits, Hamming, id lo, id hi}, then meta
        if (mem && rank < kk) {
            const uint64_t id = ids ? ids[row] : (uint64_t)row;
            uint32_t* ent = block2 + ((uint64_t)q * k + rank) * 4u;
            ent[0] = __float_as_uint(fsc[(uint64_t)q * K2 + lane]);
            ent[1] = d;
            ent[2] = (uint32_t)id;
            ent[3] = (uint32_t)(id >> 32);
        }
        if (lane == 0) {
            const uint32_t Bt = gridDim.x;
            uint32_t* meta = block2 + 4ull * Bt * k;
            meta[q] = kk;
            meta[Bt + q] = reff[q];
            if (q == 0) meta[2 * Bt] = 0u;
        }
        return;
    }
    if (mem && rank < kk) {
        out_ids[(uint64_t)q * k + rank] = ids ? ids[row] : (uint64_t)row;
        out_scores[(uint64_t)q * k + rank] = fsc[(uint64_t)q * K2 + lane];
    }
    if (lane == 0 && out_n) out_n[q] = kk;
}

hipError_t launch_deep_certify(const uint64_t* frow, const float* fsc, const uint32_t* fn, uint32_t K2,
                               const uint32_t* tcut, const uint4* codes, uint64_t cap, uint32_t W4,
                               const uint4* qcodes, uint32_t B, uint32_t k, uint32_t R, const uint64_t* ids,
                               uint64_t* out_ids,
                               float* out_scores, uint32_t* out_n, uint32_t* fail, hipStream_t s,
                               const uint32_t* kcnt, uint32_t* block2, const uint32_t* reff,
                               const uint32_t* m_rows, const uint32_t* m_dist, uint32_t mlen,
                               const uint32_t* list_fail, const uint32_t* seg_hist, uint32_t seg_n,
                               uint32_t seg_len, uint32_t seg_h, const uint16_t* dense, uint32_t dense_np) {
    if (B == 0) return hipSuccess;
    if (K2 == 0 || K2 > 64u || (block2 && !reff)) return hipErrorInvalidValue;
    if (seg_hist && (!dense || seg_n == 0 || seg_len == 0 || seg_len % 8u || seg_h == 0)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_deep_certify, dim3(B), dim3(kCertThreads), 0, s, frow, fsc, fn, K2, tcut, codes, cap, W4,
                       qcodes, k, R, ids, out_ids, out_scores, out_n, fail, kcnt, block2, reff, m_rows,
                       m_dist, mlen, list_fail, seg_hist, seg_n, seg_len, seg_h, dense, dense_np);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// The deep sharded fallback's owned rows without member lists (round 5): one block per
// query walks the dense row in order, 8 rows per thread per round; a row is owned iff
// d < T, or d == T and fewer than `quota` tied rows precede it (tcut[q] = (T, -, quota,
// mode) from k_shard_deep_own's rule form) -- the member-list compaction's set, in row
// order.  Gated like the rerank it feeds.
__global__ __launch_bounds__(kBigThreads) void k_dense_own(const uint16_t* __restrict__ dense, uint32_t np, uint32_t N,
                                                           const uint32_t* __restrict__ tcut,
                                                           const uint32_t* __restrict__ qpc,
                                                           uint32_t* __restrict__ o_rows, uint32_t* __restrict__ o_dist,
                                                           uint32_t ostride, const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ uint32_t wsum[kBigThreads / 64];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const uint32_t T = tcut[4u * q], quota = tcut[4u * q + 2u], mode = tcut[4u * q + 3u];
    const float pc = (float)qpc[q];
    // mode 2 with quota 0 and T = 0 marks "no owned row" (k_shard_deep_own: an empty rank / list)
    const bool none = mode == 2u && quota == 0u && T == 0u;
    const uint4* dq = (const uint4*)(dense + (uint64_t)q * np);
    uint32_t* orw = o_rows + (uint64_t)q * ostride;
    uint32_t* odd = o_dist + (uint64_t)q * ostride;
    const uint32_t nv = (N + 7u) / 8u;
    uint32_t ties = 0u, o = 0u;  // tied rows seen, rows written (block-uniform)
    for (uint32_t it = 0; it < nv && !none; it += kBigThreads) {
        const uint32_t v = it + tid;
        uint32_t dv[8];
        uint32_t lt = 0u, tm = 0u;
        if (v < nv) {
            const uint4 w = dq[v];
            const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t d = 8u * v + (uint32_t)j < N ? dense_d((ws[j >> 1] >> (16 * (j & 1))) & 0xffffu, pc) : ~0u;
                dv[j] = d;
                lt |= (d < T ? 1u : 0u) << j;
                tm |= (d == T ? 1u : 0u) << j;
            }
        }
        uint32_t tt;
        const uint32_t tex = ties + block_scan_u32((uint32_t)__popc(tm), wsum, &tt);
        // this thread's tied rows ranked tex, tex + 1, ...: owned while the rank < quota
        const uint32_t take = quota > tex ? min((uint32_t)__popc(tm), quota - tex) : 0u;
        uint32_t keep = lt, tk = tm;
        for (uint32_t c = 0; c < take; ++c) {
            keep |= tk & (0u - tk);  // lowest remaining tied row
            tk &= tk - 1u;
        }
        uint32_t tot;
        uint32_t pos = o + block_scan_u32((uint32_t)__popc(keep), wsum, &tot);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if ((keep >> j) & 1u) {
                orw[pos] = 8u * v + (uint32_t)j;
                odd[pos] = dv[j];
                ++pos;
            }
        }
        ties += tt;
        o += tot;
    }
}

hipError_t launch_dense_own(const uint16_t* dense, uint32_t np, uint32_t N, const uint32_t* tcut, const uint32_t* qpc,
                            uint32_t B, uint32_t* o_rows, uint32_t* o_dist, uint32_t ostride, const uint32_t* gate,
                            hipStream_t s) {
    if (B == 0) return hipSuccess;
    if (!dense || np % 8u || np < N) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_dense_own, dim3(B), dim3(kBigThreads), 0, s, dense, np, N, tcut, qpc, o_rows, o_dist, ostride,
                       gate);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ---- final: the first k of the stable cosine sort of an unordered stage-1 list
constexpr uint32_t kTopkBigMax = 1024;  // k
constexpr uint32_t kTieLds = 4096;      // tied entries sorted in LDS (more: radix select)

struct TopkLds {
    uint32_t bins[256];
    uint64_t tk[kTieLds];       // ties: (d << 32 | row)
    uint32_t sel[kTopkBigMax];  // selected entry indices
    uint32_t srt[kTopkBigMax];  // sorted order
    uint32_t su[kTopkBigMax];   // selected: ukey
    uint64_t sdr[kTopkBigMax];  // selected: (d << 32 | row)
    uint32_t s_nan, s_cut, s_below, s_nsel, s_ntie;
    uint64_t s_tcut;
};

// The first k = min(kout, n) entries of the unordered list (sc, rw, dd)[0..n)
// by (score order, Hamming, row) -- the stable score sort of the (Hamming,
// row)-ordered stage-1 list -- as entry indices into L.srt[0..k), ascending;
// L.s_nan = a NaN score among the n.  Whole block; returns k.
__device__ uint32_t big_topk_order(TopkLds& L, const float* __restrict__ sc, const uint32_t* __restrict__ rw,
                                   const uint32_t* __restrict__ dd, uint32_t n, uint32_t kout, int descending) {
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint32_t k = min(kout, n);
    auto ukey = [&](uint32_t i) {
        const uint32_t o = f32_order(sc[i]);
        return descending ? ~o : o;  // ascending = better first
    };
    if (tid == 0) {
        L.s_nan = 0u;
        L.s_nsel = 0u;
        L.s_ntie = 0u;
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += nt)
        if (sc[i] != sc[i]) L.s_nan = 1u;
    // U = the k-th smallest ukey: 4 radix passes of 8 bits
    uint32_t left = k, prefix = 0u, pmask = 0u;
    for (int pass = 0; pass < 4 && k > 0; ++pass) {
        const int shift = 24 - 8 * pass;
        for (uint32_t i = tid; i < 256; i += nt) L.bins[i] = 0u;
        __syncthreads();
        for (uint32_t i = tid; i < n; i += nt) {
            const uint32_t u = ukey(i);
            if ((u & pmask) == prefix) atomicAdd(&L.bins[(u >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid < 64) {
            const uint32_t bin = wave_find_cum(L.bins, 256, left);
            const uint32_t below = wave_sum_below(L.bins, bin);
            if (tid == 0) {
                L.s_cut = bin;
                L.s_below = below;
            }
        }
        __syncthreads();
        left -= L.s_below;
        prefix |= L.s_cut << shift;
        pmask |= 255u << shift;
        __syncthreads();
    }
    const uint32_t U = prefix, need = left;  // `need` entries tied at U complete the top k
    // entries strictly better than U (fewer than k), and the ties at U
    for (uint32_t i = tid; i < n && k > 0; i += nt) {
        const uint32_t u = ukey(i);
        if (u < U) {
            L.sel[atomicAdd(&L.s_nsel, 1u)] = i;
        } else if (u == U) {
            const uint32_t t = atomicAdd(&L.s_ntie, 1u);
            if (t < kTieLds) L.tk[t] = ((uint64_t)dd[i] << 32) | i;  // stage-1 order (d, row) resolved below
        }
    }
    __syncthreads();
    const uint32_t nties = L.s_ntie;
    if (k > 0 && nties <= kTieLds) {
        // order the ties by (d, row): re-key with the row, sort, take `need`
        for (uint32_t t = tid; t < nties; t += nt) {
            const uint32_t i = (uint32_t)L.tk[t];
            L.tk[t] = ((uint64_t)dd[i] << 52) | ((uint64_t)rw[i] << 20) | i;  // d < 2^12, row < 2^32, i < 2^20
        }
        __syncthreads();
        const uint32_t P = next_pow2(max(nties, 1u));
        for (uint32_t t = nties + tid; t < P; t += nt) L.tk[t] = ~0ull;
        __syncthreads();
        bitonic_sort_lds(L.tk, P);
        for (uint32_t t = tid; t < need; t += nt) L.sel[L.s_nsel + t] = (uint32_t)L.tk[t] & 0xfffffu;
        __syncthreads();
    } else if (k > 0) {
        // massive tie (more than kTieLds equal scores): radix select the need-th
        // smallest (d, row) among them, 64-bit key in 8 passes of 8 bits
        uint64_t tpre = 0, tmask = 0;
        uint32_t tl = need;
        for (int pass = 0; pass < 8; ++pass) {
            const int shift = 56 - 8 * pass;
            for (uint32_t i = tid; i < 256; i += nt) L.bins[i] = 0u;
            __syncthreads();
            for (uint32_t i = tid; i < n; i += nt) {
                if (ukey(i) != U) continue;
                const uint64_t key = ((uint64_t)dd[i] << 32) | rw[i];
                if ((key & tmask) == tpre) atomicAdd(&L.bins[(uint32_t)(key >> shift) & 255u], 1u);
            }
            __syncthreads();
            if (tid < 64) {
                const uint32_t bin = wave_find_cum(L.bins, 256, tl);
                const uint32_t below = wave_sum_below(L.bins, bin);
                if (tid == 0) {
                    L.s_cut = bin;
                    L.s_below = below;
                }
            }
            __syncthreads();
            tl -= L.s_below;
            tpre |= (uint64_t)L.s_cut << shift;
            tmask |= 255ull << shift;
            __syncthreads();
        }
        if (tid == 0) L.s_tcut = tpre;
        __syncthreads();
        for (uint32_t i = tid; i < n; i += nt) {
            if (ukey(i) != U) continue;
            const uint64_t key = ((uint64_t)dd[i] << 32) | rw[i];
            if (key <= L.s_tcut) L.sel[atomicAdd(&L.s_nsel, 1u)] = i;  // distinct rows: exactly `need` keys
        }
        __syncthreads();
    }
    // sort the k selected by (ukey, d, row): rank counting over LDS copies
    for (uint32_t a = tid; a < k; a += nt) {
        const uint32_t ia = L.sel[a];
        L.su[a] = ukey(ia);
        L.sdr[a] = ((uint64_t)dd[ia] << 32) | rw[ia];
    }
    __syncthreads();
    for (uint32_t a = tid; a < k; a += nt) {
        const uint32_t ua = L.su[a];
        const uint64_t da = L.sdr[a];
        uint32_t rank = 0;
        for (uint32_t c = 0; c < k; ++c) rank += L.su[c] < ua || (L.su[c] == ua && L.sdr[c] < da);
        L.srt[rank] = L.sel[a];
    }
    __syncthreads();
    return k;
}

__global__ __launch_bounds__(kBigThreads) void k_topk_big(const float* __restrict__ scores,
                                                          const uint32_t* __restrict__ s1_rows,
                                                          const uint32_t* __restrict__ s1_dist, uint32_t R,
                                                          uint32_t kout, int descending,
                                                          const uint64_t* __restrict__ ids, uint64_t row_offset,
                                                          uint64_t* __restrict__ out_ids,
                                                          float* __restrict__ out_scores, uint32_t* __restrict__ out_n,
                                                          uint32_t* __restrict__ nan_flag,
                                                          const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ TopkLds L;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const float* sc = scores + (uint64_t)q * R;
    const uint32_t* rw = s1_rows + (uint64_t)q * R;
    const uint32_t k = big_topk_order(L, sc, rw, s1_dist + (uint64_t)q * R, R, kout, descending);
    if (tid < 64) {  // take(k), then drop orphan rows (index.rs:217-228)
        uint32_t o = 0;
        for (uint32_t i0 = 0; i0 < k; i0 += 64) {
            const uint32_t i = i0 + tid;
            uint64_t id = kOrphan;
            uint32_t e = 0;
            if (i < k) {
                e = min(L.srt[i], R - 1u);  // (an index past the list would need duplicate rows in it)
                id = ids ? ids[rw[e]] : (uint64_t)rw[e] + row_offset;
            }
            const bool keep = i < k && id != kOrphan;
            const uint64_t m = __ballot(keep);
            const uint32_t before = __popcll(m & ((1ull << tid) - 1ull));
            if (keep) {
                out_ids[(uint64_t)q * kout + o + before] = id;
                out_scores[(uint64_t)q * kout + o + before] = sc[e];
            }
            o += __popcll(m);
        }
        const bool poisoned = L.s_nan && R >= 2;
        if (tid == 0) {
            if (poisoned) atomicOr(nan_flag, 1u);
            if (out_n) out_n[q] = poisoned ? GVDB_N_POISONED : o;
        }
    }
}

// Deep sharded search, step 3 (iii): this rank's local top-k of its owned
// entries (m_cos / m_rows / m_dist [B][Rl], own_cnt[q] valid) by (cosine desc,
// Hamming, row) -> the exchange-2 block: {cos bits, Hamming, id lo, id hi}
// (orphans kept: the merge drops them after the global truncation), meta.
__global__ __launch_bounds__(kBigThreads) void k_shard_deep_topk(const float* __restrict__ m_cos,
                                                                 const uint32_t* __restrict__ m_rows,
                                                                 const uint32_t* __restrict__ m_dist,
                                                                 const uint32_t* __restrict__ own_cnt,
                                                                 const uint32_t* __restrict__ reff, uint32_t B,
                                                                 uint32_t Rl, uint32_t kout,
                                                                 const uint64_t* __restrict__ ids, uint32_t err,
                                                                 uint32_t* __restrict__ block2,
                                                                 const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ TopkLds L;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const uint64_t base = (uint64_t)q * Rl;
    const uint32_t c = Rl ? min(own_cnt[q], Rl) : 0u;
    const uint32_t take = big_topk_order(L, m_cos + base, m_rows + base, m_dist + base, c, kout, 1);
    uint32_t* ent = block2 + (uint64_t)q * kout * 4u;
    for (uint32_t t = tid; t < take; t += blockDim.x) {
        const uint32_t e = min(L.srt[t], c - 1u);  // (an index past the list would need duplicate rows in it)
        const uint32_t row = m_rows[base + e];
        const uint64_t id = ids ? ids[row] : (uint64_t)row;
        ent[4 * t + 0] = __float_as_uint(m_cos[base + e]);
        ent[4 * t + 1] = m_dist[base + e];
        ent[4 * t + 2] = (uint32_t)id;
        ent[4 * t + 3] = (uint32_t)(id >> 32);
    }
    if (tid == 0) {
        uint32_t* meta = block2 + 4ull * B * kout;
        const uint32_t re = reff[q];
        meta[q] = take | ((L.s_nan && re >= 2u) ? 0x80000000u : 0u);
        meta[B + q] = re;
        if (q == 0) meta[2 * B] = err;
    }
}

hipError_t launch_shard_deep_topk(const float* m_cos, const uint32_t* m_rows, const uint32_t* m_dist,
                                  const uint32_t* own_cnt, const uint32_t* reff, uint32_t B, uint32_t Rl, uint32_t k,
                                  const uint64_t* ids, uint32_t err, uint32_t* block2, hipStream_t s,
                                  const uint32_t* gate) {
    if (B == 0) return hipSuccess;
    if (k > kTopkBigMax || Rl > kBigRMax) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_shard_deep_topk, dim3(B), dim3(kBigThreads), 0, s, m_cos, m_rows, m_dist, own_cnt, reff, B,
                       Rl, k, ids, err, block2, gate);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_topk_big(const FinalArgs& a, const uint32_t* s1_dist, hipStream_t s) {
    if (a.B == 0) return hipSuccess;
    if (a.kout > kTopkBigMax) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_topk_big, dim3(a.B), dim3(kBigThreads), 0, s, a.scores, a.s1_rows, s1_dist, a.R, a.kout,
                       a.descending, a.ids, a.row_offset, a.out_ids, a.out_scores, a.out_n, a.nan_flag, a.gate);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace gvdb
