// gvdb_flat.hip — K4: flat exact cosine search on the i8 / bf16 MFMA paths for gfx950.
//
// Replaces the per-record cosine loop of BasicVectorStore::vector_search
// (src/storage.rs:296-339, cosine_similarity 851-865) and the flat
// FaissVectorIndex::search (src/index.rs:620-640, cosine_distance 686-700)
// for an index shard held in HBM.  Results are EXACT (identical ids and
// bit-identical f32 scores to the sequential-fold oracle): the MFMA pass only
// nominates candidates, every candidate is re-scored by the exact rerank
// kernel, and a per-query certificate proves no un-nominated row can enter the
// top k (else the caller falls back to the exact full scan).
//
//   approx score  s~(q,x) = dot_bf16(q,x) * (1/|q|) * (1/|x|)   (f32 accumulate)
//   |s~ - cos| <= eps = 2^-8 (bf16 RNE of both operands, Cauchy-Schwarz)
//                      + accumulation/rounding terms (flat_eps below)
//   pass 1 (sample): s~ of every 64th row tile -> per query the m-th largest
//                    sampled score = T_q (expected ~ max(384, 4k) rows >= T_q)
//   pass 2 (emit):   every row with s~ >= T_q is a candidate
//   exact rerank of the candidates (k_rerank, sequential f32 fold)
//   certificate:     k-th best exact score >= T_q + eps  =>  every row that was
//                    not nominated has exact score < T_q + eps <= k-th: exact.
//
// Two element kinds share one kernel body (the byte geometry is identical):
//   bf16: rowsx = bf16 [KC][cap][64],  KC = ceil(D/64),  v_mfma_f32_32x32x16_bf16;
//         eps = 2^-8 (+ rounding terms, flat_eps below) for every pair.
//   i8:   rowsx = int8 [KC][cap][128], KC = ceil(D/128), v_mfma_i32_32x32x32_i8
//         (exact i32 dot of the quantised vectors).  Row x is stored as
//         xq = rint(x * 127/max|x_i|), s_x = max|x_i|/127, with
//         rscale = s_x/|x| and rho_x = |x - s_x xq| / |x| (fp64, rounded up);
//         queries likewise.  |q.x - q^.x^| <= |e_q||x| + |q^||e_x| gives, in
//         cosine units, eps_q = rho_q + (1 + rho_q) max_x rho_x (+ norm and
//         fold rounding terms): half the HBM bytes of bf16 and twice the
//         MFMA rate, for a ~4x wider (still certified) candidate margin.
// Either way a row chunk is 128 B and the mirror is TILE-major,
// [ceil(cap/256)][KC][256][128 B] (fx_off): one chunk of a 256-row tile is a
// contiguous 32 KiB block and a tile's KC chunks are adjacent, so a block
// streams one contiguous KC*32 KiB region per tile (few TLB pages in flight;
// a chunk-major [KC][cap] layout put each step 1-2 GB from the last).
// Queries are [KC][256][128 B].
// Tile = 256 rows x 256 query slots; 8 waves = 2 query halves x 4 row
// quarters, each wave 128 queries x 64 rows = 4 x 2 32x32 MFMA tiles: per
// k-step 6 ds_read_b128 feed 8 MFMAs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "gvdb_device.h"
#include "gvdb_internal.h"

namespace gvdb {

namespace {

typedef int fx_v4i __attribute__((ext_vector_type(4)));
typedef float fx_v16f __attribute__((ext_vector_type(16)));
typedef __bf16 fx_v8bf __attribute__((ext_vector_type(8)));
typedef int fx_v16i __attribute__((ext_vector_type(16)));

constexpr uint32_t kFxThreads = 512;

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// rows f32 [n][D] (rows row0.. of the index) -> rowsb bf16 [KC][cap][64]; one
// thread per (row, 8-element group).  Flags NaN elements.
__global__ __launch_bounds__(256) void k_rows_to_bf16(const float* __restrict__ rows, uint64_t n, uint32_t D,
                                                      uint16_t* __restrict__ rowsb, uint64_t cap,
                                                      uint32_t* __restrict__ nan_flag) {
    const uint32_t KC = fx_kc(D);
    const uint64_t g = (uint64_t)blockIdx.x * 256u + threadIdx.x;  // (row, group of 8) with 8*KC groups per row
    const uint64_t row = g / (8u * KC);
    if (row >= n) return;
    const uint32_t grp = (uint32_t)(g % (8u * KC));
    const uint32_t c = grp >> 3, e0 = c * 64u + (grp & 7u) * 8u;
    uint16_t v[8];
    bool bad = false;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t e = e0 + i;
        const float x = e < D ? rows[row * D + e] : 0.0f;
        bad |= !(fabsf(x) <= 3.4028235e38f);  // NaN or +-inf: the exact scan answers
        v[i] = f32_to_bf16_rne(x);
    }
    if (bad) atomicOr(nan_flag, 1u);
    uint4 o;
    o.x = v[0] | ((uint32_t)v[1] << 16);
    o.y = v[2] | ((uint32_t)v[3] << 16);
    o.z = v[4] | ((uint32_t)v[5] << 16);
    o.w = v[6] | ((uint32_t)v[7] << 16);
    *(uint4*)(rowsb + fx_off(row, c, KC) / 2u + (grp & 7u) * 8u) = o;
}

// queries f32 [B][D] -> qb bf16 [KC][256][64] (slots >= B zero), qinv = 1/|q| (0 for |q| = 0)
__global__ __launch_bounds__(256) void k_queries_to_bf16(const float* __restrict__ q, uint32_t B, uint32_t D,
                                                         const float* __restrict__ qnorm, uint16_t* __restrict__ qb,
                                                         float* __restrict__ qinv, float* __restrict__ qd, float eps) {
    const uint32_t KC = fx_kc(D);
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;  // (slot, group of 8)
    const uint32_t slot = g / (8u * KC);
    if (slot >= kFxQ) return;
    const uint32_t grp = g % (8u * KC);
    const uint32_t c = grp >> 3, e0 = c * 64u + (grp & 7u) * 8u;
    uint16_t v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t e = e0 + i;
        v[i] = f32_to_bf16_rne(slot < B && e < D ? q[(uint64_t)slot * D + e] : 0.0f);
    }
    uint4 o;
    o.x = v[0] | ((uint32_t)v[1] << 16);
    o.y = v[2] | ((uint32_t)v[3] << 16);
    o.z = v[4] | ((uint32_t)v[5] << 16);
    o.w = v[6] | ((uint32_t)v[7] << 16);
    *(uint4*)(qb + ((uint64_t)c * kFxQ + slot) * 64u + (grp & 7u) * 8u) = o;
    if (grp == 0) {
        const float nq = slot < B ? qnorm[slot] : 0.0f;
        qinv[slot] = nq == 0.0f ? 0.0f : 1.0f / nq;
        qd[slot] = eps;
    }
}

// Norm/fold rounding terms shared by both kinds: |x|_f32 vs |x| (each <= (D+2)
// 2^-24 relative) and the reference's sequential fold + division (flat_eps).
__host__ __device__ inline float fx_norm_factor(uint32_t D) { return 1.0f + 4.0f * (float)(D + 2) * 5.9604645e-8f; }
__host__ __device__ inline float fx_fold_slack(uint32_t D) { return 2.0f * (float)(D + 16) * 5.9604645e-8f + 4e-6f; }

// Per-vector symmetric int8 quantisation of one D-vector by one wave: in pass
// p lane l owns elements [1024p + 16l, +16) = 16-B piece (l & 7) of chunk
// 8p + (l >> 3), written to dst + chunk * cstride + piece * 16 (chunks < KC;
// padding elements are 0).  Returns s = max|v|/127 and rho = |v - s*vq| / |v|
// in fp64 (0 for a zero vector) on every lane, and flags non-finite values.
__device__ inline void fx_quantize_i8_wave(const float* __restrict__ v, uint32_t D, uint32_t lane, bool live,
                                           int8_t* __restrict__ dst, uint64_t cstride, float& s_out, double& rho_out,
                                           bool& bad) {
    const uint32_t KC = (D + 127u) / 128u, passes = (KC + 7u) / 8u;
    float amax = 0.0f;
    bool nf = false;
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t e0 = p * 1024u + lane * 16u;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t e = e0 + i;
            const float x = live && e < D ? v[e] : 0.0f;
            nf |= !(fabsf(x) <= 3.4028235e38f);  // NaN or +-inf
            amax = fmaxf(amax, fabsf(x));
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    const float sc = amax / 127.0f;
    const float inv = amax > 0.0f ? 127.0f / amax : 0.0f;
    double e2 = 0.0, n2 = 0.0;
    for (uint32_t p = 0; p < passes; ++p) {
        const uint32_t e0 = p * 1024u + lane * 16u, chunk = p * 8u + (lane >> 3);
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t e = e0 + i;
            const float x = live && e < D ? v[e] : 0.0f;
            float r = rintf(x * inv);
            r = fminf(127.0f, fmaxf(-127.0f, r));
            const int qi = (int)r;
            const double err = (double)x - (double)sc * (double)qi;  // the product is exact in fp64
            e2 += err * err;
            n2 += (double)x * (double)x;
            w[i >> 2] |= ((uint32_t)qi & 0xffu) << (8 * (i & 3));
        }
        if (chunk < KC) *(uint4*)(dst + (uint64_t)chunk * cstride + (lane & 7u) * 16u) = make_uint4(w[0], w[1], w[2], w[3]);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        e2 += __shfl_xor(e2, o);
        n2 += __shfl_xor(n2, o);
    }
    s_out = sc;
    // relative error, rounded up by a generous fp64 margin
    rho_out = n2 > 0.0 ? sqrt(e2 / n2) * (1.0 + 1e-12) + 1e-300 : 0.0;
    bad = __ballot(nf) != 0;
}

// rows f32 [n][D] -> rowsq int8 [KC][cap][128] (KC = ceil(D/128)); one wave per
// row.  rscale[row] = s_x/|x|_f32 (0 for a zero row), rrho[row] = rho_x
// rounded up; non-finite rows flag *bad.
__global__ __launch_bounds__(256) void k_rows_to_i8(const float* __restrict__ rows, const float* __restrict__ norms,
                                                    uint64_t n, uint32_t D, int8_t* __restrict__ rowsq, uint64_t cap,
                                                    float* __restrict__ rscale, float* __restrict__ rrho,
                                                    uint32_t* __restrict__ bad_flag) {
    const uint64_t row = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (row >= n) return;
    float sc;
    double rho;
    bool bad;
    fx_quantize_i8_wave(rows + row * D, D, lane, true, rowsq + fx_off(row, 0, (D + 127u) / 128u),
                        (uint64_t)kFxRows * 128u, sc, rho, bad);
    if (bad && lane == 0) atomicOr(bad_flag, 1u);
    if (lane == 0) {
        const float nx = norms[row];
        rscale[row] = nx == 0.0f ? 0.0f : sc / nx;
        rrho[row] = (float)(rho * (1.0 + 1e-6));
    }
}

// queries f32 [B][D] -> qq int8 [KC][256][128] (slots >= B zero); qinv = s_q/|q|,
// (qa, qd) = the query's terms of the pair bound (epilogue of k_flat_mx):
// qa = c (1 + rho_q), qd = c rho_q + fold slack, c = the norm factor.
__global__ __launch_bounds__(256) void k_queries_to_i8(const float* __restrict__ q, uint32_t B, uint32_t D,
                                                       const float* __restrict__ qnorm, int8_t* __restrict__ qq,
                                                       float* __restrict__ qinv, float* __restrict__ qa,
                                                       float* __restrict__ qd) {
    const uint32_t slot = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (slot >= kFxQ) return;
    const bool live = slot < B;
    float sc;
    double rho;
    bool bad;
    fx_quantize_i8_wave(q + (uint64_t)(live ? slot : 0) * D, D, lane, live, qq + (uint64_t)slot * 128u,
                        (uint64_t)kFxQ * 128u, sc, rho, bad);
    if (lane == 0) {
        const float nq = live ? qnorm[slot] : 0.0f;
        qinv[slot] = nq == 0.0f ? 0.0f : sc / nq;
        const double c = (double)fx_norm_factor(D) * (1.0 + 1e-6);
        qa[slot] = (float)((1.0 + rho) * c);
        // a non-finite query cannot be certified: qd = +inf forces the next tier
        qd[slot] = bad ? __builtin_inff() : (float)(rho * c) + fx_fold_slack(D);
    }
}

// The MFMA pass.  SAMPLE: every `every`-th row tile, approx scores -> smp[q][S].
// EMIT: every tile, rows with approx >= thr[q] -> cand[q][*] (counts[q]).
// Staging: global_load_lds (16 B per lane, no VGPRs), 64 k (128 B) per row and
// chunk; the query chunk (A, L2-resident) is double-buffered, the row chunk (B,
// from HBM) triple-buffered so its loads are issued two chunks ahead: the wait
// at the end of step u retires A(u+1) and B(u+1) with a counted vmcnt and leaves
// B(u+2) in flight across the raw s_barrier.  The 160 KiB of LDS hold only the
// five chunk buffers; thresholds and inverse norms are read from L1/L2 in the
// once-per-tile epilogue.  The LDS image is lane-linear, so the bank-conflict
// swizzle is applied on the global side: 16-B piece j of row r sits at slot
// j ^ ((r >> 1) & 7) of the row's 128 B (conflict-free ds_read_b128 fragments).
template <bool SAMPLE, bool I8>
__global__ __launch_bounds__(kFxThreads, 1) void k_flat_mx(FlatMxArgs a) {
    // five distinct LDS objects (not one indexed array): with every buffer index
    // a compile-time constant the waitcnt pass can tell an in-flight
    // global_load_lds into one buffer from ds_reads of another.  A chunk row is
    // 128 B (64 bf16 or 128 i8).
    __shared__ __attribute__((aligned(16))) uint16_t As0[kFxQ * 64], As1[kFxQ * 64];
    __shared__ __attribute__((aligned(16))) uint16_t Bs0[kFxRows * 64], Bs1[kFxRows * 64], Bs2[kFxRows * 64];
    const char* rowsx = (const char*)a.rowsx;
    const char* qx = (const char*)a.qx;
    auto abuf = [&](auto I) -> uint16_t* {
        if constexpr (decltype(I)::value == 0) return As0; else return As1;
    };
    auto bbuf = [&](auto I) -> uint16_t* {
        if constexpr (decltype(I)::value == 0) return Bs0;
        else if constexpr (decltype(I)::value == 1) return Bs1;
        else return Bs2;
    };

    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t wq = wv & 1u, wr = wv >> 1;  // query half (128), row quarter (64)
    const uint32_t KC = a.KC, N = a.N;
    const uint32_t ntiles_all = (N + kFxRows - 1) / kFxRows;
    const uint32_t every = SAMPLE ? a.every : 1u;
    const uint32_t ntiles = SAMPLE ? (ntiles_all + every - 1) / every : ntiles_all;  // tiles in the list
    const uint32_t G = gridDim.x;
    // tiles of this block: list entries blockIdx.x + j*G; steps u = j*KC + c
    const uint32_t nt = blockIdx.x < ntiles ? (ntiles - blockIdx.x + G - 1) / G : 0;
    const uint32_t nsteps = nt * KC;
    auto tile_of = [&](uint32_t j) { return (blockIdx.x + j * G) * every; };

    // this lane's staging slot: wave wv fills LDS rows [32*wv, 32*wv+32) of each
    // operand, 8 rows (1 KiB) per instruction; lane -> row L/8, slot L%8
    const uint32_t srow0 = wv * 32u + (lane >> 3);
    auto step_of = [&](uint32_t u, uint32_t& t, uint32_t& c) __attribute__((always_inline)) {
        const uint32_t uu = u < nsteps ? u : (nsteps ? nsteps - 1 : 0);  // clamp: branch-free
        const uint32_t j = uu / KC;
        c = uu - j * KC;
        t = tile_of(j);
    };
    auto issueA = [&](uint32_t u, auto BI) __attribute__((always_inline)) {
        uint32_t t, c;
        step_of(u, t, c);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t row = srow0 + i * 8u;
            const uint32_t piece = (lane & 7u) ^ ((row >> 1) & 7u);
            const char* ga = qx + ((uint64_t)c * kFxQ + row) * 128u + piece * 16u;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)ga,
                                             (__attribute__((address_space(3))) void*)(abuf(BI) + (wv * 32u + i * 8u) * 64u),
                                             16, 0, 0);
        }
    };
    auto issueB = [&](uint32_t u, auto BI) __attribute__((always_inline)) {
        uint32_t t, c;
        step_of(u, t, c);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t row = srow0 + i * 8u;
            const uint32_t piece = (lane & 7u) ^ ((row >> 1) & 7u);
            const uint32_t grow = min(t * kFxRows + row, N - 1u);
            const char* gb = rowsx + fx_off(grow, c, KC) + piece * 16u;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gb,
                                             (__attribute__((address_space(3))) void*)(bbuf(BI) + (wv * 32u + i * 8u) * 64u),
                                             16, 0, 0);
        }
    };

    using AccT = std::conditional_t<I8, fx_v16i, fx_v16f>;
    AccT acc[4][2];
    auto zero = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][r][e] = 0;
    };
    // Fragment reads: rows i*32 + (lane & 31) of a 32-row block all share the
    // swizzle ((lane & 31) >> 1) & 7, so a fragment address is a per-lane base,
    // plus one of 4 per-lane piece offsets (k-step s), plus a constant
    // 4 KiB * block.
    const uint32_t swz = ((lane & 31u) >> 1) & 7u;
    uint32_t poff[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) poff[s] = (((uint32_t)(2 * s) + (lane >> 5)) ^ swz) * 16u;
    const uint32_t abase = (wq * 128u + (lane & 31u)) * 128u;
    const uint32_t bbase = (wr * 64u + (lane & 31u)) * 128u;
    // 4 k-steps of 16 over one LDS chunk; fragments of step s+1 are read while
    // the 8 MFMAs of step s run
    auto mma = [&](auto AI, auto BI) __attribute__((always_inline)) {
        const char* A = (const char*)abuf(AI) + abase;
        const char* Bt = (const char*)bbuf(BI) + bbase;
        fx_v4i fa[2][4], fb[2][2];
        auto rd = [&](int s, int slot) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[slot][i] = *(const fx_v4i*)(A + poff[s] + i * 4096);
#pragma unroll
            for (int r = 0; r < 2; ++r) fb[slot][r] = *(const fx_v4i*)(Bt + poff[s] + r * 4096);
        };
        rd(0, 0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (s + 1 < 4) rd(s + 1, (s + 1) & 1);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if constexpr (I8)
                        acc[i][r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[s & 1][i], fb[s & 1][r], acc[i][r], 0, 0,
                                                                          0);
                    else
                        acc[i][r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(fx_v8bf, fa[s & 1][i]),
                                                                            __builtin_bit_cast(fx_v8bf, fb[s & 1][r]),
                                                                            acc[i][r], 0, 0, 0);
                }
        }
    };
    // Epilogue.  Per pair the exact f32 cosine is at most U = approx + qa*rho_x
    // + qd (i8: qa = (1+rho_q)*c, qd = rho_q*c + slack, rho_x per row; bf16:
    // qa = 0, qd = eps).  SAMPLE stores approx; EMIT nominates a row iff
    // U >= tau, as approx + qa*rho_x >= thr with thr = tau - qd.
    auto epilogue = [&](uint32_t j) __attribute__((always_inline)) {
        const uint32_t t = tile_of(j);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint32_t n = t * kFxRows + wr * 64u + r * 32u + (lane & 31u);
            float rinv, rho = 0.0f;
            if constexpr (I8) {
                rinv = n < N ? a.rscale[n] : 0.0f;  // s_x / |x|
                rho = n < N ? a.rrho[n] : 0.0f;
            } else {
                const float nb = n < N ? a.rnorm[n] : 0.0f;
                rinv = nb == 0.0f ? 0.0f : 1.0f / nb;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint32_t qb0 = wq * 128u + i * 32u + 4u * (lane >> 5);
                asm volatile("" : "+v"(qb0));  // keep per-slot addresses out of the tile loop
                // this lane's 16 query slots: qb0 + (e & 3) + 8 * (e >> 2)
                float qs[16], ts[16];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 qv = *(const float4*)(a.qinv + qb0 + 8 * g);
                    qs[4 * g + 0] = qv.x * rinv;
                    qs[4 * g + 1] = qv.y * rinv;
                    qs[4 * g + 2] = qv.z * rinv;
                    qs[4 * g + 3] = qv.w * rinv;
                    // EMIT: ts = thr - qa*rho (the row-dependent part of U); SAMPLE: ts = 0
                    float4 tv = make_float4(0.f, 0.f, 0.f, 0.f);
                    if constexpr (!SAMPLE) tv = *(const float4*)(a.thr + qb0 + 8 * g);
                    if constexpr (I8 && !SAMPLE) {
                        const float4 av = *(const float4*)(a.qa + qb0 + 8 * g);
                        tv.x -= av.x * rho;
                        tv.y -= av.y * rho;
                        tv.z -= av.z * rho;
                        tv.w -= av.w * rho;
                    }
                    ts[4 * g + 0] = tv.x;
                    ts[4 * g + 1] = tv.y;
                    ts[4 * g + 2] = tv.z;
                    ts[4 * g + 3] = tv.w;
                }
                if constexpr (SAMPLE) {
                    const uint32_t col = j * G + blockIdx.x;  // list position of this tile
                    const uint32_t sp = col * kFxRows + wr * 64u + r * 32u + (lane & 31u);
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        const uint32_t q = qb0 + (e & 3) + 8 * (e >> 2);
                        if (q < a.B)
                            a.smp[(uint64_t)q * a.S + sp] = n < N ? (float)acc[i][r][e] * qs[e] : -__builtin_inff();
                    }
                } else {
                    float mx = -__builtin_inff();
#pragma unroll
                    for (int e = 0; e < 16; ++e) mx = fmaxf(mx, (float)acc[i][r][e] * qs[e] - ts[e]);
                    if (!__ballot(mx >= 0.0f && n < N)) continue;
                    // rare: a candidate in this fragment (thr = +inf for slots >= B)
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        const uint32_t q = qb0 + (e & 3) + 8 * (e >> 2);
                        if (n < N && (float)acc[i][r][e] * qs[e] >= ts[e]) {
                            const uint32_t pos = atomicAdd(&a.counts[q], 1u);
                            if (pos < a.candcap) a.cand[(uint64_t)q * a.candcap + pos] = n;
                        }
                    }
                }
            }
        }
    };

    // s_waitcnt encodings (gfx9): vmcnt in [3:0], expcnt [6:4], lgkmcnt [11:8]
    constexpr int kWaitAll = 0x0000;        // vmcnt(0) expcnt(0) lgkmcnt(0)
    constexpr int kWaitKeepB = 0x0074;      // vmcnt(4) lgkmcnt(0): the 4 newest (B(u+2)) stay in flight
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
    issueA(0, C0{});
    issueB(0, C0{});
    issueB(1, C1{});
    __builtin_amdgcn_s_waitcnt(kWaitAll);
    __builtin_amdgcn_s_barrier();
    zero();
    // step u uses A buffer u%2 and B buffer u%3; six steps per loop trip keep
    // every buffer index static
    auto step = [&](uint32_t u, auto AI, auto BI) __attribute__((always_inline)) {
        using AN = std::integral_constant<int, 1 - decltype(AI)::value>;
        using BN2 = std::integral_constant<int, (decltype(BI)::value + 2) % 3>;
        if (!(a.dbg & 1)) issueA(u + 1, AN{});  // buffers of step u-1 were released by its barrier
        if (!(a.dbg & 2)) issueB(u + 2, BN2{});
        if (!(a.dbg & 4)) mma(AI, BI);
        const uint32_t j = u / KC;
        if (u - j * KC == KC - 1) {
            epilogue(j);
            zero();
            __builtin_amdgcn_s_waitcnt(kWaitAll);  // the epilogue's memory ops break the count
        } else {
            __builtin_amdgcn_s_waitcnt(kWaitKeepB);
        }
        __builtin_amdgcn_s_barrier();
    };
    for (uint32_t u = 0; u < nsteps; u += 6) {
        step(u, C0{}, C0{});
        if (u + 1 < nsteps) step(u + 1, C1{}, C1{});
        if (u + 2 < nsteps) step(u + 2, C0{}, C2{});
        if (u + 3 < nsteps) step(u + 3, C1{}, C0{});
        if (u + 4 < nsteps) step(u + 4, C0{}, C1{});
        if (u + 5 < nsteps) step(u + 5, C1{}, C2{});
    }
    __builtin_amdgcn_s_waitcnt(kWaitAll);  // drain the clamped prefetches before exit
}

// Probe selection: per query the 16 sampled rows with the largest MFMA scores
// (per-thread top-16 of (score, sample position) keys, then an LDS sort).
// They are re-scored exactly (k_rerank) and k_flat_tau takes tau_q = the mk-th
// largest exact probe score: mk rows then have exact score >= tau_q, so the
// k-th best score is >= tau_q unless the sample holds mk of the top k-1 rows
// (mk is sized for that to be a 1e-6 event, host side).
__global__ __launch_bounds__(1024) void k_flat_probes(const float* __restrict__ smp, uint32_t S, uint32_t every,
                                                      uint32_t N, uint32_t* __restrict__ probes,
                                                      uint32_t* __restrict__ pcount) {
    __shared__ uint64_t keys[256];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    // wave-cooperative top-16: lanes 0..15 hold the wave's best keys, descending
    // ((order(score) << 32) | sample position; 0 = empty); a batch of 64 values
    // costs one compare + ballot unless a lane beats the current 16th key
    uint64_t mine = 0, t16 = 0;
    const float* src = smp + (uint64_t)q * S;
    for (uint32_t i0 = wv * 64u; i0 < S; i0 += 1024u * 4u) {
        uint64_t k4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {  // 16 waves x 4 loads in flight per lane
            const uint32_t i = i0 + u * 1024u + lane;
            const float v = i < S ? src[i] : -__builtin_inff();
            k4[u] = v > -__builtin_inff() ? (((uint64_t)f32_order(v) << 32) | i) : 0ull;  // NaN / padding -> empty
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint64_t m = __ballot(k4[u] > t16);
            while (m) {
                const uint32_t l = __builtin_ctzll(m);
                m &= m - 1;
                const uint64_t key = __shfl(k4[u], l);
                if (key <= t16) continue;
                // insert into lanes 0..15: lanes holding a smaller key shift down
                const uint64_t up = __shfl_up(mine, 1);
                const bool below = lane < 16 && key > mine;
                const bool first = below && (lane == 0 || up >= key);
                mine = first ? key : (below ? up : mine);
                t16 = __shfl(mine, 15);
            }
        }
    }
    if (lane < 16) keys[wv * 16 + lane] = ~mine;  // ascending sort of ~key = descending key
    __syncthreads();
    bitonic_sort_lds(keys, 256);  // merge the 16 wave lists
    if (tid < 16) {
        const uint64_t key = ~keys[tid];
        const uint32_t sp = (uint32_t)key;
        const uint32_t row = ((sp >> 8) * every << 8) | (sp & 255u);  // sample position -> row
        const bool ok = key != 0 && row < N;
        probes[q * 16u + tid] = ok ? row : 0u;
        const uint32_t valid = (uint32_t)__ballot(ok) & 0xffffu;
        if (tid == 0) pcount[q] = __popc(valid);
    }
}

// thr_q = tau_q - qd_q with tau_q the mk-th largest exact probe score (-inf
// when fewer probes); slots q >= B get +inf (nothing is nominated for them).
__global__ __launch_bounds__(256) void k_flat_tau(const float* __restrict__ pscores, const uint32_t* __restrict__ pcount,
                                                  uint32_t B, uint32_t mk, int distance, const float* __restrict__ qd,
                                                  float* __restrict__ thr) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;
    if (q >= kFxQ) return;
    if (q >= B) {
        thr[q] = __builtin_inff();
        return;
    }
    const uint32_t c = min(pcount[q], 16u);
    float v[16];
    for (uint32_t i = 0; i < 16; ++i) {
        float x = i < c ? pscores[q * 16u + i] : -__builtin_inff();
        if (distance) x = 1.0f - x;  // the probe pass ran with the index's metric
        v[i] = x == x ? x : -__builtin_inff();
    }
    for (uint32_t i = 1; i < 16; ++i)  // insertion sort, descending
        for (uint32_t j = i; j > 0 && v[j] > v[j - 1]; --j) {
            const float t = v[j];
            v[j] = v[j - 1];
            v[j - 1] = t;
        }
    thr[q] = (c >= mk ? v[mk - 1] : -__builtin_inff()) - qd[q];
}

// Per query: sort the reranked candidates (exact score, then row ascending),
// certify, emit the first k live rows.
__global__ __launch_bounds__(256) void k_flat_final(const uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ cand, uint32_t candcap,
                                                    const float* __restrict__ scores, const float* __restrict__ thr,
                                                    const float* __restrict__ qd, uint32_t k, int descending,
                                                    const uint64_t* __restrict__ ids, uint64_t* __restrict__ out_ids,
                                                    float* __restrict__ out_scores, uint32_t* __restrict__ out_n,
                                                    uint32_t* __restrict__ fail) {
    __shared__ uint64_t keys[kFxCandCap];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const uint32_t c = counts[q];
    if (c > candcap) {  // overflow: not certifiable
        if (tid == 0) atomicOr(fail, 1u);
        return;
    }
    const uint32_t P = next_pow2(c < 2u ? 2u : c);
    for (uint32_t i = tid; i < P; i += 256u) {
        if (i < c) {
            const float sc = scores[(uint64_t)q * candcap + i];
            const uint32_t o = descending ? ~f32_order(sc) : f32_order(sc);
            keys[i] = ((uint64_t)o << 32) | cand[(uint64_t)q * candcap + i];
        } else {
            keys[i] = ~0ull;
        }
    }
    __syncthreads();
    bitonic_sort_lds(keys, P);
    if (tid == 0) {
        // first k live rows; the k-th one's exact score certifies the list
        uint32_t got = 0;
        float last = 0.0f;
        for (uint32_t i = 0; i < c && got < k; ++i) {
            const uint32_t row = (uint32_t)keys[i];
            const uint64_t id = ids ? ids[row] : row;
            if (id == kOrphan) continue;
            const uint32_t o = descending ? ~(uint32_t)(keys[i] >> 32) : (uint32_t)(keys[i] >> 32);
            const uint32_t u = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
            last = __uint_as_float(u);
            out_ids[(uint64_t)q * k + got] = id;
            out_scores[(uint64_t)q * k + got] = last;
            ++got;
        }
        // cosine (descending): rows never nominated score < T + eps.  Cosine
        // distance (ascending): their distance > 1 - (T + eps) up to one rounding.
        const float cos_k = descending ? last : 1.0f - last;
        const bool ok = k == 0 || (got == k && cos_k >= thr[q] + qd[q]);  // thr + qd = tau
        if (!ok) atomicOr(fail, 1u);
        if (out_n) out_n[q] = got;  // out_n is optional (gvdb_index_search_device)
    }
}

}  // namespace

float flat_eps(uint32_t D) {
    // bf16 RNE of both operands: |q^x^ - qx| <= (2^-8 + 2^-18)|q||x| summed by
    // Cauchy-Schwarz; f32 accumulation and the exact reference's own fold each
    // <= D * 2^-24 relative; norm/product roundings; plus slack.
    return 0.00390625f * 1.01f + fx_fold_slack(D);
}

hipError_t launch_rows_to_bf16(const float* rows, uint64_t n, uint32_t D, uint16_t* rowsb, uint64_t cap,
                               uint32_t* nan_flag, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t threads = n * 8u * fx_kc(D);
    hipLaunchKernelGGL(k_rows_to_bf16, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, rows, n, D, rowsb,
                       cap, nan_flag);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_queries_to_bf16(const float* q, uint32_t B, uint32_t D, const float* qnorm, uint16_t* qb,
                                  float* qinv, float* qd, hipStream_t s) {
    const uint32_t threads = kFxQ * 8u * fx_kc(D);
    hipLaunchKernelGGL(k_queries_to_bf16, dim3((threads + 255) / 256), dim3(256), 0, s, q, B, D, qnorm, qb, qinv,
                       qd, flat_eps(D));
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_rows_to_i8(const float* rows, const float* norms, uint64_t n, uint32_t D, int8_t* rowsq, uint64_t cap,
                             float* rscale, float* rrho, uint32_t* bad_flag, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rows_to_i8, dim3((uint32_t)((n + 3) / 4)), dim3(256), 0, s, rows, norms, n, D, rowsq, cap,
                       rscale, rrho, bad_flag);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_queries_to_i8(const float* q, uint32_t B, uint32_t D, const float* qnorm, int8_t* qq, float* qinv,
                                float* qa, float* qd, hipStream_t s) {
    hipLaunchKernelGGL(k_queries_to_i8, dim3(kFxQ / 4), dim3(256), 0, s, q, B, D, qnorm, qq, qinv, qa, qd);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

static uint32_t fx_grid(uint32_t tiles) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return tiles < (uint32_t)cus ? tiles : (uint32_t)cus;
}

hipError_t launch_flat_mx_sample(const FlatMxArgs& a, hipStream_t s) {
    const uint32_t tiles = ((a.N + kFxRows - 1) / kFxRows + a.every - 1) / a.every;
    if (tiles == 0) return hipSuccess;
    if (a.i8)
        hipLaunchKernelGGL((k_flat_mx<true, true>), dim3(fx_grid(tiles)), dim3(kFxThreads), 0, s, a);
    else
        hipLaunchKernelGGL((k_flat_mx<true, false>), dim3(fx_grid(tiles)), dim3(kFxThreads), 0, s, a);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_flat_mx_emit(const FlatMxArgs& a, hipStream_t s) {
    const uint32_t tiles = (a.N + kFxRows - 1) / kFxRows;
    if (tiles == 0) return hipSuccess;
    if (a.i8)
        hipLaunchKernelGGL((k_flat_mx<false, true>), dim3(fx_grid(tiles)), dim3(kFxThreads), 0, s, a);
    else
        hipLaunchKernelGGL((k_flat_mx<false, false>), dim3(fx_grid(tiles)), dim3(kFxThreads), 0, s, a);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_flat_probes(const float* smp, uint32_t B, uint32_t S, uint32_t every, uint32_t N, uint32_t* probes,
                              uint32_t* pcount, hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_flat_probes, dim3(B), dim3(1024), 0, s, smp, S, every, N, probes, pcount);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_flat_tau(const float* pscores, const uint32_t* pcount, uint32_t B, uint32_t mk, int distance,
                           const float* qd, float* thr, hipStream_t s) {
    hipLaunchKernelGGL(k_flat_tau, dim3((kFxQ + 255) / 256), dim3(256), 0, s, pscores, pcount, B, mk, distance, qd, thr);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_flat_final(const uint32_t* counts, const uint32_t* cand, uint32_t candcap, const float* scores,
                             const float* thr, const float* qd, uint32_t B, uint32_t k, int descending,
                             const uint64_t* ids, uint64_t* out_ids, float* out_scores, uint32_t* out_n, uint32_t* fail,
                             hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_flat_final, dim3(B), dim3(256), 0, s, counts, cand, candcap, scores, thr, qd, k, descending,
                       ids, out_ids, out_scores, out_n, fail);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace gvdb
