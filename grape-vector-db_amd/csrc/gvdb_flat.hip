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
//   bf16: rowsx = bf16 x64 per chunk row,  KC = ceil(D/64),  v_mfma_f32_32x32x16_bf16;
//         eps = 2^-8 (+ rounding terms, flat_eps below) for every pair.
//   i8:   rowsx = int8 x128 per chunk row, KC = ceil(D/128), v_mfma_i32_32x32x32_i8
//         (exact i32 dot of the quantised vectors).  Row x is stored as
//         xq = rint(x * 127/max|x_i|), s_x = max|x_i|/127, with
//         rscale = s_x/|x| and rho_x = |x - s_x xq| / |x| (fp64, rounded up);
//         queries likewise.  |q.x - q^.x^| <= |e_q||x| + |q^||e_x| gives, in
//         cosine units, eps_q = rho_q + (1 + rho_q) max_x rho_x (+ norm and
//         fold rounding terms): half the HBM bytes of bf16 and twice the
//         MFMA rate, for a ~4x wider (still certified) candidate margin.
// Either way a row chunk is 128 B and the mirror is tile-major and
// FRAGMENT-major (fx_frag, gvdb_internal.h): one chunk of a 256-row tile is a
// contiguous 32 KiB block of eight 4 KiB 32-row groups, each laid out as the
// MFMA operand fragments of its 4 k-steps, and a tile's KC chunks are
// adjacent, so a block streams one contiguous KC*32 KiB region per tile and a
// wave loads its row fragments with lane-linear 16-B loads.  Queries use the
// same layout (one 256-slot tile).
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

// rows f32 [n][D] (rows row0.. of the index) -> rowsb bf16 mirror (fx_frag); one
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
    *(uint4*)(rowsb + fx_frag(row, c, KC, grp & 7u) / 2u) = o;
}

// queries f32 [B][D] -> qb bf16 (fx_frag, slots >= B zero), qinv = 1/|q| (0 for |q| = 0)
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
    *(uint4*)(qb + fx_frag(slot, c, KC, grp & 7u) / 2u) = o;
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
// 8p + (l >> 3), written at dst + fx_frag(row, chunk, KC, piece) (chunks < KC;
// padding elements are 0).  Returns s = max|v|/127 and rho = |v - s*vq| / |v|
// in fp64 (0 for a zero vector) on every lane, and flags non-finite values.
__device__ inline void fx_quantize_i8_wave(const float* __restrict__ v, uint32_t D, uint32_t lane, bool live,
                                           int8_t* __restrict__ dst, uint64_t row, float& s_out, double& rho_out,
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
        if (chunk < KC) *(uint4*)(dst + fx_frag(row, chunk, KC, lane & 7u)) = make_uint4(w[0], w[1], w[2], w[3]);
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

// rows f32 [n][D] -> rowsq int8 mirror (fx_frag, KC = ceil(D/128)); one wave per
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
    fx_quantize_i8_wave(rows + row * D, D, lane, true, rowsq, row, sc, rho, bad);
    if (bad && lane == 0) atomicOr(bad_flag, 1u);
    if (lane == 0) {
        const float nx = norms[row];
        rscale[row] = nx == 0.0f ? 0.0f : sc / nx;
        rrho[row] = (float)(rho * (1.0 + 1e-6));
    }
}

// queries f32 [B][D] -> qq int8 (fx_frag, slots >= B zero); qinv = s_q/|q|,
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
    fx_quantize_i8_wave(q + (uint64_t)(live ? slot : 0) * D, D, lane, live, qq, slot, sc, rho, bad);
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
// Tile = 256 rows x 256 query slots; 8 waves = 2 query halves (wq) x 4 row
// quarters (wr), each wave 128 queries x 64 rows = 4 x 2 32x32 MFMA tiles.
// Rows (B operand, from HBM) go straight to VGPRs: the fragment-major mirror
// (fx_frag) makes each (32-row group, k-step) fragment 1 KiB contiguous, and
// the fragment consumed at k-step s is reloaded for the next chunk right after
// its MFMAs (one chunk of prefetch distance, 32 VGPRs).  The query chunk (A,
// 32 KiB, L2-resident) is loaded to VGPRs one chunk ahead and written to a
// 2-buffer LDS ring (plain loads, not global_load_lds: an in-flight LDS DMA
// makes the compiler drain vmcnt to 0 before every ds_read, row loads
// included).  The LDS image of a chunk is its fragment-major global image, so
// every ds_read_b128 fragment read is lane-linear (conflict-free).
// Thresholds and inverse norms are read from L1/L2 in the once-per-tile
// epilogue.
// FX_ABL (timing ablation builds only, results invalid): 1 no query loads,
// 2 no row loads, 4 no epilogue, 8 no MFMA, 16 rows loaded by one wave of
// each pair only.
#ifndef FX_ABL
#define FX_ABL 0
#endif
// FX_AMODE: how query chunks reach LDS.  1 (default): LDS DMA issued from
// inline asm two steps ahead (no staging registers; asm so that the waitcnt
// pass, which cannot tell a DMA into one buffer from ds_reads of another,
// does not drain vmcnt before every fragment read) with a counted vmcnt
// before the barrier.  0: VGPR staging + ds_write one step ahead.
#ifndef FX_AMODE
#define FX_AMODE 1
#endif
template <bool SAMPLE, bool I8>
__global__ __launch_bounds__(kFxThreads, 1) void k_flat_mx(FlatMxArgs a) {
    // three distinct LDS objects (not one indexed array), each 1 query chunk
    constexpr uint32_t kChunk = kFxQ * 128u;  // bytes of one query chunk
    __shared__ __attribute__((aligned(16))) char As0[kChunk], As1[kChunk], As2[kChunk];
    // EMIT: the block's nominations, (query << 32) | row, flushed to the
    // global per-query lists once at the end (an LDS atomic per nomination
    // instead of a global atomic round trip inside the MFMA loop)
    constexpr uint32_t kCl = SAMPLE ? 1u : 2048u;
    __shared__ uint64_t cl[kCl];
    __shared__ float cs[kCl];  // the nominations' approx scores
    __shared__ uint32_t cl_n;
    // per-slot epilogue operands, staged once: qinv, thr - (i8) qa
    __shared__ __attribute__((aligned(16))) float qinv_l[kFxQ], thr_l[kFxQ], qa_l[I8 ? kFxQ : 4];
    const char* rowsx = (const char*)a.rowsx;
    const char* qx = (const char*)a.qx;
    auto abuf = [&](auto I) -> char* {
        if constexpr (decltype(I)::value == 0) return As0;
        else if constexpr (decltype(I)::value == 1) return As1;
        else return As2;
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
    auto step_of = [&](uint32_t u, uint32_t& t, uint32_t& c) __attribute__((always_inline)) {
        const uint32_t uu = u < nsteps ? u : (nsteps ? nsteps - 1 : 0);  // clamp: branch-free
        const uint32_t j = uu / KC;
        c = uu - j * KC;
        t = tile_of(j);
    };
    // query chunk of step u: wave wv stages bytes [4 KiB wv, +4 KiB), 1 KiB per load
    constexpr bool kDma = FX_AMODE == 1;
    // kDma: every vector-memory op of the step loop is inline asm with its
    // waits placed by hand (counts below), so the compiler's waitcnt pass
    // neither drains on the DMA nor miscounts around it
    auto gload4 = [&](fx_v4i& d, const char* p) __attribute__((always_inline)) {
        if constexpr (kDma) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
        else d = *(const fx_v4i*)p;
    };
    auto gload1 = [&](float& d, const float* p) __attribute__((always_inline)) {
        if constexpr (kDma) asm volatile("global_load_dword %0, %1, off" : "=v"(d) : "v"(p) : "memory");
        else d = *p;
    };
    // DMA form: wave wv copies bytes [4 KiB wv, +4 KiB) of chunk u, 1 KiB per op
    auto issueA = [&](uint32_t u, auto BI) __attribute__((always_inline)) {
        uint32_t t, c;
        step_of(u, t, c);
        const char* ga = qx + (uint64_t)c * kChunk + wv * 4096u + lane * 16u;
        const uint32_t l0 = (uint32_t)(uintptr_t)(abuf(BI) + wv * 4096u);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(ga + i * 1024), "s"(l0 + i * 1024u)
                         : "memory");
    };
    fx_v4i qs[kDma ? 1 : 4];
    auto loadA = [&](uint32_t u) __attribute__((always_inline)) {
        uint32_t t, c;
        step_of(u, t, c);
        const char* ga = qx + (uint64_t)c * kChunk + wv * 4096u + lane * 16u;
        if constexpr (FX_ABL & 1) return;
#pragma unroll
        for (int i = 0; i < 4; ++i) qs[i] = *(const fx_v4i*)(ga + i * 1024);
    };
    auto storeA = [&](auto BI) __attribute__((always_inline)) {
        char* d = abuf(BI) + wv * 4096u + lane * 16u;
#pragma unroll
        for (int i = 0; i < 4; ++i) *(fx_v4i*)(d + i * 1024) = qs[i];
    };
    // row fragments of step u: groups 2 wr + r of tile t, chunk c; (r, s) at +4 KiB r + 1 KiB s
    auto rowbase = [&](uint32_t u) __attribute__((always_inline)) -> const char* {
        uint32_t t, c;
        step_of(u, t, c);
        return rowsx + (((uint64_t)t * KC + c) * 8u + 2u * wr) * 4096u + lane * 16u;
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
    // row fragments [ring slot][r][k-step]: bf16 keeps kRing = 2 chunks in
    // flight (slot = step parity); i8 has no registers to spare for a second
    constexpr int kRing = I8 ? 1 : 2;
    fx_v4i rf[kRing][2][4];
    const uint32_t abase = (wq * 16u * 64u + lane) * 16u;  // query groups 4 wq + i: +4 KiB i, +1 KiB s
    // query fragments, double-buffered across k-steps AND across steps: the
    // last k-step of step u reads k-step 0 of chunk u+1 (complete since the
    // barrier of step u-1), so no LDS latency follows the barrier
    fx_v4i fa[2][4];
    auto rd = [&](const char* A, int s, int slot) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[slot][i] = *(const fx_v4i*)(A + abase + i * 4096 + s * 1024);
    };
    // 4 k-steps of 16 (i8: 32) over one chunk; the query fragments of k-step
    // s+1 are read while the 8 MFMAs of k-step s run, and row fragment s is
    // reloaded for the next chunk as soon as its MFMAs have issued (pinned
    // there, so every row load has one whole chunk step to land)
    auto mma = [&](uint32_t u, auto AI, auto RI) __attribute__((always_inline)) {
        using A1 = std::integral_constant<int, (decltype(AI)::value + 1) % 3>;
        constexpr int R = decltype(RI)::value;
        const char* A = (const char*)abuf(AI);
        const char* rn = rowbase(u + kRing);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (s + 1 < 4) rd(A, s + 1, (s + 1) & 1);
            else if constexpr (!kDma) rd((const char*)abuf(A1{}), 0, 0);
            __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of this k-step's MFMAs
            if constexpr (kDma) {
                // rows k-step s of this chunk were loaded kRing steps ago after
                // that step's k-step s; younger: 2 (3 - s) rows there, 4 DMA +
                // 8 rows per step in between, then 4 DMA + 2 s rows here =
                // 10 + 12 (kRing - 1), not counting the operand loads of
                // tile-end steps (extra younger ops only make a wait stricter)
                asm volatile("s_waitcnt vmcnt(%2)"
                             : "+v"(rf[R][0][s]), "+v"(rf[R][1][s])
                             : "n"(10 + 12 * (kRing - 1)));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if constexpr (FX_ABL & 8)
                        acc[i][r][0] += __builtin_bit_cast(float, fa[s & 1][i][0] ^ rf[R][r][s][0] ^ rf[R][r][s][1] ^
                                                                      rf[R][r][s][2] ^ rf[R][r][s][3]);
                    else if constexpr (I8)
                        acc[i][r] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[s & 1][i], rf[R][r][s], acc[i][r], 0, 0, 0);
                    else
                        acc[i][r] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(fx_v8bf, fa[s & 1][i]),
                                                                            __builtin_bit_cast(fx_v8bf, rf[R][r][s]),
                                                                            acc[i][r], 0, 0, 0);
                }
            if constexpr (!(FX_ABL & 2)) {
                if (!(FX_ABL & 16) || wq == 0) {
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        gload4(rf[R][r][s], rn + r * 4096 + s * 1024);
                    }
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // Epilogue.  Per pair the exact f32 cosine is at most U = approx + qa*rho_x
    // + qd (i8: qa = (1+rho_q)*c, qd = rho_q*c + slack, rho_x per row; bf16:
    // qa = 0, qd = eps).  SAMPLE stores approx; EMIT nominates a row iff
    // U >= tau, as approx + qa*rho_x >= thr with thr = tau - qd.
    // per-row operands of the epilogue, (re)loaded every step so the
    // once-per-tile epilogue never waits on a global load: bf16 |x| (rv0),
    // i8 s_x/|x| (rv0) and rho_x (rv1), for this lane's rows r = 0, 1
    float rv0[2] = {0.0f, 0.0f}, rv1[2] = {0.0f, 0.0f};
    auto load_rowops = [&](uint32_t u) __attribute__((always_inline)) {
        uint32_t t, c;
        step_of(u, t, c);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint32_t n = min(t * kFxRows + wr * 64u + r * 32u + (lane & 31u), N - 1u);
            if constexpr (I8) {
                gload1(rv0[r], a.rscale + n);
                gload1(rv1[r], a.rrho + n);
            } else {
                gload1(rv0[r], a.rnorm + n);
            }
        }
    };
    auto epilogue = [&](uint32_t j) __attribute__((always_inline)) {
        const uint32_t t = tile_of(j);
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const uint32_t n = t * kFxRows + wr * 64u + r * 32u + (lane & 31u);
            float rinv, rho = 0.0f;
            if constexpr (I8) {
                rinv = n < N ? rv0[r] : 0.0f;  // s_x / |x|
                rho = n < N ? rv1[r] : 0.0f;
            } else {
                const float nb = n < N ? rv0[r] : 0.0f;
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
                    const float4 qv = *(const float4*)(qinv_l + qb0 + 8 * g);
                    qs[4 * g + 0] = qv.x * rinv;
                    qs[4 * g + 1] = qv.y * rinv;
                    qs[4 * g + 2] = qv.z * rinv;
                    qs[4 * g + 3] = qv.w * rinv;
                    // EMIT: ts = thr - qa*rho (the row-dependent part of U); SAMPLE: ts = 0
                    float4 tv = make_float4(0.f, 0.f, 0.f, 0.f);
                    if constexpr (!SAMPLE) tv = *(const float4*)(thr_l + qb0 + 8 * g);
                    if constexpr (I8 && !SAMPLE) {
                        const float4 av = *(const float4*)(qa_l + qb0 + 8 * g);
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
                        const float v = (float)acc[i][r][e] * qs[e];
                        if (n < N && v >= ts[e]) {
                            const uint32_t li = atomicAdd(&cl_n, 1u);
                            if (li < kCl) {
                                cl[li] = ((uint64_t)q << 32) | n;
                                cs[li] = v;
                            } else {  // block list full: straight to the global list
                                const uint32_t pos = atomicAdd(&a.counts[q], 1u);
                                if (pos < a.candcap) {
                                    a.cand[(uint64_t)q * a.candcap + pos] = n;
                                    if (a.cscore) a.cscore[(uint64_t)q * a.candcap + pos] = v;
                                }
                            }
                        }
                    }
                }
            }
        }
    };

    // Per step u: the query chunk of step u+2 is loaded to VGPRs at the start
    // and written to LDS buffer (u+2)%3 after the MFMAs (that buffer was last
    // read in step u-1 and by step u-2's tail, both before the barrier of
    // step u-1), then one barrier.  The barrier waits for LDS only (vmcnt(63)
    // lgkmcnt(0)): the row loads stay in flight.
    constexpr int kWaitLds = (3 << 14) | 0x0070 | 0xF;  // vmcnt(63) expcnt(7) lgkmcnt(0)
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
#pragma unroll
    for (int k = 0; k < kRing; ++k) {
        const char* r0 = rowbase(k);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int r = 0; r < 2; ++r) gload4(rf[k][r][s], r0 + r * 4096 + s * 1024);
    }
    if constexpr (kDma) {
        issueA(0, C0{});
        issueA(1, C1{});
        __builtin_amdgcn_s_waitcnt(0);
    } else {
        loadA(0);
        storeA(C0{});
        loadA(1);
        storeA(C1{});
    }
    if (tid == 0) cl_n = 0;
    if (tid < kFxQ) {
        qinv_l[tid] = a.qinv[tid];
        if constexpr (!SAMPLE) thr_l[tid] = a.thr[tid];
        if constexpr (I8 && !SAMPLE) qa_l[tid] = a.qa[tid];
    }
    __builtin_amdgcn_s_waitcnt(kWaitLds);
    __builtin_amdgcn_s_barrier();
    zero();
    if constexpr (!kDma) rd((const char*)As0, 0, 0);
    // step u reads A buffer u%3 (three steps per loop trip keep it static)
    auto step = [&](uint32_t u, auto AI, auto RI) __attribute__((always_inline)) {
        using AN = std::integral_constant<int, (decltype(AI)::value + 2) % 3>;
        const uint32_t j = u / KC;
        const bool tile_end = u - j * KC == KC - 1;
        __builtin_amdgcn_sched_barrier(0);
        if (tile_end) load_rowops(u);  // before the DMA: waiting for these does not wait for it
        if constexpr (kDma) issueA(u + 2, AN{});
        else loadA(u + 2);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (kDma) rd((const char*)abuf(AI), 0, 0);
        mma(u, AI, RI);
        if constexpr (!kDma) storeA(AN{});  // before the epilogue: its staging registers are free there
        if (tile_end) {
            if constexpr (kDma) {  // the operand loads: 4 DMA + 8 rows younger
#pragma unroll
                for (int r = 0; r < 2; ++r) asm volatile("s_waitcnt vmcnt(12)" : "+v"(rv0[r]), "+v"(rv1[r]));
            }
            if constexpr (!(FX_ABL & 4)) epilogue(j);
            zero();
        }
        // DMA: chunk u+1 (issued at the start of step u-1) has at least
        // 8 (step u-1) + 4 + 8 (step u) = 20 younger vector-memory ops (more
        // only make the wait stricter): vmcnt(20) retires it and leaves the
        // row loads in flight
        if constexpr (kDma) asm volatile("s_waitcnt vmcnt(20) lgkmcnt(0)" ::: "memory");
        else __builtin_amdgcn_s_waitcnt(kWaitLds);
        __builtin_amdgcn_s_barrier();
    };
    // six steps per trip keep the A buffer (u%3) and the row slot (u%kRing) static
    using R1 = std::integral_constant<int, 1 % kRing>;
    for (uint32_t u = 0; u < nsteps; u += 6) {
        step(u, C0{}, C0{});
        if (u + 1 < nsteps) step(u + 1, C1{}, R1{});
        if (u + 2 < nsteps) step(u + 2, C2{}, C0{});
        if (u + 3 < nsteps) step(u + 3, C0{}, R1{});
        if (u + 4 < nsteps) step(u + 4, C1{}, C0{});
        if (u + 5 < nsteps) step(u + 5, C2{}, R1{});
    }
    // the clamped prefetches of the last steps land before any register is reused
    if constexpr (kDma) {
#pragma unroll
        for (int k = 0; k < kRing; ++k)
#pragma unroll
            for (int s = 0; s < 4; ++s)
                asm volatile("s_waitcnt vmcnt(0)" : "+v"(rf[k][0][s]), "+v"(rf[k][1][s]) : : "memory");
    }
    if constexpr (!SAMPLE) {
        // block-aggregated (k_flat_i8q's flush): ranks within (block, query) by LDS atomics,
        // one global atomic per (block, query) -- not one per nomination on a shared counter
        __shared__ uint32_t fl_n[kFxQ], fl_b[kFxQ];
        constexpr uint32_t kPerT = (kCl + kFxThreads - 1) / kFxThreads;
        for (uint32_t q = tid; q < kFxQ; q += kFxThreads) fl_n[q] = 0u;
        __syncthreads();
        const uint32_t m = min(cl_n, kCl);
        uint32_t rk[kPerT];
#pragma unroll
        for (uint32_t j = 0; j < kPerT; ++j) {
            const uint32_t i = tid + j * kFxThreads;
            rk[j] = i < m ? atomicAdd(&fl_n[(uint32_t)(cl[i] >> 32)], 1u) : 0u;
        }
        __syncthreads();
        for (uint32_t q = tid; q < kFxQ; q += kFxThreads) {
            const uint32_t c = fl_n[q];
            if (c) fl_b[q] = atomicAdd(&a.counts[q], c);
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kPerT; ++j) {
            const uint32_t i = tid + j * kFxThreads;
            if (i < m) {
                const uint64_t v = cl[i];
                const uint32_t q = (uint32_t)(v >> 32), pos = fl_b[q] + rk[j];
                if (pos < a.candcap) {
                    a.cand[(uint64_t)q * a.candcap + pos] = (uint32_t)v;
                    if (a.cscore) a.cscore[(uint64_t)q * a.candcap + pos] = cs[i];
                }
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);  // drain the clamped prefetches before exit
}

// Probe selection: per query the 16 sampled rows with the largest MFMA scores
// (per-thread top-16 of (score, sample position) keys, then an LDS sort).
// They are re-scored exactly (k_rerank) and k_flat_tau takes tau_q = the mk-th
// largest exact probe score: mk rows then have exact score >= tau_q, so the
// k-th best score is >= tau_q unless the sample holds mk of the top k-1 rows
// (mk is sized for that to be a 1e-6 event, host side).
// Orphan rows (an id re-added elsewhere, ids[row] == kOrphan) are never probes:
// tau must be reached by mk LIVE rows, or the certificate would fail whenever
// a shadowed row of a query's own neighbourhood falls into the sample.
// gridDim.y > 1 (A/B, GVDB_PROBE_PARTS): a query's sample split over P blocks, each
// writing its top-16 keys to `part` [B][P][16]; k_flat_probes_merge picks the query's 16.
__global__ __launch_bounds__(1024) void k_flat_probes(const float* __restrict__ smp, uint32_t S, uint32_t every,
                                                      uint32_t N, const uint64_t* __restrict__ ids,
                                                      uint32_t* __restrict__ probes, uint32_t* __restrict__ pcount,
                                                      uint64_t* __restrict__ part, uint32_t chunk) {
    // Round 5: each lane keeps its own two best keys ((order(score) << 32) | sample
    // position; 0 = empty) in registers -- no cross-lane work in the scan -- and one LDS
    // sort of the block's 2048 keys picks the 16.  (The wave-cooperative top-16 it replaces
    // paid a chain of LDS shuffles per insertion, ~64 of them per wave at the start: 39 us
    // for 64 queries x 19.5K sampled rows.)  A lane holding three of the block's best 16
    // keeps two: the probes are then not the exact top 16, which only lowers tau (any 16
    // real rows bound it) -- more candidates, never a wrong certificate.
    __shared__ uint64_t keys[2048];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t P = gridDim.y, s0 = blockIdx.y * chunk, s1 = min(S, s0 + chunk);
    uint64_t k1 = 0, k2 = 0;
    const float* src = smp + (uint64_t)q * S;
    constexpr int kU = 8;  // values per lane per batch, the next batch in flight
    auto load = [&](uint32_t i0, float (&v)[kU]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t i = i0 + u * 1024u + lane;
            v[u] = i < s1 ? src[i] : -__builtin_inff();
        }
    };
    float vc[kU], vn[kU];
    load(s0 + wv * 64u, vn);
    for (uint32_t i0 = s0 + wv * 64u; i0 < s1; i0 += 1024u * kU) {
#pragma unroll
        for (int u = 0; u < kU; ++u) vc[u] = vn[u];
        load(i0 + 1024u * kU, vn);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint32_t i = i0 + u * 1024u + lane;
            const uint64_t key = vc[u] > -__builtin_inff() ? (((uint64_t)f32_order(vc[u]) << 32) | i) : 0ull;  // NaN / padding -> empty
            if (key > k2) {
                bool live = true;
                if (ids) {  // orphan rows are never probes (only when the shard holds any)
                    const uint32_t row = ((i >> 8) * every << 8) | (i & 255u);
                    live = !(row < N && ids[row] == kOrphan);
                }
                if (live) {
                    if (key > k1) {
                        k2 = k1;
                        k1 = key;
                    } else {
                        k2 = key;
                    }
                }
            }
        }
    }
    keys[2u * tid] = ~k1;  // ascending sort of ~key = descending key
    keys[2u * tid + 1u] = ~k2;
    __syncthreads();
    bitonic_sort_lds(keys, 2048);
    if (P > 1) {
        if (tid < 16) part[((uint64_t)q * P + blockIdx.y) * 16u + tid] = ~keys[tid];
        return;
    }
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

// the query's 16 best of its P partial top-16 lists (k_flat_probes with P > 1)
__global__ __launch_bounds__(256) void k_flat_probes_merge(const uint64_t* __restrict__ part, uint32_t P, uint32_t every,
                                                           uint32_t N, uint32_t* __restrict__ probes,
                                                           uint32_t* __restrict__ pcount) {
    __shared__ uint64_t keys[256];
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    keys[tid] = tid < P * 16u ? ~part[(uint64_t)q * P * 16u + tid] : ~0ull;
    __syncthreads();
    bitonic_sort_lds(keys, 256);
    if (tid < 16) {
        const uint64_t key = ~keys[tid];
        const uint32_t sp = (uint32_t)key;
        const uint32_t row = ((sp >> 8) * every << 8) | (sp & 255u);
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

// Block-wide ranks of the kk smallest 64-bit keys (one key per thread of a
// 1024-thread block, ~0ull = no key, the others distinct; kk <= 64).  Each wave
// sorts its 64 keys in registers (bitonic over lane shuffles), the sorted runs go
// to runs[]; the key at position p of run w has block rank p plus, over the other
// live runs, the number of their keys below it (a 6-step binary search of a 64-key
// run), one (w, p, run) triple per thread -- only p < kk can rank below kk.  On
// return rk[64 w + p] is that rank for p < kk (~0u otherwise).
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
    const uint32_t lo = __shfl_xor((uint32_t)x, m), hi = __shfl_xor((uint32_t)(x >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void block_rank_smallest(uint64_t key, uint32_t kk, uint32_t nw, uint64_t* runs,
                                                    uint32_t* rk) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
#pragma unroll
    for (uint32_t k2 = 2; k2 <= 64; k2 <<= 1)
#pragma unroll
        for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
            const uint64_t y = shfl_xor_u64(key, (int)j);
            const bool keep_min = ((lane & j) == 0u) == ((lane & k2) == 0u);
            key = keep_min ? (key < y ? key : y) : (key < y ? y : key);
        }
    runs[tid] = key;
    rk[tid] = lane < kk && key != ~0ull ? lane : ~0u;
    __syncthreads();
    const uint32_t npairs = nw * kk * nw;
    for (uint32_t t = tid; t < npairs; t += blockDim.x) {
        const uint32_t v = t % nw, wp = t / nw, p = wp % kk, w = wp / kk;
        if (v == w) continue;
        const uint64_t x = runs[w * 64u + p];
        if (x == ~0ull) continue;
        const uint64_t* r = runs + v * 64u;
        uint32_t pos = 0;
#pragma unroll
        for (uint32_t st = 32; st > 0; st >>= 1)
            if (r[pos + st - 1u] < x) pos += st;
        pos += r[pos] < x ? 1u : 0u;
        if (pos) atomicAdd(&rk[w * 64u + p], pos);
    }
    __syncthreads();
}

// One LDS counter reservation per wave: the position of this lane's entry among
// the keeping lanes (the caller's list is unordered).  Every lane of the wave calls it.
__device__ __forceinline__ uint32_t wave_append(bool keep, uint32_t* ctr) {
    const uint64_t m = __ballot(keep);
    if (m == 0ull) return 0u;
    const uint32_t lane = threadIdx.x & 63u, lead = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __shfl(base, (int)lead);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// The kk smallest of up to 8 keys per thread (lists up to 8192 = kFxCandCap
// entries): T = the kk-th smallest of the threads' own minima bounds the
// kk-th smallest key from above (kk threads hold a key <= T), and only those kk
// threads can hold keys <= T, so at most 8 kk <= 512 keys survive the filter; they
// are compacted into surv[] and ranked again.  On return runs[] / rk[] are the
// second pass's (rk[t] = the block rank of runs[t] for the kk smallest).
template <int P>  // kk >= 1
__device__ __forceinline__ void block_smallest_multi(const uint64_t (&key)[P], uint32_t kk, uint32_t c, uint64_t* runs,
                                                     uint32_t* rk, uint64_t* surv, uint32_t* s_n, uint64_t* s_T) {
    const uint32_t tid = threadIdx.x;
    uint64_t m = key[0];
#pragma unroll
    for (int j = 1; j < P; ++j) m = key[j] < m ? key[j] : m;
    if (tid == 0) {
        *s_n = 0u;
        *s_T = ~0ull - 1u;  // fewer than kk live minima: every live key survives
    }
    block_rank_smallest(m, kk, (min(c, blockDim.x) + 63u) / 64u, runs, rk);
    if (rk[tid] == kk - 1u) *s_T = runs[tid];
    __syncthreads();
    const uint64_t T = *s_T;
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const uint32_t pos = wave_append(key[j] <= T, s_n);
        if (key[j] <= T) surv[pos] = key[j];
    }
    __syncthreads();
    const uint32_t n = *s_n;
    block_rank_smallest(tid < n ? surv[tid] : ~0ull, kk, (n + 63u) / 64u, runs, rk);
}

// Candidate pruning between the emit pass and the exact rerank.  Each
// nomination carries its approx score v, and the emit pass's own bound puts the
// exact f32 cosine in [v - m, v + m], m = qa*rho_x + qd (bf16: m = qd).  With L
// the k-th largest lower bound v - m over the live (non-orphan) candidates, k
// live rows have exact cosine >= L, so the k-th best exact cosine is >= L, and a
// candidate whose upper bound v + m is below L can neither be in the top k nor
// tie its k-th score: it is dropped without a rerank, as are the orphans that
// k_flat_final skips anyway.  Both bounds are widened by kPruneSlack against
// the f32 roundings of v, m and the sums here.  The survivors keep the list's
// (unordered) form; k_flat_final sorts them and its certificate (k-th exact
// score >= tau) is unchanged.  L by a 4 x 8-bit radix select over the
// order-mapped lower bounds; one block per query.
constexpr float kPruneSlack = 2e-6f;
constexpr uint32_t kPrThreads = 1024;
constexpr uint32_t kPrPer = kFxCandCap / kPrThreads;
__global__ __launch_bounds__(kPrThreads) void k_flat_prune(uint32_t* __restrict__ counts, uint32_t* __restrict__ cand,
                                                          const float* __restrict__ cscore, uint32_t candcap,
                                                          uint32_t k, const float* __restrict__ qa,
                                                          const float* __restrict__ qd,
                                                          const float* __restrict__ rrho,
                                                          const uint64_t* __restrict__ ids) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t sel[2];  // chosen key prefix, rank still to find below it
    __shared__ uint32_t live_n, out_n;
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u;
    const uint32_t c = counts[q];
    if (k == 0 || c <= k || c > candcap) return;  // nothing to drop / overflow (k_flat_final fails it)
    const float qaq = qa ? qa[q] : 0.0f, qdq = qd[q];
    uint32_t row[kPrPer], key[kPrPer];
    float ub[kPrPer];
    uint32_t live = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPrPer; ++j) {
        const uint32_t i = tid + j * kPrThreads;
        row[j] = 0;
        key[j] = 0;  // below every live key (f32_order of a finite or infinite value is > 0)
        ub[j] = -__builtin_inff();
        if (i < c) {
            const uint32_t r = cand[(uint64_t)q * candcap + i];
            const float v = cscore[(uint64_t)q * candcap + i];
            const float m = (rrho ? qaq * rrho[r] : 0.0f) + qdq;
            row[j] = r;
            if (!(ids && ids[r] == kOrphan)) {
                ub[j] = (v + m) + kPruneSlack;
                key[j] = f32_order((v - m) - kPruneSlack);
                ++live;
            }
        }
    }
    if (tid == 0) {
        live_n = 0;
        out_n = 0;
        sel[0] = 0;
        sel[1] = k;
    }
    __syncthreads();
    if (live) atomicAdd(&live_n, live);
    __syncthreads();
    float L = -__builtin_inff();  // fewer than k live rows: keep them all
    if (live_n >= k) {
        for (int sh = 24; sh >= 0; sh -= 8) {
            if (tid < 256) hist[tid] = 0;
            __syncthreads();
            const uint32_t pre = sel[0];
            const uint32_t hm = sh == 24 ? 0u : ~0u << (sh + 8);
#pragma unroll
            for (uint32_t j = 0; j < kPrPer; ++j)
                if (key[j] && (key[j] & hm) == (pre & hm)) atomicAdd(&hist[(key[j] >> sh) & 255u], 1u);
            __syncthreads();
            if (tid < 64) {  // digit of the rem-th largest: lane l holds bins 4l .. 4l+3
                const uint32_t rem = sel[1];
                const uint32_t h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2],
                               h3 = hist[4 * lane + 3];
                const uint32_t t = h0 + h1 + h2 + h3;
                uint32_t x = t;  // inclusive suffix sum over lanes >= l
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_down(x, o);
                    if (lane + o < 64) x += y;
                }
                uint32_t above = x - t;  // keys in higher lanes' bins
                const uint32_t hb[4] = {h0, h1, h2, h3};
#pragma unroll
                for (int b = 3; b >= 0; --b) {
                    if (above < rem && rem <= above + hb[b]) {
                        sel[0] = pre | ((4u * lane + (uint32_t)b) << sh);
                        sel[1] = rem - above;
                    }
                    above += hb[b];
                }
            }
            __syncthreads();
        }
        const uint32_t o = sel[0];  // f32_order of the k-th largest lower bound
        L = __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
    }
    // every entry is in registers: compact in place
#pragma unroll
    for (uint32_t j = 0; j < kPrPer; ++j) {
        // -inf (orphans, empty slots) never passes a finite L; -inf L keeps the live rows
        const bool keep = ub[j] >= L && !(ub[j] == -__builtin_inff());
        const uint32_t pos = wave_append(keep, &out_n);
        if (keep) cand[(uint64_t)q * candcap + pos] = row[j];
    }
    __syncthreads();
    if (tid == 0) counts[q] = out_n;
}

// Per query: order the reranked candidates by (exact score, then row ascending),
// certify, emit the first k live rows.  k <= 64: orphans become the ~0
// sentinel (their ids loaded in parallel), block_smallest_multi ranks the first
// k keys and a live key of rank r < k is output r (shard flat pass, k = 32:
// 34.5 -> 25.0 us).  The first version sorted the keys bitonically and walked them
// on thread 0, one dependent ids[] load per emitted row; k > 64 keeps that form.
// (The same selection for k_flat_prune's L measured 27.7 -> 38.2 us: not used.)
__global__ __launch_bounds__(1024) void k_flat_final(const uint32_t* __restrict__ counts,
                                                    const uint32_t* __restrict__ cand, uint32_t candcap,
                                                    const float* __restrict__ scores, const float* __restrict__ thr,
                                                    const float* __restrict__ qd, uint32_t k, int descending,
                                                    const uint64_t* __restrict__ ids, uint64_t* __restrict__ out_ids,
                                                    float* __restrict__ out_scores, uint32_t* __restrict__ out_n,
                                                    uint32_t* __restrict__ fail) {
    __shared__ __attribute__((aligned(16))) uint64_t keys[kFxCandCap];
    __shared__ uint32_t s_live;
    __shared__ float s_last;
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    const uint32_t c = counts[q];
    if (c > candcap) {  // overflow: not certifiable
        if (tid == 0) atomicOr(fail, 1u);
        return;
    }
    uint32_t got = 0;
    float last = 0.0f;
    if (k >= 1u && k <= 64u) {
        constexpr int kFP = (int)(kFxCandCap / 1024u);
        uint64_t mk[kFP];
#pragma unroll
        for (int j = 0; j < kFP; ++j) {
            const uint32_t i = tid + (uint32_t)j * 1024u;
            mk[j] = ~0ull;
            if (i < c) {
                const float sc = scores[(uint64_t)q * candcap + i];
                const uint32_t row = cand[(uint64_t)q * candcap + i];
                const uint32_t o = descending ? ~f32_order(sc) : f32_order(sc);
                if (!(ids && ids[row] == kOrphan)) mk[j] = ((uint64_t)o << 32) | row;
            }
        }
        if (tid == 0) {
            s_live = 0;
            s_last = 0.0f;
        }
        __syncthreads();
        uint32_t nl = 0;
#pragma unroll
        for (int j = 0; j < kFP; ++j) nl += mk[j] != ~0ull ? 1u : 0u;
        if (nl) atomicAdd(&s_live, nl);
        uint32_t* rk = (uint32_t*)(keys + 1024);
        uint64_t* surv = keys + 1536;
        uint32_t* s_n = (uint32_t*)(keys + 2048);
        uint64_t* s_T = keys + 2049;
        block_smallest_multi<kFP>(mk, k, c, keys, rk, surv, s_n, s_T);  // its barriers publish s_live
        got = min(k, s_live);
        const uint32_t r = rk[tid];
        if (r < got) {
            const uint64_t x = keys[tid];
            const uint32_t row = (uint32_t)x;
            const uint32_t o = descending ? ~(uint32_t)(x >> 32) : (uint32_t)(x >> 32);
            const float sc = __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
            out_ids[(uint64_t)q * k + r] = ids ? ids[row] : row;
            out_scores[(uint64_t)q * k + r] = sc;
            if (r + 1u == got) s_last = sc;
        }
        __syncthreads();
        if (tid != 0) return;
        last = s_last;
    } else {
        const uint32_t P = next_pow2(c);
        for (uint32_t i = tid; i < P; i += blockDim.x) {
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
        if (tid != 0) return;
        // first k live rows; the k-th one's exact score certifies the list
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
    }
    // thread 0: cosine (descending): rows never nominated score < T + eps.  Cosine
    // distance (ascending): their distance > 1 - (T + eps) up to one rounding.
    const float cos_k = descending ? last : 1.0f - last;
    const bool ok = k == 0 || (got == k && cos_k >= thr[q] + qd[q]);  // thr + qd = tau
    if (!ok) atomicOr(fail, 1u);
    if (out_n) out_n[q] = got;  // out_n is optional (gvdb_index_search_device)
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

// ---------------------------------------------------------------------------
// k_flat_i8q: the i8 EMIT pass with the QUERY operands in registers (KC = 6, i.e.
// D in (640, 768]).  k_flat_mx streams a 32 KiB query chunk through LDS per
// step and holds the rows in VGPRs; here the roles swap.  Wave w owns query
// tile w (32 of the 256 slots): its A fragments for all 4*KC k-steps live in
// 96 VGPRs for the whole launch, as do its 16 slots' epilogue operands.  The
// rows stream HBM -> LDS by DMA (global_load_lds_dwordx4, no staging registers)
// in sub-tiles of two 32-row groups (48 KiB, the fragment-major mirror's own
// 1 KiB pieces), three LDS buffers deep: sub-tiles i+1 and i+2 are in flight
// while every wave reads sub-tile i's B fragments from LDS (48 ds_read_b128,
// 256 B/clk) for its 2 x 24 MFMAs (v_mfma_i32_32x32x32_i8).  One barrier per
// sub-tile; the mirror is read from HBM exactly once.  Epilogue, candidate rule
// (U = approx + qa*rho_x + qd >= tau) and the block nomination list are
// k_flat_mx's; all vector-memory ops of the loop are inline asm with counted vmcnt.
// Round-3/4 A/B results behind these constants: an L2 line
// prefetch of later sub-tiles slowed the row DMA stream itself (memory-only
// 1.30 -> 2.02 ms); the skewed epilogue of waves 4..7 saved 4 %; 32-row
// sub-tiles with 6 buffers (a deeper DMA pipeline) were 7 % slower; issuing a
// wave's 6 row pieces of sub-tile i+2 one per 2 k-steps of step i's MFMAs
// instead of all after the barrier saved 7 % (every 1, 2, 3 or 4 k-steps, at
// any offset: the same within noise).
// GVDB_I8Q_T (experimental, default 0): the MFMA operands swapped -- rows as A, queries
// as B -- so a lane's 16 accumulators are ONE query against 16 rows (k_scan_mx7's trick),
// and the candidate test starts from a per-lane bound (largest dot x the rows' largest
// qinv * rinv against thr - qa * the rows' largest rho; both monotone in f32, so no pair
// the exact test nominates is missed).  GVDB_I8Q_NOPASS: timing probe, bound never passes.
#ifndef GVDB_I8Q_T
#define GVDB_I8Q_T 0
#endif
constexpr int kI8qBr = 4;           // B-fragment ring depth in k-steps
constexpr int kI8qSpread = 2;       // a row piece of the sub-tile two ahead every kI8qSpread k-steps
constexpr uint32_t kI8qSub = 2;     // 32-row groups per LDS sub-tile
constexpr uint32_t kI8qBufs = 3;    // LDS sub-tile buffers (kI8qBufs - 1 sub-tiles in flight)
constexpr uint32_t kI8qCl = 1024;  // block nomination list, u32 entries + scores (flushed at a barrier once half full)
// SPLIT (batches of <= 128 queries, round 5): the 4 live query tiles take two waves
// each, wave w tile w % 4 and row group w / 4 of every sub-tile -- half the MFMAs and
// B-fragment reads per wave instead of 4 waves computing padded slots.
template <int KC, bool SPLIT>
__global__ __launch_bounds__(kFxThreads, 1) void k_flat_i8q(FlatMxArgs a) {
    constexpr int KS = 4 * KC;                          // k-steps of 32 per row group
    constexpr uint32_t NGI = SPLIT ? 1u : kI8qSub;      // row groups per wave and sub-tile
    constexpr uint32_t kPieces = kI8qSub * KC * 4;      // 1 KiB pieces per sub-tile
    constexpr uint32_t kPerWave = kPieces / 8;          // row DMAs per wave per sub-tile
    constexpr uint32_t kSubBytes = kPieces * 1024u;
    constexpr uint32_t kRows = kI8qSub * 32u;           // rows per sub-tile (one per lane)
    constexpr uint32_t kBufBytes = kSubBytes;
    constexpr uint32_t kOps = kPerWave + 1u;            // vector-memory ops per stage of a wave with an operand DMA
    constexpr uint32_t kOpsWaves = kRows == 64 ? 2u : 1u;  // waves that DMA the rows' s_x/|x| and rho_x
    static_assert((kPerWave - 1u) * kI8qSpread < (uint32_t)KS, "every row piece issued within its step");
    static_assert(kPieces % 8 == 0, "pieces split evenly over the waves");
    static_assert(kRows == 64 || kRows == 32, "one operand word per lane");
    __shared__ __attribute__((aligned(16))) char Bs[kI8qBufs][kBufBytes];
    // the rows' s_x/|x| and rho_x of sub-tile i, in a ring one deeper than the row buffers (the
    // transposed form's late waves read step i-1's after the barrier of step i)
    constexpr uint32_t kOpsRing = kI8qBufs + 1u;
    __shared__ __attribute__((aligned(16))) float opsr[kOpsRing][2u * kRows];
    // nomination (slot q, block step i, row group gi, row j) as q << 24 | i << 6 | gi << 5 | j
    __shared__ uint32_t cl[kI8qCl];
    __shared__ float cs[kI8qCl];  // their approx scores
    __shared__ uint32_t cl_n;
    __shared__ __attribute__((aligned(16))) float qinv_l[kFxQ], thr_l[kFxQ], qa_l[kFxQ];
    __shared__ uint32_t fl_n[kFxQ], fl_b[kFxQ];  // flush: entries per query, their global base
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t qtile = SPLIT ? (wv & 3u) : wv;   // this wave's 32 query slots
    const uint32_t gi0 = SPLIT ? (wv >> 2) : 0u;     // its first row group of a sub-tile
    const uint32_t N = a.N, G = gridDim.x;
    const uint32_t nsub_all = ((N + kFxRows - 1) / kFxRows) * (kFxRows / 32u / kI8qSub);
    const uint32_t ns = blockIdx.x < nsub_all ? (nsub_all - blockIdx.x + G - 1) / G : 0u;  // sub-tiles b, b+G, ...
    const char* rowsx = (const char*)a.rowsx;
    constexpr uint32_t kSubPerTile = kFxRows / 32u / kI8qSub;
    auto sub_of = [&](uint32_t i, uint32_t& t, uint32_t& u) __attribute__((always_inline)) {
        const uint32_t ii = i < ns ? i : (ns ? ns - 1 : 0);  // clamped: a valid read, never used
        const uint32_t v = blockIdx.x + ii * G;
        t = v / kSubPerTile;
        u = v % kSubPerTile;
    };
    // stage i: the block's i-th sub-tile -> buffer i % kI8qBufs, as kPerWave 1 KiB row
    // pieces per wave (piece p = (gi*KC + c)*4 + s4: row group kI8qSub*u + gi of tile
    // t), plus one op of the operand waves: the rows' s_x/|x| and rho_x
    auto piece = [&](uint32_t i, uint32_t k) __attribute__((always_inline)) {
        uint32_t t, u;
        sub_of(i, t, u);
        const uint32_t l0 = (uint32_t)(uintptr_t)Bs[i % kI8qBufs];
        const uint32_t p = wv * kPerWave + k, s4 = p & 3u, c = (p >> 2) % KC, gi = (p >> 2) / KC;
        const char* ga = rowsx + ((((uint64_t)t * KC + c) * 8u + kI8qSub * u + gi) * 4u + s4) * 1024u + lane * 16u;
        asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(ga), "s"(l0 + p * 1024u)
                     : "memory");
    };
    auto stage_ops = [&](uint32_t i) __attribute__((always_inline)) {
        uint32_t t, u;
        sub_of(i, t, u);
        const uint32_t l0 = (uint32_t)(uintptr_t)opsr[i % kOpsRing];
        if (wv < kOpsWaves) {
            // 64 rows: wave 0 s_x/|x|, wave 1 rho_x; 32 rows: wave 0, lanes 0-31 / 32-63
            const uint32_t r = kRows == 64 ? lane : (lane & 31u);
            const uint32_t n = min(t * kFxRows + u * kRows + r, N - 1u);
            const bool rho = kRows == 64 ? wv == 1 : lane >= 32u;
            const float* src = (rho ? a.rrho : a.rscale) + n;
            asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(src),
                         "s"(l0 + (kRows == 64 ? wv * kRows * 4u : 0u))
                         : "memory");
        }
    };
    auto stage = [&](uint32_t i) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t k = 0; k < kPerWave; ++k) piece(i, k);
        stage_ops(i);
    };
    // this wave's query fragments (A) and per-slot epilogue operands
    fx_v4i A[KS];
    {
        const char* qx = (const char*)a.qx;
#pragma unroll
        for (int s = 0; s < KS; ++s)
            A[s] = *(const fx_v4i*)(qx + (((uint32_t)(s >> 2) * 8u + qtile) * 4u + (uint32_t)(s & 3)) * 1024u + lane * 16u);
        // landed here, once: otherwise the waitcnt pass defers these waits into the
        // loop, where its counts (blind to the asm DMAs) drain the row prefetch
#pragma unroll
        for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(A[s]));
    }
    if (tid < kFxQ) {
        qinv_l[tid] = a.qinv[tid];
        thr_l[tid] = a.thr[tid];
        qa_l[tid] = a.qa[tid];
    }
    if (tid == 0) cl_n = 0;
    __syncthreads();  // the compiler-visible loads above are complete from here on
    constexpr bool kT = GVDB_I8Q_T != 0;
    // transposed: this lane's query slot and its epilogue operands, for the whole launch
    const uint32_t lq = qtile * 32u + (lane & 31u);
    const float lqinv = qinv_l[lq], lthr = thr_l[lq], lqa = qa_l[lq];
    if (ns)
#pragma unroll
        for (uint32_t j = 0; j + 1 < kI8qBufs; ++j) stage(j);
    fx_v16i acc[NGI];
    auto row_of = [&](uint32_t e) {  // a list entry's row
        const uint32_t v = blockIdx.x + ((e >> 6) & 0x3ffffu) * G;
        return (v / kSubPerTile) * kFxRows + (kI8qSub * (v % kSubPerTile) + ((e >> 5) & 1u)) * 32u + (e & 31u);
    };
    // the block's list -> the per-query global lists, block-aggregated (round 5): ranks within
    // (block, query) by LDS atomics, ONE global atomic per (block, query) reserves the slots.
    // One global atomic per entry put ~1000 serialised atomics on each query's counter at the
    // end of a 1.25M-row shard's pass (K2 = 32: ~1000 nominations per query, all blocks
    // flushing together).  Every thread calls it (block-uniform).
    constexpr uint32_t kPerT = (kI8qCl + kFxThreads - 1) / kFxThreads;
    auto flush = [&](uint32_t m) {
        for (uint32_t q = tid; q < kFxQ; q += kFxThreads) fl_n[q] = 0u;
        __syncthreads();
        uint32_t rk[kPerT];
#pragma unroll
        for (uint32_t j = 0; j < kPerT; ++j) {
            const uint32_t x = tid + j * kFxThreads;
            rk[j] = x < m ? atomicAdd(&fl_n[cl[x] >> 24], 1u) : 0u;
        }
        __syncthreads();
        for (uint32_t q = tid; q < kFxQ; q += kFxThreads) {
            const uint32_t c = fl_n[q];
            if (c) fl_b[q] = atomicAdd(&a.counts[q], c);
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kPerT; ++j) {
            const uint32_t x = tid + j * kFxThreads;
            if (x < m) {
                const uint32_t e = cl[x], q = e >> 24, pos = fl_b[q] + rk[j];
                if (pos < a.candcap) {
                    a.cand[(uint64_t)q * a.candcap + pos] = row_of(e);
                    if (a.cscore) a.cscore[(uint64_t)q * a.candcap + pos] = cs[x];
                }
            }
        }
    };
    // The candidate test of step i's accumulators.  Per pair the exact f32 cosine is at most
    // U = approx + qa*rho_x + qd; a row is nominated iff U >= tau (thr = tau - qd).
    auto epilogue = [&](uint32_t i, uint32_t t, uint32_t u, const float* rv, const float* rh)
                        __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t ga = 0; ga < NGI; ++ga) {
            const uint32_t gi = gi0 + ga;
            const uint32_t n = t * kFxRows + (kI8qSub * u + gi) * 32u + (lane & 31u);
            const float rinv = n < N ? rv[ga] : 0.0f, rho = n < N ? rh[ga] : 0.0f;
            // this lane's 16 slots: qb0 + (e & 3) + 8 (e >> 2)
            uint32_t qb0 = qtile * 32u + 4u * (lane >> 5);
            asm volatile("" : "+v"(qb0));  // keep the per-slot addresses out of the loop
            float qs[16], ts[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 qv = *(const float4*)(qinv_l + qb0 + 8 * g);
                const float4 tv = *(const float4*)(thr_l + qb0 + 8 * g);
                const float4 av = *(const float4*)(qa_l + qb0 + 8 * g);
                qs[4 * g + 0] = qv.x * rinv;
                qs[4 * g + 1] = qv.y * rinv;
                qs[4 * g + 2] = qv.z * rinv;
                qs[4 * g + 3] = qv.w * rinv;
                ts[4 * g + 0] = tv.x - av.x * rho;
                ts[4 * g + 1] = tv.y - av.y * rho;
                ts[4 * g + 2] = tv.z - av.z * rho;
                ts[4 * g + 3] = tv.w - av.w * rho;
            }
            float mx = -__builtin_inff();
#pragma unroll
            for (int e = 0; e < 16; ++e) mx = fmaxf(mx, (float)acc[ga][e] * qs[e] - ts[e]);
            if (!__ballot(mx >= 0.0f && n < N)) continue;
            // rare: a candidate in this fragment (thr = +inf for slots >= B)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const uint32_t q = qb0 + (e & 3) + 8u * (e >> 2);
                const float v = (float)acc[ga][e] * qs[e];
                if (n < N && v >= ts[e]) {
                    const uint32_t li = atomicAdd(&cl_n, 1u);
                    if (li < kI8qCl) {
                        cl[li] = (q << 24) | (i << 6) | (gi << 5) | (lane & 31u);
                        cs[li] = v;
                    } else {  // block list full (a burst within one sub-tile): straight to the global list
                        const uint32_t pos = atomicAdd(&a.counts[q], 1u);
                        if (pos < a.candcap) {
                            a.cand[(uint64_t)q * a.candcap + pos] = n;
                            if (a.cscore) a.cscore[(uint64_t)q * a.candcap + pos] = v;
                        }
                    }
                }
            }
        }
    };
    auto set_stats = [&](const float* ops, float* rmx, float* rmn, float* pmx) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t ga = 0; ga < NGI; ++ga) {
            const uint32_t b = (gi0 + ga) * 32u + 4u * (lane >> 5);
            float hi = 0.0f, lo = __builtin_inff(), ph = 0.0f;
#pragma unroll
            for (uint32_t g = 0; g < 4; ++g) {
                const float4 r = *(const float4*)(ops + b + 8u * g);
                const float4 h = *(const float4*)(ops + kRows + b + 8u * g);
                hi = fmaxf(fmaxf(hi, fmaxf(r.x, r.y)), fmaxf(r.z, r.w));
                lo = fminf(fminf(lo, fminf(r.x, r.y)), fminf(r.z, r.w));
                ph = fmaxf(fmaxf(ph, fmaxf(h.x, h.y)), fmaxf(h.z, h.w));
            }
            rmx[ga] = hi;
            rmn[ga] = lo;
            pmx[ga] = ph;
        }
    };
    auto epilogue_t = [&](uint32_t i, uint32_t t, uint32_t u, const float* rmx, const float* rmn, const float* pmx,
                          const float* ops) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t ga = 0; ga < NGI; ++ga) {
            const uint32_t gi = gi0 + ga;
            int m = acc[ga][0];
#pragma unroll
            for (int e = 1; e < 16; ++e) m = max(m, acc[ga][e]);
            const float bnd = (float)m * (m >= 0 ? lqinv * rmx[ga] : lqinv * rmn[ga]);
            const float tmin = lthr - lqa * pmx[ga];
#ifdef GVDB_I8Q_NOPASS
            const bool pass = bnd >= tmin && bnd < -1.0e30f;
#else
            const bool pass = bnd >= tmin;
#endif
            if (!__ballot(pass)) continue;
            if (!pass) continue;
            const uint32_t r0 = 4u * (lane >> 5), nb = t * kFxRows + (kI8qSub * u + gi) * 32u + r0;
            const float* ro = ops + gi * 32u + r0;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const uint32_t rr = (uint32_t)(e & 3) + 8u * (uint32_t)(e >> 2);
                const uint32_t n = nb + rr;
                if (n >= N) continue;
                const float v = (float)acc[ga][e] * (lqinv * ro[rr]);
                if (v >= lthr - lqa * ro[kRows + rr]) {
                    const uint32_t li = atomicAdd(&cl_n, 1u);
                    if (li < kI8qCl) {
                        cl[li] = (lq << 24) | (i << 6) | (gi << 5) | (r0 + rr);
                        cs[li] = v;
                    } else {
                        const uint32_t pos = atomicAdd(&a.counts[lq], 1u);
                        if (pos < a.candcap) {
                            a.cand[(uint64_t)lq * a.candcap + pos] = n;
                            if (a.cscore) a.cscore[(uint64_t)lq * a.candcap + pos] = v;
                        }
                    }
                }
            }
        }
    };
    // Waves 4..7 (the second wave of each SIMD) run step i-1's epilogue right after the
    // barrier of step i, before step i's MFMAs: on every SIMD one wave's candidate test
    // overlaps the other wave's MFMAs instead of both testing while the matrix core idles.
    const bool late = wv >= 4;
    float lrv[NGI] = {}, lrh[NGI] = {};  // step i-1's row operands (late waves)
    float lmx[NGI] = {}, lmn[NGI] = {}, lpx[NGI] = {};  // transposed: step i-1's bound operands
    for (uint32_t i = 0; i < ns; ++i) {
        // stage i landed (stages i+1 .. i+kI8qBufs-2 are the younger ops), then every wave's part
        if (wv < kOpsWaves)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kI8qBufs - 2u) * kOps) : "memory");
        else  // no operand op in this wave's stages
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kI8qBufs - 2u) * (kOps - 1u)) : "memory");
        __syncthreads();
        // every wave reads the list count before any wave adds to it again (the late waves'
        // epilogue follows right after this), so the flush decision is block-uniform
        const bool full = cl_n >= kI8qCl / 2;
        __syncthreads();
        if (full) {  // rare: empty the list before it can overflow
            flush(min(cl_n, kI8qCl));
            __syncthreads();
            if (tid == 0) cl_n = 0;
            __syncthreads();
        }
        stage_ops(i + kI8qBufs - 1u);  // into the buffer read in step i-1 (its row pieces: below)
        uint32_t t, u;
        sub_of(i, t, u);
        const char* Bb = Bs[i % kI8qBufs] + lane * 16u;
        const float* ops = opsr[i % kOpsRing];
        if (late && i > 0) {
            uint32_t tp, up;
            sub_of(i - 1, tp, up);
            if constexpr (kT)
                epilogue_t(i - 1, tp, up, lmx, lmn, lpx, opsr[(i - 1) % kOpsRing]);
            else
                epilogue(i - 1, tp, up, lrv, lrh);
        }
#pragma unroll
        for (uint32_t ga = 0; ga < NGI; ++ga)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[ga][e] = 0;
        // B fragments from LDS, kI8qBr k-steps ahead of their MFMAs (LDS latency > the
        // ~64 cycles of one k-step's two MFMAs)
        constexpr int BR = kI8qBr;
        fx_v4i bf[BR][NGI];
#pragma unroll
        for (int s = 0; s < BR - 1; ++s)
#pragma unroll
            for (uint32_t ga = 0; ga < NGI; ++ga)
                bf[s][ga] = *(const fx_v4i*)(Bb + ((gi0 + ga) * KC * 4u + (uint32_t)s) * 1024u);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s + BR - 1 < KS) {
#pragma unroll
                for (uint32_t ga = 0; ga < NGI; ++ga)
                    bf[(s + BR - 1) % BR][ga] =
                        *(const fx_v4i*)(Bb + ((gi0 + ga) * KC * 4u + (uint32_t)(s + BR - 1)) * 1024u);
            }
            __builtin_amdgcn_sched_barrier(0);  // the reads stay BR - 1 k-steps ahead (no sinking)
            // the row pieces of sub-tile i + kI8qBufs - 1 spread over the MFMAs rather than
            // issued together after the barrier (the DMA issue of all waves at once left the
            // matrix cores idle: emit 2.26 -> 2.09 ms, profiles/r04/flat_spread/); all of them
            // within this step, which the vmcnt count at the next barrier assumes
            if (s % kI8qSpread == 0 && (uint32_t)(s / kI8qSpread) < kPerWave)
                piece(i + kI8qBufs - 1u, (uint32_t)(s / kI8qSpread));
#pragma unroll
            for (uint32_t ga = 0; ga < NGI; ++ga) {
                if constexpr (kT)  // rows x queries: lane = one query, 16 rows
                    acc[ga] = __builtin_amdgcn_mfma_i32_32x32x32_i8(bf[s % BR][ga], A[s], acc[ga], 0, 0, 0);
                else
                    acc[ga] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s], bf[s % BR][ga], acc[ga], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (kT) {
            if (!late) {
                float mx[NGI], mn[NGI], px[NGI];
                set_stats(ops, mx, mn, px);
                epilogue_t(i, t, u, mx, mn, px, ops);
            } else {
                set_stats(ops, lmx, lmn, lpx);
            }
        } else if (!late) {
            float rv[NGI], rh[NGI];
#pragma unroll
            for (uint32_t ga = 0; ga < NGI; ++ga) {
                rv[ga] = ops[(gi0 + ga) * 32u + (lane & 31u)];
                rh[ga] = ops[kRows + (gi0 + ga) * 32u + (lane & 31u)];
            }
            epilogue(i, t, u, rv, rh);
        } else {  // this step's operands to registers: buffer i % 3 is refilled after the next barrier
#pragma unroll
            for (uint32_t ga = 0; ga < NGI; ++ga) {
                lrv[ga] = ops[(gi0 + ga) * 32u + (lane & 31u)];
                lrh[ga] = ops[kRows + (gi0 + ga) * 32u + (lane & 31u)];
            }
        }
    }
    if (late && ns) {
        uint32_t t, u;
        sub_of(ns - 1, t, u);
        if constexpr (kT)
            epilogue_t(ns - 1, t, u, lmx, lmn, lpx, opsr[(ns - 1) % kOpsRing]);
        else
            epilogue(ns - 1, t, u, lrv, lrh);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped prefetches land before exit
    __syncthreads();
    flush(min(cl_n, kI8qCl));
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
    static const bool i8r = [] {  // GVDB_FLAT_I8R=0: k_flat_mx, the streamed-query kernel (A/B)
        const char* e = getenv("GVDB_FLAT_I8R");
        return !(e && e[0] == '0');
    }();
    const uint64_t nsub = (uint64_t)tiles * (kFxRows / 32u / kI8qSub);
    const uint32_t g = fx_grid((uint32_t)std::min<uint64_t>(nsub, 0xffffffffull));
    if (a.i8 && a.KC == 6 && i8r && nsub < (uint64_t)g << 18) {  // one block per CU over the 64-row sub-tiles
        if (a.B <= 128u)  // 4 live query tiles: two waves per tile, one row group each
            hipLaunchKernelGGL((k_flat_i8q<6, true>), dim3(g), dim3(kFxThreads), 0, s, a);
        else
            hipLaunchKernelGGL((k_flat_i8q<6, false>), dim3(g), dim3(kFxThreads), 0, s, a);
    } else if (a.i8)
        hipLaunchKernelGGL((k_flat_mx<false, true>), dim3(fx_grid(tiles)), dim3(kFxThreads), 0, s, a);
    else
        hipLaunchKernelGGL((k_flat_mx<false, false>), dim3(fx_grid(tiles)), dim3(kFxThreads), 0, s, a);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_flat_prune(uint32_t* counts, uint32_t* cand, const float* cscore, uint32_t candcap, uint32_t B,
                             uint32_t k, const float* qa, const float* qd, const float* rrho, const uint64_t* ids,
                             hipStream_t s) {
    if (B == 0 || k == 0 || candcap > kFxCandCap) return hipSuccess;
    hipLaunchKernelGGL(k_flat_prune, dim3(B), dim3(kPrThreads), 0, s, counts, cand, cscore, candcap, k, qa, qd, rrho,
                       ids);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_flat_probes(const float* smp, uint32_t B, uint32_t S, uint32_t every, uint32_t N, const uint64_t* ids,
                              uint32_t* probes, uint32_t* pcount, uint64_t* part, hipStream_t s) {
    if (B == 0) return hipSuccess;
    // GVDB_PROBE_PARTS: blocks per query (A/B).  Default 1: every block starts from an empty
    // top-16 and its first insertions dominate (10M, batch 256: 86 / 169 / 336 us at 1 / 4 / 10
    // blocks per query; the 1.25M shard with K2 = 32: 0.517 / 0.519 / 0.544 ms per batch)
    static const uint32_t P_env = [] {
        const char* e = getenv("GVDB_PROBE_PARTS");
        return e ? (uint32_t)atoi(e) : 1u;
    }();
    uint32_t P = P_env;
    P = part ? std::max<uint32_t>(1u, std::min<uint32_t>(kFxProbeParts, P)) : 1u;
    const uint32_t chunk = (((S + P - 1u) / P) + 63u) & ~63u;
    hipLaunchKernelGGL(k_flat_probes, dim3(B, P), dim3(1024), 0, s, smp, S, every, N, ids, probes, pcount, part, chunk);
    GVDB_LAUNCH_CHECK();
    if (P > 1) {
        hipLaunchKernelGGL(k_flat_probes_merge, dim3(B), dim3(256), 0, s, part, P, every, N, probes, pcount);
        GVDB_LAUNCH_CHECK();
    }
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
    hipLaunchKernelGGL(k_flat_final, dim3(B), dim3(1024), 0, s, counts, cand, candcap, scores, thr, qd, k, descending,
                       ids, out_ids, out_scores, out_n, fail);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace gvdb
