// gvdb_kernels.hip — gfx950 (MI355X, CDNA4) kernels of the grape-vector-db
// ANN hot path.  Wave64 throughout; no CUDA-isms, no dual paths.
//
//   K1  k_pack / k_bytes_to_*        BinaryQuantizer::quantize  (quantization.rs:86-122)
//   K2  k_sample_hist, k_threshold,  multi_stage_search stage 1 (quantization.rs:165-179):
//       k_scan (hot), k_select       exact top-R by (Hamming asc, row asc) == the
//                                    reference's stable sort by similarity desc
//   K3  k_rerank, k_final_sort       stage 2 (quantization.rs:177-190) with
//                                    cosine_similarity_manual (206-216) computed in
//                                    the reference's exact sequential f32 order
//   flat k_flat_scores              storage.rs:296-339 / index.rs:620-640
//   merge k_topk_merge               shard.rs:776-784
//
// Floating point: this file is compiled with -ffp-contract=off and without
// fast-math; every f32 reduction that produces a reported score runs
// sequentially in one lane, in the reference's order, so scores are
// bit-identical to the Rust fold (sum starts at -0.0f, `impl Sum for f32`).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include <type_traits>

#include "gvdb_device.h"
#include "gvdb_internal.h"

namespace gvdb {


// ============================================================================
// K1: sign/threshold packing
// ============================================================================
// A ballot over 64 consecutive dims gives bit l = dim (base + l), LSB-first.
// Msb0 (bitvec::order::Msb0) stores dim 8b+i at bit (7-i) of byte b; read as
// a little-endian u32 that is a per-byte bit reversal.
__device__ __forceinline__ uint32_t msb0_word(uint32_t lsb) { return __builtin_bswap32(__builtin_bitreverse32(lsb)); }

__global__ __launch_bounds__(256) void k_pack(const float* __restrict__ rows, uint64_t n, uint32_t D, float thr,
                                              void* __restrict__ out, int layout, uint64_t cap, uint64_t row0,
                                              uint32_t W4) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t chunks = (D + 63u) / 64u;             // 64-dim units per row
    const uint32_t nbytes = (D + 7u) / 8u;
    const uint32_t nwords_pad = 4u * W4;                 // padded u32 words per row
    const uint64_t units = n * (uint64_t)chunks;
    for (uint64_t u = wave; u < units; u += nwaves) {
        const uint64_t r = u / chunks;
        const uint32_t c = (uint32_t)(u - r * chunks);
        const uint32_t dim = c * 64u + lane;
        // NaN > thr is false, like Rust's `value > threshold`.
        const bool bit = dim < D && rows[r * D + dim] > thr;
        const uint64_t m = __ballot(bit);
        if (lane < 2) {
            const uint32_t w = 2u * c + lane;
            const uint32_t word = msb0_word(lane == 0 ? (uint32_t)m : (uint32_t)(m >> 32));
            if (layout == kPackBytesAoS) {
                uint8_t* o = (uint8_t*)out + r * nbytes;
                for (uint32_t b = 0; b < 4; ++b)
                    if (4u * w + b < nbytes) o[4u * w + b] = (uint8_t)(word >> (8u * b));
            } else if (layout == kPackWordsAoS) {
                if (w < nwords_pad) ((uint32_t*)out)[r * nwords_pad + w] = word;
            } else {
                if (w < nwords_pad) {
                    uint32_t* planes = (uint32_t*)out;
                    planes[(((uint64_t)(w >> 2) * cap) + row0 + r) * 4u + (w & 3u)] = word;
                }
            }
        }
        // zero the pad words beyond the last 64-dim unit (SoA / words layouts)
        if (c == chunks - 1 && layout != kPackBytesAoS) {
            for (uint32_t w = 2u * chunks + lane; w < nwords_pad; w += 64u) {
                if (layout == kPackWordsAoS) ((uint32_t*)out)[r * nwords_pad + w] = 0u;
                else ((uint32_t*)out)[(((uint64_t)(w >> 2) * cap) + row0 + r) * 4u + (w & 3u)] = 0u;
            }
        }
    }
}

hipError_t launch_pack(const float* rows, uint64_t n, uint32_t D, float thr, void* out, int layout, uint64_t cap,
                       uint64_t row0, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t units = n * ((D + 63u) / 64u);
    uint64_t blocks = (units + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(k_pack, dim3((uint32_t)blocks), dim3(256), 0, s, rows, n, D, thr, out, layout, cap, row0,
                       code_w4(D));
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

__global__ void k_bytes_to_soa(const uint8_t* __restrict__ bytes, uint64_t n, uint32_t nbytes, uint32_t nwords,
                               uint32_t* __restrict__ planes, uint64_t cap, uint64_t row0) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n * nwords) return;
    const uint64_t r = t / nwords;
    const uint32_t w = (uint32_t)(t - r * nwords);
    uint32_t word = 0;
    for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t idx = 4u * w + b;
        if (idx < nbytes) word |= (uint32_t)bytes[r * nbytes + idx] << (8u * b);
    }
    planes[(((uint64_t)(w >> 2) * cap) + row0 + r) * 4u + (w & 3u)] = word;
}

hipError_t launch_bytes_to_soa(const uint8_t* bytes, uint64_t n, uint32_t D, uint4* codes, uint64_t cap,
                               uint64_t row0, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t nwords = 4u * code_w4(D);
    const uint64_t total = n * nwords;
    hipLaunchKernelGGL(k_bytes_to_soa, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, bytes, n,
                       (D + 7u) / 8u, nwords, (uint32_t*)codes, cap, row0);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

__global__ void k_bytes_to_words(const uint8_t* __restrict__ bytes, uint64_t n, uint32_t nbytes, uint32_t nwords,
                                 uint32_t* __restrict__ words) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n * nwords) return;
    const uint64_t r = t / nwords;
    const uint32_t w = (uint32_t)(t - r * nwords);
    uint32_t word = 0;
    for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t idx = 4u * w + b;
        if (idx < nbytes) word |= (uint32_t)bytes[r * nbytes + idx] << (8u * b);
    }
    words[r * nwords + w] = word;
}

hipError_t launch_bytes_to_words(const uint8_t* bytes, uint64_t n, uint32_t D, uint32_t* words, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t nwords = 4u * code_w4(D);
    const uint64_t total = n * nwords;
    hipLaunchKernelGGL(k_bytes_to_words, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, bytes, n,
                       (D + 7u) / 8u, nwords, words);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// hamming 0.1.3 distance over byte slices (quantization.rs:139).
__global__ void k_hamming_pairs(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, uint64_t n,
                                uint32_t nbytes, uint32_t* __restrict__ out) {
    const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (r >= n) return;
    uint32_t d = 0;
    const uint8_t* pa = a + r * nbytes;
    const uint8_t* pb = b + r * nbytes;
    for (uint32_t i = 0; i < nbytes; ++i) d += __builtin_popcount((uint32_t)(pa[i] ^ pb[i]));
    out[r] = d;
}

hipError_t launch_hamming_pairs(const uint8_t* a, const uint8_t* b, uint64_t n, uint32_t D, uint32_t* out,
                                hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hamming_pairs, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, a, b, n, (D + 7u) / 8u,
                       out);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ============================================================================
// Sequential-order f32 reductions through an LDS row tile.
//
// One lane owns one row and folds it left to right, exactly like Rust's
// `iter().map(..).sum::<f32>()`.  To keep the HBM reads coalesced, each wave
// first stages a [64 rows][32 dims] tile in LDS (16-B loads, 8 lanes per
// 128-B row segment), then every lane reads its own row back with
// ds_read_b128.  Row stride 36 floats: conflict-free for both the
// ds_write_b128 (8-lane groups) and the ds_read_b128 (16-lane groups).
// ============================================================================
constexpr int kCh = 32;        // dims per staged chunk
constexpr int kTileLd = 36;    // padded LDS row stride (floats)

// Stage rows[row_of(r)][c0 .. c0+32) for r = 0..63 into tile[r][0..32).
// row_base[r] = element offset of row r, or UINT64_MAX for an absent row.
// Elements at/after `len` are written as 0 (never read by the fold).
__device__ __forceinline__ void stage_tile(float* tile, const float* __restrict__ src, const uint64_t* row_base,
                                           uint64_t c0, uint64_t len, bool vec4, uint32_t lane) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const uint32_t idx = it * 64u + lane;
        const uint32_t r = idx >> 3;
        const uint32_t c4 = idx & 7u;
        const uint64_t base = row_base[r];
        const uint64_t j = c0 + 4u * c4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (base != ~0ull) {
            if (vec4 && j + 3 < len) {
                v = *(const float4*)(src + base + j);
            } else {
                if (j + 0 < len) v.x = src[base + j + 0];
                if (j + 1 < len) v.y = src[base + j + 1];
                if (j + 2 < len) v.z = src[base + j + 2];
                if (j + 3 < len) v.w = src[base + j + 3];
            }
        }
        *(float4*)(tile + r * kTileLd + 4u * c4) = v;
    }
}

// sqrt(sum x*x) per row, bit-identical to `a.iter().map(|x| x*x).sum::<f32>().sqrt()`.
__global__ __launch_bounds__(256) void k_row_norms(const float* __restrict__ rows, uint64_t n, uint32_t D,
                                                   float* __restrict__ out, const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ __attribute__((aligned(16))) float tiles[4][64 * kTileLd];
    __shared__ uint64_t bases[4][64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    float* tile = tiles[wv];
    const uint64_t r0 = ((uint64_t)blockIdx.x * 4u + wv) * 64u;
    const uint64_t myrow = r0 + lane;
    bases[wv][lane] = myrow < n ? myrow * D : ~0ull;
    __syncthreads();
    const bool vec4 = (D & 3u) == 0;
    float s = -0.0f;
    for (uint64_t c0 = 0; c0 < D; c0 += kCh) {
        stage_tile(tile, rows, bases[wv], c0, D, vec4, lane);
        __syncthreads();
        const uint32_t m = (uint32_t)((D - c0) < (uint64_t)kCh ? (D - c0) : kCh);
        const float* tr = tile + lane * kTileLd;
        if (m == kCh) {
#pragma unroll
            for (int j = 0; j < kCh; j += 4) {
                const float4 v = *(const float4*)(tr + j);
                s = s + v.x * v.x;
                s = s + v.y * v.y;
                s = s + v.z * v.z;
                s = s + v.w * v.w;
            }
        } else {
            for (uint32_t j = 0; j < m; ++j) s = s + tr[j] * tr[j];
        }
        __syncthreads();
    }
    if (myrow < n) out[myrow] = sqrtf(s);
}

// The same norms for FEW rows (a query batch): k_row_norms runs them in one
// block whose per-chunk staging round trips serialise (~120 us for 256 x 768).
// Here a block of 256 threads stages RB whole rows in LDS with one round trip
// (all loads in flight), then lane r < RB folds row r from -0.0 in order.
constexpr uint32_t kRnSmallFloats = 16384;  // LDS floats per block (64 KiB)
// D % 4 == 0: rows staged at a stride of D + 4 floats (16-B aligned, conflict-free across 16
// lanes at D = 768) and folded from float4 reads, 8 in flight -- the same sequential sum.
__global__ __launch_bounds__(256) void k_row_norms_few(const float* __restrict__ rows, uint64_t n, uint32_t D,
                                                       uint32_t RB, float* __restrict__ out,
                                                       const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    extern __shared__ __attribute__((aligned(16))) float stage[];  // [RB][ld]
    const uint64_t r0 = (uint64_t)blockIdx.x * RB;
    const bool v4 = (D & 3u) == 0;
    const uint32_t nr = (uint32_t)min((uint64_t)RB, n - r0), ld = v4 ? D + 4u : D + 1u;
    const float* src = rows + r0 * D;
    for (uint32_t i = threadIdx.x; i < nr * D; i += 256u) stage[(i / D) * ld + i % D] = src[i];
    __syncthreads();
    if (threadIdx.x < nr) {
        const float* tr = stage + threadIdx.x * ld;
        float s = -0.0f;
        if (v4) {
            const float4* t4 = (const float4*)tr;
#pragma unroll 8
            for (uint32_t j = 0; j < D / 4u; ++j) {
                const float4 x = t4[j];
                s = s + x.x * x.x;
                s = s + x.y * x.y;
                s = s + x.z * x.z;
                s = s + x.w * x.w;
            }
        } else {
            for (uint32_t j = 0; j < D; ++j) s = s + tr[j] * tr[j];
        }
        out[r0 + threadIdx.x] = sqrtf(s);
    }
}

hipError_t launch_row_norms(const float* rows, uint64_t n, uint32_t D, float* out, hipStream_t s,
                            const uint32_t* gate) {
    if (n == 0) return hipSuccess;
    const uint32_t ld = (D & 3u) == 0 ? D + 4u : D + 1u;
    const uint32_t rb = kRnSmallFloats / ld;
    if (n <= 4096 && rb >= 1) {  // few rows: one staging round trip per block
        const uint32_t RB = std::min<uint32_t>(rb, 16u);
        hipLaunchKernelGGL(k_row_norms_few, dim3((uint32_t)((n + RB - 1) / RB)), dim3(256),
                           (size_t)RB * ld * 4u, s, rows, n, D, RB, out, gate);
        GVDB_LAUNCH_CHECK();
        return hipSuccess;
    }
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_row_norms, dim3((uint32_t)blocks), dim3(256), 0, s, rows, n, D, out, gate);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ============================================================================
// K2: BQ Hamming stage 1
// ============================================================================
// popcount(x) + acc as ONE v_bcnt_u32_b32 (the accumulate form).  Written as
// inline asm because LLVM otherwise re-associates the chain into
// v_bcnt(x, 0) + v_add3 trees: +1 VALU op per 2 words on the hot loop.
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
// Streaming read of one 16-B code word that is not re-read by this launch:
// non-temporal (no L2 retention): 6.66 vs 5.94 TB/s for a 960 MB batch-1 code
// sweep in isolation (tools/scan_probe.hip).
__device__ __forceinline__ uint4 load_code_nt(const uint4* p) {
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    const u4v v = __builtin_nontemporal_load((const u4v*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t ham4(const uint4& c, const uint4& q, uint32_t acc) {
    acc = bcnt_acc(c.x ^ q.x, acc);
    acc = bcnt_acc(c.y ^ q.y, acc);
    acc = bcnt_acc(c.z ^ q.z, acc);
    acc = bcnt_acc(c.w ^ q.w, acc);
    return acc;
}

// Sample histogram: blockIdx.x = sample chunk (4096 contiguous rows starting
// at chunk*stride), blockIdx.y = query tile of QT queries.  LDS histogram per
// query, flushed with global atomics (non-zero bins only).
template <int W4>
__global__ __launch_bounds__(256) void k_sample_hist(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                     uint32_t D, uint32_t stride, const uint4* __restrict__ qcodes,
                                                     uint32_t B, uint32_t QT, uint32_t* __restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lh[];  // [QT][D+1] histograms, then [QT][W4] query codes
    const uint32_t nb = D + 1u;
    uint4* qs = (uint4*)(lh + ((QT * nb + 3u) & ~3u));
    const uint64_t start = (uint64_t)blockIdx.x * stride;
    const uint32_t q0 = blockIdx.y * QT;
    const uint32_t qn = (B - q0) < QT ? (B - q0) : QT;
    for (uint32_t i = threadIdx.x; i < QT * nb; i += 256) lh[i] = 0u;
    for (uint32_t i = threadIdx.x; i < qn * W4; i += 256) qs[i] = qcodes[(uint64_t)q0 * W4 + i];
    __syncthreads();
    // the next row's code planes are in flight while the current row is
    // compared with the block's queries (about one wave per SIMD here: a
    // load -> use chain would expose one HBM latency per row)
    uint4 c[W4], cn[W4];
    {
        const uint64_t row = min(start + threadIdx.x, (uint64_t)N - 1);
#pragma unroll
        for (int w = 0; w < W4; ++w) c[w] = load_code_nt(codes + (uint64_t)w * cap + row);
    }
    for (uint32_t it = 0; it < 16; ++it) {
        const uint64_t row = start + it * 256u + threadIdx.x;
        if (row >= N) break;
        const uint64_t nrow = min(row + 256u, (uint64_t)N - 1);
        if (it + 1 < 16) {
#pragma unroll
            for (int w = 0; w < W4; ++w) cn[w] = load_code_nt(codes + (uint64_t)w * cap + nrow);
        }
        uint32_t qi = 0;
        for (; qi < qn; ++qi) {
            const uint4* qc = qs + qi * W4;
            uint32_t d = 0;
#pragma unroll
            for (int w = 0; w < W4; ++w) d = ham4(c[w], qc[w], d);
            atomicAdd(&lh[qi * nb + d], 1u);
        }
#pragma unroll
        for (int w = 0; w < W4; ++w) c[w] = cn[w];
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < qn * nb; i += 256) {
        const uint32_t v = lh[i];
        if (v) atomicAdd(&hist[(uint64_t)(q0 + i / nb) * nb + (i % nb)], v);
    }
}

// T[q] = smallest t with (sample count of d <= t) >= target; D if never.
// One wave per query.
__global__ __launch_bounds__(256) void k_threshold(const uint32_t* __restrict__ hist, uint32_t B, uint32_t D,
                                                   uint32_t target, uint32_t* __restrict__ thr) {
    const uint32_t q = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (q >= B) return;
    const uint32_t t = wave_find_cum(hist + (uint64_t)q * (D + 1u), D + 1u, target);
    if ((threadIdx.x & 63u) == 0) thr[q] = t;
}

// The hot loop.  Each lane holds CPL rows' codes in VGPRs (coalesced 16-B
// loads from the SoA planes); the batch's query codes are wave-uniform and
// arrive through scalar loads, so one pair costs W4*4 x (v_xor_b32 +
// v_bcnt_u32_b32) plus one compare per CPL rows.  Rows with d <= T[q] are
// appended to the query's candidate buffer as (d << 32 | row).
template <int W4, int CPL>
__global__ __launch_bounds__(256) void k_scan(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                              const uint4* __restrict__ qcodes, const uint32_t* __restrict__ thr,
                                              uint32_t B, uint32_t* __restrict__ counts, uint64_t* __restrict__ buf,
                                              uint32_t bufcap) {
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * (256u * CPL);
    uint4 c[CPL][W4];
    uint32_t bias[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const uint64_t n = base + (uint64_t)k * 256u + tid;
        const bool ok = n < N;
        const uint64_t nc = ok ? n : (uint64_t)(N - 1);
        bias[k] = ok ? 0u : 0x01000000u;  // out-of-range rows never pass the threshold
#pragma unroll
        for (int w = 0; w < W4; ++w) c[k][w] = load_code_nt(codes + (uint64_t)w * cap + nc);
    }
    // query codes are wave-uniform: scalar loads.  For narrow codes the next
    // query is prefetched into SGPRs so the s_load latency hides under the
    // current query's VALU work; wide codes would not fit the SGPR file.
    constexpr bool kPrefetch = W4 <= 6;
    uint4 qw[W4];
    uint32_t T = thr[0];
#pragma unroll
    for (int w = 0; w < W4; ++w) qw[w] = qcodes[w];
    for (uint32_t q = 0; q < B; ++q) {
        const uint32_t qnext = (q + 1 < B) ? q + 1 : q;
        uint4 qn[W4];
        uint32_t Tn = 0;
        if constexpr (kPrefetch) {
#pragma unroll
            for (int w = 0; w < W4; ++w) qn[w] = qcodes[(uint64_t)qnext * W4 + w];
            Tn = thr[qnext];
        } else {
#pragma unroll
            for (int w = 0; w < W4; ++w) qw[w] = qcodes[(uint64_t)q * W4 + w];
            T = thr[q];
        }
        uint32_t d[CPL];
#pragma unroll
        for (int k = 0; k < CPL; ++k) d[k] = bias[k];
#pragma unroll
        for (int w = 0; w < W4; ++w) {
#pragma unroll
            for (int k = 0; k < CPL; ++k) d[k] = ham4(c[k][w], qw[w], d[k]);
        }
        uint32_t dmin = d[0];
#pragma unroll
        for (int k = 1; k < CPL; ++k) dmin = min(dmin, d[k]);
        if (dmin <= T) {
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                if (d[k] <= T) {
                    const uint32_t pos = atomicAdd(&counts[q], 1u);
                    if (pos < bufcap)
                        buf[(uint64_t)q * bufcap + pos] =
                            ((uint64_t)d[k] << 32) | (uint32_t)(base + (uint64_t)k * 256u + tid);
                }
            }
        }
        if constexpr (kPrefetch) {
#pragma unroll
            for (int w = 0; w < W4; ++w) qw[w] = qn[w];
            T = Tn;
        }
    }
}

// Generic scan for codes wider than the templated set: codes re-read per
// query (L1/L2 resident within the block).
__global__ __launch_bounds__(256) void k_scan_generic(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                      uint32_t W4, const uint4* __restrict__ qcodes,
                                                      const uint32_t* __restrict__ thr, uint32_t B,
                                                      uint32_t* __restrict__ counts, uint64_t* __restrict__ buf,
                                                      uint32_t bufcap) {
    const uint64_t n = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (n >= N) return;
    for (uint32_t q = 0; q < B; ++q) {
        const uint4* qc = qcodes + (uint64_t)q * W4;
        uint32_t d = 0;
        for (uint32_t w = 0; w < W4; ++w) d = ham4(codes[(uint64_t)w * cap + n], qc[w], d);
        if (d <= thr[q]) {
            const uint32_t pos = atomicAdd(&counts[q], 1u);
            if (pos < bufcap) buf[(uint64_t)q * bufcap + pos] = ((uint64_t)d << 32) | (uint32_t)n;
        }
    }
}

__global__ void k_sample_hist_generic(const uint4* __restrict__ codes, uint64_t cap, uint32_t N, uint32_t D,
                                      uint32_t W4, uint32_t stride, const uint4* __restrict__ qcodes, uint32_t B,
                                      uint32_t* __restrict__ hist) {
    const uint64_t start = (uint64_t)blockIdx.x * stride;
    const uint32_t q = blockIdx.y;
    const uint4* qc = qcodes + (uint64_t)q * W4;
    for (uint32_t it = 0; it < 16; ++it) {
        const uint64_t row = start + it * 256u + threadIdx.x;
        if (row >= N) break;
        uint32_t d = 0;
        for (uint32_t w = 0; w < W4; ++w) d = ham4(codes[(uint64_t)w * cap + row], qc[w], d);
        atomicAdd(&hist[(uint64_t)q * (D + 1u) + d], 1u);
    }
}


// Block-wide exclusive prefix of a per-thread flag in thread order (one
// ballot per wave + the wave totals in LDS).  *total = the block's count.
__device__ __forceinline__ uint32_t block_prefix_flag(bool f, uint32_t* wcnt, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = (blockDim.x + 63u) >> 6;
    const uint64_t m = __ballot(f);
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), tot = 0;
    for (uint32_t i = 0; i < nw; ++i) {
        const uint32_t c = wcnt[i];
        if (i < w) pre += c;
        tot += c;
    }
    __syncthreads();  // wcnt is rewritten by the next call
    *total = tot;
    return pre;
}

__device__ __forceinline__ uint32_t code_dist(const uint4* __restrict__ codes, uint64_t cap, uint32_t W4,
                                              const uint4* __restrict__ qc, uint64_t n) {
    uint32_t d = 0;
    for (uint32_t w = 0; w < W4; ++w) d = ham4(codes[(uint64_t)w * cap + n], qc[w], d);
    return d;
}

// sk[0..n) -> sorted ascending (padded to a power of two with ~0).  Keys
// must be distinct (they carry the row).  Up to kRankSortMax keys: rank
// counting (key i goes to #{j : key_j < key_i}; no barrier inside, LDS
// broadcast reads) through `tmp`; larger sets: the LDS bitonic network.
constexpr uint32_t kRankSortMax = 512;
__device__ __forceinline__ void select_sort(uint64_t* sk, uint32_t n, uint64_t* tmp) {
    if (n <= kRankSortMax && tmp) {
        uint64_t mine[kRankSortMax / 256];
        uint32_t rank[kRankSortMax / 256];
#pragma unroll
        for (int u = 0; u < (int)(kRankSortMax / 256); ++u) {
            const uint32_t i = threadIdx.x + u * 256u;
            mine[u] = i < n ? sk[i] : ~0ull;
            rank[u] = 0u;
        }
        for (uint32_t j = 0; j < n; ++j) {
            const uint64_t kj = sk[j];
#pragma unroll
            for (int u = 0; u < (int)(kRankSortMax / 256); ++u) rank[u] += kj < mine[u];
        }
#pragma unroll
        for (int u = 0; u < (int)(kRankSortMax / 256); ++u)
            if (threadIdx.x + u * 256u < n) tmp[rank[u]] = mine[u];
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) sk[i] = tmp[i];
        __syncthreads();
        return;
    }
    const uint32_t P = next_pow2(n);
    for (uint32_t i = n + threadIdx.x; i < P; i += blockDim.x) sk[i] = ~0ull;
    __syncthreads();
    bitonic_sort_lds(sk, P);
}

// Exact stage-1 top-R of ALL rows for one query by this block alone: pass 1
// histograms every distance -> T_R; pass 2 walks the rows in order keeping
// d < T_R and the first (R - count(d < T_R)) rows with d == T_R -- the
// reference's stable sort by (similarity desc, index) restricted to its first
// R.  The rare fallback of the certified fast path (threshold estimate too
// tight, candidate buffer overflow); no host round trip.
__device__ __noinline__ void select_rescan(const uint4* __restrict__ codes, uint64_t cap, uint32_t N, uint32_t D,
                                           uint32_t W4, const uint4* __restrict__ qc, uint32_t R, uint64_t* sk,
                                           uint32_t* hist) {
    __shared__ uint32_t s_T, s_lt, s_n, s_tie, wcnt[16];
    for (uint32_t i = threadIdx.x; i <= D; i += blockDim.x) hist[i] = 0u;
    __syncthreads();
    for (uint64_t n = threadIdx.x; n < N; n += blockDim.x) atomicAdd(&hist[code_dist(codes, cap, W4, qc, n)], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t t = wave_find_cum(hist, D + 1u, R);
        const uint32_t lt = wave_sum_below(hist, t);
        if (threadIdx.x == 0) {
            s_T = t;
            s_lt = lt;
            s_n = 0u;
            s_tie = 0u;
        }
    }
    __syncthreads();
    const uint32_t T = s_T, need = R - s_lt;  // R <= N, so count(d <= T) >= R
    for (uint64_t base = 0; base < N; base += blockDim.x) {
        const uint64_t n = base + threadIdx.x;
        const uint32_t d = n < N ? code_dist(codes, cap, W4, qc, n) : ~0u;
        if (d < T) sk[atomicAdd(&s_n, 1u)] = ((uint64_t)d << 32) | (uint32_t)n;
        uint32_t tot;
        const uint32_t rank = s_tie + block_prefix_flag(d == T, wcnt, &tot);
        if (d == T && rank < need) sk[atomicAdd(&s_n, 1u)] = ((uint64_t)d << 32) | (uint32_t)n;
        __syncthreads();
        if (threadIdx.x == 0) s_tie += tot;
        __syncthreads();
    }
    select_sort(sk, s_n, nullptr);
}

constexpr uint32_t kNoIdx = (1u << 21) - 1u;
__device__ __forceinline__ uint64_t pack_key_idx(uint64_t key, uint32_t idx) {
    return ((key >> 32) << 53) | ((key & 0xffffffffull) << 21) | (uint64_t)idx;
}

// Exact top-R of one query from its candidate buffer, left SORTED in
// sk[0..R) as (d << 32 | row) keys: histogram -> T_R (R-th smallest d); if the
// keys with d <= T_R fit the LDS sort, gather and sort them; otherwise (many
// rows tied at T_R) a radix select over the row index picks the first
// R - count(d < T_R) tied rows in row order, so the sorted list is still the
// reference's stable order.  A query whose buffer cannot hold its top-R (fewer
// than R keys passed the estimated threshold, or the buffer overflowed) is
// answered by select_rescan in the same block: every path is exact and none
// needs the host.  Returns true when the rescan ran.
// LDS: sk [kSelectLdsCap] keys, hist [(D+4)&~3], bins [2048].
__device__ __forceinline__ bool select_topr(uint32_t cnt, const uint64_t* __restrict__ b, uint32_t bufcap,
                                            uint32_t D, uint32_t R, const uint4* __restrict__ codes, uint64_t cap,
                                            uint32_t N, uint32_t W4, const uint4* __restrict__ qc, bool force_rescan,
                                            uint64_t* sk, uint32_t* hist, uint32_t* bins, bool with_idx = false) {
    // with_idx (batch-1 tail; D <= 2047, bufcap <= 2^21): the sorted keys carry
    // their buffer index, (d << 53) | (row << 21) | idx -- the same (d, row)
    // order, plus where the row's exact score was published.  A rescan's keys
    // carry idx = kNoIdx.
    __shared__ uint32_t s_T, s_lt, s_n, s_cut;
    const uint32_t nt = blockDim.x;
    // small buffers (the common case) stay in registers: one global read, issued
    // with the count's (slots past the count are masked below)
    constexpr int KPT = 8;
    uint64_t kk[KPT];
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
        const uint32_t i = threadIdx.x + u * nt;
        kk[u] = i < bufcap ? b[i] : ~0ull;
    }
    if (cnt < R || cnt > bufcap || force_rescan) {
        select_rescan(codes, cap, N, D, W4, qc, R, sk, hist);
        if (with_idx) {
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < R; i += blockDim.x) sk[i] = pack_key_idx(sk[i], kNoIdx);
            __syncthreads();
        }
        return true;
    }
    const bool inreg = cnt <= KPT * nt;
    if (inreg) {
#pragma unroll
        for (int u = 0; u < KPT; ++u)
            if (threadIdx.x + u * nt >= cnt) kk[u] = ~0ull;
    }
    for (uint32_t i = threadIdx.x; i <= D; i += nt) hist[i] = 0u;
    if (threadIdx.x == 0) s_n = 0u;
    __syncthreads();
    if (inreg) {
#pragma unroll
        for (int u = 0; u < KPT; ++u)
            if (kk[u] != ~0ull) atomicAdd(&hist[(uint32_t)(kk[u] >> 32)], 1u);
    } else {
        for (uint32_t i = threadIdx.x; i < cnt; i += nt) atomicAdd(&hist[(uint32_t)(b[i] >> 32)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t t = wave_find_cum(hist, D + 1u, R);
        const uint32_t lt = wave_sum_below(hist, t);
        if (threadIdx.x == 0) {
            s_T = t;
            s_lt = lt;
        }
    }
    __syncthreads();
    const uint32_t T = s_T;
    uint32_t cut = ~0u;  // rows tied at T with row <= cut are kept
    if (s_lt + hist[T] > kSelectLdsCap) {
        // the need-th smallest row among the keys with d == T: radix select,
        // 11 + 11 + 10 bits of the row index (rows in the buffer are distinct)
        uint32_t need = R - s_lt, prefix = 0u, pmask = 0u;
        for (int pass = 0; pass < 3; ++pass) {
            const int shift = pass == 0 ? 21 : pass == 1 ? 10 : 0;
            const uint32_t nb = pass == 2 ? 1024u : 2048u, dm = nb - 1u;
            for (uint32_t i = threadIdx.x; i < nb; i += nt) bins[i] = 0u;
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < cnt; i += nt) {
                const uint64_t key = b[i];
                const uint32_t row = (uint32_t)key;
                if ((uint32_t)(key >> 32) == T && (row & pmask) == prefix) atomicAdd(&bins[(row >> shift) & dm], 1u);
            }
            __syncthreads();
            if (threadIdx.x < 64) {
                const uint32_t bin = wave_find_cum(bins, nb, need);
                const uint32_t below = wave_sum_below(bins, bin);
                if (threadIdx.x == 0) {
                    s_cut = bin;
                    s_n = below;
                }
            }
            __syncthreads();
            need -= s_n;
            prefix |= s_cut << shift;
            pmask |= dm << shift;
            __syncthreads();
        }
        cut = prefix;
        if (threadIdx.x == 0) s_n = 0u;
        __syncthreads();
    }
    if (inreg) {  // wave-aggregated append: one LDS atomic per wave and round
        const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
        for (int u = 0; u < KPT; ++u) {
            const uint64_t key = kk[u];
            const uint32_t d = (uint32_t)(key >> 32);
            const bool keep = key != ~0ull && (d < T || (d == T && (uint32_t)key <= cut));
            const uint64_t m = __ballot(keep);
            if (m == 0) continue;  // wave-uniform
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&s_n, (uint32_t)__popcll(m));
            base = __shfl(base, 0);
            const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (keep && pos < kSelectLdsCap)
                sk[pos] = with_idx ? pack_key_idx(key, threadIdx.x + u * nt) : key;
        }
    } else {
        for (uint32_t i = threadIdx.x; i < cnt; i += nt) {
            const uint64_t key = b[i];
            const uint32_t d = (uint32_t)(key >> 32);
            if (d < T || (d == T && (uint32_t)key <= cut)) {
                const uint32_t pos = atomicAdd(&s_n, 1u);
                if (pos < kSelectLdsCap) sk[pos] = with_idx ? pack_key_idx(key, i) : key;
            }
        }
    }
    __syncthreads();
    // rank-count scratch: the radix bins + whatever follows them (>= 4 KiB)
    select_sort(sk, min(s_n, kSelectLdsCap), (uint64_t*)bins);
    return false;
}

// One block per query: select_topr, then the first R keys -> s1_rows / s1_dist.
// fail[q] / any_fail record the device-side rescans (diagnostics).
__global__ __launch_bounds__(256) void k_select(const uint32_t* __restrict__ counts, const uint64_t* __restrict__ buf,
                                                uint32_t bufcap, uint32_t D, uint32_t R,
                                                const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                uint32_t W4, const uint4* __restrict__ qcodes,
                                                uint32_t* __restrict__ fail, uint32_t* __restrict__ any_fail,
                                                uint32_t* __restrict__ s1_rows, uint32_t* __restrict__ s1_dist,
                                                int force_rescan, uint64_t* __restrict__ keys_out,
                                                uint32_t keys_stride) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];  // kSelectLdsCap keys, then hist, then radix bins
    uint32_t* hist = (uint32_t*)(sk + kSelectLdsCap);
    uint32_t* bins = hist + ((D + 4u) & ~3u);
    const uint32_t q = blockIdx.x;
    const bool rescanned = select_topr(counts[q], buf + (uint64_t)q * bufcap, bufcap, D, R, codes, cap, N, W4,
                                       qcodes + (uint64_t)q * W4, force_rescan != 0, sk, hist, bins);
    if (rescanned && threadIdx.x == 0) {
        fail[q] = 1u;
        atomicOr(any_fail, 1u);
    }
    for (uint32_t i = threadIdx.x; i < R; i += 256) {
        const uint64_t key = sk[i];
        s1_rows[(uint64_t)q * R + i] = (uint32_t)key;
        s1_dist[(uint64_t)q * R + i] = (uint32_t)(key >> 32);
        if (keys_out) keys_out[(uint64_t)q * keys_stride + i] = key;  // sharded search: the exchange-1 block
    }
    // ... whose per-query counts follow the B x keys_stride keys
    if (keys_out && threadIdx.x == 0) ((uint32_t*)(keys_out + (uint64_t)gridDim.x * keys_stride))[q] = R;
}

// ----------------------------------------------------------------------------
// k_scan_mfma — the same stage-1 filter for LARGE batches on the matrix cores.
//
// Hamming as a +/-1 dot product: with s(b) = 1 - 2b per bit,
//   sum_k s(q_k) s(c_k) = Kpad - 2 * hamming(q, c)
// (pad bits are 0 in both codes and cancel), so one 32-bit code word is one
// K=32 step of v_mfma_i32_32x32x32_i8 and the distances stay exact integers.
// Which k-slot a lane's 16 bytes occupy never matters: A (queries) and B
// (candidates) are fed with the same bit->slot map, and the dot product sums
// over all slots.
//
// Block = 8 waves, one CU.  Wave w keeps the +/-1 fragments of query tile w
// (32 queries x all KS k-steps, KS = 4*W4) in VGPRs for the whole launch.
// The block walks candidate tiles of 64 rows (persistent grid): all 512
// threads expand the tile's codes (coalesced SoA 16-B loads) into a
// double-buffered LDS image laid out so every B fragment is one contiguous
// ds_read_b128 per wave; each wave then runs KS x 2 MFMAs (2 sub-tiles of 32
// candidates) and compares its 2 x 16 i32 results with its queries'
// thresholds.  Per pair: 768/1024 of an i8 MFMA slot at D=768, instead of
// 48 VALU ops on the popcount path.
// ----------------------------------------------------------------------------
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));

// 4 code bits -> 4 bytes of +/-1 (bit 0 -> 0x01, bit 1 -> 0xFF): spread the
// bits to bit 0 of each byte with one 24-bit multiply, then byte*255 | 1.
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pm1_x4(uint32_t nib) {
    const uint32_t t = __umul24(nib, 0x00204081u) & 0x01010101u;
    // byte*255 per 16-bit half (v_pk_mul_lo_u16: full rate; a 32-bit t*255
    // would become a quarter-rate v_mul_lo_u32)
    const u16x2_t m = __builtin_bit_cast(u16x2_t, t) * (u16x2_t){255, 255};
    return __builtin_bit_cast(uint32_t, m) | 0x01010101u;
}
__device__ __forceinline__ v4i_t pm1_x16(uint32_t h16) {
    v4i_t r;
    r.x = (int)pm1_x4(h16 & 15u);
    r.y = (int)pm1_x4((h16 >> 4) & 15u);
    r.z = (int)pm1_x4((h16 >> 8) & 15u);
    r.w = (int)pm1_x4((h16 >> 12) & 15u);
    return r;
}


// ----------------------------------------------------------------------------
// k_scan_mx — the large-batch stage-1 filter on block-scaled FP4 MFMA.
// Same +/-1 identity as k_scan_mfma, with each code bit an e2m1 value
// (+1.0 = 0b0010, -1.0 = 0b1010) and unit E8M0 scales (0x7f):
// v_mfma_scale_f32_32x32x64_f8f6f4 runs K=64 per instruction at twice the
// i8 rate, sums exactly in f32 (|dot| <= D < 2^24), and its operands are
// half the LDS bytes.  One k-step = two 32-bit code words; lane half h of a
// fragment carries word (2s + h) as 32 nibbles (verified exact on gfx950 by
// tools/mx_fp4_probe.hip).
// ----------------------------------------------------------------------------
typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef float v16f_t __attribute__((ext_vector_type(16)));

// 8 code bits -> 8 e2m1 nibbles: spread bit i to bit 4i, then (b<<3) | 0x2.
// 32 code bits -> 32 e2m1 nibbles: bit 1 -> -1.0 (0b1010), bit 0 -> +1.0 (0b0010).
// Nibble i of output dword j takes bit 4i+j of w: a fixed permutation of the
// bits, applied identically to query and candidate words, so the dot product
// (and the Hamming distance it encodes) is unchanged; 2 VALU ops per dword.
__device__ __forceinline__ v4i_t fp4_x32(uint32_t w) {
    v4i_t r;
    r.x = (int)(((w << 3) & 0x88888888u) | 0x22222222u);
    r.y = (int)(((w << 2) & 0x88888888u) | 0x22222222u);
    r.z = (int)(((w << 1) & 0x88888888u) | 0x22222222u);
    r.w = (int)((w & 0x88888888u) | 0x22222222u);
    return r;
}
__device__ __forceinline__ v16f_t mfma_fp4(const v4i_t& a, const v4i_t& b, const v16f_t& c) {
    const v8i_t a8 = {a.x, a.y, a.z, a.w, 0, 0, 0, 0};
    const v8i_t b8 = {b.x, b.y, b.z, b.w, 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
}

// The same instruction as inline asm with 4-VGPR fp4 operands.  Through the
// builtin, hipcc hoists the (v4i, 0,0,0,0) -> v8i operand construction out of
// the k-loop and keeps 8-register tuples live per query fragment, which
// spills the two-tile consumer waves.  Hazards handled here (hipcc pads
// nothing inside asm): the chain's first MFMA takes C = literal 0 (no VALU
// write -> srcC hazard), later ones take the previous D whole as C (no wait
// states), and mfma_fp4_drain() puts 32 wait states after a chain's last
// MFMA before any VALU reads D.
__device__ __forceinline__ void mfma_fp4_first(v16f_t& d, const v4i_t& a, const v4i_t& b, int scale) {
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                 : "=&v"(d)
                 : "v"(a), "v"(b), "v"(scale));
}
// an MFMA whose B operand may have just been written by VALU: the two wait
// states of the VALU-write -> MFMA-operand hazard inside the string
__device__ __forceinline__ void mfma_fp4_first_nop(v16f_t& d, const v4i_t& a, const v4i_t& b, int scale) {
    asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                 : "=&v"(d)
                 : "v"(a), "v"(b), "v"(scale));
}
__device__ __forceinline__ void mfma_fp4_acc_nop(v16f_t& d, const v4i_t& a, const v4i_t& b, int scale) {
    asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                 : "+v"(d)
                 : "v"(a), "v"(b), "v"(scale));
}
__device__ __forceinline__ void mfma_fp4_acc(v16f_t& d, const v4i_t& a, const v4i_t& b, int scale) {
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                 : "+v"(d)
                 : "v"(a), "v"(b), "v"(scale));
}
__device__ __forceinline__ void mfma_fp4_drain() { asm volatile("s_nop 15\n\ts_nop 15" ::: "memory"); }
// the same drain naming the accumulators as operands: no compiler read of them
// can be scheduled above it (plain C++ reads of asm-MFMA results otherwise can)
template <int NA>
__device__ __forceinline__ void mfma_fp4_drain_acc(v16f_t (&acc)[NA]) {
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#pragma unroll
    for (int i = 0; i < NA; ++i) asm volatile("" : "+v"(acc[i]));
}


// k_scan_mx2: the FP4 scan with staggered wave halves.  8 waves per CU, one
// 32-query tile each; waves w and w+4 share a SIMD.  Every tile both halves
// run the same work in opposite order:
//   waves 0-3:  issue loads(t+1) -> MFMAs(t) -> threshold test -> expand(t+1, half)
//   waves 4-7:  expand(t+1, half, from registers loaded one tile earlier)
//               -> issue loads(t+2) -> MFMAs(t) -> threshold test
// so on each SIMD one wave's expansion VALU runs beside the other wave's
// MFMAs instead of all waves alternating between the two phases together.
// Each half keeps ONE register set for its codes (expanded, then reloaded:
// no register moves, which would wait on the loads).  One barrier per tile.

// Block-aggregated flush of the per-wave staged emits (k_scan_mx3/mx4): one
// LDS atomic per entry gives its rank within (block, query), then ONE global
// atomicAdd per (block, query) reserves the block's slots in the query's
// candidate buffer.  The per-entry global atomics this replaces all target the
// same <= 256 counters at the end of the kernel and serialise there (53 us of
// the 822 us 10M x 768 scan).  Counters still advance by every emit, so an
// overflow (counts[q] > bufcap) is detected exactly as before.  Call from all
// threads; qcnt[0..nq) must be zero.
template <int kWaves, int kStage>
__device__ __forceinline__ void flush_stage_block(const uint64_t (*st_key)[kStage], const uint8_t (*st_q)[kStage],
                                                  uint32_t wv, uint32_t lane, uint32_t wcnt, uint32_t nq,
                                                  uint32_t* qcnt, uint32_t* qbase, uint32_t* __restrict__ counts,
                                                  uint64_t* __restrict__ buf, uint32_t bufcap) {
    constexpr int kPer = kStage / 64;
    const uint32_t ns = min(wcnt, (uint32_t)kStage);
    uint32_t rk[kPer];
    __syncthreads();  // every wave's stage complete
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint32_t e = lane + 64u * i;
        if (e < ns) rk[i] = atomicAdd(&qcnt[st_q[wv][e]], 1u);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nq; q += kWaves * 64) {
        const uint32_t c = qcnt[q];
        if (c) qbase[q] = atomicAdd(&counts[q], c);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const uint32_t e = lane + 64u * i;
        if (e < ns) {
            const uint32_t qi = st_q[wv][e];
            const uint32_t pos = qbase[qi] + rk[i];
            if (pos < bufcap) buf[(uint64_t)qi * bufcap + pos] = st_key[wv][e];
        }
    }
}

// geometry of k_scan_mx4: 8 waves per CU (2 per SIMD), 32-row sub-tiles
constexpr int kMx3Rows = 32;  // candidates per wave sub-tile
constexpr int kMx3Threads = 512;


// ---------------------------------------------------------------------------
// The FP4 stage-1 operands (k_scan_mx5, the round-2/3 scan, replaced by
// k_scan_mx7 below; k_sample_dense / k_sample_mx use them too).  mx5 had the
// same contract as k_scan_mx3 (emit (d << 32 | row) for every row with Hamming
// d <= thr[q]), three changes measured against it:
//  * {0,1} x {+-1} operands: a row bit b becomes e2m1 {0, v_c} and a query bit
//    e2m1 +-1/v_c, so dot = sum over the row's set bits of (q ? +1 : -1)
//    = 2 pop(q & x) - |x| and Hamming = |q| - dot exactly (|q| per query in
//    LDS).  The row expansion is then one AND per dword (class c = bit 4j+c of
//    the word, v = 0.5 / 1 / 2 / 2; the last class needs one shift): 5 VALU per
//    k-step instead of 12 (shift/and/or per dword plus the half select).
//  * each lane half loads only its own words (uint2 per plane: half h takes
//    components 2h, 2h+1, k-step s uses plane s/2, component 2h + (s&1); the
//    query fragments use the same map), so a ring slot is 2*W4 VGPRs and there
//    is no per-k-step word select.
//  * the code loads are inline asm into a static 3-deep ring with hand-placed
//    s_waitcnt vmcnt(2*W4): hipcc drained vmcnt to 0 at the top of every
//    k_scan_mx3 sub-tile (register copies of the ring across the loop back
//    edge), exposing a full HBM round trip per sub-tile.  Any younger or older
//    vector-memory op (the rare overflow emit) only makes that wait stricter.
// The next k-step's row fragment is expanded between the current k-step's
// MFMAs, so a wave's own VALU runs under its MFMA pipe time.
constexpr int kMx5Threads = 512;  // 8 waves per CU (2 per SIMD): the FP4 stage-1 kernels
__device__ __forceinline__ v4i_t fp4_row01(uint32_t w) {
    v4i_t r;
    r.x = (int)(w & 0x11111111u);         // 0.5
    r.y = (int)(w & 0x22222222u);         // 1.0
    r.z = (int)(w & 0x44444444u);         // 2.0
    r.w = (int)((w >> 1) & 0x44444444u);  // 2.0 (bit 4j+3)
    return r;
}
__device__ __forceinline__ v4i_t fp4_query_pm(uint32_t w) {
    // +-2 / +-1 / +-0.5 / +-0.5 against the row classes above (sign = query bit clear)
    const uint32_t nw = ~w;
    v4i_t r;
    r.x = (int)(((nw & 0x11111111u) << 3) | 0x44444444u);
    r.y = (int)(((nw & 0x22222222u) << 2) | 0x22222222u);
    r.z = (int)(((nw & 0x44444444u) << 1) | 0x11111111u);
    r.w = (int)((nw & 0x88888888u) | 0x11111111u);
    return r;
}
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float d;
    asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
// Query operands of the FP4-MFMA stage-1 kernels (k_sample_dense, k_scan_mx5),
// expanded ONCE per batch instead of once per block: for query group g (256
// queries), qfrag[g][(s*8 + qt)*64 + l] = fp4_query_pm(word 4(s/2) + 2(l/32) +
// (s&1) of query 256g + 32qt + (l&31)), zero words past B; qpc[256g + j] = |q|.
// The kernels' prologue is then a straight 16-B copy of the group's fragments
// (L2-resident, 96 KiB at D = 768) into LDS.
template <int W4>
__global__ __launch_bounds__(256) void k_qfrag(const uint32_t* __restrict__ qwords, uint32_t B, uint32_t ngroups,
                                               v4i_t* __restrict__ qfrag, uint32_t* __restrict__ qpc,
                                               uint32_t* __restrict__ zero, uint32_t nzero,
                                               const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    constexpr int KW = 4 * W4, KS = KW / 2, QT = 8;
    constexpr uint32_t kPer = QT * KS * 64;
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < nzero) zero[i] = 0u;  // the stage-1 flags / counts (instead of a memset launch)
    if (i < ngroups * kPer) {
        const uint32_t g = i / kPer, f = i % kPer, l = f & 63u, st = f >> 6, qt = st % QT, qs = st / QT;
        const uint32_t q = g * 256u + qt * 32u + (l & 31u);
        const uint32_t wi = 4u * (qs >> 1) + 2u * (l >> 5) + (qs & 1u);
        qfrag[i] = fp4_query_pm(q < B ? qwords[(uint64_t)q * KW + wi] : 0u);
    }
    if (i < ngroups * 256u) {
        uint32_t pc = 0;
        if (i < B)
            for (int w = 0; w < KW; ++w) pc += __popc(qwords[(uint64_t)i * KW + w]);
        qpc[i] = pc;
    }
}

// ---------------------------------------------------------------------------
// k_scan_mx7: k_scan_mx6 with the MFMA operands swapped (A = the rows' FP4
// fragment, B = the queries'), so D is transposed: lane l holds query
// 32 qt + (l & 31) and 16 corpus rows.  A lane's 16 accumulators then share
// ONE threshold, so the sub-tile's first MFMA of a tile takes C = 0 (no seed
// tile read from LDS right before it, no seed registers) and the test compares
// the max of the 16 dots with the lane's cq = |q| - thr: d = |q| - dot <= thr
// <=> dot >= cq.  Same speed as mx6 (0.645 vs 0.649 ms at 10M x 768 x 256,
// same box), less code; mx6 / mx5 history in DESIGN.md §4.
//
// From k_scan_mx6: k_scan_mx5 with the sub-tile boundary software-pipelined.
// mx5 drains every accumulator after a sub-tile's last k-step, then runs the
// threshold epilogue of all 8 query tiles, re-seeds them and restarts the
// A-fragment ring: a boundary with the matrix pipe idle (ablations: epilogue
// 15 %, seeds 7 % of the scan).  Here each wave's sub-tiles form ONE MFMA
// stream: in k-step 0 of sub-tile i+1, tile qt of sub-tile i is tested and
// re-seeded right before its first MFMA of sub-tile i+1, i.e. between the
// MFMAs of the other tiles (its last MFMA of sub-tile i is 7 MFMAs old
// there), and the A-fragment ring runs on across sub-tiles (its sequence is
// periodic in the sub-tile).
// One wave per SIMD (4 per CU): the 128 accumulator registers live in AGPRs
// (the MFMAs take them as "+a"), which leaves the architectural VGPRs to the
// code ring, the A ring and the tests -- mx5's 2 waves per SIMD had 256
// registers each and no room to keep the A ring live through the tests.
// Tail: the full rounds give every wave the same number of sub-tiles; the
// last partial round (nsub mod waves sub-tiles) is split into (sub-tile,
// query tile) units of KS MFMAs spread over all waves.
// Same emit contract as mx5: (d << 32 | row) for every row with d <= thr[q].
constexpr int kMx7Threads = 512;  // 8 waves per CU, 2 per SIMD
#ifdef GVDB_MX7_CLK
// timing study (variant builds only, scripts/build_variant.sh -DGVDB_MX7_CLK): per wave
// of the last non-dense launch, s_memrealtime (100 MHz) at kernel start, after the
// prologue, after the full rounds, after the tail units, at the end; and the number
// of tile tests that took the hit path
__device__ unsigned long long g_mx7_clk[4096][6];
#define MX7_CLK(i)                                                                              \
    do {                                                                                        \
        if (!DENSE && lane == 0 && gw < 4096u) g_mx7_clk[gw][i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define MX7_CLK(i) \
    do {           \
    } while (0)
#endif
// DENSE (the reference's default depth, R/N >= 1/64): no threshold test; every
// tile's 16 dots per lane go to dense[q][row] as f16 (exact: |dot| <= 768),
// four consecutive rows per 8-byte store; the select reads d = |q| - dot.
// QT: query tiles of 32 per launch (8 = a full 256-query group; smaller batches take
// 1 / 2 / 4 instead of multiplying padded slots: the MFMAs per row scale with QT).
// D8 (with DENSE, round 6: the certified default depth's rule form): one BYTE per pair
// instead of an f16 -- b = clamp(d - base[q], 0, 255) with the query's window base
// passed in `thr` (k_dense_base) -- half the dense block's writes and its histogram
// pass's reads; the rule (k_dense_rule8) checks that T lies strictly inside the window.
// The bytes are BLOCKED: pair (q, n) at ((n / 256) * B + q) * 256 + 32 (n % 256 / 32) + the
// position of row n % 32 within its sub-tile (16 h + 4 g + r for row 8 g + 4 h + r).
template <int W4, bool DENSE, int QT = 8, bool D8 = false>
__global__ __launch_bounds__(kMx7Threads, 1) void k_scan_mx7(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                           const v4i_t* __restrict__ qfrag_g,
                                                           const uint32_t* __restrict__ qpc,
                                                           const uint32_t* __restrict__ thr, uint32_t B,
                                                           uint32_t* __restrict__ counts, uint64_t* __restrict__ buf,
                                                           uint32_t bufcap, uint16_t* __restrict__ dense,
                                                           uint32_t dense_np, const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    constexpr int KW = 4 * W4;  // 32-bit code words per row
    constexpr int KS = KW / 2;  // k-steps of 64 bits
    constexpr int NM = KS * QT;  // MFMAs per sub-tile
#ifdef GVDB_MX7_CLK
    uint32_t n_hit = 0;
#endif
    constexpr int NW = kMx7Threads / 64;
    constexpr int PF = NM % 4 == 0 ? 4 : NM % 3 == 0 ? 3 : 2;  // A-fragment ring depth (in MFMAs; 8: same time)
    constexpr int kExpandAt = QT > 1 ? 1 : 0;  // the next k-step's row fragment is expanded after this tile's MFMA
    static_assert(NM % PF == 0, "the A ring's slot of MFMA m must not depend on the sub-tile");
    // Hit records (the threshold scan): a tile test that hits appends, per hitting LANE,
    // its 16 dots as f16 (exact: |dot| <= 768) + (first row, query) to the wave's LDS
    // record list -- two ds_write_b128 and one ds_write_b64, no read-back -- and the
    // per-value tests, keys and buffer slots are worked out once, at the end (the
    // round-4 hit path staged all 16 values, read them back and emitted per value inside
    // the MFMA stream: ~0.4 us per hit, ~20 % of the scan at the 1.25M-row shard where
    // 29 % of the tile tests hit).  A full list drains to the global buffer.
    constexpr uint32_t kRec = 176;  // records per wave (10M x 768 x 256: ~105 used on average)
    __shared__ __attribute__((aligned(16))) v4i_t qfrag[QT * KS * 64];
    __shared__ float cq_lds[QT * 32];  // |q| - thr (a query past B: never reached)
    __shared__ float pc_lds[QT * 32];  // |q|
    __shared__ uint32_t qcnt[QT * 32], qbase[QT * 32];
    __shared__ uint32_t blk_next;  // the block's sub-tile pool: next free slot
    constexpr uint32_t kRecBytes = NW * kRec * 40u, kTscrBytes = NW * 16u * 64u * 4u;
    __shared__ __attribute__((aligned(16))) char scr_raw[DENSE ? kTscrBytes : kRecBytes];
    // DENSE: a tile's transposed f16 dots per wave; else the hit records: dots [NW][kRec][16] f16 | meta [NW][kRec]
    float(*tscr)[16 * 64] = (float(*)[16 * 64])scr_raw;
    uint4(*rec_v)[kRec][2] = (uint4(*)[kRec][2])scr_raw;
    uint2(*rec_m)[kRec] = (uint2(*)[kRec])(scr_raw + NW * kRec * 32u);
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t h = lane >> 5;
    const uint32_t nsub = (N + 31u) / 32u;
    const uint32_t W = gridDim.x * NW;        // waves in the grid
    const uint32_t nround = nsub / W;         // full rounds (every wave the same count)
    const uint32_t gw = blockIdx.x * NW + wv;
    MX7_CLK(0);
    uint2 ring[2][W4];
    auto load = [&](uint32_t sb, uint2 (&c)[W4]) __attribute__((always_inline)) {
        const uint32_t n = min(sb * 32u + (lane & 31u), N - 1u);  // clamped: branch-free ring
        const uint32_t voff = n * 16u + h * 8u;
#pragma unroll
        for (int p = 0; p < W4; ++p) {
            const uint4* base = codes + (uint64_t)p * cap;
            asm volatile("global_load_dwordx2 %0, %1, %2" : "=v"(c[p]) : "v"(voff), "s"(base));
        }
    };
    // the first two sub-tiles' codes are in flight during the prologue
    if (nround > 0) {
        load(gw, ring[0]);
        load(gw + W, ring[1]);
    }
    // the group's fragments are laid out for 8 tiles: (k-step, tile, lane) at (s * 8 + qt) * 64 + l
#pragma unroll 4
    for (uint32_t i = tid; i < (uint32_t)(QT * KS * 64); i += kMx7Threads)
        qfrag[i] = QT == 8 ? qfrag_g[i] : qfrag_g[((i >> 6) / QT * 8u + (i >> 6) % QT) * 64u + (i & 63u)];
    constexpr uint32_t kPadBits = 32u * KW;
    if (tid < QT * 32) {
        const uint32_t q = tid;
        const uint32_t pc = qpc[q];
        // D8: |q| - base (the byte of a pair is |q| - base - dot, clamped)
        cq_lds[q] = DENSE ? (D8 && q < B ? (float)pc - (float)thr[q] : 0.0f)
                          : q < B ? (float)pc - (float)min(thr[q], kPadBits) : 1.0e9f;
        pc_lds[q] = (float)pc;
        qcnt[q] = 0u;
    }
    if (tid == 0) blk_next = 2u * NW;  // slots wv and NW + wv: the prologue's loads
    __syncthreads();
    float cq[QT];  // this lane's query of each tile
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) cq[qt] = cq_lds[qt * 32 + (lane & 31u)];
    const uint32_t nqt = (B + 31u) / 32u;
    uint32_t wrec = 0;  // this wave's hit records (wave-uniform)
    v16f_t acc[QT];
    // global (address space 1) pointers: a flat atomic / store in the stream would count in
    // lgkmcnt too and make every later LDS wait of the stream a full lgkmcnt(0)
    typedef __attribute__((address_space(1))) uint32_t g_u32;
    typedef __attribute__((address_space(1))) uint64_t g_u64;
    // a record's hits: value r is row nb + 8 (r / 4) + (r % 4) of query qi; hit iff dot >= cq[qi], row < N
    auto rec_hits = [&](uint32_t e, uint32_t& qi, uint32_t& nb, float (&v)[16]) __attribute__((always_inline)) {
        const uint2 m = rec_m[wv][e];
        nb = m.x;
        qi = m.y;
        const uint4 a0 = rec_v[wv][e][0], a1 = rec_v[wv][e][1];
        const uint32_t w[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float c = cq_lds[qi];
        uint32_t hm = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            v[r] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w[r >> 1] >> (16 * (r & 1))));
            const uint32_t n = nb + 8u * (uint32_t)(r >> 2) + (uint32_t)(r & 3);
            hm |= (v[r] >= c && n < N) ? 1u << r : 0u;
        }
        return hm;
    };
    // the wave's full list -> the global buffer, one atomic per emit (rare: a burst of hits)
    auto drain = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the lanes' record writes before the reads
        g_u32* cnt = (g_u32*)counts;
        g_u64* bf = (g_u64*)buf;
        uint32_t bcap = bufcap;
        asm volatile("" : "+s"(cnt), "+s"(bf), "+s"(bcap));
#pragma unroll 1
        for (uint32_t e = lane; e < wrec; e += 64u) {
            uint32_t qi, nb;
            float v[16];
            uint32_t hm = rec_hits(e, qi, nb, v);
            const float pcl = pc_lds[qi];
#pragma unroll 1
            while (hm) {
                const uint32_t r = __builtin_ctz(hm);
                hm &= hm - 1u;
                float vr = v[0];
#pragma unroll
                for (int j = 1; j < 16; ++j) vr = (uint32_t)j == r ? v[j] : vr;
                const uint32_t pos = __hip_atomic_fetch_add(cnt + qi, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t n = nb + 8u * (r >> 2) + (r & 3u);
                if (pos < bcap) bf[(uint64_t)qi * bcap + pos] = ((uint64_t)(uint32_t)(int)(pcl - vr) << 32) | n;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        wrec = 0;
    };
    const int scale1 = 0x7f7f7f7f;
    // threshold test of one query tile (a hit: dot >= cq).  Common path: the max
    // of the lane's 16 dots against its cq and one ballot.  Rare hit path, kept
    // compact: the tile's values go to the wave's LDS scratch, then a runtime
    // loop over the groups of 4 registers (4 consecutive rows) that hold a hit.
    // Register r holds row 8 (r / 4) + 4 h + (r % 4) of the sub-tile at n0.
    auto test = [&](const v16f_t& A, uint32_t qt, uint32_t n0) __attribute__((always_inline)) {
        if constexpr (DENSE && D8) {
            // no transpose: within each 32-row sub-tile the bytes are stored PERMUTED --
            // position 16 h + 4 g + r holds row 8 g + 4 h + r (register 4 g + r of lane half h)
            // -- so a lane's 16 bytes (one query) are one contiguous 16-B store, with no LDS
            // round trip or wave barrier in the MFMA stream; the readers (k_dense_seg_hist8,
            // k_dense_rule8) undo the permutation
#ifdef GVDB_D8_NOEPI
            return;  // timing probe (variant builds only): the MFMA stream without the epilogue
#endif
            const uint32_t qi = qt * 32u + (lane & 31u);
            if (qt < nqt && qi < B) {
                const float cb = cq[qt];  // |q| - base: the byte is cb - dot (an exact integer)
                typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
                u4v_t v0;
#pragma unroll
                for (int g = 0; g < 4; ++g) {  // word g: rows 8g + 4h .. +3
                    uint32_t x = 0u;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        x = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(cb - A[4 * g + r], 0.0f, 255.0f),
                                                           (uint32_t)r, x);
                    v0[g] = x;
                }
                typedef __attribute__((address_space(1))) u4v_t g_u4;
                // blocked layout [row / 256][query][row % 256 (permuted per sub-tile)]: a block's 8
                // consecutive sub-tiles fill one 64-KiB region (B = 256)
                g_u4* dst = (g_u4*)((uint8_t*)dense + ((uint64_t)(n0 >> 8) * B + qi) * 256u + (n0 & 255u) + 16u * h);
#ifndef GVDB_D8_NOSTORE  // timing probe (variant builds only): the epilogue without its stores
                dst[0] = v0;
#endif
            }
            return;
        } else if constexpr (DENSE) {
            // the tile's 32 x 32 f16 dots go through the wave's LDS scratch ([query][row
            // pair], padded rows) so that lane L stores rows 16 (L & 1) .. +15 of query
            // L / 2 as 32 contiguous bytes: 64-B segments per query instead of 8-B pieces
            // (rows past N land in the block's padding: its row stride is N rounded up to 32)
            if (qt < nqt) {
                constexpr uint32_t kLd = 18;  // u32 per query row of the scratch (16 + 2 pad)
                uint32_t* tw = (uint32_t*)tscr[wv];
                const uint32_t j = lane & 31u;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const uint32_t p = 4u * (uint32_t)g + 2u * h;  // row pair of rows 8g + 4h, 8g + 4h + 1
                    tw[j * kLd + p] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[4 * g], A[4 * g + 1]));
                    tw[j * kLd + p + 1u] =
                        __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[4 * g + 2], A[4 * g + 3]));
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                const uint32_t qo = lane >> 1, half = lane & 1u;
                const uint32_t* src = tw + qo * kLd + 8u * half;
                typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
                const u4v_t v0 = {src[0], src[1], src[2], src[3]};
                const u4v_t v1 = {src[4], src[5], src[6], src[7]};
                const uint32_t qi = qt * 32u + qo;
                if (qi < B) {
                    typedef __attribute__((address_space(1))) u4v_t g_u4;
                    g_u4* dst = (g_u4*)(dense + (uint64_t)qi * dense_np + n0 + 16u * half);
                    dst[0] = v0;
                    dst[1] = v1;
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
            return;
        }
        // (v_max3_f32 through asm: the dots are finite, no canonicalisation needed)
        const float m0 = max3f(A[0], A[1], A[2]), m1 = max3f(A[3], A[4], A[5]), m2 = max3f(A[6], A[7], A[8]);
        const float m3 = max3f(A[9], A[10], A[11]), m4 = max3f(A[12], A[13], A[14]);
        const float mx = max3f(max3f(m0, m1, m2), m3, max3f(m4, A[15], A[15]));
        const float c = cq[qt];
        const bool ok = qt < nqt;  // padded query tile: no emits (a query past B has cq = 1e9)
        const bool hit = ok && mx >= c;
        const uint64_t hb = __ballot(hit);
        if (hb) {
#ifdef GVDB_MX7_CLK
            ++n_hit;
#endif
            const uint32_t nh = (uint32_t)__popcll(hb);
            if (wrec + nh > kRec) drain();
            if (hit) {
                const uint32_t e = wrec + __builtin_amdgcn_mbcnt_hi((uint32_t)(hb >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)hb, 0u));
                uint4 a0, a1;
                a0.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[0], A[1]));
                a0.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[2], A[3]));
                a0.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[4], A[5]));
                a0.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[6], A[7]));
                a1.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[8], A[9]));
                a1.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[10], A[11]));
                a1.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[12], A[13]));
                a1.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(A[14], A[15]));
                rec_v[wv][e][0] = a0;
                rec_v[wv][e][1] = a1;
                rec_m[wv][e] = make_uint2(n0 + 4u * h, qt * 32u + (lane & 31u));
            }
            wrec += nh;
        }
    };
    MX7_CLK(1);
    const v4i_t* qf = qfrag + lane;
    // A fragment mm of the sub-tile: two base registers, one per 64 KiB of
    // fragments (a ds_read offset is 16 bits; without the split hipcc keeps one
    // address VGPR per fragment past 64 KiB)
    typedef __attribute__((address_space(3))) const v4i_t lds_v4i_t;
    const uint32_t qf_lo = (uint32_t)(uintptr_t)qf;  // LDS byte address
    uint32_t qf_hi = qf_lo + 64u * 64u * 16u;
    asm volatile("" : "+v"(qf_hi));  // opaque: hipcc folds it back into qf_lo otherwise
    auto afrag = [&](int mm) __attribute__((always_inline)) -> v4i_t {
        const uint32_t ad = mm < 64 ? qf_lo + (uint32_t)mm * 1024u : qf_hi + (uint32_t)(mm - 64) * 1024u;
        return *(lds_v4i_t*)ad;
    };
    // The full rounds are shared out DYNAMICALLY inside the block: the block owns the
    // sub-tiles b*NW + w + r*W (r < nround, w < NW) -- pool slot j = r*NW + w -- and a
    // wave takes the next free slot (an LDS atomic, issued a whole sub-tile ahead of
    // its use) for each ring refill.  With a static share the second wave of every
    // SIMD (waves 4..7, lower MFMA-issue priority) finished its rounds 39 % after the
    // first (601 vs 432 us at 10M x 768 x 256, profiles/r05/mx7clk) and the kernel
    // ended with it.
    const uint32_t npool = nround * (uint32_t)NW;
    auto slot_sb = [&](uint32_t j) { return (j / NW) * W + blockIdx.x * NW + (j % NW); };
    const uint32_t blk_addr = (uint32_t)(uintptr_t)&blk_next;  // LDS byte address
    if (nround > 0) {
        v4i_t ar[PF];
#pragma unroll
        for (int m = 0; m < PF; ++m) ar[m] = afrag(m);
        // one sub-tile of the stream: slot c holds its codes; tile qt of the
        // previous sub-tile (rows of sub-tile sbp) is tested just before its
        // first MFMA here; the slot is refilled with the next pool sub-tile (nx,
        // valid iff nv; else a clamped dummy) after its last expansion
        auto step = [&](uint2 (&c)[W4], uint32_t sb, bool prev, uint32_t sbp, uint32_t& nx, bool& nv)
                        __attribute__((always_inline)) {
            const uint32_t np = sbp * 32u;  // the previous sub-tile's first row
#pragma unroll
            for (int p = 0; p < W4; ++p)  // this slot's loads are the older of the two in flight
                asm volatile("s_waitcnt vmcnt(%1)" : "+v"(c[p]) : "n"(W4));
            // the pool grab through asm: the compiler's atomic (wave-reduced by its atomic
            // optimizer) waited lgkmcnt(0) right here, draining the A ring at every step;
            // this one is waited at the refill (LDS ops complete in order, so the
            // compiler's own counted waits only get stricter)
            uint32_t jn = 0;
            if (lane == 0)
                asm volatile("ds_add_rtn_u32 %0, %1, %2" : "=v"(jn) : "v"(blk_addr), "v"(1u) : "memory");
            v4i_t bcur = fp4_row01(c[0].x);
            v4i_t bnext;
            // k-step 0, peeled (its control flow would stop the k-loop unroll):
            // position qt tests tile qt of the previous sub-tile (its last MFMA is
            // 7 MFMAs old; the pad + the asm naming acc[qt] keep every read below
            // it), re-seeds it, then issues its first MFMA of this sub-tile
#define GVDB_MX7_POS0(qt)                                                      \
            {                                                                  \
                __builtin_amdgcn_sched_barrier(0);                             \
                if (prev) {                                                    \
                    asm volatile("s_nop 4" : "+v"(acc[qt]));                   \
                    test(acc[qt], (uint32_t)(qt), np);                         \
                }                                                              \
                const v4i_t a = ar[(qt) % PF];                                 \
                ar[(qt) % PF] = afrag(((qt) + PF) % NM);                        \
                mfma_fp4_first_nop(acc[qt], bcur, a, scale1);                 \
                if ((qt) == kExpandAt) {                                       \
                    const uint2 v = c[0];                                      \
                    bnext = fp4_row01(v.y);                                    \
                }                                                              \
            }
            if constexpr (QT > 0) GVDB_MX7_POS0(0)
            if constexpr (QT > 1) GVDB_MX7_POS0(1)
            if constexpr (QT > 2) GVDB_MX7_POS0(2)
            if constexpr (QT > 3) GVDB_MX7_POS0(3)
            if constexpr (QT > 4) GVDB_MX7_POS0(4)
            if constexpr (QT > 5) GVDB_MX7_POS0(5)
            if constexpr (QT > 6) GVDB_MX7_POS0(6)
            if constexpr (QT > 7) GVDB_MX7_POS0(7)
#undef GVDB_MX7_POS0
            bcur = bnext;
#pragma unroll
            for (int s = 1; s < KS; ++s) {
                __builtin_amdgcn_sched_barrier(0);
                bnext = bcur;
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    const int m = s * QT + qt;
                    const v4i_t a = ar[m % PF];
                    ar[m % PF] = afrag((m + PF) % NM);  // the ring runs on into the next sub-tile
                    mfma_fp4_acc(acc[qt], bcur, a, scale1);
                    if (qt == kExpandAt && s + 1 < KS) {  // next k-step's row fragment under this one's MFMAs
                        const uint2 v = c[(s + 1) >> 1];
                        bnext = fp4_row01(((s + 1) & 1) ? v.y : v.x);
                    }
                }
                bcur = bnext;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(jn)::"memory");
            jn = __builtin_amdgcn_readfirstlane(jn);
            nv = jn < npool;
            nx = nv ? slot_sb(jn) : nsub;  // nsub: rows past N, clamped (a dummy refill)
            load(nx, c);  // every expansion of this slot is done
        };
        // two inlined copies of step() (one per ring slot); the first sub-tile
        // has no predecessor to test
        uint32_t s0 = gw, s1 = gw + W, sbp = 0, nx;
        bool v0 = true, v1 = nround > 1, prev = false, nv;
        while (v0) {
            step(ring[0], s0, prev, sbp, nx, nv);
            prev = true;
            sbp = s0;
            s0 = nx;
            v0 = nv;
            if (!v1) break;
            step(ring[1], s1, true, sbp, nx, nv);
            sbp = s1;
            s1 = nx;
            v1 = nv;
        }
        asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
        const uint32_t nl = sbp * 32u;
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            asm volatile("" : "+v"(acc[qt]));
            test(acc[qt], (uint32_t)qt, nl);
        }
        // the refills past the end (clamped rows) must land before the registers are reused
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int p = 0; p < W4; ++p) asm volatile("s_waitcnt vmcnt(0)" : "+v"(ring[k][p]));
    }
    MX7_CLK(2);
    // the partial last round: (sub-tile, query tile) units of KS MFMAs over all waves
    const uint32_t sb0 = nround * W;
    const uint32_t nunits = (nsub - sb0) * nqt;
    for (uint32_t u = gw; u < nunits; u += W) {
        const uint32_t sb = sb0 + u / nqt, qt = u % nqt;
        const uint32_t n = sb * 32u + (lane & 31u);
        const uint32_t voff = min(n, N - 1u) * 16u + h * 8u;
        uint2 c[W4];
#pragma unroll
        for (int p = 0; p < W4; ++p) c[p] = *(const uint2*)((const char*)(codes + (uint64_t)p * cap) + voff);
        v16f_t& A = acc[0];
        const v4i_t* qa = qf + qt * 64u;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint2 v = c[s >> 1];
            const v4i_t b = fp4_row01((s & 1) ? v.y : v.x);
            const v4i_t a = qa[s * QT * 64];
            if (s == 0)
                mfma_fp4_first_nop(A, b, a, scale1);
            else
                mfma_fp4_acc_nop(A, b, a, scale1);
        }
        asm volatile("s_nop 15\n\ts_nop 15" : "+v"(A));
        test(A, qt, sb * 32u);
    }
    MX7_CLK(3);
    if constexpr (!DENSE) {
        // the records' emits, block-aggregated: per record its hit count ranks it within
        // (block, query) by one LDS atomic, ONE global atomicAdd per (block, query)
        // reserves the block's slots, then every record writes its keys
        constexpr uint32_t kPer = (kRec + 63u) / 64u;
        uint32_t rk[kPer];
        __syncthreads();  // qcnt zeroed in the prologue; every wave's records complete
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint32_t e = lane + 64u * i;
            rk[i] = 0u;
            if (e < wrec) {
                uint32_t qi, nb;
                float v[16];
                const uint32_t hm = rec_hits(e, qi, nb, v);
                if (hm) rk[i] = atomicAdd(&qcnt[qi], (uint32_t)__popc(hm));
            }
        }
        __syncthreads();
        for (uint32_t q = tid; q < min(B, (uint32_t)QT * 32u); q += kMx7Threads) {
            const uint32_t c = qcnt[q];
            if (c) qbase[q] = atomicAdd(&counts[q], c);
        }
        __syncthreads();
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
            const uint32_t e = lane + 64u * i;
            if (e < wrec) {
                uint32_t qi, nb;
                float v[16];
                const uint32_t hm = rec_hits(e, qi, nb, v);
                uint32_t pos = qbase[qi] + rk[i];
                const float pcl = pc_lds[qi];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    if (!((hm >> r) & 1u)) continue;
                    const uint32_t n = nb + 8u * (uint32_t)(r >> 2) + (uint32_t)(r & 3);
                    if (pos < bufcap) buf[(uint64_t)qi * bufcap + pos] = ((uint64_t)(uint32_t)(int)(pcl - v[r]) << 32) | n;
                    ++pos;
                }
            }
        }
    }
    MX7_CLK(4);
#ifdef GVDB_MX7_CLK
    if (!DENSE && lane == 0 && gw < 4096u) g_mx7_clk[gw][5] = n_hit;
#endif
}

#ifdef GVDB_MX7_CLK
extern "C" int gvdb_debug_mx7_clock(unsigned long long* out, uint32_t n) {  // [n][6]
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mx7_clk), (size_t)std::min(n, 4096u) * 48) == hipSuccess ? 0 : -2;
}
#endif

// CUs of the current device (cached per device: read on every launch)
static uint32_t cu_count() {
    static int cached[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (!cached[dev]) {
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        cached[dev] = cus > 0 ? cus : 256;
    }
    return (uint32_t)cached[dev];
}

// k_qfrag with the query packing fused in: one wave per query slot of the
// groups (ceil(B/256)*256 slots).  The wave packs its query like k_pack (a
// ballot per 64 dims: bit = x > thr, Msb0 words, pad bits 0), writes the words
// [B][4*W4] (the VALU rescan / k_select read them), |q|, and the query's 2*KS
// FP4 fragments (slots past B: zero words) -- one launch instead of two.
template <int W4>
__global__ __launch_bounds__(64) void k_qprep(const float* __restrict__ qf, uint32_t D, float thr, uint32_t B,
                                              uint32_t* __restrict__ qwords, v4i_t* __restrict__ qfrag,
                                              uint32_t* __restrict__ qpc, uint32_t* __restrict__ zero,
                                              uint32_t nzero, const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    constexpr int KW = 4 * W4, KS = KW / 2, QT = 8;
    constexpr uint32_t kPer = QT * KS * 64;
    __shared__ uint32_t w[KW];
    const uint32_t slot = blockIdx.x, lane = threadIdx.x;
    for (uint32_t i = slot * 64u + lane; i < nzero; i += gridDim.x * 64u) zero[i] = 0u;
    const bool live = slot < B;
    // every load of the query row in flight at once (a load -> ballot chain per
    // 64 dims serialised 12 HBM round trips at D = 768)
    float v[KW / 2];
#pragma unroll
    for (int c = 0; c < KW / 2; ++c) {
        const uint32_t d = 64u * (uint32_t)c + lane;
        v[c] = live && d < D ? qf[(uint64_t)slot * D + d] : 0.0f;
    }
#pragma unroll
    for (int c = 0; c < KW / 2; ++c) {  // 64 dims per ballot = 2 words
        const uint32_t d = 64u * (uint32_t)c + lane;
        const uint64_t m = __ballot(live && d < D && v[c] > thr);
        if (lane == 0) {
            w[2 * c] = msb0_word((uint32_t)m);
            w[2 * c + 1] = msb0_word((uint32_t)(m >> 32));
        }
    }
    __syncthreads();
    if (live && lane < (uint32_t)KW) qwords[(uint64_t)slot * KW + lane] = w[lane];
    if (lane == 0) {
        uint32_t pc = 0;
#pragma unroll
        for (int i = 0; i < KW; ++i) pc += __popc(w[i]);
        qpc[slot] = live ? pc : 0u;
    }
    // fragment (s, qt, l) with l = 32 h + j holds word 4(s/2) + 2h + (s&1) of query 32 qt + j
    const uint32_t g = slot / 256u, qt = (slot % 256u) / 32u, j = slot % 32u;
    for (uint32_t t = lane; t < (uint32_t)(2 * KS); t += 64u) {
        const uint32_t s = t >> 1, h = t & 1u;
        const uint32_t wi = 4u * (s >> 1) + 2u * h + (s & 1u);
        qfrag[(uint64_t)g * kPer + (s * QT + qt) * 64u + h * 32u + j] = fp4_query_pm(w[wi]);
    }
}

template <int W4>
static void launch_qfrag_t(const Stage1Args& a, hipStream_t s) {
    if (a.qf32) {
        const uint32_t ng = (a.B + 255u) / 256u;
        hipLaunchKernelGGL((k_qprep<W4>), dim3(ng * 256u), dim3(64), 0, s, a.qf32, a.D, a.qthr, a.B,
                           (uint32_t*)a.qcodes, (v4i_t*)a.qfrag, a.qpc, a.zero, a.nzero, a.gate);
        return;
    }
    constexpr uint32_t kPer = 8u * (2u * W4) * 64u;
    const uint32_t ng = (a.B + 255u) / 256u;
    const uint32_t n = std::max<uint32_t>(ng * kPer, a.nzero);
    hipLaunchKernelGGL((k_qfrag<W4>), dim3((n + 255u) / 256u), dim3(256), 0, s, (const uint32_t*)a.qcodes, a.B, ng,
                       (v4i_t*)a.qfrag, a.qpc, a.zero, a.nzero, a.gate);
}

template <int W4>
static hipError_t launch_scan_mx7_t(const Stage1Args& a, hipStream_t s) {
    constexpr uint64_t kPer = 8u * (2u * W4) * 64u;
    for (uint32_t g = 0; g < a.B; g += 256) {
        const uint32_t bg = min(256u, a.B - g);
        const v4i_t* qf = (const v4i_t*)a.qfrag + (g / 256u) * kPer;
        // the query tiles this group needs (a batch of 64 pays 2 tiles' MFMAs, not 8)
        const uint32_t qt = bg <= 32u ? 1u : bg <= 64u ? 2u : bg <= 128u ? 4u : 8u;
        if (a.dense_sel) {  // every distance of the group, then its members (the dense block is reused per group)
            auto kern = a.dense8 ? (qt == 1 ? k_scan_mx7<W4, true, 1, true> : qt == 2 ? k_scan_mx7<W4, true, 2, true>
                                  : qt == 4 ? k_scan_mx7<W4, true, 4, true> : k_scan_mx7<W4, true, 8, true>)
                                 : (qt == 1 ? k_scan_mx7<W4, true, 1> : qt == 2 ? k_scan_mx7<W4, true, 2>
                                  : qt == 4 ? k_scan_mx7<W4, true, 4> : k_scan_mx7<W4, true, 8>);
            // few tiles: little MFMA work per code load, two blocks per CU keep more loads in flight
            uint16_t* dn = a.dense + (a.dense_keep ? (uint64_t)g * a.dense_np : 0ull);
            // dense8: the window bases in the threshold slot
            const uint32_t* th = a.dense8 ? a.qwin + g : a.thr + g;
            hipLaunchKernelGGL(kern, dim3(cu_count() * (qt <= 2u ? 2u : 1u)), dim3(kMx7Threads), 0, s, a.codes, a.cap,
                               a.N, qf, a.qpc + g, th, bg, a.counts + g, a.buf, a.bufcap, dn, a.dense_np, a.gate);
            GVDB_LAUNCH_CHECK();
            const hipError_t e = launch_select_dense(a, g, bg, s);
            if (e != hipSuccess) return e;
        } else {
            auto kern = qt <= 4 ? k_scan_mx7<W4, false, 4> : k_scan_mx7<W4, false, 8>;
            hipLaunchKernelGGL(kern, dim3(cu_count()), dim3(kMx7Threads), 0, s, a.codes, a.cap, a.N, qf, a.qpc + g,
                               a.thr + g, bg, a.counts + g, a.buf + (uint64_t)g * a.bufcap, a.bufcap, nullptr, 0u,
                               a.gate);
            GVDB_LAUNCH_CHECK();
        }
    }
    return hipSuccess;
}


// k_scan_mx4: k_scan_mx3 for WIDE codes (D > 768, e.g. 3072 bits = 24 planes,
// SURVEY config 4).  The whole batch's expanded query fragments no longer fit
// in LDS (8 tiles x 96 k-steps x 1 KiB = 768 KiB at D = 3072), so a launch
// holds QT query tiles (QT x KS KiB of LDS) and the batch is covered by
// ceil(B / 32QT) launches, each streaming the code planes once.  A row's W4
// planes are split into NC chunks of CH planes; the registers hold one whole
// sub-tile (NC slots of CH planes) and slot c is refilled with chunk c of the
// wave's NEXT sub-tile as soon as chunk c has been consumed, so NC - 1 chunks
// of MFMA work cover each chunk's HBM latency.  The QT accumulators live
// across the chunks; threshold epilogue and emits are those of k_scan_mx3.
//
// Round 5: ONE launch covers every query tile group ("pair" of QT tiles) of the batch.
// Block L runs on XCD L % 8; its slot L / 8 on that XCD names (pair, row block), with
// the row block's npairs blocks on the SAME XCD -- they stream the same code rows at
// about the same time, so 3 of 4 row reads hit that XCD's L2 instead of HBM (the
// launch-per-pair form read the planes ceil(B / 32QT) times from HBM: 4 x 480 MB per
// batch-256 step at the 1.25M-row shard of config 4).
template <int W4, int CH, int QT>
__global__ __launch_bounds__(kMx3Threads, 1) void k_scan_mx4(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                           const uint32_t* __restrict__ qwords_all,
                                                           const uint32_t* __restrict__ thr_all, uint32_t Bt,
                                                           uint32_t* __restrict__ counts_all,
                                                           uint64_t* __restrict__ buf_all, uint32_t bufcap,
                                                           uint32_t npairs) {
    constexpr int KW = 4 * W4;  // 32-bit code words per row
    const uint32_t xcd = blockIdx.x % 8u, slot = blockIdx.x / 8u;
    const uint32_t pair = slot % npairs, rb = (slot / npairs) * 8u + xcd, nrb = gridDim.x / npairs;
    const uint32_t qg0 = pair * 32u * QT;
    const uint32_t B = min(32u * QT, Bt - qg0);
    const uint32_t* __restrict__ qwords = qwords_all + (uint64_t)qg0 * KW;
    const uint32_t* __restrict__ thr = thr_all + qg0;
    uint32_t* __restrict__ counts = counts_all + qg0;
    uint64_t* __restrict__ buf = buf_all + (uint64_t)qg0 * bufcap;
    constexpr int KS = KW / 2;  // k-steps of 64 bits
    constexpr int NC = W4 / CH;
    constexpr int KC = 2 * CH;  // k-steps per chunk
    static_assert(W4 % CH == 0, "chunks must tile the code planes");
    constexpr uint32_t kWaveStage = 512;
    __shared__ __attribute__((aligned(16))) v4i_t qfrag[QT * KS * 64];
    __shared__ __attribute__((aligned(16))) float tf_lds[QT * 32];
    __shared__ float pc_lds[QT * 32];  // |q|
    __shared__ float tmin_lds[QT * 2];
    __shared__ uint64_t st_key[kMx3Threads / 64][kWaveStage];
    __shared__ uint8_t st_q[kMx3Threads / 64][kWaveStage];
    __shared__ uint32_t qcnt[QT * 32], qbase[QT * 32];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int scale1 = 0x7f7f7f7f;
    // round 5: mx7's {0,1} x {+-1} operands (fp4_row01 / fp4_query_pm: dot = 2 pop(q & x) - |x|,
    // Hamming = |q| - dot) and its word map (k-step s, lane half h: word 4 (s / 2) + 2 h + s % 2,
    // one uint2 per plane and half) -- 5 VALU per row fragment and no word select, instead of
    // fp4_x32's 8 plus a select on the uint4 (7.7 VALU per MFMA by PMC at 10M x 3072)
    for (uint32_t i = tid; i < (uint32_t)(QT * KS * 64); i += kMx3Threads) {
        const uint32_t l = i & 63u, st = i >> 6, qs = st % KS, qt = st / KS;
        const uint32_t q = qt * 32u + (l & 31u);
        const uint32_t wi = 4u * (qs >> 1) + 2u * (l >> 5) + (qs & 1u);
        qfrag[i] = fp4_query_pm(q < B ? qwords[(uint64_t)q * KW + wi] : 0u);
    }
    if (tid < QT * 32) {
        uint32_t pc = 0;
        if (tid < B)
            for (int w = 0; w < KW; ++w) pc += __popc(qwords[(uint64_t)tid * KW + w]);
        pc_lds[tid] = (float)pc;
        // a hit: d = |q| - dot <= thr  <=>  dot >= |q| - thr
        tf_lds[tid] = tid < B ? (float)pc - (float)thr[tid] : __builtin_inff();
        qcnt[tid] = 0u;
    }
    __syncthreads();
    if (tid < QT * 2) {
        const float* tq = tf_lds + (tid >> 1) * 32 + 4u * (tid & 1u);
        float m = tq[0];
        for (int r = 1; r < 16; ++r) m = fminf(m, tq[(r & 3) + 8 * (r >> 2)]);
        tmin_lds[tid] = m;
    }
    __syncthreads();
    const uint32_t nsub = (N + kMx3Rows - 1) / kMx3Rows;
    const uint32_t W = nrb * (kMx3Threads / 64);
    const uint32_t h = lane >> 5;
    uint2 cr[NC][CH];  // this lane half's two words of each plane
    auto load = [&](uint32_t sb, int c) __attribute__((always_inline)) {
        const uint32_t n = min(sb * (uint32_t)kMx3Rows + (lane & 31u), N - 1u);  // clamped: branch-free ring
#pragma unroll
        for (int p = 0; p < CH; ++p) cr[c][p] = ((const uint2*)(codes + (uint64_t)(c * CH + p) * cap))[2u * n + h];
    };
    auto word = [&](int c, int s) __attribute__((always_inline)) {
        const uint2 v = cr[c][s >> 1];
        return (s & 1) ? v.y : v.x;
    };
    uint32_t wcnt = 0;
    v16f_t acc[QT];
    auto chunk = [&](int c) __attribute__((always_inline)) {
        const v4i_t* qf = qfrag + lane;
        constexpr int PF = 4;  // A-fragment LDS ring depth
        constexpr int M = KC * QT;  // MFMAs of this chunk: m = s*QT + qt
        v4i_t ar[PF];
        auto aidx = [&](int m) { return ((m % QT) * KS + c * KC + m / QT) * 64; };
#pragma unroll
        for (int m = 0; m < PF; ++m)
            if (m < M) ar[m] = qf[aidx(m)];
#pragma unroll
        for (int s = 0; s < KC; ++s) {
            __builtin_amdgcn_sched_barrier(0);
            const v4i_t b = fp4_row01(word(c, s));
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const int m = s * QT + qt;
                const v4i_t a = ar[m % PF];
                if (m + PF < M) ar[m % PF] = qf[aidx(m + PF)];
                if (c == 0 && s == 0)
                    mfma_fp4_first(acc[qt], a, b, scale1);
                else
                    mfma_fp4_acc(acc[qt], a, b, scale1);
            }
        }
    };
    auto epilogue = [&](uint32_t sb) __attribute__((always_inline)) {
        const uint32_t n = sb * (uint32_t)kMx3Rows + (lane & 31u);
        // opaque copies of the emit pointers: otherwise the per-(tile, row)
        // overflow addresses are hoisted out of the sub-tile loop (64 VGPR pairs)
        uint32_t* cnt = counts;
        uint64_t* bf = buf;
        uint32_t bcap = bufcap;
        asm volatile("" : "+s"(cnt), "+s"(bf), "+s"(bcap));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            __builtin_amdgcn_sched_barrier(0);
            float amax = acc[qt][0];
#pragma unroll
            for (int r = 1; r < 16; ++r) amax = fmaxf(amax, acc[qt][r]);
            if (!__ballot(amax >= tmin_lds[qt * 2 + h] && n < N)) continue;
            float Tf[16];
            const float* tq = tf_lds + qt * 32 + 4u * h;
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const float4 v = *(const float4*)(tq + 8 * g4);
                Tf[4 * g4 + 0] = v.x;
                Tf[4 * g4 + 1] = v.y;
                Tf[4 * g4 + 2] = v.z;
                Tf[4 * g4 + 3] = v.w;
            }
            const uint32_t rb = qt * 32u + 4u * h;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool hit = acc[qt][r] >= Tf[r] && n < N;
                const uint64_t m = __ballot(hit);
                if (m) {
                    if (hit) {
                        const uint32_t sp = wcnt + __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        const uint32_t qi = rb + (r & 3) + 8 * (r >> 2);
                        const uint32_t d = (uint32_t)(int)(pc_lds[qi] - acc[qt][r]);  // exact: integers
                        const uint64_t key = ((uint64_t)d << 32) | n;
                        if (sp < kWaveStage) {
                            st_key[wv][sp] = key;
                            st_q[wv][sp] = (uint8_t)qi;
                        } else {
                            const uint32_t pos = atomicAdd(&cnt[qi], 1u);
                            if (pos < bcap) bf[(uint64_t)qi * bcap + pos] = key;
                        }
                    }
                    wcnt += (uint32_t)__popcll(m);
                }
            }
        }
    };
    uint32_t sb = rb * (kMx3Threads / 64) + wv;
#pragma unroll
    for (int c = 0; c < NC; ++c) load(sb, c);
    for (; sb < nsub; sb += W) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            __builtin_amdgcn_sched_barrier(0);
            chunk(c);
            load(sb + W, c);  // slot c now free: chunk c of the next sub-tile
        }
        mfma_fp4_drain();
        __builtin_amdgcn_sched_barrier(0);
        epilogue(sb);
        __builtin_amdgcn_sched_barrier(0);
    }
    flush_stage_block<kMx3Threads / 64, kWaveStage>(st_key, st_q, wv, lane, wcnt, min(B, (uint32_t)QT * 32u), qcnt,
                                                     qbase, counts, buf, bufcap);
}

#ifndef GVDB_MX4_CH24
#define GVDB_MX4_CH24 6  // code planes per chunk at W4 = 24 (variant builds: -DGVDB_MX4_CH24=N)
#endif
template <int W4, int CH, int QT>
static void launch_scan_mx4_t(const Stage1Args& a, hipStream_t s) {
    const uint32_t cus = cu_count();
    const uint32_t nsub = (a.N + kMx3Rows - 1) / kMx3Rows;
    const uint32_t wpb = kMx3Threads / 64;
    constexpr uint32_t QB = 32u * QT;  // queries per tile group
    const uint32_t npairs = (a.B + QB - 1u) / QB;
    // row blocks: a multiple of 8 (one per XCD per slot row), all resident (one block per CU)
    uint32_t nrbl = std::max<uint32_t>(1u, cus / (8u * npairs));                    // row blocks per XCD
    nrbl = std::min<uint32_t>(nrbl, std::max<uint32_t>(1u, (nsub + 8u * wpb - 1u) / (8u * wpb)));
    const uint32_t grid = 8u * nrbl * npairs;
    hipLaunchKernelGGL((k_scan_mx4<W4, CH, QT>), dim3(grid), dim3(kMx3Threads), 0, s, a.codes, a.cap, a.N,
                       (const uint32_t*)a.qcodes, a.thr, a.B, a.counts, a.buf, a.bufcap, npairs);
}




// The stage-1 sample of WIDE codes on the FP4 matrix cores (round 5): the
// VALU k_sample_hist re-read every 4096-row chunk once per query tile and spent
// 2 x W4 x 4 xor/popcount per (row, query) -- 0.30 ms of the 0.93 ms per-rank
// step of config 4 (10M x 3072, 8 shards of 1.25M rows, batch 256).  Here a block
// holds QT query tiles' fragments (k_scan_mx4's operands and layout: A = queries
// from LDS, B = the row's code words), a wave takes 32 sample positions at a time
// (position p is row (p / 4096) * stride + p % 4096: plan_sampling's chunks), and
// every Hamming distance d = (32 KW - dot) / 2 (exact) goes to dsm[q][p] as u16;
// k_sample_thr then takes T[q] = the smallest t with #{d <= t} >= target from a
// per-query histogram -- k_sample_hist + k_threshold's T, bit for bit (positions past
// the shard's last row, in a shard of <= kExactN rows, are written as 0xffff: not counted).
template <int W4, int QT>
__global__ __launch_bounds__(kMx3Threads, 1) void k_sample_wide(const uint4* __restrict__ codes, uint64_t cap,
                                                               uint32_t N, uint32_t S, uint32_t stride,
                                                               const uint32_t* __restrict__ qwords, uint32_t B,
                                                               uint16_t* __restrict__ dsm) {
    constexpr int KW = 4 * W4;  // 32-bit code words per row
    constexpr int KS = KW / 2;  // k-steps of 64 bits
    __shared__ __attribute__((aligned(16))) v4i_t qfrag[QT * KS * 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, h = lane >> 5;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t q0 = blockIdx.y * 32u * QT;
    for (uint32_t i = tid; i < (uint32_t)(QT * KS * 64); i += kMx3Threads) {
        const uint32_t l = i & 63u, st = i >> 6, qs = st % KS, qt = st / KS;
        const uint32_t q = q0 + qt * 32u + (l & 31u);
        qfrag[i] = fp4_x32(q < B ? qwords[(uint64_t)q * KW + 2u * qs + (l >> 5)] : 0u);
    }
    __syncthreads();
    constexpr float kPadF = (float)(32 * KW);
    const int scale1 = 0x7f7f7f7f;
    const uint32_t nsub = (S + 31u) / 32u, W = gridDim.x * (kMx3Threads / 64);
    for (uint32_t sb = blockIdx.x * (kMx3Threads / 64) + wv; sb < nsub; sb += W) {
        const uint32_t p = sb * 32u + (lane & 31u), pc = min(p, S - 1u);
        const uint32_t raw = (pc >> 12) * stride + (pc & 4095u), row = min(raw, N - 1u);
        const bool live = raw < N;  // a shard of <= kExactN rows: its last chunk runs past N
        uint4 c[W4];
#pragma unroll
        for (int w = 0; w < W4; ++w) c[w] = codes[(uint64_t)w * cap + row];
        v16f_t acc[QT];
#pragma unroll
        for (int st = 0; st < KS; ++st) {
            const uint4 v = c[st >> 1];
            const v4i_t b = fp4_x32((st & 1) ? (h ? v.w : v.z) : (h ? v.y : v.x));
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const v4i_t a = qfrag[(qt * KS + st) * 64 + lane];
                if (st == 0)
                    mfma_fp4_first_nop(acc[qt], a, b, scale1);
                else
                    mfma_fp4_acc_nop(acc[qt], a, b, scale1);
            }
        }
        mfma_fp4_drain_acc(acc);
        if (p < S) {
#pragma unroll
            for (int qt = 0; qt < QT; ++qt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const uint32_t q = q0 + (uint32_t)qt * 32u + 4u * h + (uint32_t)(r & 3) + 8u * (uint32_t)(r >> 2);
                    if (q < B)
                        dsm[(uint64_t)q * S + p] = live ? (uint16_t)((uint32_t)(kPadF - acc[qt][r]) >> 1) : (uint16_t)0xffffu;
                }
        }
    }
}

// T[q] from the query's S sampled distances (k_sample_wide): smallest t with
// #{d <= t} >= target, D if never -- k_threshold's rule on the same counts
__global__ __launch_bounds__(256) void k_sample_thr(const uint16_t* __restrict__ dsm, uint32_t S, uint32_t D,
                                                    uint32_t target, uint32_t* __restrict__ thr) {
    extern __shared__ uint32_t sh[];  // [D + 1]
    const uint32_t q = blockIdx.x, tid = threadIdx.x;
    for (uint32_t t = tid; t <= D; t += 256u) sh[t] = 0u;
    __syncthreads();
    const uint4* src = (const uint4*)(dsm + (uint64_t)q * S);  // S % 8 == 0 (4096-row chunks)
    const uint32_t nv = S / 8u;
    for (uint32_t v = tid; v < nv; v += 256u) {
        const uint4 w = src[v];
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t d = (ws[j >> 1] >> (16 * (j & 1))) & 0xffffu;
            if (d <= D) atomicAdd(&sh[d], 1u);  // 0xffff: a position past the shard's rows
        }
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t t = wave_find_cum(sh, D + 1u, target);
        if (tid == 0) thr[q] = t;
    }
}

template <int W4, int QT>
static void launch_sample_wide_t(const Stage1Args& a, hipStream_t s) {
    const uint32_t S = a.sample_chunks * 4096u;
    const uint32_t npairs = (a.B + 32u * QT - 1u) / (32u * QT);
    const uint32_t bx = std::max<uint32_t>(1u, std::min<uint32_t>(cu_count() / std::max<uint32_t>(1u, npairs),
                                                                  (S / 32u + 7u) / 8u));
    hipLaunchKernelGGL((k_sample_wide<W4, QT>), dim3(bx, npairs), dim3(kMx3Threads), 0, s, a.codes, a.cap, a.N, S,
                       a.sample_stride, (const uint32_t*)a.qcodes, a.B, a.smp);
    hipLaunchKernelGGL(k_sample_thr, dim3(a.B), dim3(256), (size_t)(a.D + 1u) * 4u, s, a.smp, S, a.D, a.target, a.thr);
}

template <int W4, int CPL>
static void launch_scan_t(const Stage1Args& a, hipStream_t s) {
    const uint64_t per_block = 256ull * CPL;
    const uint32_t blocks = (uint32_t)((a.N + per_block - 1) / per_block);
    hipLaunchKernelGGL((k_scan<W4, CPL>), dim3(blocks), dim3(256), 0, s, a.codes, a.cap, a.N, a.qcodes, a.thr, a.B,
                       a.counts, a.buf, a.bufcap);
}

// k_sample_mx: the sample histogram of a large batch on the FP4 MFMA (the
// k_scan_mx5 operands; accumulators seeded with -|q|, so acc = -Hamming).
// The VALU form (k_sample_hist) re-reads the sample once per group of ~13
// queries (LDS holds 13 full histograms) and spends ~48 VALU per pair: 0.10 ms
// per 10M x 768 batch.  Here a block holds 128 queries' fragments (48 KiB) and
// their histograms of d < cap = min(D+1, 384) as packed u16 pairs (96 KiB), so
// the sample is read once per 128 queries.  Flush: each query's bins only up
// to the block's own target-th smallest distance t_b (all bins below cap if the
// block never reaches target).  The global threshold T = smallest t with
// sum_b cnt_b(<= t) >= target satisfies T <= t_b for every block that reached
// target, so the flushed histogram gives k_threshold exactly the T of the full
// one (T >= cap reads as D: a looser, still valid threshold).  Only used for
// sampled shards (N > kExactN, target << sample rows); correctness of the
// search never depends on T (k_select certifies the top-R).
constexpr int kSmxThreads = 512;
constexpr uint32_t kSmxCap = 384;  // histogram bins per query (d < cap)
constexpr uint32_t kSmxHW = kSmxCap / 2;
template <int W4>
__global__ __launch_bounds__(kSmxThreads, 1) void k_sample_mx(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                            uint32_t D, uint32_t stride, uint32_t nsub,
                                                            const uint32_t* __restrict__ qwords, uint32_t B,
                                                            uint32_t target, uint32_t* __restrict__ hist) {
    constexpr int KW = 4 * W4;
    constexpr int KS = KW / 2;
    constexpr int QT = 4;  // query tiles per block (128 queries)
    constexpr int NW = kSmxThreads / 64;
    __shared__ __attribute__((aligned(16))) v4i_t qfrag[KS * QT * 64];
    __shared__ __attribute__((aligned(16))) float seed_lds[QT * 2 * 16];
    __shared__ uint32_t hl[QT * 32 * kSmxHW];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t h = lane >> 5;
    const uint32_t q0 = blockIdx.y * (QT * 32u);
    const uint32_t binc = min(D + 1u, kSmxCap);
    for (uint32_t i = tid; i < (uint32_t)(KS * QT * 64); i += kSmxThreads) {
        const uint32_t l = i & 63u, st = i >> 6, qt = st % QT, qs = st / QT;
        const uint32_t q = q0 + qt * 32u + (l & 31u);
        const uint32_t wi = 4u * (qs >> 1) + 2u * (l >> 5) + (qs & 1u);
        qfrag[i] = fp4_query_pm(q < B ? qwords[(uint64_t)q * KW + wi] : 0u);
    }
    for (uint32_t i = tid; i < (uint32_t)(QT * 32 * kSmxHW); i += kSmxThreads) hl[i] = 0u;
    if (tid < QT * 32) {
        const uint32_t q = q0 + tid;
        uint32_t pc = 0;
        if (q < B)
            for (int w = 0; w < KW; ++w) pc += __popc(qwords[(uint64_t)q * KW + w]);
        const uint32_t qt = tid >> 5, j = tid & 31u, hh = (j >> 2) & 1u, r = (j & 3u) + 4u * (j >> 3);
        // padding queries: acc stays hugely negative -> d >= cap, never counted
        seed_lds[(qt * 2 + hh) * 16 + r] = q < B ? -(float)pc : -1.0e6f;
    }
    __syncthreads();
    const uint32_t W = gridDim.x * NW;
    const int scale1 = 0x7f7f7f7f;
    v16f_t acc[QT];
    for (uint32_t sb = blockIdx.x * NW + wv; sb < nsub; sb += W) {
        // sample sub-tile sb: chunk (32 sb) / 4096 at stride rows, 32 consecutive rows
        const uint32_t s0 = sb * 32u;
        const uint32_t n = (s0 >> 12) * stride + (s0 & 4095u) + (lane & 31u);
        const uint32_t nc = min(n, N - 1u);
        uint2 c[W4];
#pragma unroll
        for (int p = 0; p < W4; ++p) c[p] = ((const uint2*)(codes + (uint64_t)p * cap + nc))[h];
#pragma unroll
        for (int t = 0; t < QT; ++t) {
            const float4* sp = (const float4*)(seed_lds + (t * 2 + h) * 16);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 v = sp[g];
                acc[t][4 * g + 0] = v.x;
                acc[t][4 * g + 1] = v.y;
                acc[t][4 * g + 2] = v.z;
                acc[t][4 * g + 3] = v.w;
            }
        }
        const v4i_t* qf = qfrag + lane;
        constexpr int PF = 6;  // A-fragment LDS ring depth (in MFMAs)
        v4i_t ar[PF];
#pragma unroll
        for (int m = 0; m < PF; ++m) ar[m] = qf[m * 64];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint2 v = c[s >> 1];
            const v4i_t b = fp4_row01((s & 1) ? v.y : v.x);
#pragma unroll
            for (int t = 0; t < QT; ++t) {
                const int m = s * QT + t;
                const v4i_t a = ar[m % PF];
                if (m + PF < KS * QT) ar[m % PF] = qf[(m + PF) * 64];
                if (t == 0)
                    mfma_fp4_acc_nop(acc[t], a, b, scale1);
                else
                    mfma_fp4_acc(acc[t], a, b, scale1);
            }
        }
        mfma_fp4_drain_acc(acc);
        const uint32_t lim = n < N ? binc : 0u;  // rows past N (defensive: sampled chunks lie inside the shard)
#pragma unroll
        for (int t = 0; t < QT; ++t) {
            uint32_t rb = t * 32u + 4u * h;
            asm volatile("" : "+v"(rb));
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint32_t d = (uint32_t)(int)(-acc[t][r]);
                if (d < lim) {
                    const uint32_t ql = rb + (r & 3) + 8 * (r >> 2);
                    atomicAdd(&hl[ql * kSmxHW + (d >> 1)], 1u << ((d & 1u) << 4));
                }
            }
        }
    }
    __syncthreads();
    // flush: one wave per query; lane l holds bins [6l, 6l + 6)
    const uint32_t nb = D + 1u;
    for (uint32_t ql = wv; ql < QT * 32u; ql += NW) {
        const uint32_t q = q0 + ql;
        if (q >= B) break;
        uint32_t cnt[6], sum = 0;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint32_t wi = lane * 3u + i;
            const uint32_t w = wi < kSmxHW ? hl[ql * kSmxHW + wi] : 0u;
            cnt[2 * i] = w & 0xffffu;
            cnt[2 * i + 1] = w >> 16;
            sum += cnt[2 * i] + cnt[2 * i + 1];
        }
        uint32_t incl = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t v = __shfl_up(incl, off);
            if ((int)lane >= off) incl += v;
        }
        const uint64_t m = __ballot(incl >= target);
        uint32_t tb = binc - 1u;
        if (m) {
            const uint32_t first = __ffsll((long long)m) - 1;
            uint32_t t = 0;
            if (lane == first) {
                uint32_t cum = incl - sum;
                for (int i = 0; i < 6; ++i) {
                    cum += cnt[i];
                    if (cum >= target) {
                        t = lane * 6u + i;
                        break;
                    }
                }
            }
            tb = __shfl(t, first);
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const uint32_t bin = lane * 6u + i;
            if (bin <= tb && bin < binc && cnt[i]) atomicAdd(&hist[(uint64_t)q * nb + bin], cnt[i]);
        }
    }
}

template <int W4>
static void launch_sample_mx_t(const Stage1Args& a, hipStream_t s) {
    const uint32_t nsub = a.sample_chunks * (4096u / 32u);
    const uint32_t gy = (a.B + 127u) / 128u;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    // about one block per CU over the query groups; >= 8 x-blocks keeps a
    // block's per-bin count below 2^16 for any sample (<= 262144 rows)
    const uint32_t gx = std::max<uint32_t>(8u, std::min<uint32_t>((uint32_t)cus / gy, (nsub + 7u) / 8u));
    hipLaunchKernelGGL((k_sample_mx<W4>), dim3(gx, gy), dim3(kSmxThreads), 0, s, a.codes, a.cap, a.N, a.D,
                       a.sample_stride, nsub, (const uint32_t*)a.qcodes, a.B, a.target, a.hist);
}

// k_sample_dense + k_sample_select: the stage-1 threshold estimate of a large
// batch without histogram atomics.  k_sample_mx spends most of its time in
// the per-pair LDS-atomic histogram epilogue (~1 atomic per 2 pairs on i.i.d.
// codes); here the FP4 MFMA (k_scan_mx5's operands, accumulators seeded with
// -|q|, so acc = -Hamming) computes every sampled distance and keeps, per
// query and group of 16 consecutive sample rows, their MINIMUM (u16, via a
// per-wave LDS transpose): a dense [B][S/16] block, 1/16 of the distances.
// One block per query then takes the target-th smallest group minimum: a min
// pass, then histograms of narrow windows above the min (only the low tail
// does LDS atomics; the window doubles while the target is not reached).
// Every group whose minimum is <= T holds a row with d <= T, so at least
// `target` sample rows lie at or below T: T is never below the VALU form's
// threshold (equal unless two of the target smallest distances share a
// group), and k_select certifies the top-R whatever T is.
template <int W4>
__global__ __launch_bounds__(kMx5Threads, 1) void k_sample_dense(const uint4* __restrict__ codes, uint64_t cap,
                                                               uint32_t N, uint32_t stride, uint32_t nsub,
                                                               const v4i_t* __restrict__ qfrag_g,
                                                               const uint32_t* __restrict__ qpc, uint32_t B,
                                                               uint16_t* __restrict__ dsm, uint32_t S) {
    constexpr int KW = 4 * W4;
    constexpr int KS = KW / 2;
    constexpr int QT = 8;
    constexpr int NW = kMx5Threads / 64;
    __shared__ __attribute__((aligned(16))) v4i_t qfrag[QT * KS * 64];
    __shared__ __attribute__((aligned(16))) float seed_lds[QT * 2 * 16];
    __shared__ __attribute__((aligned(16))) uint16_t tr_lds[NW][32 * 32];  // per wave: [query][row] of one tile
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t h = lane >> 5;
#pragma unroll 4
    for (uint32_t i = tid; i < (uint32_t)(QT * KS * 64); i += kMx5Threads) qfrag[i] = qfrag_g[i];
    if (tid < QT * 32) {
        const uint32_t q = tid;
        const uint32_t qt = q >> 5, j = q & 31u, hh = (j >> 2) & 1u, r = (j & 3u) + 4u * (j >> 3);
        seed_lds[(qt * 2 + hh) * 16 + r] = q < B ? -(float)qpc[q] : -1.0e6f;
    }
    uint16_t* tw = tr_lds[wv];
    __syncthreads();
    const uint32_t nqt = (B + 31u) / 32u;
    const uint32_t W = gridDim.x * NW;
    const int scale1 = 0x7f7f7f7f;
    v16f_t acc[QT];
    for (uint32_t sb = blockIdx.x * NW + wv; sb < nsub; sb += W) {
        // sample sub-tile sb: chunk (32 sb) / 4096 at `stride` rows, 32 consecutive rows
        const uint32_t s0 = sb * 32u;
        const uint32_t n = (s0 >> 12) * stride + (s0 & 4095u) + (lane & 31u);
        const uint32_t nc = min(n, N - 1u);
        uint2 c[W4];
#pragma unroll
        for (int p = 0; p < W4; ++p) c[p] = ((const uint2*)(codes + (uint64_t)p * cap + nc))[h];
#pragma unroll
        for (int t = 0; t < QT; ++t) {
            const float4* sp = (const float4*)(seed_lds + (t * 2 + h) * 16);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 v = sp[g];
                acc[t][4 * g + 0] = v.x;
                acc[t][4 * g + 1] = v.y;
                acc[t][4 * g + 2] = v.z;
                acc[t][4 * g + 3] = v.w;
            }
        }
        const v4i_t* qf = qfrag + lane;
        constexpr int PF = 8;  // A-fragment LDS ring depth (in MFMAs)
        v4i_t ar[PF];
#pragma unroll
        for (int m = 0; m < PF; ++m) ar[m] = qf[m * 64];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const uint2 v = c[s >> 1];
            const v4i_t b = fp4_row01((s & 1) ? v.y : v.x);
#pragma unroll
            for (int t = 0; t < QT; ++t) {
                const int m = s * QT + t;
                const v4i_t a = ar[m % PF];
                if (m + PF < KS * QT) ar[m % PF] = qf[(m + PF) * 64];
                if (t == 0)
                    mfma_fp4_acc_nop(acc[t], a, b, scale1);
                else
                    mfma_fp4_acc(acc[t], a, b, scale1);
            }
        }
        mfma_fp4_drain_acc(acc);
        // lane (h, j) holds row s0 + j of queries qt*32 + 8(r/4) + 4h + (r%4).
        // Transposed through the wave's LDS tile so that each lane stores 32
        // contiguous bytes (16 rows of one query) instead of 16 scattered u16.
        // Rows past N (the last chunk of an unsampled small shard) read as 0xffff.
        const float lim = n < N ? 65535.0f : -1.0f;
        const uint32_t jj = lane & 31u;
#pragma unroll
        for (int t = 0; t < QT; ++t) {
            if (t < (int)nqt) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const uint32_t qo = 8u * (r >> 2) + 4u * h + (r & 3);
                    const float dv = -acc[t][r];
                    tw[qo * 32u + jj] = lim < 0.0f ? (uint16_t)0xffffu : (uint16_t)min(dv, lim);
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                // lane L: query L/2 of the tile, rows 16 (L%2) .. +15 -> their minimum
                const uint32_t qo = lane >> 1, rh = lane & 1u;
                const uint4 v0 = *(const uint4*)(tw + qo * 32u + rh * 16u);
                const uint4 v1 = *(const uint4*)(tw + qo * 32u + rh * 16u + 8u);
                uint32_t mn = 0xffffu;
                {
                    const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
                    for (int e = 0; e < 8; ++e) mn = min(mn, min(w[e] & 0xffffu, w[e] >> 16));
                }
                uint32_t qg = t * 32u + qo;
                asm volatile("" : "+v"(qg));  // keeps the per-tile row addresses from being hoisted
                if (qg < B) dsm[(uint64_t)qg * (S >> 4) + (s0 >> 4) + rh] = (uint16_t)mn;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
        }
    }
}

// One block per query over its S dense values (S % 8 == 0; here the group minima): the
// query's values are loaded once into registers (kSsPer uint4 = 8 u16 each per
// thread, all loads in flight together), then a min pass and windowed
// histograms run on the registers.  Larger samples stream from memory.
constexpr int kSsThreads = 512;
constexpr int kSsPer = 8;  // uint4 per thread: S <= 512 * 8 * 8 = 32768 values in registers (more stream)
__device__ __forceinline__ void ss_count(uint32_t w, uint32_t base, uint32_t win, uint32_t* hist) {
    const uint32_t o0 = (w & 0xffffu) - base, o1 = (w >> 16) - base;  // wrap below base: outside
    if (o0 < win) atomicAdd(&hist[o0], 1u);
    if (o1 < win) atomicAdd(&hist[o1], 1u);
}
__global__ __launch_bounds__(kSsThreads) void k_sample_select(const uint16_t* __restrict__ dsm, uint32_t S, uint32_t D,
                                                              uint32_t target, uint32_t* __restrict__ thr) {
    constexpr uint32_t kMaxWin = 1024;
    __shared__ uint32_t hist[kMaxWin];
    __shared__ uint32_t red[kSsThreads / 64];
    __shared__ uint32_t s_T, s_cum;
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u;
    const uint4* v = (const uint4*)(dsm + (uint64_t)q * S);
    const uint32_t nv = S / 8u;
    const bool inreg = nv <= (uint32_t)kSsThreads * kSsPer;
    uint4 x[kSsPer];
    uint32_t mn = 0xffffu;
    // register slots in use (block-uniform): the loops over x stop there -- a
    // 1.25M-row shard's sample fills one slot of 40, 10M rows three
    const int jn = (int)((nv + kSsThreads - 1) / kSsThreads);
    if (inreg) {
#pragma unroll
        for (int j = 0; j < kSsPer; ++j) {
            if (j >= jn) continue;
            const uint32_t i = tid + (uint32_t)j * kSsThreads;
            x[j] = i < nv ? v[i] : make_uint4(~0u, ~0u, ~0u, ~0u);
        }
#pragma unroll
        for (int j = 0; j < kSsPer; ++j) {
            if (j >= jn) continue;
            const uint32_t a = min(min(x[j].x & 0xffffu, x[j].x >> 16), min(x[j].y & 0xffffu, x[j].y >> 16));
            const uint32_t b = min(min(x[j].z & 0xffffu, x[j].z >> 16), min(x[j].w & 0xffffu, x[j].w >> 16));
            mn = min(mn, min(a, b));
        }
    } else {
        for (uint32_t i = tid; i < nv; i += kSsThreads) {
            const uint4 y = v[i];
            const uint32_t a = min(min(y.x & 0xffffu, y.x >> 16), min(y.y & 0xffffu, y.y >> 16));
            const uint32_t b = min(min(y.z & 0xffffu, y.z >> 16), min(y.w & 0xffffu, y.w >> 16));
            mn = min(mn, min(a, b));
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, off));
    if (lane == 0) red[tid >> 6] = mn;
    if (tid == 0) {
        s_T = ~0u;
        s_cum = 0u;
    }
    __syncthreads();
    uint32_t base = red[0];
#pragma unroll
    for (int w = 1; w < kSsThreads / 64; ++w) base = min(base, red[w]);
    uint32_t win = 64;  // one round in the common case: the target-th minimum lies within ~40 of the minimum
    while (true) {
        for (uint32_t i = tid; i < win; i += kSsThreads) hist[i] = 0u;
        __syncthreads();
        if (inreg) {
#pragma unroll
            for (int j = 0; j < kSsPer; ++j) {
                if (j >= jn) continue;
                // the bulk of the values lies above the window: one test per 8
                const uint32_t a = min(min(x[j].x & 0xffffu, x[j].x >> 16), min(x[j].y & 0xffffu, x[j].y >> 16));
                const uint32_t b = min(min(x[j].z & 0xffffu, x[j].z >> 16), min(x[j].w & 0xffffu, x[j].w >> 16));
                if (min(a, b) - base >= win && min(a, b) >= base) continue;
                ss_count(x[j].x, base, win, hist);
                ss_count(x[j].y, base, win, hist);
                ss_count(x[j].z, base, win, hist);
                ss_count(x[j].w, base, win, hist);
            }
        } else {
            for (uint32_t i = tid; i < nv; i += kSsThreads) {
                const uint4 y = v[i];
                ss_count(y.x, base, win, hist);
                ss_count(y.y, base, win, hist);
                ss_count(y.z, base, win, hist);
                ss_count(y.w, base, win, hist);
            }
        }
        __syncthreads();
        if (tid < 64) {  // first bin whose running count reaches the target
            const uint32_t seg = (win + 63u) / 64u, b0 = lane * seg, b1 = min(b0 + seg, win);
            uint32_t sum = 0;
            for (uint32_t i = b0; i < b1; ++i) sum += hist[i];
            uint32_t incl = sum;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t t = __shfl_up(incl, off);
                if ((int)lane >= off) incl += t;
            }
            const uint32_t cum0 = s_cum;
            const uint64_t m = __ballot(cum0 + incl >= target);
            if (m) {
                const uint32_t first = __ffsll((long long)m) - 1;
                if (lane == first) {
                    uint32_t cum = cum0 + incl - sum;
                    for (uint32_t i = b0; i < b1; ++i) {
                        cum += hist[i];
                        if (cum >= target) {
                            s_T = base + i;
                            break;
                        }
                    }
                }
            } else if (lane == 63) {
                s_cum = cum0 + incl;
            }
        }
        __syncthreads();
        if (s_T != ~0u || base + win > D) break;
        base += win;
        win = min(win * 2u, kMaxWin);
        __syncthreads();
    }
    if (tid == 0) thr[q] = min(s_T, D);
}

// k_sample_prep: k_qprep and k_sample_dense in ONE launch (the large-batch
// stage 1 with the dense sample; round 5).  k_qprep (one 64-thread block per
// query slot, ~4.6 us) only fed k_sample_dense, whose every block then copied the
// whole group's 96 KiB of FP4 query fragments into LDS to run one sub-tile per
// wave at the 1.25M-row shard: two launches of mostly latency.  Here block
// f = 8 s + qt (32 slices s x 8 query tiles qt of one 256-query group; the 32
// blocks of a tile share blockIdx % 8) packs its tile's 32 queries itself (a
// ballot per 64 dims, as k_qprep: Msb0 words, pad bits 0), keeps the tile's 2*W4
// FP4 A fragments in REGISTERS (no LDS reads in the MFMA stream), and computes
// the dense sample of its slice for those 32 queries: per wave a contiguous run of
// sample sub-tiles, two accumulator chains at a time (acc = -|q| + dot =
// -Hamming), then the minimum of every 16 rows per query through the wave's LDS
// transpose -> dsm[q][S/16], the layout k_sample_select reads (the same values
// as k_sample_dense's, so the same thresholds).  The slice-0 block of each tile
// also writes what the scan and the select read: the query words [B][4 W4], |q|
// per slot and the tile's fragments in the scan's layout (slots past B: zero
// words); and the blocks zero the stage-1 flags / counts (k_qprep's duty).
#ifdef GVDB_PREP_CLK
__device__ unsigned long long g_prep_clk[256 * 8][5];  // timing study (variant builds): per wave phase clocks
#define PREP_CLK(i)                                                                                  \
    do {                                                                                             \
        if (lane == 0) g_prep_clk[blockIdx.x * 8u + wv][i] = __builtin_amdgcn_s_memrealtime();      \
    } while (0)
extern "C" int gvdb_debug_prep_clock(unsigned long long* out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prep_clk), sizeof(g_prep_clk)) == hipSuccess ? 0 : -2;
}
#else
#define PREP_CLK(i) \
    do {            \
    } while (0)
#endif
template <int W4>
__global__ __launch_bounds__(kMx5Threads, 1) void k_sample_prep(
    const float* __restrict__ qf, uint32_t D, float qthr, uint32_t B, uint32_t* __restrict__ qwords,
    v4i_t* __restrict__ qfrag, uint32_t* __restrict__ qpc, uint32_t* __restrict__ zero, uint32_t nzero,
    const uint4* __restrict__ codes, uint64_t cap, uint32_t N, uint32_t stride, uint32_t nsub, uint32_t pw,
    uint16_t* __restrict__ dsm, uint32_t S) {
    constexpr int KW = 4 * W4, KS = KW / 2, QT = 8, NW = kMx5Threads / 64;
    __shared__ uint32_t qw_lds[32][KW + 1];
    __shared__ uint32_t pc_lds[32];
    __shared__ __attribute__((aligned(16))) uint16_t tr_lds[NW][32 * 32];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t f = blockIdx.x, qt = f % QT, sl = f / QT, h = lane >> 5;
    PREP_CLK(0);
    for (uint32_t i = f * kMx5Threads + tid; i < nzero; i += gridDim.x * kMx5Threads) zero[i] = 0u;
    // the slice's sample sub-tiles: wave (sl, wv) takes the contiguous run [wg * pw, +pw), two
    // at a time (two accumulator chains); the codes of the next pair load under the current
    // pair's MFMAs, the first pair's under the query packing
    const uint32_t wg = sl * NW + wv;
    const uint32_t j0 = min(wg * pw, nsub), j1 = min(j0 + pw, nsub);
    auto rown = [&](uint32_t j) { const uint32_t s0 = j * 32u; return (s0 >> 12) * stride + (s0 & 4095u) + (lane & 31u); };
    uint2 cc[2][2][W4];  // [buffer][chain][plane]
    auto load_pair = [&](uint32_t j, uint2 (&c)[2][W4]) __attribute__((always_inline)) {
        const uint32_t n0 = min(rown(j), N - 1u), n1 = min(rown(j + 1 < j1 ? j + 1 : j), N - 1u);
#pragma unroll
        for (int p = 0; p < W4; ++p) {
            c[0][p] = ((const uint2*)(codes + (uint64_t)p * cap + n0))[h];
            c[1][p] = ((const uint2*)(codes + (uint64_t)p * cap + n1))[h];
        }
    };
    const bool live_tile = qt * 32u < B;
    // 1. the tile's 32 queries: wave wv packs queries 4 wv .. 4 wv + 3, every load in flight
    {
        float v[4][KW / 2];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t q = qt * 32u + wv * 4u + (uint32_t)u;
#pragma unroll
            for (int c = 0; c < KW / 2; ++c) {
                const uint32_t d = 64u * (uint32_t)c + lane;
                v[u][c] = q < B && d < D ? qf[(uint64_t)q * D + d] : 0.0f;
            }
        }
        // the first pair's codes: issued after the query loads, so the ballots wait only for
        // those (vector loads complete in order)
        load_pair(j0, cc[0]);  // unconditional (clamped rows): a branch here made the ballots wait for it
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t x = wv * 4u + (uint32_t)u, q = qt * 32u + x;
#pragma unroll
            for (int c = 0; c < KW / 2; ++c) {
                const uint32_t d = 64u * (uint32_t)c + lane;
                const uint64_t m = __ballot(q < B && d < D && v[u][c] > qthr);
                if (lane == 0) {
                    qw_lds[x][2 * c] = msb0_word((uint32_t)m);
                    qw_lds[x][2 * c + 1] = msb0_word((uint32_t)(m >> 32));
                }
            }
        }
    }
    __syncthreads();
    PREP_CLK(1);
    if (tid < 32) {
        uint32_t pc = 0;
#pragma unroll
        for (int i = 0; i < KW; ++i) pc += __popc(qw_lds[tid][i]);
        pc_lds[tid] = pc;  // 0 past B (zero words)
    }
    __syncthreads();
    if (sl == 0) {  // the scan's and the select's operands for this tile
        for (uint32_t i = tid; i < 32u * KW; i += kMx5Threads) {
            const uint32_t x = i / KW, w = i % KW, q = qt * 32u + x;
            if (q < B) qwords[(uint64_t)q * KW + w] = qw_lds[x][w];
        }
        if (tid < 32) qpc[qt * 32u + tid] = pc_lds[tid];
        for (uint32_t i = tid; i < (uint32_t)KS * 64u; i += kMx5Threads) {
            const uint32_t sk = i >> 6, l = i & 63u;
            const uint32_t wi = 4u * (sk >> 1) + 2u * (l >> 5) + (sk & 1u);
            qfrag[(sk * QT + qt) * 64u + l] = fp4_query_pm(qw_lds[l & 31u][wi]);
        }
    }
    // this lane's A fragments (query l & 31, k-half h) and the accumulator seeds -|q|
    v4i_t A[KS];
#pragma unroll
    for (int sk = 0; sk < KS; ++sk) A[sk] = fp4_query_pm(qw_lds[lane & 31u][4 * (sk >> 1) + 2 * (int)h + (sk & 1)]);
    float seed[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const uint32_t x = 8u * (uint32_t)(r >> 2) + 4u * h + (uint32_t)(r & 3);
        seed[r] = qt * 32u + x < B ? -(float)pc_lds[x] : -1.0e6f;
    }
    PREP_CLK(2);
    if (!live_tile) return;  // a tile past B: fragments written, nothing to sample
    // 2. the sample
    uint16_t* tw = tr_lds[wv];
    const int scale1 = 0x7f7f7f7f;
    auto epi = [&](const v16f_t& acc, uint32_t j) __attribute__((always_inline)) {
        // rows past N (an unsampled small shard's last chunk) read as 0xffff
        const uint32_t n = rown(j);
        const float lim = n < N ? 65535.0f : -1.0f;
        const uint32_t jj = lane & 31u;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const uint32_t qo = 8u * (uint32_t)(r >> 2) + 4u * h + (uint32_t)(r & 3);
            const float dv = -acc[r];
            tw[qo * 32u + jj] = lim < 0.0f ? (uint16_t)0xffffu : (uint16_t)min(dv, lim);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // lane L: query L / 2 of the tile, rows 16 (L % 2) .. +15 -> their minimum
        const uint32_t qo = lane >> 1, rh = lane & 1u;
        const uint4 v0 = *(const uint4*)(tw + qo * 32u + rh * 16u);
        const uint4 v1 = *(const uint4*)(tw + qo * 32u + rh * 16u + 8u);
        uint32_t mn = 0xffffu;
        const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) mn = min(mn, min(w[e] & 0xffffu, w[e] >> 16));
        const uint32_t qg = qt * 32u + qo;
        if (qg < B) dsm[(uint64_t)qg * (S >> 4) + 2u * j + rh] = (uint16_t)mn;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    };
    auto pair = [&](uint32_t j, const uint2 (&cb)[2][W4]) __attribute__((always_inline)) {
        const bool two = j + 1 < j1;
        const uint2(&c0)[W4] = cb[0];
        const uint2(&c1)[W4] = cb[1];
        v16f_t acc[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            acc[0][r] = seed[r];
            acc[1][r] = seed[r];
        }
#pragma unroll
        for (int sk = 0; sk < KS; ++sk) {
            const v4i_t b0 = fp4_row01((sk & 1) ? c0[sk >> 1].y : c0[sk >> 1].x);
            const v4i_t b1 = fp4_row01((sk & 1) ? c1[sk >> 1].y : c1[sk >> 1].x);
            mfma_fp4_acc_nop(acc[0], A[sk], b0, scale1);
            mfma_fp4_acc_nop(acc[1], A[sk], b1, scale1);
        }
        mfma_fp4_drain_acc(acc);
        epi(acc[0], j);
        if (two) epi(acc[1], j + 1);
    };
    // two inlined copies (one per code buffer)
    for (uint32_t j = j0; j < j1; j += 4) {
        if (j + 2 < j1) load_pair(j + 2, cc[1]);
        pair(j, cc[0]);
        if (j + 2 >= j1) break;
        if (j + 4 < j1) load_pair(j + 4, cc[0]);
        pair(j + 2, cc[1]);
    }
    PREP_CLK(3);
}

template <int W4>
static void launch_sample_prep_t(const Stage1Args& a, hipStream_t s) {
    const uint32_t S = a.sample_chunks * 4096u;
    const uint32_t nsub = S / 32u;
    constexpr uint32_t kBlocks = 32u * 8u, kWaves = kBlocks / 8u * (kMx5Threads / 64u);  // per query tile: 256 waves
    const uint32_t pw = (nsub + kWaves - 1u) / kWaves;
    constexpr uint64_t kPer = 8u * (2u * W4) * 64u;
    for (uint32_t g = 0; g < a.B; g += 256) {
        const uint32_t bg = min(256u, a.B - g);
        hipLaunchKernelGGL((k_sample_prep<W4>), dim3(kBlocks), dim3(kMx5Threads), 0, s, a.qf32 + (uint64_t)g * a.D,
                           a.D, a.qthr, bg, (uint32_t*)a.qcodes + (uint64_t)g * 4u * W4,
                           (v4i_t*)a.qfrag + (g / 256u) * kPer, a.qpc + g, g == 0 ? a.zero : nullptr,
                           g == 0 ? a.nzero : 0u, a.codes, a.cap, a.N, a.sample_stride, nsub, pw,
                           a.smp + (uint64_t)g * (S / 16u), S);
    }
    hipLaunchKernelGGL(k_sample_select, dim3(a.B), dim3(kSsThreads), 0, s, a.smp, S / 16u, a.D, a.target, a.thr);
}

template <int W4>
static void launch_sample_dense_t(const Stage1Args& a, hipStream_t s) {
    const uint32_t S = a.sample_chunks * 4096u;
    const uint32_t nsub = S / 32u;
    const uint32_t wpb = kMx5Threads / 64;
    const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>(cu_count(), (nsub + wpb - 1) / wpb));
    constexpr uint64_t kPer = 8u * (2u * W4) * 64u;
    for (uint32_t g = 0; g < a.B; g += 256) {
        const uint32_t bg = min(256u, a.B - g);
        hipLaunchKernelGGL((k_sample_dense<W4>), dim3(grid), dim3(kMx5Threads), 0, s, a.codes, a.cap, a.N,
                           a.sample_stride, nsub, (const v4i_t*)a.qfrag + (g / 256u) * kPer, a.qpc + g, bg,
                           a.smp + (uint64_t)g * (S / 16u), S);
    }
    hipLaunchKernelGGL(k_sample_select, dim3(a.B), dim3(kSsThreads), 0, s, a.smp, S / 16u, a.D, a.target, a.thr);
}

template <int W4>
static void launch_hist_t(const Stage1Args& a, hipStream_t s) {
    // GVDB_HIST_LDS_WORDS: LDS histogram words per block (timing knob; default 12288)
    static const uint32_t words = [] {
        const char* e = getenv("GVDB_HIST_LDS_WORDS");
        const long v = e ? atol(e) : 0;
        return v >= 1024 && v <= 36864 ? (uint32_t)v : 12288u;
    }();
    uint32_t QT = words / (a.D + 1u);
    if (!getenv("GVDB_HIST_LDS_WORDS")) {
        // about three blocks per CU: fewer queries per block when the sample has
        // few chunks (1.25M-row shard, 16 chunks: 6 queries per block, 0.282 ->
        // 0.260 ms per batch-256 step; 10M: 13, unchanged -- profiles/r02)
        int dev = 0, cus = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const uint32_t want = (uint32_t)(((uint64_t)a.B * a.sample_chunks + 3ull * cus - 1) / (3ull * cus));
        QT = std::min(QT, std::max(want, 4u));
    }
    if (QT < 1) QT = 1;
    if (QT > 32) QT = 32;
    if (QT > a.B) QT = a.B;
    const size_t lds = (((size_t)QT * (a.D + 1u) + 3u) & ~(size_t)3) * 4u + (size_t)QT * W4 * 16u;
    hipLaunchKernelGGL((k_sample_hist<W4>), dim3(a.sample_chunks, (a.B + QT - 1) / QT), dim3(256), lds, s, a.codes,
                       a.cap, a.N, a.D, a.sample_stride, a.qcodes, a.B, QT, a.hist);
}

static bool getenv_flag_eq(const char* name, const char* v) {  // read per launch (tests switch it)
    const char* e = getenv(name);
    return e && strcmp(e, v) == 0;
}

size_t stage1_plan(Stage1Args& a) {
    const uint32_t W4 = code_w4(a.D);
    const uint64_t S = (uint64_t)a.sample_chunks * 4096u;
    const bool big = a.use_mfma == 1 && a.B >= kMfmaMinB && mfma_scan_supported(W4);
    a.mfma_scan = big;
    a.sample_mode = kSampleValu;
    // wide codes (k_scan_mx4): the FP4 sample when the scan is the FP4 one (GVDB_SAMPLE=valu: the VALU form)
    if (a.use_mfma == 1 && a.B >= kMfmaMinB && mx4_scan_supported(W4) && !getenv_flag_eq("GVDB_SAMPLE", "valu") &&
        (uint64_t)a.B * a.sample_chunks * 4096u * 2u <= (1ull << 30))
        a.sample_mode = kSampleWide;
    // GVDB_SAMPLE=valu / =mx / =dense force a sample form (tests, A/B).  Default
    // for large batches: the dense FP4 sample (any shard size: for N <= kExactN
    // the "sample" is the whole shard and T is the exact R-th distance); the
    // FP4 histogram only when the dense block would exceed 1 GiB.
    if (big && !getenv_flag_eq("GVDB_SAMPLE", "valu")) {
        const bool sampled = a.target < S / 2u && a.N > S;
        // the dense sample keeps one minimum per 16 rows: S/16 values, so it can
        // only reach a target well below that (at R/N above ~1/64 -- the
        // reference's default ratio 0.1 -- it would leave thr = D and every row
        // would be emitted); such depths take the FP4 histogram / VALU form
        const bool dense_fits = (uint64_t)a.B * (S / 16u) * 2u <= (1ull << 30);
        const bool dense_reach = (uint64_t)a.target * 4u <= S / 16u;
        if (getenv_flag_eq("GVDB_SAMPLE", "mx")) {
            if (sampled) a.sample_mode = kSampleMxHist;
        } else if (dense_fits && (dense_reach || getenv_flag_eq("GVDB_SAMPLE", "dense"))) {
            a.sample_mode = kSampleDense;
        } else if (sampled) {
            a.sample_mode = kSampleMxHist;
        }
    }
    // the reference's default depth (R = 0.1 N): at R/N >= 1/64 the threshold scan would emit
    // a large share of all (row, query) pairs through its hit path; write every distance
    // instead (one f16 per pair, 256 queries at a time) and select from the dense block
    a.dense_sel = a.big_select && a.use_mfma == 1 && mfma_scan_supported(W4) && (uint64_t)a.R * 64u >= a.N &&
                  !getenv_flag_eq("GVDB_DENSE_SEL", "0");
    if (a.dense_sel) {
        a.mfma_scan = true;  // the FP4 scan at any batch size (padded query slots)
        a.sample_mode = kSampleValu;
        a.dense_np = (a.N + 31u) & ~31u;
    }
    size_t bytes = 0;
    if (a.mfma_scan) {
        const uint64_t ng = (a.B + 255u) / 256u;
        bytes += ng * (8u * 2u * W4 * 64u * 16u + 256u * 4u);
    }
    if (a.sample_mode == kSampleDense) bytes += (size_t)a.B * (S / 16u) * 2u + 256u;
    if (a.sample_mode == kSampleWide) bytes += (size_t)a.B * S * 2u + 256u;
    if (a.dense_sel && !a.dense_keep) bytes += (size_t)std::min<uint32_t>(a.B, 256u) * a.dense_np * 2u + 256u;
    return bytes;
}

// GVDB_PREP=0: k_qprep + k_sample_dense instead of the fused k_sample_prep (A/B, tests)
static bool prep_enabled() {
    const char* e = getenv("GVDB_PREP");
    return !(e && e[0] == '0');
}

hipError_t launch_stage1_fast(const Stage1Args& a, hipStream_t s) {
    const uint32_t W4 = code_w4(a.D);
    // a tier gate is carried by the dense FP4 form's kernels only (the deep fallback)
    if (a.gate && !(a.dense_sel && a.mfma_scan)) return hipErrorInvalidValue;
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    // the query packing fused into the dense sample (one launch instead of two)
    const bool prep = a.mfma_scan && !a.dense_sel && a.sample_mode == kSampleDense && a.qf32 && prep_enabled();
    if (a.mfma_scan && !prep) {
        switch (W4) {
            case 2: launch_qfrag_t<2>(a, s); break;
            case 3: launch_qfrag_t<3>(a, s); break;
            case 4: launch_qfrag_t<4>(a, s); break;
            default: launch_qfrag_t<6>(a, s); break;
        }
        GVDB_LAUNCH_CHECK();
    }
    if (a.dense_sel) {
        // no threshold: every distance is written and selected exactly (the scan below)
        hipError_t e = hipSuccess;
        if (a.dense8 && (e = launch_dense_base(a, s)) != hipSuccess) return e;  // the byte windows
        if (a.ev) (void)hipEventRecord(a.ev[1], s);
        switch (W4) {
            case 2: e = launch_scan_mx7_t<2>(a, s); break;
            case 3: e = launch_scan_mx7_t<3>(a, s); break;
            case 4: e = launch_scan_mx7_t<4>(a, s); break;
            default: e = launch_scan_mx7_t<6>(a, s); break;
        }
        if (e != hipSuccess) return e;
        if (a.ev) {
            (void)hipEventRecord(a.ev[2], s);
            (void)hipEventRecord(a.ev[3], s);
        }
        return hipSuccess;
    }
    if (prep) {
        switch (W4) {
            case 2: launch_sample_prep_t<2>(a, s); break;
            case 3: launch_sample_prep_t<3>(a, s); break;
            case 4: launch_sample_prep_t<4>(a, s); break;
            default: launch_sample_prep_t<6>(a, s); break;
        }
    } else if (a.sample_mode == kSampleDense) {
        switch (W4) {
            case 2: launch_sample_dense_t<2>(a, s); break;
            case 3: launch_sample_dense_t<3>(a, s); break;
            case 4: launch_sample_dense_t<4>(a, s); break;
            default: launch_sample_dense_t<6>(a, s); break;
        }
    } else if (a.sample_mode == kSampleWide) {
        switch (W4) {
            case 8: launch_sample_wide_t<8, 4>(a, s); break;
            case 12: launch_sample_wide_t<12, 4>(a, s); break;
            case 16: launch_sample_wide_t<16, 3>(a, s); break;
            case 24: launch_sample_wide_t<24, 2>(a, s); break;
            default: launch_sample_wide_t<32, 1>(a, s); break;
        }
    } else if (a.sample_mode == kSampleMxHist) {
        switch (W4) {
            case 2: launch_sample_mx_t<2>(a, s); break;
            case 3: launch_sample_mx_t<3>(a, s); break;
            case 4: launch_sample_mx_t<4>(a, s); break;
            default: launch_sample_mx_t<6>(a, s); break;
        }
    } else switch (W4) {
#define GVDB_CASE(w, cpl)            \
    case w:                          \
        launch_hist_t<w>(a, s);      \
        break;
        GVDB_CASE(1, 8)
        GVDB_CASE(2, 8)
        GVDB_CASE(3, 8)
        GVDB_CASE(4, 4)
        GVDB_CASE(6, 4)
        GVDB_CASE(8, 2)
        GVDB_CASE(12, 2)
        GVDB_CASE(16, 1)
        GVDB_CASE(24, 1)
        GVDB_CASE(32, 1)
#undef GVDB_CASE
        default:
            hipLaunchKernelGGL(k_sample_hist_generic, dim3(a.sample_chunks, a.B), dim3(256), 0, s, a.codes, a.cap,
                               a.N, a.D, W4, a.sample_stride, a.qcodes, a.B, a.hist);
    }
    GVDB_LAUNCH_CHECK();
    if (a.sample_mode != kSampleDense && a.sample_mode != kSampleWide) {
        hipLaunchKernelGGL(k_threshold, dim3((a.B + 3) / 4), dim3(256), 0, s, a.hist, a.B, a.D, a.target, a.thr);
        GVDB_LAUNCH_CHECK();
    }
    if (a.ev) (void)hipEventRecord(a.ev[1], s);
    const bool mfma = a.use_mfma && a.B >= kMfmaMinB && mfma_scan_supported(W4);
    const bool wide = a.use_mfma == 1 && a.B >= kMfmaMinB && mx4_scan_supported(W4);
    if (wide) {  // FP4 MFMA for wide codes: query tiles per launch bounded by LDS
        switch (W4) {
            case 8: launch_scan_mx4_t<8, 4, 4>(a, s); break;
            case 12: launch_scan_mx4_t<12, 6, 4>(a, s); break;
            case 16: launch_scan_mx4_t<16, 8, 3>(a, s); break;
            case 24: launch_scan_mx4_t<24, GVDB_MX4_CH24, 2>(a, s); break;
            default: launch_scan_mx4_t<32, 8, 1>(a, s); break;
        }
    } else if (mfma) {  // FP4 block-scaled MFMA, {0,1} x {+-1} operands (default for large batches)
        hipError_t e = hipSuccess;
        switch (W4) {
            case 2: e = launch_scan_mx7_t<2>(a, s); break;
            case 3: e = launch_scan_mx7_t<3>(a, s); break;
            case 4: e = launch_scan_mx7_t<4>(a, s); break;
            default: e = launch_scan_mx7_t<6>(a, s); break;
        }
        if (e != hipSuccess) return e;
    } else switch (W4) {
#define GVDB_CASE(w, cpl)             \
    case w:                           \
        launch_scan_t<w, cpl>(a, s);  \
        break;
        GVDB_CASE(1, 8)
        GVDB_CASE(2, 8)
        GVDB_CASE(3, 8)
        GVDB_CASE(4, 4)
        GVDB_CASE(6, 4)
        GVDB_CASE(8, 2)
        GVDB_CASE(12, 2)
        GVDB_CASE(16, 1)
        GVDB_CASE(24, 1)
        GVDB_CASE(32, 1)
#undef GVDB_CASE
        default:
            hipLaunchKernelGGL(k_scan_generic, dim3((a.N + 255) / 256), dim3(256), 0, s, a.codes, a.cap, a.N, W4,
                               a.qcodes, a.thr, a.B, a.counts, a.buf, a.bufcap);
    }
    GVDB_LAUNCH_CHECK();
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    if (a.big_select) {
        hipError_t e = launch_select_big(a, s);
        if (e != hipSuccess) return e;
    } else {
        const size_t lds = (size_t)kSelectLdsCap * 8u + (size_t)((a.D + 4u) & ~3u) * 4u + 2048u * 4u;
        hipLaunchKernelGGL(k_select, dim3(a.B), dim3(256), lds, s, a.counts, a.buf, a.bufcap, a.D, a.R, a.codes,
                           a.cap, a.N, W4, a.qcodes, a.fail, a.any_fail, a.s1_rows, a.s1_dist, a.force_rescan,
                           a.keys_out, a.keys_stride);
        GVDB_LAUNCH_CHECK();
    }
    if (a.ev) (void)hipEventRecord(a.ev[3], s);
    return hipSuccess;
}

// ---- exact slow path (one query) --------------------------------------------------
__global__ void k_dist_all(const uint4* __restrict__ codes, uint64_t cap, uint32_t N, uint32_t W4,
                           const uint4* __restrict__ qc, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint64_t n = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    uint32_t d = 0;
    for (uint32_t w = 0; w < W4; ++w) d = ham4(codes[(uint64_t)w * cap + n], qc[w], d);
    keys[n] = d;
    vals[n] = (uint32_t)n;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static size_t cub_pairs_u32_bytes(uint32_t N) {
    size_t bytes = 0;
    hipcub::DoubleBuffer<uint32_t> k(nullptr, nullptr), v(nullptr, nullptr);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, k, v, (int)N, 0, 32);
    return bytes;
}

size_t stage1_slow_bytes(uint32_t N) { return 4 * align256((size_t)N * 4) + align256(cub_pairs_u32_bytes(N)); }

hipError_t launch_stage1_slow(const uint4* codes, uint64_t cap, uint32_t N, uint32_t D, const uint4* qcode, uint32_t R,
                              uint32_t* out_rows, uint32_t* out_dist, void* tmp, size_t tmp_bytes, hipStream_t s) {
    char* p = (char*)tmp;
    const size_t a = align256((size_t)N * 4);
    uint32_t* k0 = (uint32_t*)p;
    uint32_t* k1 = (uint32_t*)(p + a);
    uint32_t* v0 = (uint32_t*)(p + 2 * a);
    uint32_t* v1 = (uint32_t*)(p + 3 * a);
    void* ctmp = p + 4 * a;
    size_t cbytes = tmp_bytes - 4 * a;
    hipLaunchKernelGGL(k_dist_all, dim3((N + 255) / 256), dim3(256), 0, s, codes, cap, N, code_w4(D), qcode, k0, v0);
    GVDB_LAUNCH_CHECK();
    int end_bit = 1;
    while ((1u << end_bit) <= D) ++end_bit;
    hipcub::DoubleBuffer<uint32_t> kb(k0, k1), vb(v0, v1);
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(ctmp, cbytes, kb, vb, (int)N, 0, end_bit, s);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(out_rows, vb.Current(), (size_t)R * 4, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    return hipMemcpyAsync(out_dist, kb.Current(), (size_t)R * 4, hipMemcpyDeviceToDevice, s);
}

__global__ void k_iota_rows(uint32_t* rows, uint32_t B, uint32_t R) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)B * R) return;
    rows[t] = (uint32_t)(t % R);
}

hipError_t launch_iota_rows(uint32_t* rows, uint32_t B, uint32_t R, hipStream_t s) {
    const uint64_t total = (uint64_t)B * R;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_iota_rows, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, rows, B, R);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ============================================================================
// K3: exact rerank.  A work item = 64 consecutive candidates of one query; a
// block of 512 threads takes items from a compact list (grid-stride over the
// prefix sum of the per-query counts, so no block is launched for an empty
// slot).  All 8 waves stream the item's rows through a double-buffered LDS
// tile ([64 rows][128 dims], 16-B loads, one 512-B row segment per 32 lanes;
// the next chunk's loads are in flight while the current one is folded); wave
// 0 folds: lane r owns candidate r and accumulates q_j*x_j (or (q_j-x_j)^2)
// left to right, and every lane also folds q_j*q_j for the query norm -- the
// reference's exact sequential order, so cosine / L2 are bit-identical to
// cosine_similarity_manual / VectorPoint::distance.  Row stride 132 floats:
// conflict-free ds_read_b128 / ds_write_b128.  67 KiB of LDS: two blocks per
// CU.
// ============================================================================
constexpr int kRrRows = 64;
constexpr int kRrCh = 128;
constexpr int kRrLd = kRrCh + 4;
constexpr int kRrThreads = 512;
constexpr int kRrPer = kRrRows * (kRrCh / 4) / kRrThreads;  // float4 per thread per chunk (4)
constexpr uint32_t kRrMaxB = 1024;                            // queries per launch (prefix in LDS)

__device__ __forceinline__ float4 load4_guarded(const float* __restrict__ src, uint64_t base, uint64_t j, uint64_t len,
                                               bool vec4) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (base == ~0ull) return v;
    if (vec4 && j + 3 < len) return *(const float4*)(src + base + j);
    if (j + 0 < len) v.x = src[base + j + 0];
    if (j + 1 < len) v.y = src[base + j + 1];
    if (j + 2 < len) v.z = src[base + j + 2];
    if (j + 3 < len) v.w = src[base + j + 3];
    return v;
}

__global__ __launch_bounds__(kRrThreads, 2) void k_rerank(const float* __restrict__ rows, uint64_t clen,
                                                          const float* __restrict__ norms, const float* __restrict__ q,
                                                          uint64_t qlen, const uint32_t* __restrict__ s1_rows,
                                                          uint32_t B, uint32_t R, const uint32_t* __restrict__ counts,
                                                          int kind, float* __restrict__ scores,
                                                          const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ __attribute__((aligned(16))) float tiles[2][kRrRows * kRrLd];
    __shared__ __attribute__((aligned(16))) float qs[2][kRrCh];
    __shared__ uint64_t bases[kRrRows];
    __shared__ uint32_t pre[kRrMaxB + 1];  // items before query i
    const uint32_t tid = threadIdx.x;
    // exclusive prefix of per-query item counts (B <= kRrMaxB), block-wide
    {
        const uint32_t per = (B + kRrThreads - 1) / kRrThreads;
        const uint32_t b0 = tid * per;
        uint32_t loc = 0;
        for (uint32_t i = 0; i < per && b0 + i < B; ++i) {
            const uint32_t c = counts ? min(counts[b0 + i], R) : R;
            loc += (c + kRrRows - 1) / kRrRows;
        }
        // inclusive scan of the per-thread sums through LDS (Hillis-Steele)
        __shared__ uint32_t part[kRrThreads];
        part[tid] = loc;
        __syncthreads();
        for (uint32_t o = 1; o < kRrThreads; o <<= 1) {
            const uint32_t v = tid >= o ? part[tid - o] : 0u;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        uint32_t run = part[tid] - loc;
        for (uint32_t i = 0; i < per && b0 + i < B; ++i) {
            pre[b0 + i] = run;
            const uint32_t c = counts ? min(counts[b0 + i], R) : R;
            run += (c + kRrRows - 1) / kRrRows;
        }
        if (tid == kRrThreads - 1) pre[B] = part[tid];
        __syncthreads();
    }
    const uint32_t items = pre[B];
    const uint64_t len = qlen < clen ? qlen : clen;  // zip() truncates
    const bool vec4 = (clen & 3u) == 0;
    const uint32_t nch = (uint32_t)((len + kRrCh - 1) / kRrCh);
    for (uint32_t item = blockIdx.x; item < items; item += gridDim.x) {
        // item -> (query qi, first candidate r0): last qi with pre[qi] <= item
        uint32_t lo = 0, hi = B;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= item) lo = mid; else hi = mid;
        }
        const uint32_t qi = lo;
        const uint32_t r0 = (item - pre[qi]) * kRrRows;
        const uint32_t Rq = counts ? min(counts[qi], R) : R;  // valid entries of this query's list
        if (tid < kRrRows) {
            const uint32_t r = r0 + tid;
            bases[tid] = r < Rq ? (uint64_t)s1_rows[(uint64_t)qi * R + r] * clen : ~0ull;
        }
        __syncthreads();
        const float* qv = q + (uint64_t)qi * qlen;
        const bool qvec4 = (qlen & 3u) == 0 && (((uintptr_t)qv) & 15u) == 0;
        float4 rg[kRrPer];
        float4 qg = make_float4(0.f, 0.f, 0.f, 0.f);
        auto load = [&](uint32_t c) {
#pragma unroll
            for (int it = 0; it < kRrPer; ++it) {
                const uint32_t idx = it * kRrThreads + tid;
                rg[it] = load4_guarded(rows, bases[idx >> 5], (uint64_t)c * kRrCh + 4u * (idx & 31u), len, vec4);
            }
            if (tid < kRrCh / 4) qg = load4_guarded(qv, 0, (uint64_t)c * kRrCh + 4u * tid, len, qvec4);
        };
        auto store = [&](uint32_t c) {
            float* t = tiles[c & 1];
#pragma unroll
            for (int it = 0; it < kRrPer; ++it) {
                const uint32_t idx = it * kRrThreads + tid;
                *(float4*)(t + (idx >> 5) * kRrLd + 4u * (idx & 31u)) = rg[it];
            }
            if (tid < kRrCh / 4) *(float4*)(qs[c & 1] + 4u * tid) = qg;
        };
        float acc = -0.0f, qq = -0.0f;
        if (nch) {
            load(0);
            store(0);
        }
        __syncthreads();
        for (uint32_t c = 0; c < nch; ++c) {
            if (c + 1 < nch) load(c + 1);
            if (tid < 64) {
                const float* tr = tiles[c & 1] + tid * kRrLd;
                const float* qc = qs[c & 1];
                const uint32_t m = (uint32_t)min((uint64_t)kRrCh, len - (uint64_t)c * kRrCh);
                if (kind == kScoreL2) {
                    for (uint32_t j = 0; j < m; ++j) {
                        const float d = qc[j] - tr[j];
                        acc = acc + d * d;
                    }
                } else if (m == kRrCh) {
#pragma unroll 8
                    for (int j = 0; j < kRrCh; j += 4) {
                        const float4 x = *(const float4*)(tr + j);
                        const float4 w = *(const float4*)(qc + j);
                        acc = acc + w.x * x.x;
                        acc = acc + w.y * x.y;
                        acc = acc + w.z * x.z;
                        acc = acc + w.w * x.w;
                        qq = qq + w.x * w.x;
                        qq = qq + w.y * w.y;
                        qq = qq + w.z * w.z;
                        qq = qq + w.w * w.w;
                    }
                } else {
                    for (uint32_t j = 0; j < m; ++j) {
                        acc = acc + qc[j] * tr[j];
                        qq = qq + qc[j] * qc[j];
                    }
                }
            }
            if (c + 1 < nch) store(c + 1);
            __syncthreads();
        }
        if (tid < 64) {
            const uint32_t r = r0 + tid;
            if (r < Rq) {
                float score;
                if (kind == kScoreL2) {
                    score = sqrtf(acc);
                } else {
                    for (uint64_t j = len; j < qlen; ++j) qq = qq + qv[j] * qv[j];  // query longer than rows
                    const float na = sqrtf(qq);
                    const float nb = norms[s1_rows[(uint64_t)qi * R + r]];
                    if (kind == kScoreCosine) {
                        score = (na == 0.0f || nb == 0.0f) ? 0.0f : acc / (na * nb);
                    } else {
                        score = (na == 0.0f || nb == 0.0f) ? __builtin_inff() : 1.0f - (acc / (na * nb));
                    }
                }
                scores[(uint64_t)qi * R + r] = score;
            }
        }
        __syncthreads();  // bases / tiles are rewritten by the next item
    }
}

// k_rerank2: the same exact re-scoring with NO block barrier in the loop.
// Every wave owns one work item (64 candidates of one query) at a time and a
// private LDS tile: per 32-dimension chunk it loads the 64 rows' slices with
// coalesced float4 loads (8 lanes per 128-B row slice) two chunks ahead into
// registers, writes the current one to its tile, and each lane then folds its
// own row in order (acc = acc + q_j * x_j, the reference's sequential f32 sum;
// the query is wave-uniform and comes through scalar loads).  Waves never wait
// for each other, so 16 waves per CU keep ~256 KiB of gathers in flight (the
// block-synchronous form above was latency-bound: waves parked 88 % of their
// cycles).
constexpr int kRr2Ch = 32;                  // dimensions per chunk
constexpr int kRr2Ld = kRr2Ch + 4;          // padded row stride (conflict-free b128)
constexpr int kRr2Threads = 256;            // 4 independent waves
constexpr int kRr2Per = 64 * kRr2Ch / 4 / 64;  // float4 per lane per chunk (8)

__global__ __launch_bounds__(kRr2Threads, 4) void k_rerank2(const float* __restrict__ rows, uint64_t clen,
                                                            const float* __restrict__ norms,
                                                            const float* __restrict__ q, uint64_t qlen,
                                                            const uint32_t* __restrict__ s1_rows, uint32_t B,
                                                            uint32_t R, const uint32_t* __restrict__ counts, int kind,
                                                            float* __restrict__ scores,
                                                            const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ __attribute__((aligned(16))) float tiles[kRr2Threads / 64][64 * kRr2Ld];
    __shared__ uint64_t bases[kRr2Threads / 64][64];
    __shared__ uint32_t pre[kRrMaxB + 1];  // work items before query i
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    {
        const uint32_t per = (B + kRr2Threads - 1) / kRr2Threads;
        const uint32_t b0 = tid * per;
        uint32_t loc = 0;
        for (uint32_t i = 0; i < per && b0 + i < B; ++i) {
            const uint32_t c = counts ? min(counts[b0 + i], R) : R;
            loc += (c + 63u) / 64u;
        }
        __shared__ uint32_t part[kRr2Threads];
        part[tid] = loc;
        __syncthreads();
        for (uint32_t o = 1; o < kRr2Threads; o <<= 1) {
            const uint32_t v = tid >= o ? part[tid - o] : 0u;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        uint32_t run = part[tid] - loc;
        for (uint32_t i = 0; i < per && b0 + i < B; ++i) {
            pre[b0 + i] = run;
            const uint32_t c = counts ? min(counts[b0 + i], R) : R;
            run += (c + 63u) / 64u;
        }
        if (tid == kRr2Threads - 1) pre[B] = part[tid];
        __syncthreads();
    }
    const uint32_t items = pre[B];
    const uint64_t len = qlen < clen ? qlen : clen;  // zip() truncates
    const bool vec4 = (clen & 3u) == 0;
    const uint32_t nch = (uint32_t)((len + kRr2Ch - 1) / kRr2Ch);
    float* tile = tiles[wv];
    uint64_t* wb = bases[wv];
    const uint32_t W = gridDim.x * (kRr2Threads / 64);
    for (uint32_t item = blockIdx.x * (kRr2Threads / 64) + wv; item < items; item += W) {
        uint32_t lo = 0, hi = B;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= item) lo = mid; else hi = mid;
        }
        const uint32_t qi = __builtin_amdgcn_readfirstlane(lo);
        const uint32_t r0 = (item - pre[qi]) * 64u;
        const uint32_t Rq = counts ? min(counts[qi], R) : R;
        const uint32_t r = r0 + lane;
        const uint32_t row = r < Rq ? s1_rows[(uint64_t)qi * R + r] : 0u;
        const float nbv = (r < Rq && kind != kScoreL2) ? norms[row] : 0.0f;
        wb[lane] = r < Rq ? (uint64_t)row * clen : ~0ull;  // read back by other lanes of this wave only
        __builtin_amdgcn_wave_barrier();
        const float* qv = q + (uint64_t)qi * qlen;
        // slice s of a chunk: lane L loads float4 (L & 7) of row 8 s + (L >> 3)
        float4 rg[2][kRr2Per];
        auto load = [&](uint32_t c, int sl) __attribute__((always_inline)) {
#pragma unroll
            for (int s = 0; s < kRr2Per; ++s) {
                const uint32_t rr = 8u * s + (lane >> 3);
                rg[sl][s] = load4_guarded(rows, wb[rr], (uint64_t)c * kRr2Ch + 4u * (lane & 7u), len, vec4);
            }
        };
        auto store = [&](int sl) __attribute__((always_inline)) {
#pragma unroll
            for (int s = 0; s < kRr2Per; ++s) {
                const uint32_t rr = 8u * s + (lane >> 3);
                *(float4*)(tile + rr * kRr2Ld + 4u * (lane & 7u)) = rg[sl][s];
            }
        };
        float acc = -0.0f, qq = -0.0f;
        if (nch) load(0, 0);
        if (nch > 1) load(1, 1);
        for (uint32_t c = 0; c < nch; ++c) {
            if (c & 1) store(1); else store(0);
            __builtin_amdgcn_wave_barrier();
            if (c + 2 < nch) {
                if (c & 1) load(c + 2, 1); else load(c + 2, 0);
            }
            const float* tr = tile + lane * kRr2Ld;
            const uint64_t j0 = (uint64_t)c * kRr2Ch;
            const uint32_t m = (uint32_t)min((uint64_t)kRr2Ch, len - j0);
            if (kind == kScoreL2) {
                for (uint32_t j = 0; j < m; ++j) {
                    const float d = qv[j0 + j] - tr[j];
                    acc = acc + d * d;
                }
            } else if (m == kRr2Ch) {
#pragma unroll
                for (int j = 0; j < kRr2Ch; j += 4) {
                    const float4 x = *(const float4*)(tr + j);
                    const float w0 = qv[j0 + j], w1 = qv[j0 + j + 1], w2 = qv[j0 + j + 2], w3 = qv[j0 + j + 3];
                    acc = acc + w0 * x.x;
                    acc = acc + w1 * x.y;
                    acc = acc + w2 * x.z;
                    acc = acc + w3 * x.w;
                    qq = qq + w0 * w0;
                    qq = qq + w1 * w1;
                    qq = qq + w2 * w2;
                    qq = qq + w3 * w3;
                }
            } else {
                for (uint32_t j = 0; j < m; ++j) {
                    const float w = qv[j0 + j];
                    acc = acc + w * tr[j];
                    qq = qq + w * w;
                }
            }
            __builtin_amdgcn_wave_barrier();  // the tile is rewritten next chunk
        }
        if (r < Rq) {
            float score;
            if (kind == kScoreL2) {
                score = sqrtf(acc);
            } else {
                for (uint64_t j = len; j < qlen; ++j) qq = qq + qv[j] * qv[j];  // query longer than rows
                const float na = sqrtf(qq);
                if (kind == kScoreCosine)
                    score = (na == 0.0f || nbv == 0.0f) ? 0.0f : acc / (na * nbv);
                else
                    score = (na == 0.0f || nbv == 0.0f) ? __builtin_inff() : 1.0f - (acc / (na * nbv));
            }
            scores[(uint64_t)qi * R + r] = score;
        }
        __builtin_amdgcn_wave_barrier();  // wb is rewritten by the next item
    }
}

// k_rerank_small: the exact re-scoring for SMALL candidate sets (batch-1 and
// few-query batches, D <= 1024).  The block-synchronous k_rerank walks 128-dim
// chunks with one chunk of loads in flight, so its time is a chain of gather
// latencies (34 us for one query's 100 rows at D = 768).  Here a block takes
// 16 candidates of one query, issues ALL their row loads at once into LDS
// (16 x D floats, <= 64 KiB) together with the query, and 16 lanes then fold
// their rows left to right (acc = acc + q_j*x_j, qq = qq + q_j*q_j: the same
// sequential order as k_rerank / cosine_similarity_manual, so scores are
// bit-identical).  One block per (query, 16-candidate slot); empty slots exit.
constexpr int kRsRows = 16;
constexpr int kRsThreads = 256;
constexpr uint32_t kRsMaxLen = 1024;
// Exact re-score of up to 16 rows (rows[r] for r < nr) by lanes 0..15: every
// row load in flight at once into LDS, then each lane folds its row left to
// right (acc = acc + q_j*x_j, qq = qq + q_j*q_j; the reference's order) with
// the next 8 float4 of its row prefetched from LDS while the current 8 fold.
__device__ __forceinline__ float rerank16(const float* __restrict__ rows, uint64_t clen, const float* __restrict__ norms,
                          const float* __restrict__ qv, uint64_t qlen, int kind, const uint32_t* rowid, uint32_t nr,
                          float4* tile4, float4* qs4, unsigned long long* t_staged = nullptr) {
    __shared__ uint64_t bases[kRsRows];
    const uint32_t tid = threadIdx.x;
    const uint64_t len = qlen < clen ? qlen : clen;
    const uint32_t L4 = (uint32_t)((len + 3) / 4), ld4 = L4 + 1;
    const bool vec4 = (clen & 3u) == 0;
    const bool qvec4 = (qlen & 3u) == 0 && (((uintptr_t)qv) & 15u) == 0;
    if (tid < kRsRows) bases[tid] = tid < nr ? (uint64_t)rowid[tid] * clen : ~0ull;
    __syncthreads();
    constexpr int kPer = kRsRows * (kRsMaxLen / 4) / kRsThreads;
    float4 v[kPer];
    const float4 qv4 = tid < L4 ? load4_guarded(qv, 0, 4ull * tid, len, qvec4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = tid + k * kRsThreads, r = i / L4, c = i - r * L4;
        v[k] = i < kRsRows * L4 ? load4_guarded(rows, bases[r], 4ull * c, len, vec4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t i = tid + k * kRsThreads, r = i / L4, c = i - r * L4;
        if (i < kRsRows * L4) tile4[r * ld4 + c] = v[k];
    }
    if (tid < L4) qs4[tid] = qv4;
    __syncthreads();
    if (t_staged) *t_staged = wall_clock64();
    if (kind != kScoreL2 && (len & 3u) == 0) {
        // one chain per lane: lanes 0..15 fold q_j*x_j of their row, lane 16
        // folds q_j*q_j (the query norm, same for every row); the products of
        // a float4 go out as packed multiplies, the sums stay sequential
        if (tid > kRsRows) return 0.0f;
        typedef float f2_t __attribute__((ext_vector_type(2)));
        const float4* src = tid < kRsRows ? tile4 + tid * ld4 : qs4;
        float acc = -0.0f;
#pragma unroll 8
        for (uint32_t c = 0; c < L4; ++c) {
            const float4 x = src[c];
            const float4 w = qs4[c];
            const f2_t p01 = (f2_t){w.x, w.y} * (f2_t){x.x, x.y};
            const f2_t p23 = (f2_t){w.z, w.w} * (f2_t){x.z, x.w};
            acc = acc + p01.x;
            acc = acc + p01.y;
            acc = acc + p23.x;
            acc = acc + p23.y;
        }
        float qq = __shfl(acc, kRsRows);
        if (tid >= nr) return 0.0f;
        for (uint64_t j = len; j < qlen; ++j) qq = qq + qv[j] * qv[j];  // query longer than rows
        const float na = sqrtf(qq);
        const float nb = norms[rowid[tid]];
        if (kind == kScoreCosine) return (na == 0.0f || nb == 0.0f) ? 0.0f : acc / (na * nb);
        return (na == 0.0f || nb == 0.0f) ? __builtin_inff() : 1.0f - (acc / (na * nb));
    }
    if (tid >= nr) return 0.0f;
    const float4* tr4 = tile4 + tid * ld4;
    float acc = -0.0f, qq = -0.0f;
    if (kind == kScoreL2) {
        const float* tr = (const float*)tr4;
        const float* qc = (const float*)qs4;
        for (uint32_t j = 0; j < len; ++j) {
            const float d = qc[j] - tr[j];
            acc = acc + d * d;
        }
    } else {
        const float* tr = (const float*)tr4;
        const float* qc = (const float*)qs4;
        for (uint32_t j = 0; j < len; ++j) {
            acc = acc + qc[j] * tr[j];
            qq = qq + qc[j] * qc[j];
        }
    }
    if (kind == kScoreL2) return sqrtf(acc);
    for (uint64_t j = len; j < qlen; ++j) qq = qq + qv[j] * qv[j];  // query longer than rows
    const float na = sqrtf(qq);
    const float nb = norms[rowid[tid]];
    if (kind == kScoreCosine) return (na == 0.0f || nb == 0.0f) ? 0.0f : acc / (na * nb);
    return (na == 0.0f || nb == 0.0f) ? __builtin_inff() : 1.0f - (acc / (na * nb));
}

__global__ __launch_bounds__(kRsThreads) void k_rerank_small(const float* __restrict__ rows, uint64_t clen,
                                                            const float* __restrict__ norms,
                                                            const float* __restrict__ q, uint64_t qlen,
                                                            const uint32_t* __restrict__ s1_rows, uint32_t B,
                                                            uint32_t R, const uint32_t* __restrict__ counts, int kind,
                                                            float* __restrict__ scores,
                                                            const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ float4 tile4[kRsRows * (kRsMaxLen / 4 + 1)];
    __shared__ float4 qs4[kRsMaxLen / 4];
    __shared__ uint32_t rowid[kRsRows];
    const uint32_t tid = threadIdx.x;
    const uint32_t ipq = (R + kRsRows - 1) / kRsRows;
    const uint32_t qi = blockIdx.x / ipq;
    const uint32_t r0 = (blockIdx.x % ipq) * kRsRows;
    if (qi >= B) return;
    const uint32_t Rq = counts ? min(counts[qi], R) : R;
    if (r0 >= Rq) return;  // block-uniform
    const uint32_t nr = min((uint32_t)kRsRows, Rq - r0);
    if (tid < kRsRows) rowid[tid] = tid < nr ? s1_rows[(uint64_t)qi * R + r0 + tid] : 0u;
    __syncthreads();
    const float sc = rerank16(rows, clen, norms, q + (uint64_t)qi * qlen, qlen, kind, rowid, nr, tile4, qs4);
    if (tid < nr) scores[(uint64_t)qi * R + r0 + tid] = sc;
}

// k_rerank_small over device-side counts (round 5): a fixed grid of blocks walks the
// (query, 16-candidate) items of the prefix of min(counts, R) / 16 -- every row load
// of an item in flight at once, instead of k_rerank2's 64-row wave items whose 24
// chunk gathers are serial (at ~900 candidates per query the items are fewer than
// the waves and the kernel is one item's latency: 130 us for 58K rows).
__global__ __launch_bounds__(kRsThreads) void k_rerank_small_items(
    const float* __restrict__ rows, uint64_t clen, const float* __restrict__ norms, const float* __restrict__ q,
    uint64_t qlen, const uint32_t* __restrict__ s1_rows, uint32_t B, uint32_t R, const uint32_t* __restrict__ counts,
    int kind, float* __restrict__ scores, const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ float4 tile4[kRsRows * (kRsMaxLen / 4 + 1)];
    __shared__ float4 qs4[kRsMaxLen / 4];
    __shared__ uint32_t rowid[kRsRows];
    __shared__ uint32_t pre[kRrMaxB + 1];  // items before query i
    __shared__ uint32_t part[kRsThreads];
    const uint32_t tid = threadIdx.x;
    {
        const uint32_t per = (B + kRsThreads - 1) / kRsThreads, b0 = tid * per;
        uint32_t loc = 0;
        for (uint32_t i = 0; i < per && b0 + i < B; ++i) loc += (min(counts[b0 + i], R) + kRsRows - 1) / kRsRows;
        part[tid] = loc;
        __syncthreads();
        for (uint32_t o = 1; o < kRsThreads; o <<= 1) {
            const uint32_t v = tid >= o ? part[tid - o] : 0u;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        uint32_t run = part[tid] - loc;
        for (uint32_t i = 0; i < per && b0 + i < B; ++i) {
            pre[b0 + i] = run;
            run += (min(counts[b0 + i], R) + kRsRows - 1) / kRsRows;
        }
        if (tid == kRsThreads - 1) pre[B] = part[tid];
        __syncthreads();
    }
    const uint32_t items = pre[B];
    for (uint32_t item = blockIdx.x; item < items; item += gridDim.x) {  // block-uniform
        uint32_t lo = 0, hi = B;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= item) lo = mid; else hi = mid;
        }
        const uint32_t qi = lo, r0 = (item - pre[qi]) * kRsRows;
        const uint32_t Rq = min(counts[qi], R), nr = min((uint32_t)kRsRows, Rq - r0);
        if (tid < kRsRows) rowid[tid] = tid < nr ? s1_rows[(uint64_t)qi * R + r0 + tid] : 0u;
        __syncthreads();
        const float sc = rerank16(rows, clen, norms, q + (uint64_t)qi * qlen, qlen, kind, rowid, nr, tile4, qs4);
        if (tid < nr) scores[(uint64_t)qi * R + r0 + tid] = sc;
        __syncthreads();  // rowid / the tiles are rewritten by the next item
    }
}

// k_rerank_dma (round 5): k_rerank2's wave items (64 candidates of one query, one row
// per lane, the reference's sequential fold) with the row gathers made asynchronous:
// each 32-dimension chunk of the 64 rows (8 KiB) is DMA'd straight into LDS by eight
// global_load_lds_dwordx4 (one 16-B piece per lane, any row address), kRdBufs - 1
// chunks ahead of the fold -- k_rerank2 held two chunks in registers and waited on each
// gather in turn (at ~850 candidates per query its 64-row items are fewer than the
// waves, and the kernel was one item's serial latency).  A lane writes float4 f of row r
// to slot f ^ ((r >> 1) & 7) of the row, so the fold's per-lane row reads hit 16 distinct
// bank groups per 16 lanes.  The query is DMA'd once per item.  Cosine / cosine
// distance, rows and queries of one length D % 32 == 0, D <= 1024, 16-B aligned.
constexpr int kRdThreads = 256;  // 4 independent waves
constexpr int kRdBufs = 4;       // chunk buffers per wave
constexpr uint32_t kRdMaxD = 1024;
__global__ __launch_bounds__(kRdThreads, 1) void k_rerank_dma(const float* __restrict__ rows, uint32_t D,
                                                             const float* __restrict__ norms,
                                                             const float* __restrict__ q,
                                                             const uint32_t* __restrict__ s1_rows, uint32_t B,
                                                             uint32_t R, const uint32_t* __restrict__ counts, int kind,
                                                             float* __restrict__ scores,
                                                             const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ __attribute__((aligned(16))) float4 tile[kRdThreads / 64][kRdBufs][64 * 8];
    __shared__ __attribute__((aligned(16))) float4 qs[kRdThreads / 64][kRdMaxD / 4];
    __shared__ uint32_t pre[kRrMaxB + 1];
    __shared__ uint32_t part[kRdThreads];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    {  // items (64 candidates of one query) before query i
        const uint32_t per = (B + kRdThreads - 1) / kRdThreads, b0 = tid * per;
        uint32_t loc = 0;
        for (uint32_t i = 0; i < per && b0 + i < B; ++i) loc += ((counts ? min(counts[b0 + i], R) : R) + 63u) / 64u;
        part[tid] = loc;
        __syncthreads();
        for (uint32_t o = 1; o < kRdThreads; o <<= 1) {
            const uint32_t v = tid >= o ? part[tid - o] : 0u;
            __syncthreads();
            part[tid] += v;
            __syncthreads();
        }
        uint32_t run = part[tid] - loc;
        for (uint32_t i = 0; i < per && b0 + i < B; ++i) {
            pre[b0 + i] = run;
            run += ((counts ? min(counts[b0 + i], R) : R) + 63u) / 64u;
        }
        if (tid == kRdThreads - 1) pre[B] = part[tid];
        __syncthreads();
    }
    const uint32_t items = pre[B], nch = D / 32u, L4 = D / 4u;
    const uint32_t tb = (uint32_t)(uintptr_t)&tile[wv][0][0];  // LDS byte addresses
    const uint32_t qb = (uint32_t)(uintptr_t)&qs[wv][0];
    const uint32_t W = gridDim.x * (kRdThreads / 64);
    // chunk c of the item's rows -> buffer c % kRdBufs: instruction s, lane l fills slot
    // (8 s + l / 8, l % 8) with float4 (l % 8) ^ ((row >> 1) & 7) of row 8 s + l / 8
    const uint32_t lr = lane >> 3, lp = lane & 7u;
    for (uint32_t item = blockIdx.x * (kRdThreads / 64) + wv; item < items; item += W) {  // wave-uniform
        uint32_t lo = 0, hi = B;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= item) lo = mid; else hi = mid;
        }
        const uint32_t qi = __builtin_amdgcn_readfirstlane(lo);
        const uint32_t r0 = (item - pre[qi]) * 64u, Rq = counts ? min(counts[qi], R) : R;
        const uint32_t* srow = s1_rows + (uint64_t)qi * R;
        const uint32_t my_r = r0 + lane;
        const bool live = my_r < Rq;
        // the source row of each of this lane's 8 DMA pieces: row 8 s + l / 8 of the item
        uint64_t src[8];
#pragma unroll
        for (int st = 0; st < 8; ++st) {
            const uint32_t rr = r0 + 8u * (uint32_t)st + lr;
            const uint32_t row = srow[rr < Rq ? rr : r0];  // past the list: a valid row, never used
            const uint32_t f = lp ^ (((8u * (uint32_t)st + lr) >> 1) & 7u);
            src[st] = (uint64_t)(uintptr_t)(rows + (uint64_t)row * D + 4u * f);
        }
        // the query (a piece per lane per 1 KiB), then the first chunks
        const float* qv = q + (uint64_t)qi * D;
        for (uint32_t k = 0; k * 64u < L4; ++k) {
            const uint32_t idx = min(k * 64u + lane, L4 - 1u);
            asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(qv + 4u * idx),
                         "s"(qb + k * 1024u)
                         : "memory");
        }
        auto issue = [&](uint32_t c) __attribute__((always_inline)) {
            const uint32_t b = tb + (c % kRdBufs) * 8192u;
#pragma unroll
            for (int st = 0; st < 8; ++st)
                asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src[st] + 128ull * c),
                             "s"(b + (uint32_t)st * 1024u)
                             : "memory");
        };
#pragma unroll
        for (int c = 0; c < kRdBufs - 1; ++c)
            if ((uint32_t)c < nch) issue((uint32_t)c);
        float acc = -0.0f, qq = -0.0f;
        const uint32_t rsw = (lane >> 1) & 7u;  // this lane's row swizzle
        for (uint32_t c = 0; c < nch; ++c) {
            // chunk c (and the query) landed: the younger DMAs are the next kRdBufs - 2 chunks
            if (c + kRdBufs - 2 < nch)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((kRdBufs - 2) * 8) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (c + kRdBufs - 1 < nch) issue(c + kRdBufs - 1);  // into the buffer chunk c - 1 used
            const float4* tr = (const float4*)&tile[wv][c % kRdBufs][8u * lane];
            const float4* qc = &qs[wv][8u * c];
#pragma unroll
            for (uint32_t f = 0; f < 8u; ++f) {
                const float4 x = tr[f ^ rsw];
                const float4 w = qc[f];
                acc = acc + w.x * x.x;
                acc = acc + w.y * x.y;
                acc = acc + w.z * x.z;
                acc = acc + w.w * x.w;
                qq = qq + w.x * w.x;
                qq = qq + w.y * w.y;
                qq = qq + w.z * w.z;
                qq = qq + w.w * w.w;
            }
        }
        if (live) {
            const uint32_t row = srow[my_r];
            const float na = sqrtf(qq), nb = norms[row];
            scores[(uint64_t)qi * R + my_r] = kind == kScoreCosine
                                                  ? ((na == 0.0f || nb == 0.0f) ? 0.0f : acc / (na * nb))
                                                  : ((na == 0.0f || nb == 0.0f) ? __builtin_inff()
                                                                               : 1.0f - (acc / (na * nb)));
        }
        // every lane's LDS reads of this item are done before the next item's DMAs land
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// GVDB_RERANK=v1: always the block-synchronous k_rerank (A/B)
static bool rerank_v2() {
    static const bool v = [] {
        const char* e = getenv("GVDB_RERANK");
        return !(e && strcmp(e, "v1") == 0);
    }();
    return v;
}
// k_rerank_small slots (query x 16 candidates) up to which it replaces
// k_rerank; GVDB_RERANK_SMALL=<n> overrides (0 disables; A/B timing)
static uint64_t rerank_small_max() {
    static const uint64_t v = [] {
        const char* e = getenv("GVDB_RERANK_SMALL");
        return e ? (uint64_t)atoll(e) : (uint64_t)256;
    }();
    return v;
}

hipError_t launch_rerank(const RerankArgs& a, hipStream_t s) {
    if (a.B == 0 || a.R == 0) return hipSuccess;
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t small_slots = (uint64_t)a.B * ((a.R + kRsRows - 1) / kRsRows);
    if ((small_slots <= rerank_small_max() || (a.short_lists && a.counts)) && std::min(a.qlen, a.clen) <= kRsMaxLen &&
        small_slots < (1ull << 31)) {
        hipLaunchKernelGGL(k_rerank_small, dim3((uint32_t)small_slots), dim3(kRsThreads), 0, s, a.rows, a.clen,
                           a.norms, a.q, a.qlen, a.s1_rows, a.B, a.R, a.counts, a.kind, a.scores, a.gate);
        GVDB_LAUNCH_CHECK();
        return hipSuccess;
    }
    // device-counted lists (D <= 1024): the item-walking k_rerank_small (flat candidates at the 8-GPU
    // shard, k 32, batch 64: 132 -> 84 us; neutral at 10M, batch 256); GVDB_RERANK=v2 / v1: the
    // 64-row wave items / the block-synchronous form (A/B)
    static const bool counted = [] {
        const char* e = getenv("GVDB_RERANK");
        return !(e && (strcmp(e, "v2") == 0 || strcmp(e, "v1") == 0));
    }();
    // lists at D % 32 == 0 (counted or full): k_rerank_dma (flat candidates at the 1.25M-row shard,
    // k = 32, batch 64: 84 -> 38 us; 10M, batch 256: flat group 2.65 -> 2.53 ms); GVDB_RERANK_DMA=0:
    // the item-walking k_rerank_small below (A/B)
    static const bool dma = [] {
        const char* e = getenv("GVDB_RERANK_DMA");
        return !(e && e[0] == '0');
    }();
    if (dma && a.qlen == a.clen && a.clen % 32u == 0 && a.clen <= kRdMaxD &&
        (a.kind == kScoreCosine || a.kind == kScoreCosineDistance) && (((uintptr_t)a.q | (uintptr_t)a.rows) & 15u) == 0) {
        for (uint32_t b0 = 0; b0 < a.B; b0 += kRrMaxB) {
            const uint32_t nb = std::min<uint32_t>(kRrMaxB, a.B - b0);
            const uint64_t waves = (uint64_t)nb * ((a.R + 63u) / 64u);
            const uint32_t grid = (uint32_t)std::min<uint64_t>((waves + 3u) / 4u, (uint64_t)cus);
            hipLaunchKernelGGL(k_rerank_dma, dim3(grid), dim3(kRdThreads), 0, s, a.rows, (uint32_t)a.clen, a.norms,
                               a.q + (uint64_t)b0 * a.qlen, a.s1_rows + (uint64_t)b0 * a.R, nb, a.R,
                               a.counts ? a.counts + b0 : nullptr, a.kind, a.scores + (uint64_t)b0 * a.R, a.gate);
            GVDB_LAUNCH_CHECK();
        }
        return hipSuccess;
    }
    if (a.counts && std::min(a.qlen, a.clen) <= kRsMaxLen && counted) {
        for (uint32_t b0 = 0; b0 < a.B; b0 += kRrMaxB) {
            const uint32_t nb = std::min<uint32_t>(kRrMaxB, a.B - b0);
            const uint64_t slots = (uint64_t)nb * ((a.R + kRsRows - 1) / kRsRows);
            const uint32_t grid = (uint32_t)std::min<uint64_t>(slots, 2ull * cus);
            hipLaunchKernelGGL(k_rerank_small_items, dim3(grid), dim3(kRsThreads), 0, s, a.rows, a.clen, a.norms,
                               a.q + (uint64_t)b0 * a.qlen, a.qlen, a.s1_rows + (uint64_t)b0 * a.R, nb, a.R,
                               a.counts + b0, a.kind, a.scores + (uint64_t)b0 * a.R, a.gate);
            GVDB_LAUNCH_CHECK();
        }
        return hipSuccess;
    }
    for (uint32_t b0 = 0; b0 < a.B; b0 += kRrMaxB) {
        const uint32_t nb = std::min<uint32_t>(kRrMaxB, a.B - b0);
        // upper bound of the work items (counts are on the device): every item
        // slot up to 2 resident blocks per CU, the loop takes the rest
        const uint64_t max_items = (uint64_t)nb * ((a.R + kRrRows - 1) / kRrRows);
        // k_rerank2 (wave-independent, 32-dim chunks) wins on large gathers
        // (flat candidate lists: ~13 % on 560K rows); the block-synchronous
        // k_rerank (128-dim chunks, shorter serial chain per item) on small
        // ones (batch-1: 34 us vs 60 us)
        static const uint64_t v2_min = [] {  // GVDB_RERANK2_MIN: items from which k_rerank2 is used (A/B)
            const char* e = getenv("GVDB_RERANK2_MIN");
            return e ? (uint64_t)atoll(e) : (uint64_t)2048;
        }();
        if (rerank_v2() && max_items >= v2_min) {
            // one item per wave; up to 4 resident blocks (16 waves) per CU
            const uint64_t blocks = (max_items + 3) / 4;
            const uint32_t grid = (uint32_t)std::min<uint64_t>(blocks, 4ull * cus);
            hipLaunchKernelGGL(k_rerank2, dim3(grid), dim3(kRr2Threads), 0, s, a.rows, a.clen, a.norms,
                               a.q + (uint64_t)b0 * a.qlen, a.qlen, a.s1_rows + (uint64_t)b0 * a.R, nb, a.R,
                               a.counts ? a.counts + b0 : nullptr, a.kind, a.scores + (uint64_t)b0 * a.R, a.gate);
        } else {
            const uint32_t grid = (uint32_t)std::min<uint64_t>(max_items, 2ull * cus);
            hipLaunchKernelGGL(k_rerank, dim3(grid), dim3(kRrThreads), 0, s, a.rows, a.clen, a.norms,
                               a.q + (uint64_t)b0 * a.qlen, a.qlen, a.s1_rows + (uint64_t)b0 * a.R, nb, a.R,
                               a.counts ? a.counts + b0 : nullptr, a.kind, a.scores + (uint64_t)b0 * a.R, a.gate);
        }
        GVDB_LAUNCH_CHECK();
    }
    return hipSuccess;
}


__global__ __launch_bounds__(256) void k_final_sort(const float* __restrict__ scores,
                                                    const uint32_t* __restrict__ s1_rows, uint32_t R, uint32_t kout,
                                                    int descending, const uint64_t* __restrict__ ids,
                                                    uint64_t row_offset, uint64_t* __restrict__ out_ids,
                                                    float* __restrict__ out_scores, uint32_t* __restrict__ out_n,
                                                    uint32_t* __restrict__ nan_flag) {
    __shared__ uint64_t sk[kSortLdsCap];
    __shared__ uint64_t tmp[kRankSortMax];
    __shared__ uint32_t s_nan;
    const uint32_t q = blockIdx.x;
    const float* sc = scores + (uint64_t)q * R;
    if (threadIdx.x == 0) s_nan = 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < R; i += 256) {
        const float f = sc[i];
        if (f != f) s_nan = 1u;
        uint32_t o = f32_order(f);
        if (descending) o = ~o;
        sk[i] = ((uint64_t)o << 32) | i;  // ties: stage-1 rank ascending (stable sort)
    }
    __syncthreads();
    if (s_nan && R >= 2) {
        if (threadIdx.x == 0) atomicOr(nan_flag, 1u);
    }
    select_sort(sk, R, tmp);  // rank counting up to kRankSortMax keys, bitonic beyond
    const uint32_t take = kout < R ? kout : R;
    // take(k) then drop orphan rows (index.rs:217-228); order-preserving
    // compaction by wave 0 with a ballot prefix.
    if (threadIdx.x < 64) {
        uint32_t o = 0;
        for (uint32_t i0 = 0; i0 < take; i0 += 64) {
            const uint32_t i = i0 + threadIdx.x;
            uint64_t id = kOrphan;
            uint32_t rank = 0;
            if (i < take) {
                rank = (uint32_t)sk[i];
                const uint32_t row = s1_rows[(uint64_t)q * R + rank];
                id = ids ? ids[row] : (uint64_t)row + row_offset;
            }
            const bool keep = i < take && id != kOrphan;
            const uint64_t m = __ballot(keep);
            const uint32_t before = __popcll(m & ((1ull << threadIdx.x) - 1ull));
            if (keep) {
                out_ids[(uint64_t)q * kout + o + before] = id;
                out_scores[(uint64_t)q * kout + o + before] = sc[rank];
            }
            o += __popcll(m);
        }
        // a NaN score would make the reference's sort panic: the query is poisoned
        if (threadIdx.x == 0 && out_n) out_n[q] = (s_nan && R >= 2) ? GVDB_N_POISONED : o;
    }
}

hipError_t launch_final_sort(const FinalArgs& a, hipStream_t s) {
    if (a.B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_final_sort, dim3(a.B), dim3(256), 0, s, a.scores, a.s1_rows, a.R, a.kout, a.descending, a.ids,
                       a.row_offset, a.out_ids, a.out_scores, a.out_n, a.nan_flag);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// Large-R variant: per query, radix-sort (order key, rank) pairs in HBM.
__global__ void k_make_keys(const float* __restrict__ sc, uint32_t R, int descending, uint32_t* __restrict__ keys,
                            uint32_t* __restrict__ vals, uint32_t* __restrict__ nan_flag) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const float f = sc[i];
    if (f != f && R >= 2) {
        atomicOr(nan_flag, 1u);
        atomicOr(nan_flag + 1, 1u);  // this query's flag, read and cleared by k_emit_sorted
    }
    uint32_t o = f32_order(f);
    keys[i] = descending ? ~o : o;
    vals[i] = i;
}

__global__ void k_emit_sorted(const uint32_t* __restrict__ ranks, const float* __restrict__ sc,
                              const uint32_t* __restrict__ s1_rows, uint32_t take, const uint64_t* __restrict__ ids,
                              uint64_t row_offset, uint64_t* __restrict__ out_ids, float* __restrict__ out_scores,
                              uint32_t* __restrict__ out_n, uint32_t* __restrict__ qnan) {
    // single wave: order-preserving compaction of orphans via ballot prefix.
    uint32_t o = 0;
    for (uint32_t i0 = 0; i0 < take; i0 += 64) {
        const uint32_t i = i0 + threadIdx.x;
        uint64_t id = kOrphan;
        uint32_t rank = 0;
        if (i < take) {
            rank = ranks[i];
            const uint32_t row = s1_rows[rank];
            id = ids ? ids[row] : (uint64_t)row + row_offset;
        }
        const bool keep = i < take && id != kOrphan;
        const uint64_t m = __ballot(keep);
        const uint32_t before = __popcll(m & ((1ull << threadIdx.x) - 1ull));
        if (keep) {
            out_ids[o + before] = id;
            out_scores[o + before] = sc[rank];
        }
        o += __popcll(m);
    }
    if (threadIdx.x == 0) {
        if (out_n) *out_n = *qnan ? GVDB_N_POISONED : o;
        *qnan = 0u;
    }
}

static size_t cub_pairs_bytes_u32(uint32_t n) { return cub_pairs_u32_bytes(n); }

size_t final_sort_global_bytes(uint32_t R) { return 4 * align256((size_t)R * 4) + align256(cub_pairs_bytes_u32(R)); }

hipError_t launch_final_sort_global(const FinalArgs& a, void* tmp, size_t tmp_bytes, hipStream_t s) {
    char* p = (char*)tmp;
    const size_t al = align256((size_t)a.R * 4);
    uint32_t* k0 = (uint32_t*)p;
    uint32_t* k1 = (uint32_t*)(p + al);
    uint32_t* v0 = (uint32_t*)(p + 2 * al);
    uint32_t* v1 = (uint32_t*)(p + 3 * al);
    void* ctmp = p + 4 * al;
    const uint32_t take = a.kout < a.R ? a.kout : a.R;
    for (uint32_t q = 0; q < a.B; ++q) {
        size_t cbytes = tmp_bytes - 4 * al;
        const float* sc = a.scores + (uint64_t)q * a.R;
        hipLaunchKernelGGL(k_make_keys, dim3((a.R + 255) / 256), dim3(256), 0, s, sc, a.R, a.descending, k0, v0,
                           a.nan_flag);
        GVDB_LAUNCH_CHECK();
        hipcub::DoubleBuffer<uint32_t> kb(k0, k1), vb(v0, v1);
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(ctmp, cbytes, kb, vb, (int)a.R, 0, 32, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_emit_sorted, dim3(1), dim3(64), 0, s, vb.Current(), sc, a.s1_rows + (uint64_t)q * a.R,
                           take, a.ids, a.row_offset, a.out_ids + (uint64_t)q * a.kout,
                           a.out_scores + (uint64_t)q * a.kout, a.out_n ? a.out_n + q : nullptr, a.nan_flag + 1);
        GVDB_LAUNCH_CHECK();
    }
    return hipSuccess;
}

// ============================================================================
// Flat exact scan: scores[q][row] for a tile of QT queries per block, each
// lane folding its row in order (bit-identical to storage.rs:851-865 /
// index.rs:686-700 / index.rs:69-78).
// ============================================================================
constexpr int kFlatQT = 16;

__global__ __launch_bounds__(256) void k_flat_scores(const float* __restrict__ q, uint32_t B,
                                                     const float* __restrict__ qnorm, const float* __restrict__ rows,
                                                     uint32_t N, uint32_t D, const float* __restrict__ norms, int kind,
                                                     const uint32_t* __restrict__ list, float* __restrict__ scores,
                                                     const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    __shared__ __attribute__((aligned(16))) float tiles[4][64 * kTileLd];
    __shared__ __attribute__((aligned(16))) float qs[kFlatQT][kCh];
    __shared__ uint64_t bases[4][64];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    // grid-stride over 256-row tiles (a bounded grid: a gated launch exits cheaply)
    for (uint32_t tile_i = blockIdx.x; tile_i < (N + 255u) / 256u; tile_i += gridDim.x) {
        // row: position in the scan (scores column); src: the shard row it reads
        // (list[row] for a filtered scan, else row itself)
        const uint64_t row = (uint64_t)tile_i * 256u + threadIdx.x;
        const uint64_t src = row < N ? (list ? (uint64_t)list[row] : row) : 0;
        const uint32_t q0 = blockIdx.y * kFlatQT;
        const uint32_t qn = (B - q0) < (uint32_t)kFlatQT ? (B - q0) : (uint32_t)kFlatQT;
        bases[wv][lane] = row < N ? src * D : ~0ull;
        float* tile = tiles[wv];
        const bool vec4 = (D & 3u) == 0;
        float acc[kFlatQT];
#pragma unroll
        for (int i = 0; i < kFlatQT; ++i) acc[i] = -0.0f;
        __syncthreads();
        for (uint64_t c0 = 0; c0 < D; c0 += kCh) {
            stage_tile(tile, rows, bases[wv], c0, D, vec4, lane);
            for (uint32_t t = threadIdx.x; t < kFlatQT * kCh; t += 256) {
                const uint32_t qi = t / kCh, j = t % kCh;
                qs[qi][j] = (qi < qn && c0 + j < D) ? q[(uint64_t)(q0 + qi) * D + c0 + j] : 0.0f;
            }
            __syncthreads();
            const uint32_t m = (uint32_t)((D - c0) < (uint64_t)kCh ? (D - c0) : kCh);
            const float* tr = tile + lane * kTileLd;
            for (uint32_t j = 0; j < m; ++j) {
                const float x = tr[j];
                if (kind == kScoreL2) {
#pragma unroll
                    for (int i = 0; i < kFlatQT; ++i) {
                        const float d = qs[i][j] - x;
                        acc[i] = acc[i] + d * d;
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < kFlatQT; ++i) acc[i] = acc[i] + qs[i][j] * x;
                }
            }
            __syncthreads();
        }
        if (row < N) {
            const float nb = norms ? norms[src] : 0.0f;
#pragma unroll
            for (int i = 0; i < kFlatQT; ++i) {
                if ((uint32_t)i >= qn) break;
                float score;
                if (kind == kScoreL2) {
                    score = sqrtf(acc[i]);
                } else {
                    const float na = qnorm[q0 + i];
                    if (kind == kScoreCosine)
                        score = (na == 0.0f || nb == 0.0f) ? 0.0f : acc[i] / (na * nb);
                    else
                        score = (na == 0.0f || nb == 0.0f) ? __builtin_inff() : 1.0f - (acc[i] / (na * nb));
                }
                scores[(uint64_t)(q0 + i) * N + row] = score;
            }
        }
        __syncthreads();  // bases[] is rewritten by the next tile
    }
}

hipError_t launch_flat_scores(const float* q, uint32_t B, const float* qnorm, const float* rows, uint32_t N, uint32_t D,
                              const float* norms, int kind, const uint32_t* list, float* scores, hipStream_t s,
                              const uint32_t* gate) {
    if (B == 0 || N == 0) return hipSuccess;
    const uint32_t qg = (B + kFlatQT - 1) / kFlatQT;
    // about 8 blocks per CU over all query groups; each block walks its row tiles
    const uint32_t gx = std::max<uint32_t>(1u, std::min<uint32_t>((N + 255) / 256, (8u * cu_count() + qg - 1) / qg));
    hipLaunchKernelGGL(k_flat_scores, dim3(gx, qg), dim3(256), 0, s, q, B, qnorm, rows, N, D, norms, kind, list,
                       scores, gate);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

size_t flat_select_bytes(uint32_t N) { return final_sort_global_bytes(N); }

__global__ void k_emit_flat(const uint32_t* __restrict__ ranks, const float* __restrict__ sc, uint32_t N,
                            uint32_t limit, int has_threshold, float threshold, const uint64_t* __restrict__ ids,
                            uint64_t* __restrict__ out_idx, float* __restrict__ out_scores,
                            uint32_t* __restrict__ out_n) {
    // Walk the sorted list; rows without an id are skipped BEFORE truncation
    // (index.rs:626-631 iterates only mapped rows); with a threshold the
    // sorted-descending list is cut at the first score < threshold
    // (storage.rs:313-317 drops them before sorting: same survivors, same order).
    uint32_t o = 0;
    for (uint32_t i0 = 0; i0 < N && o < limit; i0 += 64) {
        const uint32_t i = i0 + threadIdx.x;
        bool keep = false;
        float f = 0.f;
        uint64_t id = 0;
        if (i < N) {
            const uint32_t rank = ranks[i];
            f = sc[rank];
            id = ids ? ids[rank] : (uint64_t)rank;
            keep = (!has_threshold || !(f < threshold)) && id != kOrphan;
        }
        const uint64_t m = __ballot(keep);
        const uint32_t before = __popcll(m & ((1ull << threadIdx.x) - 1ull));
        if (keep && o + before < limit) {
            out_idx[o + before] = id;
            out_scores[o + before] = f;
        }
        o += __popcll(m);
    }
    if (threadIdx.x == 0 && out_n) *out_n = o < limit ? o : limit;
}

// The same selection for limit <= kFlatTopkCap and N <= kFlatTopkMaxN, every
// query of the batch in ONE launch (one block per query) instead of a radix
// sort per query: the kept entries' (order key, row) pairs are totally ordered
// exactly as the stable key sort orders them, so the first `limit` kept
// entries are the `limit` smallest pairs.  The keys are staged in LDS (N <=
// kFlatTopkStage; else re-read from L2), a 4-digit radix select finds the
// limit-th smallest key K, then the entries below K and the lowest-row entries
// equal to K (ordered compaction, chunk by chunk) are collected and sorted in
// LDS.  NaN flags as k_make_keys.
constexpr uint32_t kFlatTopkCap = 1024;
constexpr uint32_t kFlatTopkBuf = 2048;  // collected entries (>= kFlatTopkCap)
constexpr uint32_t kFlatTopkStage = 16384;
constexpr uint32_t kFlatTopkMaxN = 262144;
constexpr uint32_t kFlatTopkThreads = 1024;
template <bool STAGED>
__global__ __launch_bounds__(kFlatTopkThreads) void k_flat_topk(const float* __restrict__ scores, uint32_t N, uint32_t limit,
                                                   int descending, int has_threshold, float threshold,
                                                   const uint64_t* __restrict__ ids, uint64_t* __restrict__ out_idx,
                                                   float* __restrict__ out_scores, uint32_t* __restrict__ out_n,
                                                   uint32_t* __restrict__ nan_flag,
                                                   const uint32_t* __restrict__ gate) {
    if (gate_closed(gate)) return;
    constexpr uint32_t kKeys = STAGED ? kFlatTopkStage : 1u;
    __shared__ uint32_t s_key[kKeys];
    __shared__ uint32_t s_kept[STAGED ? kFlatTopkStage / 32 : 1u];
    __shared__ uint32_t hist[256];
    __shared__ uint64_t cand[kFlatTopkBuf];
    __shared__ uint32_t s_total, s_nan, s_prefix, s_need, s_nc, s_wc[kFlatTopkThreads / 64];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const float* sc = scores + (uint64_t)q * N;
    auto load = [&](uint32_t i, uint32_t& key, bool& nan) {  // kept (threshold, mapped row) and its order key
        const float f = sc[i];
        const uint64_t id = ids ? ids[i] : (uint64_t)i;
        const uint32_t o = f32_order(f);
        key = descending ? ~o : o;
        nan = f != f;
        return (!has_threshold || !(f < threshold)) && id != kOrphan;
    };
    auto get = [&](uint32_t i, uint32_t& key) {
        if constexpr (STAGED) {
            key = s_key[i];
            return ((s_kept[i >> 5] >> (i & 31u)) & 1u) != 0u;
        } else {
            bool nan;
            return load(i, key, nan);
        }
    };
    if (tid == 0) {
        s_total = 0;
        s_nan = 0;
        s_prefix = 0;
        s_nc = 0;
    }
    __syncthreads();
    uint32_t kept = 0;
    bool nan = false;
    constexpr uint32_t kU = 8;  // loads in flight per thread
    for (uint32_t i0 = tid; i0 < N; i0 += kFlatTopkThreads * kU) {
        uint32_t key[kU];
        bool kp[kU], nn[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t i = i0 + kFlatTopkThreads * u;
            kp[u] = i < N && load(min(i, N - 1), key[u], nn[u]);
            nn[u] = i < N && nn[u];
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t i = i0 + kFlatTopkThreads * u;
            kept += kp[u] ? 1u : 0u;
            nan |= nn[u];
            if constexpr (STAGED) {  // the wave's 64 consecutive rows: two bitmap words
                if (i < N) s_key[i] = key[u];
                const uint64_t b = __ballot(kp[u]);
                const uint32_t w0 = (i - lane) >> 5;
                if (lane == 0 && w0 < kFlatTopkStage / 32) s_kept[w0] = (uint32_t)b;
                if (lane == 32 && w0 + 1 < kFlatTopkStage / 32) s_kept[w0 + 1] = (uint32_t)(b >> 32);
            }
        }
    }
    atomicAdd(&s_total, kept);
    if (nan) s_nan = 1u;
    __syncthreads();
    const uint32_t want = min(s_total, limit);
    if (tid == 0) {
        if (s_nan && N >= 2) {
            atomicOr(nan_flag, 1u);
            atomicOr(nan_flag + 1, 1u);
        }
        if (out_n) out_n[q] = want;
        s_need = want;
    }
    if (want == 0) return;
    // radix select of the want-th smallest key among the kept entries
    uint32_t mask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
        if (tid < 256) hist[tid] = 0;
        __syncthreads();
        const uint32_t prefix = s_prefix;
        for (uint32_t i = tid; i < N; i += kFlatTopkThreads) {
            uint32_t key;
            if (get(i, key) && (key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
        }
        __syncthreads();
        // the digit whose cumulative count reaches s_need: a scan of the 256 bins (waves 0-3)
        const uint32_t v = tid < 256 ? hist[tid] : 0u, need = s_need;
        uint32_t incl = v;
#pragma unroll
        for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(incl, off);
            if (lane >= off) incl += t;
        }
        if (lane == 63 && wv < 4) s_wc[wv] = incl;
        __syncthreads();
        for (uint32_t w = 0; w < wv && w < 4; ++w) incl += s_wc[w];
        const uint32_t excl = incl - v;
        if (tid < 256 && excl < need && need <= incl) {
            s_need = need - excl;
            s_prefix = prefix | (tid << shift);
        }
        mask |= 255u << shift;
        __syncthreads();
    }
    const uint32_t K = s_prefix;
    // collect every kept entry below K and those equal to K (their sort by row
    // keeps the lowest rows first); past the buffer (massive ties) the equal
    // ones are taken again in row order, chunk by chunk
    for (uint32_t i = tid; i < N; i += kFlatTopkThreads) {
        uint32_t key;
        if (get(i, key) && key <= K) {
            const uint32_t c = atomicAdd(&s_nc, 1u);
            if (c < kFlatTopkBuf) cand[c] = ((uint64_t)key << 32) | i;
        }
    }
    __syncthreads();
    uint32_t nc = s_nc;
    if (nc > kFlatTopkBuf) {
        __syncthreads();
        if (tid == 0) s_nc = 0;
        __syncthreads();
        uint32_t eq_left = s_need;
        for (uint32_t base = 0; base < N; base += kFlatTopkThreads) {
            const uint32_t i = base + tid;
            uint32_t key = 0;
            const bool k = i < N && get(i, key);
            if (k && key < K) cand[atomicAdd(&s_nc, 1u)] = ((uint64_t)key << 32) | i;
            if (eq_left == 0) continue;  // (block-uniform)
            const bool eq = k && key == K;
            const uint64_t m = __ballot(eq);
            if (lane == 0) s_wc[wv] = (uint32_t)__popcll(m);
            __syncthreads();
            uint32_t before = 0, tot = 0;
            for (uint32_t w = 0; w < kFlatTopkThreads / 64; ++w) {
                before += w < wv ? s_wc[w] : 0u;
                tot += s_wc[w];
            }
            const uint32_t r = before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (eq && r < eq_left) cand[atomicAdd(&s_nc, 1u)] = ((uint64_t)key << 32) | i;
            eq_left = tot < eq_left ? eq_left - tot : 0u;
            __syncthreads();
        }
        __syncthreads();
        nc = s_nc;  // == want
    }
    const uint32_t P = next_pow2(nc);
    for (uint32_t j = nc + tid; j < P; j += kFlatTopkThreads) cand[j] = ~0ull;
    __syncthreads();
    bitonic_sort_lds(cand, P);
    for (uint32_t j = tid; j < want; j += kFlatTopkThreads) {
        const uint32_t i = (uint32_t)cand[j];
        out_idx[(uint64_t)q * limit + j] = ids ? ids[i] : (uint64_t)i;
        out_scores[(uint64_t)q * limit + j] = sc[i];
    }
}

hipError_t launch_flat_select(const float* scores, uint32_t B, uint32_t N, uint32_t limit, int descending,
                              int has_threshold, float threshold, const uint64_t* ids, uint64_t* out_idx,
                              float* out_scores, uint32_t* out_n, void* tmp, size_t tmp_bytes, uint32_t* nan_flag,
                              hipStream_t s, const uint32_t* gate) {
    if (B == 0) return hipSuccess;
    // a gated (device-decided fallback) select takes the one-launch form at any N:
    // the per-query radix sorts below are B launches each
    if (limit <= kFlatTopkCap && (gate || (N <= kFlatTopkMaxN && !getenv("GVDB_FLAT_SORT")))) {
        if (N <= kFlatTopkStage)
            hipLaunchKernelGGL(k_flat_topk<true>, dim3(B), dim3(kFlatTopkThreads), 0, s, scores, N, limit, descending,
                               has_threshold, threshold, ids, out_idx, out_scores, out_n, nan_flag, gate);
        else
            hipLaunchKernelGGL(k_flat_topk<false>, dim3(B), dim3(kFlatTopkThreads), 0, s, scores, N, limit, descending,
                               has_threshold, threshold, ids, out_idx, out_scores, out_n, nan_flag, gate);
        GVDB_LAUNCH_CHECK();
        return hipSuccess;
    }
    if (gate) return hipErrorInvalidValue;  // a gated select needs limit <= kFlatTopkCap
    char* p = (char*)tmp;
    const size_t al = align256((size_t)N * 4);
    uint32_t* k0 = (uint32_t*)p;
    uint32_t* k1 = (uint32_t*)(p + al);
    uint32_t* v0 = (uint32_t*)(p + 2 * al);
    uint32_t* v1 = (uint32_t*)(p + 3 * al);
    void* ctmp = p + 4 * al;
    for (uint32_t q = 0; q < B; ++q) {
        size_t cbytes = tmp_bytes - 4 * al;
        const float* sc = scores + (uint64_t)q * N;
        hipLaunchKernelGGL(k_make_keys, dim3((N + 255) / 256), dim3(256), 0, s, sc, N, descending, k0, v0, nan_flag);
        GVDB_LAUNCH_CHECK();
        hipcub::DoubleBuffer<uint32_t> kb(k0, k1), vb(v0, v1);
        hipError_t e = hipcub::DeviceRadixSort::SortPairs(ctmp, cbytes, kb, vb, (int)N, 0, 32, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_emit_flat, dim3(1), dim3(64), 0, s, vb.Current(), sc, N, limit, has_threshold, threshold,
                           ids, out_idx + (uint64_t)q * limit, out_scores + (uint64_t)q * limit,
                           out_n ? out_n + q : nullptr);
        GVDB_LAUNCH_CHECK();
    }
    return hipSuccess;
}

// ============================================================================
// Shard merge (shard.rs:776-784): per query concat the shards' lists in shard
// order, stable sort by score, truncate.  One workgroup per query, LDS sort.
// ============================================================================
__global__ __launch_bounds__(256) void k_topk_merge(const uint64_t* __restrict__ ids, const float* __restrict__ scores,
                                                    const uint32_t* __restrict__ counts, uint32_t n_shards, uint32_t B,
                                                    uint32_t stride, uint32_t limit, int descending,
                                                    uint64_t* __restrict__ out_ids, float* __restrict__ out_scores,
                                                    uint32_t* __restrict__ out_n) {
    __shared__ uint64_t sk[kSortLdsCap];
    __shared__ uint32_t s_n;
    const uint32_t q = blockIdx.x;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    // position in the concatenation = shard * stride + i (monotone in concat order)
    for (uint32_t t = threadIdx.x; t < n_shards * stride; t += 256) {
        const uint32_t sh = t / stride, i = t % stride;
        if (i < counts[(uint64_t)sh * B + q]) {
            const float f = scores[((uint64_t)sh * B + q) * stride + i];
            uint32_t o = f32_order(f);
            if (descending) o = ~o;
            const uint32_t pos = atomicAdd(&s_n, 1u);
            sk[pos] = ((uint64_t)o << 32) | t;
        }
    }
    __syncthreads();
    const uint32_t n = s_n;
    const uint32_t P = next_pow2(n);
    for (uint32_t i = n + threadIdx.x; i < P; i += 256) sk[i] = ~0ull;
    __syncthreads();
    bitonic_sort_lds(sk, P);
    const uint32_t take = limit < n ? limit : n;
    for (uint32_t i = threadIdx.x; i < take; i += 256) {
        const uint32_t t = (uint32_t)sk[i];
        const uint32_t sh = t / stride, j = t % stride;
        out_ids[(uint64_t)q * limit + i] = ids[((uint64_t)sh * B + q) * stride + j];
        out_scores[(uint64_t)q * limit + i] = scores[((uint64_t)sh * B + q) * stride + j];
    }
    if (threadIdx.x == 0 && out_n) out_n[q] = take;
}

hipError_t launch_topk_merge(const uint64_t* ids, const float* scores, const uint32_t* counts, uint32_t n_shards,
                             uint32_t B, uint32_t stride, uint32_t limit, int descending, uint64_t* out_ids,
                             float* out_scores, uint32_t* out_n, hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_topk_merge, dim3(B), dim3(256), 0, s, ids, scores, counts, n_shards, B, stride, limit,
                       descending, out_ids, out_scores, out_n);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

__global__ void k_widen(const uint32_t* __restrict__ a, uint64_t* __restrict__ b, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

hipError_t launch_widen(const uint32_t* a, uint64_t* b, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_widen, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, a, b, n);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// Stage-1-ordered candidate list with exact scores (sharded search input).
// Output row stride out_stride >= R (a shard with fewer rows than the global
// R fills the first R of each stride-R row of the all-gather send block).
__global__ void k_emit_candidates(const uint32_t* __restrict__ s1_rows, const uint32_t* __restrict__ s1_dist,
                                  const float* __restrict__ scores, uint32_t B, uint32_t R, uint64_t out_stride,
                                  const uint64_t* __restrict__ ids, uint64_t* __restrict__ out_ids,
                                  uint32_t* __restrict__ out_dist, float* __restrict__ out_scores) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)B * R) return;
    const uint64_t o = (t / R) * out_stride + t % R;
    out_ids[o] = ids ? ids[s1_rows[t]] : (uint64_t)s1_rows[t];
    out_dist[o] = s1_dist[t];
    out_scores[o] = scores[t];
}

hipError_t launch_emit_candidates(const uint32_t* s1_rows, const uint32_t* s1_dist, const float* scores, uint32_t B,
                                  uint32_t R, const uint64_t* ids, uint64_t* out_ids, uint32_t* out_dist,
                                  float* out_scores, hipStream_t s, uint64_t out_stride) {
    const uint64_t total = (uint64_t)B * R;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_emit_candidates, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, s, s1_rows, s1_dist,
                       scores, B, R, out_stride ? out_stride : (uint64_t)R, ids, out_ids, out_dist, out_scores);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ============================================================================
// Exact sharded multi-stage merge.  Each shard sends, per query, its LOCAL
// stage-1 top-R (Hamming d, global id) with the exact cosine of each; the
// union of the local top-R lists contains the global top-R, so one exchange
// suffices.  Per query: sort the union by (d asc, gid asc) == the reference's
// stable stage-1 sort over the concatenated corpus, keep R, then sort those by
// (cosine desc, global stage-1 rank asc), keep k.  Bit-identical to running
// multi_stage_search on one device over all shards (ids = global row numbers).
// ============================================================================
__device__ void bitonic_sort_pairs_lds(uint64_t* s, uint32_t* v, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = s[i], b = s[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        s[i] = b;
                        s[ixj] = a;
                        const uint32_t t = v[i];
                        v[i] = v[ixj];
                        v[ixj] = t;
                    }
                }
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(256) void k_bq_shard_merge(const uint64_t* __restrict__ gids,
                                                        const uint32_t* __restrict__ dist,
                                                        const float* __restrict__ cosv,
                                                        const uint32_t* __restrict__ counts, uint32_t G, uint32_t B,
                                                        uint32_t stride, uint64_t gs_id, uint64_t gs_w, uint64_t gs_c,
                                                        uint32_t R, uint32_t kout, uint64_t* __restrict__ out_ids,
                                                        float* __restrict__ out_scores, uint32_t* __restrict__ out_n,
                                                        uint32_t* __restrict__ nan_flag, int mark_nan) {
    // rank g's list for query q starts at gids + g*gs_id + q*stride (dist/cosv: g*gs_w),
    // its count is counts[g*gs_c + q].  mark_nan: a query whose top-R holds a NaN
    // cosine (the reference's sort would panic) gets out_n[q] = GVDB_N_POISONED.
    __shared__ uint64_t sk[kSortLdsCap];
    __shared__ uint32_t sv[kSortLdsCap];
    __shared__ uint32_t s_n;
    const uint32_t q = blockIdx.x;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < G * stride; t += 256) {
        const uint32_t g = t / stride, i = t % stride;
        if (i < counts[(uint64_t)g * gs_c + q]) {
            const uint64_t at = (uint64_t)q * stride + i;
            const uint32_t pos = atomicAdd(&s_n, 1u);
            sk[pos] = ((uint64_t)dist[g * gs_w + at] << 40) | (gids[g * gs_id + at] & ((1ull << 40) - 1));
            sv[pos] = t;
        }
    }
    __syncthreads();
    const uint32_t n = s_n;
    uint32_t P = next_pow2(n);
    for (uint32_t i = n + threadIdx.x; i < P; i += 256) {
        sk[i] = ~0ull;
        sv[i] = 0;
    }
    __syncthreads();
    bitonic_sort_pairs_lds(sk, sv, P);
    const uint32_t r = R < n ? R : n;
    // second key: cosine desc, then global stage-1 rank
    __shared__ uint32_t s_nan;
    if (threadIdx.x == 0) s_nan = 0;
    __syncthreads();
    const uint32_t P2 = next_pow2(r);
    for (uint32_t i = threadIdx.x; i < P2; i += 256) {
        uint64_t key = ~0ull;
        uint32_t val = 0;
        if (i < r) {
            const uint32_t t = sv[i];
            const uint32_t g = t / stride, j = t % stride;
            const float f = cosv[g * gs_w + (uint64_t)q * stride + j];
            if (f != f) s_nan = 1u;
            key = ((uint64_t)(~f32_order(f)) << 32) | i;
            val = t;
        }
        sk[i] = key;  // thread i reads and rewrites only slot i
        sv[i] = val;
    }
    __syncthreads();
    const bool poisoned = s_nan && r >= 2;
    if (poisoned && threadIdx.x == 0 && nan_flag) atomicOr(nan_flag, 1u);
    bitonic_sort_pairs_lds(sk, sv, P2);
    const uint32_t take = kout < r ? kout : r;
    for (uint32_t i = threadIdx.x; i < take; i += 256) {
        const uint32_t t = sv[i];
        const uint32_t g = t / stride, j = t % stride;
        const uint64_t at = (uint64_t)q * stride + j;
        out_ids[(uint64_t)q * kout + i] = gids[g * gs_id + at];
        out_scores[(uint64_t)q * kout + i] = cosv[g * gs_w + at];
    }
    if (threadIdx.x == 0 && out_n) out_n[q] = (poisoned && mark_nan) ? GVDB_N_POISONED : take;
}

hipError_t launch_bq_shard_merge(const uint64_t* gids, const uint32_t* dist, const float* cosv, const uint32_t* counts,
                                 uint32_t G, uint32_t B, uint32_t stride, uint32_t R, uint32_t kout, uint64_t* out_ids,
                                 float* out_scores, uint32_t* out_n, uint32_t* nan_flag, hipStream_t s,
                                 uint64_t gs_id, uint64_t gs_w, uint64_t gs_c, int mark_nan) {
    if (B == 0) return hipSuccess;
    const uint64_t dense = (uint64_t)B * stride;  // [G][B][stride] when no rank strides are given
    hipLaunchKernelGGL(k_bq_shard_merge, dim3(B), dim3(256), 0, s, gids, dist, cosv, counts, G, B, stride,
                       gs_id ? gs_id : dense, gs_w ? gs_w : dense, gs_c ? gs_c : (uint64_t)B, R, kout, out_ids,
                       out_scores, out_n, nan_flag, mark_nan);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ============================================================================
// Order-preserving gather (remove_vector compaction, index.rs:245-266)
// ============================================================================
__global__ void k_gather_rows(const float* __restrict__ src, float* __restrict__ dst, const uint64_t* __restrict__ map,
                              uint64_t m, uint32_t D) {
    const uint64_t r = blockIdx.y * (uint64_t)gridDim.x + blockIdx.x;
    if (r >= m) return;
    const float* s = src + map[r] * D;
    float* d = dst + r * D;
    for (uint32_t j = threadIdx.x; j < D; j += blockDim.x) d[j] = s[j];
}

__global__ void k_gather_meta(const uint4* __restrict__ codes, uint4* __restrict__ ncodes, const float* __restrict__ norms,
                              float* __restrict__ nnorms, const uint64_t* __restrict__ ids, uint64_t* __restrict__ nids,
                              const uint64_t* __restrict__ map, uint64_t m, uint64_t cap, uint32_t W4) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const uint64_t o = map[r];
    for (uint32_t w = 0; w < W4; ++w) ncodes[(uint64_t)w * cap + r] = codes[(uint64_t)w * cap + o];
    nnorms[r] = norms[o];
    nids[r] = ids[o];
}

// Filtered BQ search: the allowed rows' code planes, compacted (row list
// ascending, so the subset keeps the index's row order), and the stage-1
// candidates mapped back to index rows before the rerank.
__global__ void k_gather_code_rows(const uint4* __restrict__ codes, uint64_t cap, const uint32_t* __restrict__ rows,
                                   uint32_t m, uint32_t W4, uint4* __restrict__ ncodes) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    const uint64_t o = rows[r];
    for (uint32_t w = 0; w < W4; ++w) ncodes[(uint64_t)w * m + r] = codes[(uint64_t)w * cap + o];
}

__global__ void k_map_rows(uint32_t* __restrict__ s1_rows, uint64_t n, const uint32_t* __restrict__ rows) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) s1_rows[i] = rows[s1_rows[i]];
}

hipError_t launch_gather_code_rows(const uint4* codes, uint64_t cap, const uint32_t* rows, uint32_t m, uint32_t D,
                                   uint4* ncodes, hipStream_t s) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_code_rows, dim3((m + 255) / 256), dim3(256), 0, s, codes, cap, rows, m, code_w4(D),
                       ncodes);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_map_rows(uint32_t* s1_rows, uint64_t n, const uint32_t* rows, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_map_rows, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, s1_rows, n, rows);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

hipError_t launch_gather(const float* rows, float* nrows, const uint4* codes, uint4* ncodes, const float* norms,
                         float* nnorms, const uint64_t* ids, uint64_t* nids, const uint64_t* map, uint64_t m,
                         uint64_t cap, uint32_t D, hipStream_t s) {
    if (m == 0) return hipSuccess;
    const uint32_t gx = (uint32_t)(m < 65535 ? m : 65535);
    const uint32_t gy = (uint32_t)((m + gx - 1) / gx);
    hipLaunchKernelGGL(k_gather_rows, dim3(gx, gy), dim3(256), 0, s, rows, nrows, map, m, D);
    GVDB_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_gather_meta, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, s, codes, ncodes, norms, nnorms,
                       ids, nids, map, m, cap, code_w4(D));
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

// ============================================================================
// Batch-1 fast path: three launches, no host round trip.
//
//   k_b1_sample  packs the query (ballots, Msb0 words) in every block and
//                histograms the Hamming distance of a sample of ~N/32 rows
//                (1024-row chunks spread over the shard; the whole shard when
//                N <= kExactN), flushed into one global histogram;
//   k_b1_scan    the HBM-bound pass over every code: each block derives the
//                threshold T from that histogram while its code loads are in
//                flight, rows with d <= T go to the candidate buffer;
//   k_b1_tail    ceil(R/16) blocks: each one selects the exact top-R from the
//                buffer (select_topr, with its device-side rescan), re-scores
//                its 16 rows (sequential f32 fold = cosine_similarity_manual),
//                publishes the scores, and the last block to arrive sorts all
//                R scores (stable by stage-1 rank) and writes the top-k.  The
//                last block also zeroes the histogram and the counter for the
//                next call (the path is self-cleaning).
// Hand-off inside k_b1_tail: scores stored `sc1` (agent-scope relaxed atomic
// stores), the storing waves drain (`s_waitcnt vmcnt(0)`) before one agent
// atomic add per block, and the block whose add came last reads them with
// agent-scope atomic loads (MI355X_MICROARCH.md, valid hand-off forms, row 1).
// ============================================================================

// Query -> 4*W4 Msb0 code words in LDS (pad words zero), by the whole block.
// 256-thread blocks, D <= 1024: every query load is issued before the first
// ballot (one memory latency, not one per 64-dim unit).
template <int W4>
__device__ __forceinline__ void pack_query_lds(const float* __restrict__ q, uint32_t D, float thr, uint32_t* qw) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t chunks = (D + 63u) / 64u;
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t dim = (wv + 4u * u) * 64u + lane;
        v[u] = dim < D ? q[dim] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t c = wv + 4u * u;
        const uint32_t dim = c * 64u + lane;
        const bool bit = dim < D && v[u] > thr;  // NaN > thr is false (Rust `value > threshold`)
        const uint64_t m = __ballot(bit);
        if (c < chunks && lane < 2) {
            const uint32_t w = 2u * c + lane;
            if (w < 4u * W4) qw[w] = msb0_word(lane == 0 ? (uint32_t)m : (uint32_t)(m >> 32));
        }
    }
    for (uint32_t w = 2u * chunks + threadIdx.x; w < 4u * W4; w += blockDim.x) qw[w] = 0u;
}

// Only bins <= this block's own target-th smallest distance are flushed: the
// global target-th smallest T^ is <= every block's (each block alone holds
// target rows at or below its own), so every bin <= T^ still receives every
// block's count -- exact where it matters, with a fraction of the global atomics.
template <int W4>
__global__ __launch_bounds__(256) void k_b1_sample(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                   uint32_t D, uint32_t stride, const float* __restrict__ q, float thr,
                                                   uint32_t target, uint32_t* __restrict__ qwords_out,
                                                   uint32_t* __restrict__ hist) {
    __shared__ uint32_t s_top;
    __shared__ uint4 qc[W4];
    __shared__ uint32_t lh[kRsMaxLen + 1];  // D <= 1024 on this path
    const uint32_t tid = threadIdx.x;
    const uint64_t start = (uint64_t)blockIdx.x * stride;
    uint4 c[4][W4];
    bool ok[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {  // loads first: they fly while the query is packed
        const uint64_t row = start + (uint64_t)it * 256u + tid;
        ok[it] = row < N;
        const uint64_t r = ok[it] ? row : 0;
#pragma unroll
        for (int w = 0; w < W4; ++w) c[it][w] = load_code_nt(codes + (uint64_t)w * cap + r);
    }
    pack_query_lds<W4>(q, D, thr, (uint32_t*)qc);
    for (uint32_t i = tid; i <= D; i += 256) lh[i] = 0u;
    __syncthreads();
    if (blockIdx.x == 0 && tid < 4u * W4) qwords_out[tid] = ((const uint32_t*)qc)[tid];
    uint4 qv[W4];
#pragma unroll
    for (int w = 0; w < W4; ++w) qv[w] = qc[w];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        if (!ok[it]) continue;
        uint32_t d = 0;
#pragma unroll
        for (int w = 0; w < W4; ++w) d = ham4(c[it][w], qv[w], d);
        atomicAdd(&lh[d], 1u);
    }
    __syncthreads();
    if (tid < 64) {
        const uint32_t t = wave_find_cum(lh, D + 1u, target);  // D when the block holds fewer rows
        if (tid == 0) s_top = t;
    }
    __syncthreads();
    const uint32_t top = s_top;
    for (uint32_t i = tid; i <= top; i += 256) {
        const uint32_t v = lh[i];
        if (v) atomicAdd(&hist[i], v);
    }
}

template <int W4, int CPL>
__global__ __launch_bounds__(256) void k_b1_scan(const uint4* __restrict__ codes, uint64_t cap, uint32_t N, uint32_t D,
                                                 const uint32_t* __restrict__ qwords, const uint32_t* __restrict__ hist,
                                                 uint32_t target, uint32_t* __restrict__ counts,
                                                 uint64_t* __restrict__ buf, uint32_t bufcap) {
    __shared__ uint32_t s_T;
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * (256u * CPL);
    uint4 c[CPL][W4];
    uint32_t bias[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const uint64_t n = base + (uint64_t)k * 256u + tid;
        const bool ok = n < N;
        const uint64_t nc = ok ? n : (uint64_t)(N - 1);
        bias[k] = ok ? 0u : 0x01000000u;  // out-of-range rows never pass the threshold
#pragma unroll
        for (int w = 0; w < W4; ++w) c[k][w] = load_code_nt(codes + (uint64_t)w * cap + nc);
    }
    // the threshold from the sample histogram, while the code loads fly
    if (tid < 64) {
        const uint32_t t = wave_find_cum(hist, D + 1u, target);
        if (tid == 0) s_T = t;
    }
    const uint4* qc = (const uint4*)qwords;
    uint4 qw[W4];
#pragma unroll
    for (int w = 0; w < W4; ++w) qw[w] = qc[w];
    __syncthreads();
    const uint32_t T = s_T;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        uint32_t d = bias[k];
#pragma unroll
        for (int w = 0; w < W4; ++w) d = ham4(c[k][w], qw[w], d);
        if (d <= T) {
            const uint32_t pos = atomicAdd(counts, 1u);
            if (pos < bufcap) buf[pos] = ((uint64_t)d << 32) | (uint32_t)(base + (uint64_t)k * 256u + tid);
        }
    }
}

struct B1TailArgs {
    const uint32_t* counts;   // [0] candidates in buf; zeroed by the last block
    const uint64_t* buf;
    uint32_t bufcap, D, R, N, W4, kout;
    const uint4* codes;
    uint64_t cap;
    const uint32_t* qwords;
    const float* rows;
    uint64_t clen;
    const float* norms;
    const float* q;
    uint64_t qlen;
    int kind, descending, force_rescan;
    const uint64_t* ids;
    uint64_t row_offset;
    float* scores;            // [bufcap] published exact scores of the buffered candidates
    float* rscores;           // [R] scores of a rescan's rows
    uint64_t* topr;           // [R] published sorted top-R keys (d, row, buffer index)
    uint32_t* ticket;         // arrival counter, reset by the last block
    uint32_t* rescans;        // diagnostics: device-side rescans
    uint32_t* hist;           // [D+1] sample histogram, zeroed by the last block
    uint64_t* out_ids;
    float* out_scores;
    uint32_t* out_n;
    unsigned long long* clk;  // timing study only (GVDB_B1_CLK): [block0 | last block][8] wall clocks
};

// k_b1_tail: block 0 selects the exact top-R from the candidate buffer while
// blocks 1..G re-score EVERY buffered candidate (16 per block and round), so the
// select and the row gathers + sequential folds overlap; the last block to
// arrive sorts the top-R by exact score.  A rescan (buffer cannot hold the
// top-R) re-scores its R rows in block 0 itself (rare; slow, still exact).
__global__ __launch_bounds__(256) void k_b1_tail(B1TailArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t sk[];  // keys | hist | bins | tile | query
    uint32_t* hist = (uint32_t*)(sk + kSelectLdsCap);
    uint32_t* bins = hist + ((a.D + 4u) & ~3u);
    float4* tile4 = (float4*)(bins + 2048);
    float4* qs4 = tile4 + kRsRows * (kRsMaxLen / 4 + 1);
    __shared__ uint32_t s_last, s_nan, rowid[kRsRows];
    const uint32_t tid = threadIdx.x, R = a.R;
    unsigned long long ck[6];
    ck[0] = wall_clock64();
    const uint32_t cnt = a.counts[0];
    unsigned long long t_staged = 0;
    if (blockIdx.x == 0) {
        const bool resc = select_topr(cnt, a.buf, a.bufcap, a.D, R, a.codes, a.cap, a.N, a.W4,
                                      (const uint4*)a.qwords, a.force_rescan != 0, sk, hist, bins, true);
        ck[1] = wall_clock64();
        for (uint32_t i = tid; i < R; i += 256)
            __hip_atomic_store(a.topr + i, sk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (resc) {  // rows not from the buffer: score them here, 16 at a time
            if (tid == 0) atomicAdd(a.rescans, 1u);
            for (uint32_t r0 = 0; r0 < R; r0 += kRsRows) {
                const uint32_t nr = min((uint32_t)kRsRows, R - r0);
                __syncthreads();
                if (tid < kRsRows) rowid[tid] = tid < nr ? (uint32_t)((sk[r0 + tid] >> 21) & 0xffffffffull) : 0u;
                __syncthreads();
                const float sc = rerank16(a.rows, a.clen, a.norms, a.q, a.qlen, a.kind, rowid, nr, tile4, qs4);
                if (tid < nr)
                    __hip_atomic_store(a.rscores + r0 + tid, sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        ck[2] = wall_clock64();
    } else if (cnt <= a.bufcap) {
        // candidates j = 16 (blockIdx.x - 1) + 16 G i: their exact scores
        const uint32_t G = gridDim.x - 1;
        for (uint32_t j0 = (blockIdx.x - 1) * kRsRows; j0 < cnt; j0 += G * kRsRows) {
            const uint32_t nr = min((uint32_t)kRsRows, cnt - j0);
            __syncthreads();
            if (tid < kRsRows) rowid[tid] = tid < nr ? (uint32_t)a.buf[j0 + tid] : 0u;
            __syncthreads();
            const float sc = rerank16(a.rows, a.clen, a.norms, a.q, a.qlen, a.kind, rowid, nr, tile4, qs4,
                                      &t_staged);
            if (tid < nr) __hip_atomic_store(a.scores + j0 + tid, sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        ck[1] = t_staged;
        ck[2] = wall_clock64();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const uint32_t t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = t == gridDim.x - 1;
        s_nan = 0u;
    }
    __syncthreads();
    ck[3] = wall_clock64();
    if (a.clk && tid == 0 && blockIdx.x <= 1)
        for (int i = 0; i < 4; ++i) a.clk[blockIdx.x * 4 + i] = ck[i];
    if (!s_last) return;
    // the last block: stable sort of the top-R by exact score (ties: stage-1 rank)
    for (uint32_t i = tid; i < R; i += 256)
        sk[i] = __hip_atomic_load(a.topr + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    uint64_t* fk = (uint64_t*)tile4;                  // R <= kSortLdsCap keys (32 KiB of the tile region)
    float* fsc = (float*)(fk + kSortLdsCap);          // R scores (16 KiB after them)
    for (uint32_t i = tid; i < R; i += 256) {
        const uint32_t idx = (uint32_t)(sk[i] & kNoIdx);
        const float f = __hip_atomic_load(idx == kNoIdx ? a.rscores + i : a.scores + idx, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
        if (f != f) s_nan = 1u;
        uint32_t o = f32_order(f);
        if (a.descending) o = ~o;
        fk[i] = ((uint64_t)o << 32) | i;  // ties: stage-1 rank
        fsc[i] = f;
    }
    __syncthreads();
    select_sort(fk, R, (uint64_t*)hist);  // hist (>= 4 KiB free now) as the rank-sort scratch
    ck[4] = wall_clock64();
    const uint32_t take = a.kout < R ? a.kout : R;
    if (tid < 64) {  // take(k) then drop orphan rows (index.rs:217-228), order-preserving
        uint32_t o = 0;
        for (uint32_t i0 = 0; i0 < take; i0 += 64) {
            const uint32_t i = i0 + tid;
            uint64_t id = kOrphan;
            uint32_t rank = 0;
            if (i < take) {
                rank = (uint32_t)fk[i];
                const uint32_t row = (uint32_t)((sk[rank] >> 21) & 0xffffffffull);
                id = a.ids ? a.ids[row] : (uint64_t)row + a.row_offset;
            }
            const bool keep = i < take && id != kOrphan;
            const uint64_t m = __ballot(keep);
            const uint32_t before = __popcll(m & ((1ull << tid) - 1ull));
            if (keep) {
                a.out_ids[o + before] = id;
                a.out_scores[o + before] = fsc[rank];
            }
            o += __popcll(m);
        }
        if (tid == 0 && a.out_n) a.out_n[0] = (s_nan && R >= 2) ? GVDB_N_POISONED : o;
    }
    // self-cleaning for the next call (visible to it across the kernel boundary)
    for (uint32_t i = tid; i <= a.D; i += 256) a.hist[i] = 0u;
    if (tid == 0) {
        *(uint32_t*)a.counts = 0u;
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.clk) {
            ck[5] = wall_clock64();
            for (int i = 0; i < 6; ++i) a.clk[8 + i] = ck[i];
            a.clk[14] = cnt;
        }
    }
}

size_t b1_tail_lds(uint32_t D) {
    return (size_t)kSelectLdsCap * 8u + (size_t)((D + 4u) & ~3u) * 4u + 2048u * 4u +
           (size_t)(kRsRows * (kRsMaxLen / 4 + 1) + kRsMaxLen / 4) * 16u;
}

hipError_t launch_b1_search(const B1Args& b, hipStream_t s) {
    const uint32_t W4 = code_w4(b.D);
    if (b.ev) (void)hipEventRecord(b.ev[0], s);
    switch (W4) {
#define GVDB_CASE(w)                                                                                            \
    case w:                                                                                                     \
        hipLaunchKernelGGL((k_b1_sample<w>), dim3(b.sample_chunks), dim3(256), 0, s, b.codes, b.cap, b.N, b.D, \
                           b.sample_stride, b.q, b.thr, b.target, b.qwords, b.hist);                           \
        break;
        GVDB_CASE(1) GVDB_CASE(2) GVDB_CASE(3) GVDB_CASE(4) GVDB_CASE(6) GVDB_CASE(8)
#undef GVDB_CASE
        default: return hipErrorInvalidValue;
    }
    GVDB_LAUNCH_CHECK();
    if (b.ev) (void)hipEventRecord(b.ev[1], s);
    switch (W4) {
#define GVDB_CASE(w, cpl)                                                                                        \
    case w:                                                                                                      \
        hipLaunchKernelGGL((k_b1_scan<w, cpl>), dim3((uint32_t)((b.N + 256ull * cpl - 1) / (256ull * cpl))),    \
                           dim3(256), 0, s, b.codes, b.cap, b.N, b.D, b.qwords, b.hist, b.target, b.counts, b.buf, \
                           b.bufcap);                                                                            \
        break;
        GVDB_CASE(1, 8) GVDB_CASE(2, 8) GVDB_CASE(3, 8) GVDB_CASE(4, 4) GVDB_CASE(6, 4) GVDB_CASE(8, 2)
#undef GVDB_CASE
    }
    GVDB_LAUNCH_CHECK();
    if (b.ev) {
        (void)hipEventRecord(b.ev[2], s);
        (void)hipEventRecord(b.ev[3], s);
    }
    B1TailArgs t{};
    t.counts = b.counts;
    t.buf = b.buf;
    t.bufcap = b.bufcap;
    t.D = b.D;
    t.R = b.R;
    t.N = b.N;
    t.W4 = W4;
    t.kout = b.kout;
    t.codes = b.codes;
    t.cap = b.cap;
    t.qwords = b.qwords;
    t.rows = b.rows;
    t.clen = b.clen;
    t.norms = b.norms;
    t.q = b.q;
    t.qlen = b.qlen;
    t.kind = b.kind;
    t.descending = b.descending;
    t.force_rescan = b.force_rescan;
    t.ids = b.ids;
    t.row_offset = b.row_offset;
    t.scores = b.scores;
    t.rscores = b.rscores;
    t.topr = b.topr;
    t.ticket = b.ticket;
    t.rescans = b.rescans;
    t.hist = b.hist;
    t.out_ids = b.out_ids;
    t.out_scores = b.out_scores;
    t.out_n = b.out_n;
    t.clk = b.clk;
    const uint32_t G = std::min<uint32_t>((b.bufcap + kRsRows - 1) / kRsRows, kB1RerankBlocks);
    hipLaunchKernelGGL(k_b1_tail, dim3(1 + G), dim3(256), b1_tail_lds(b.D), s, t);
    GVDB_LAUNCH_CHECK();
    return hipSuccess;
}

}  // namespace gvdb

