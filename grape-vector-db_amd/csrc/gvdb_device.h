// gvdb_device.h — device helpers shared by the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gvdb {

#define GVDB_LAUNCH_CHECK() \
    do {                    \
        hipError_t e__ = hipGetLastError(); \
        if (e__ != hipSuccess) return e__;  \
    } while (0)

// Device-side tier gate of the host-sync-free searches: a fallback tier is
// enqueued unconditionally behind the tier it backs up, with that tier's
// failure word as its gate; while the word is 0 (the earlier tier certified
// its batch) every block of the fallback returns at once.  nullptr = ungated.
// (Written by an earlier kernel of the same stream: visible at kernel start.)
__device__ __forceinline__ bool gate_closed(const uint32_t* gate) { return gate && *gate == 0u; }

// Total order key for f32 scores: -0.0 == +0.0 (Rust partial_cmp), ascending.
__device__ __forceinline__ uint32_t f32_order(float f) {
    uint32_t u = __float_as_uint(f);
    if (u == 0x80000000u) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// In-LDS bitonic sort (ascending) of P = power-of-two u64 keys by a whole
// workgroup.  Each stage walks the P/2 compare-exchange PAIRS (lo has bit j
// clear, hi = lo | j), so no thread iteration is spent on the idle half.
__device__ inline void bitonic_sort_lds(uint64_t* s, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t p = threadIdx.x; p < P / 2; p += blockDim.x) {
                const uint32_t lo = ((p & ~(j - 1)) << 1) | (p & (j - 1));
                const uint32_t hi = lo | j;
                const uint64_t a = s[lo], b = s[hi];
                const bool up = (lo & k) == 0;
                if ((a > b) == up) {
                    s[lo] = b;
                    s[hi] = a;
                }
            }
            __syncthreads();
        }
    }
}

__host__ __device__ __forceinline__ uint32_t next_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Smallest t in [0, nb) with sum(h[0..t]) >= target (nb-1 if never), by one
// full wave: each lane sums a contiguous segment, a shuffle scan finds the
// segment that crosses the target, that lane walks its segment.
__device__ inline uint32_t wave_find_cum(const uint32_t* h, uint32_t nb, uint32_t target) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t seg = (nb + 63u) / 64u;
    const uint32_t b0 = lane * seg;
    const uint32_t b1 = min(b0 + seg, nb);
    uint32_t s = 0;
    for (uint32_t i = b0; i < b1; ++i) s += h[i];
    uint32_t incl = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off);
        if ((int)lane >= off) incl += v;
    }
    const uint64_t m = __ballot(incl >= target);
    if (m == 0) return nb - 1;
    const uint32_t first = __ffsll((long long)m) - 1;
    uint32_t t = nb - 1;
    if (lane == first) {
        uint32_t cum = incl - s;
        for (uint32_t i = b0; i < b1; ++i) {
            cum += h[i];
            if (cum >= target) {
                t = i;
                break;
            }
        }
    }
    return __shfl(t, first);
}

// Sum of h[0..t) by one full wave.
__device__ inline uint32_t wave_sum_below(const uint32_t* h, uint32_t t) {
    uint32_t s = 0;
    for (uint32_t i = threadIdx.x & 63u; i < t; i += 64) s += h[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    return s;
}

// Block-wide exclusive prefix of a flag in thread order; *total = block count.
__device__ __forceinline__ uint32_t big_prefix(bool f, uint32_t* wcnt, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint64_t m = __ballot(f);
    if (lane == 0) wcnt[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), tot = 0;
    for (uint32_t i = 0; i < nw; ++i) {
        const uint32_t c = wcnt[i];
        if (i < w) pre += c;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return pre;
}

// Block-wide exclusive prefix of a per-thread count in thread order; *total = the block sum.
// wsum: [blockDim.x / 64] LDS words.
__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t* wsum, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
        if ((int)lane >= off) incl += y;
    }
    if (lane == 63u) wsum[w] = incl;
    __syncthreads();
    uint32_t pre = incl - v, tot = 0;
    for (uint32_t i = 0; i < nw; ++i) {
        const uint32_t c = wsum[i];
        if (i < w) pre += c;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return pre;
}

}  // namespace gvdb
