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

__device__ __forceinline__ uint32_t next_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace gvdb
