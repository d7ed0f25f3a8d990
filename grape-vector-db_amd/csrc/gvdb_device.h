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
// workgroup.
__device__ inline void bitonic_sort_lds(uint64_t* s, uint32_t P) {
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
                    }
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
