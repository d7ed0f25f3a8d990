// Streaming-pattern probe for the K4 emit pass (tools only, not product):
// 10M x 768 bf16 rows in the fragment-major mirror (15.4 GB), read by 256
// blocks x 8 waves in the k_flat_mx order; variants isolate the access
// pattern from the MFMA/LDS work.
//   mode 0: each wave loads its pair's 8 KiB per step (pairs duplicate), no barrier
//   mode 1: as 0 with a barrier per step
//   mode 2: each wave loads a distinct 4 KiB per step, no barrier
//   mode 3: as 2 with a barrier per step
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef int v4i __attribute__((ext_vector_type(4)));
template <int MODE>
__global__ __launch_bounds__(512, 1) void k(const char* __restrict__ rows, uint32_t ntiles, uint32_t KC, int* out) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wr = wv >> 1, wq = wv & 1;
    const uint32_t G = gridDim.x;
    v4i acc = {0, 0, 0, 0};
    for (uint32_t t = blockIdx.x; t < ntiles; t += G) {
        for (uint32_t c = 0; c < KC; ++c) {
            const char* base = rows + ((uint64_t)t * KC + c) * 32768;
            v4i v[8];
            if (MODE <= 1) {
                const char* p = base + (2 * wr) * 4096 + lane * 16;
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = *(const v4i*)(p + (i >> 2) * 4096 + (i & 3) * 1024);
            } else {
                const char* p = base + wv * 4096 + lane * 16;
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = *(const v4i*)(p + i * 1024);
#pragma unroll
                for (int i = 4; i < 8; ++i) v[i] = v[i - 4];
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) acc ^= v[i];
            if (MODE & 1) __syncthreads();
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) out[0] = 1;
    (void)wq;
}
int main() {
    const uint64_t N = 10000000, KC = 12, ntiles = (N + 255) / 256;
    const uint64_t bytes = ntiles * KC * 32768;
    char* d;
    int* o;
    if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) return 1;
    hipMemset(d, 1, bytes);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 4; ++rep) {
            hipEventRecord(a);
            switch (mode) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(512), 0, 0, d, (uint32_t)ntiles, (uint32_t)KC, o); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(512), 0, 0, d, (uint32_t)ntiles, (uint32_t)KC, o); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(512), 0, 0, d, (uint32_t)ntiles, (uint32_t)KC, o); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(512), 0, 0, d, (uint32_t)ntiles, (uint32_t)KC, o); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep == 3) printf("mode %d: %.3f ms  %.0f GB/s\n", mode, ms, bytes / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
