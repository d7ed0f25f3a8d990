// Batch-1 scan probe (tools only, not product): the k_b1_scan access pattern
// (W4 = 6 uint4 planes of N = 10M codes, 960 MB, one query) under different
// launch geometries, to find the HBM-streaming optimum for the batch-1 pass.
//   grid  : one block per 256*CPL rows (CPL = 2, 4, 8)
//   persist: G = k * CUs blocks looping over 256*CPL-row tiles (k = 1, 2, 4),
//            next tile's loads issued before the current tile's popcounts
//   nt    : as grid CPL=4 with non-temporal loads
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
__device__ __forceinline__ uint32_t ham4(const uint4& c, const uint4& q, uint32_t acc) {
    acc = bcnt_acc(c.x ^ q.x, acc);
    acc = bcnt_acc(c.y ^ q.y, acc);
    acc = bcnt_acc(c.z ^ q.z, acc);
    return bcnt_acc(c.w ^ q.w, acc);
}

template <int CPL, bool NT>
__global__ __launch_bounds__(256) void k_grid(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                              const uint4* __restrict__ qc, uint32_t T, uint32_t* cnt) {
    constexpr int W4 = 6;
    const uint64_t base = (uint64_t)blockIdx.x * (256u * CPL);
    uint4 c[CPL][W4];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        uint64_t n = base + (uint64_t)k * 256u + threadIdx.x;
        if (n >= N) n = N - 1;
#pragma unroll
        for (int w = 0; w < W4; ++w)
        {
            typedef unsigned int u4v __attribute__((ext_vector_type(4)));
            if (NT) {
                const u4v v = __builtin_nontemporal_load((const u4v*)(codes + (uint64_t)w * cap + n));
                c[k][w] = make_uint4(v.x, v.y, v.z, v.w);
            } else {
                c[k][w] = codes[(uint64_t)w * cap + n];
            }
        }
    }
    uint4 q[W4];
#pragma unroll
    for (int w = 0; w < W4; ++w) q[w] = qc[w];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        uint32_t d = 0;
#pragma unroll
        for (int w = 0; w < W4; ++w) d = ham4(c[k][w], q[w], d);
        if (d <= T) atomicAdd(cnt, 1u);
    }
}

template <int CPL>
__global__ __launch_bounds__(256) void k_persist(const uint4* __restrict__ codes, uint64_t cap, uint32_t N,
                                                 const uint4* __restrict__ qc, uint32_t T, uint32_t* cnt) {
    constexpr int W4 = 6;
    const uint32_t tiles = (N + 256u * CPL - 1) / (256u * CPL);
    uint4 q[W4];
#pragma unroll
    for (int w = 0; w < W4; ++w) q[w] = qc[w];
    uint4 c[CPL][W4], nx[CPL][W4];
    uint32_t t = blockIdx.x;
    auto load = [&](uint4 (&dst)[CPL][W4], uint32_t tile) {
        const uint64_t base = (uint64_t)tile * (256u * CPL);
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            uint64_t n = base + (uint64_t)k * 256u + threadIdx.x;
            if (n >= N) n = N - 1;
#pragma unroll
            for (int w = 0; w < W4; ++w) dst[k][w] = codes[(uint64_t)w * cap + n];
        }
    };
    if (t < tiles) load(c, t);
    for (; t < tiles; t += gridDim.x) {
        const uint32_t tn = t + gridDim.x;
        if (tn < tiles) load(nx, tn);
        uint32_t hits = 0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            uint32_t d = 0;
#pragma unroll
            for (int w = 0; w < W4; ++w) d = ham4(c[k][w], q[w], d);
            hits += d <= T;
        }
        if (hits) atomicAdd(cnt, hits);
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int w = 0; w < W4; ++w) c[k][w] = nx[k][w];
    }
}

int main() {
    const uint32_t N = 10000000;
    const uint64_t cap = N;
    uint4 *codes, *qc;
    uint32_t* cnt;
    if (hipMalloc(&codes, cap * 6 * 16) != hipSuccess || hipMalloc(&qc, 6 * 16) != hipSuccess ||
        hipMalloc(&cnt, 4) != hipSuccess)
        return 1;
    hipMemset(codes, 0x5a, cap * 6 * 16);
    hipMemset(qc, 0x33, 6 * 16);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const double bytes = (double)N * 96.0;
    auto run = [&](const char* name, auto launch) {
        float best = 1e9f, sum = 0;
        for (int rep = 0; rep < 25; ++rep) {
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep >= 5) {
                sum += ms;
                if (ms < best) best = ms;
            }
        }
        printf("%-22s avg %.1f us  best %.1f us  %.0f GB/s (avg)\n", name, 1e3 * sum / 20, 1e3 * best,
               bytes / (sum / 20 * 1e-3) / 1e9);
    };
#define GRID(CPL, NT, NAME) \
    run(NAME, [&] { hipLaunchKernelGGL((k_grid<CPL, NT>), dim3((N + 256 * CPL - 1) / (256 * CPL)), dim3(256), 0, 0, codes, cap, N, qc, 300u, cnt); })
    GRID(2, false, "grid CPL=2");
    GRID(4, false, "grid CPL=4");
    GRID(8, false, "grid CPL=8");
    GRID(4, true, "grid CPL=4 nt");
    GRID(8, true, "grid CPL=8 nt");
#define PERS(CPL, K, NAME) \
    run(NAME, [&] { hipLaunchKernelGGL((k_persist<CPL>), dim3(K * cus), dim3(256), 0, 0, codes, cap, N, qc, 300u, cnt); })
    PERS(2, 2, "persist CPL=2 x2/CU");
    PERS(2, 4, "persist CPL=2 x4/CU");
    PERS(4, 1, "persist CPL=4 x1/CU");
    PERS(4, 2, "persist CPL=4 x2/CU");
    PERS(4, 3, "persist CPL=4 x3/CU");
    return 0;
}
