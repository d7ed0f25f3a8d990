// FP4 MFMA ceiling probe (tools only, not product): what the stage-1 scan's
// MFMA loop can reach on this part, with the clock measured in-kernel
// (s_memtime cycles / s_memrealtime 100 MHz ticks on wave 0 of block 0).
//   pure   : 8 independent accumulators, v_mfma_scale_f32_32x32x64_f8f6f4 (fp4) back to back
//   lds    : + one ds_read_b128 A fragment per MFMA (ring of 4, as k_scan_mx5)
//   lds2   : + one ds_read_b128 per TWO MFMAs (as k_scan_mx6)
//   valu   : lds + 5 VALU per 8 MFMAs (the row-fragment expansion)
// One 512-thread block per CU (2 waves per SIMD), like the scan.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mfma(v16f& d, const v4i& a, const v4i& b, int sc) {
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                 : "+v"(d)
                 : "v"(a), "v"(b), "v"(sc));
}

template <int MODE>
__global__ __launch_bounds__(512, 1) void k_probe(int iters, float* out, unsigned long long* clk) {
    __shared__ v4i lds[8 * 64 * 12];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 8 * 64 * 12; i += 512) lds[i] = v4i{i * 0x01010101, i ^ 0x22222222, i, 0x11111111};
    __syncthreads();
    unsigned long long t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && tid == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    v16f acc[8];
    for (int t = 0; t < 8; ++t) acc[t] = v16f{0};
    v4i b = v4i{0x22222222 ^ lane, 0x11111111, 0x44444444, lane};
    v4i a = b;
    const int sc = 0x7f7f7f7f;
    const v4i* qf = lds + lane;
    uint32_t w = lane * 2654435761u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 12; ++s) {
            v4i ar[4];
            if (MODE >= 1) {
#pragma unroll
                for (int m = 0; m < 4; ++m) ar[m] = qf[((s * 8 + m) % 96) * 64];
            }
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                v4i x = a;
                if (MODE == 1 || MODE == 3) {
                    x = ar[t & 3];
                    if (t + 4 < 8) ar[t & 3] = qf[((s * 8 + t + 4) % 96) * 64];
                } else if (MODE == 2) {
                    x = ar[(t >> 1) & 3];
                }
                mfma(acc[t], x, b, sc);
                if (MODE == 3 && t == 1) {
                    w = w * 1664525u + 1013904223u;
                    b = v4i{(int)(w & 0x11111111u), (int)(w & 0x22222222u), (int)(w & 0x44444444u),
                            (int)((w >> 1) & 0x44444444u)};
                }
            }
        }
    }
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
    float s = 0;
    for (int t = 0; t < 8; ++t)
        for (int r = 0; r < 16; ++r) s += acc[t][r];
    if (s == 1.2345f) out[blockIdx.x * 512 + tid] = s;
    __syncthreads();
    if (blockIdx.x == 0 && tid == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int MODE>
static void run(const char* name, int cus, float* out, unsigned long long* clk) {
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k_probe<MODE>, dim3(cus), dim3(512), 0, 0, iters, out, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long h[2];
        hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
        const double mfmas = (double)cus * 8 * iters * 12 * 8;  // waves x MFMAs per wave
        const double tflops = mfmas * 32 * 32 * 64 * 2 / (ms * 1e-3) / 1e12;
        const double ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 0.0;
        const double cyc_per_mfma = ghz * 1e9 * ms * 1e-3 / (mfmas / (cus * 4.0));
        printf("%-6s %8.3f ms  %7.1f TFLOP/s  clock %.3f GHz  %.1f cycles per MFMA per SIMD\n", name, ms, tflops, ghz,
               cyc_per_mfma);
    }
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, (size_t)cus * 512 * 4);
    hipMalloc(&clk, 16);
    run<0>("pure", cus, out, clk);
    run<1>("lds", cus, out, clk);
    run<2>("lds2", cus, out, clk);
    run<3>("valu", cus, out, clk);
    return 0;
}
