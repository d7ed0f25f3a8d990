// Probe: sustained issue rate of the MFMA forms the scan kernels use, chip-wide
// (256 blocks x WAVES waves, back-to-back MFMAs on 2 accumulators, operands in
// registers).  Prints cycles per MFMA per SIMD (from wall time and the
// shader clock) and the achieved dense rate.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

constexpr int kIters = 2000;

template <int KIND>
__global__ __launch_bounds__(512) void k(float* out, int seed, unsigned long long* clk) {
    const int l = threadIdx.x;
    v4i a = {seed + l, seed ^ l, l * 3, l + 7};
    v4i b = {l, seed, l ^ 5, seed * 3};
    v16f acc0 = {0}, acc1 = {0};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
        if constexpr (KIND == 0) {  // fp4 32x32x64 block-scaled, inline asm (as the scan)
            asm volatile(
                "v_mfma_scale_f32_32x32x64_f8f6f4 %0, %2, %3, %0, %4, %4 op_sel_hi:[0,0,0] cbsz:4 blgp:4\n"
                "v_mfma_scale_f32_32x32x64_f8f6f4 %1, %2, %3, %1, %4, %4 op_sel_hi:[0,0,0] cbsz:4 blgp:4"
                : "+v"(acc0), "+v"(acc1)
                : "v"(a), "v"(b), "v"(0x7f7f7f7f));
        } else if constexpr (KIND == 1) {  // bf16 32x32x16
            v8bf ab = __builtin_bit_cast(v8bf, v4i{a.x, a.y, a.z, a.w});
            v8bf bb = __builtin_bit_cast(v8bf, v4i{b.x, b.y, b.z, b.w});
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ab, bb, acc1, 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int r = 0; r < 16; ++r) s += acc0[r] + acc1[r];
    out[blockIdx.x * 512 + l] = s;
    if (blockIdx.x == 0 && l == 0) clk[0] = t1 - t0;
}

template <int KIND>
void run(const char* name, double flops_per_mfma) {
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, 256 * 512 * 4);
    hipMalloc(&clk, 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k<KIND>, dim3(256), dim3(512), 0, 0, out, 1, clk);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<KIND>, dim3(256), dim3(512), 0, 0, out, 2, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c = 0;
    hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
    const double mfma_per_simd = 2.0 * kIters * 2;  // 2 waves per SIMD (8 waves / 4 SIMDs), 2 MFMAs per iter
    const double total = 256.0 * 8 * kIters * 2;
    printf("%-10s %.3f ms  %.1f cyc/MFMA/SIMD @2.4GHz  memtime %.1f clk/MFMA/wave  %.1f TFLOP/s\n", name, ms,
           ms * 1e-3 * 2.4e9 / mfma_per_simd, (double)c / (2.0 * kIters), total * flops_per_mfma / (ms * 1e-3) / 1e12);
}

int main() {
    run<0>("fp4", 2.0 * 32 * 32 * 64);
    run<1>("bf16", 2.0 * 32 * 32 * 16);
    return 0;
}
