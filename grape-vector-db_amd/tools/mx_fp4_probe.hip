// Probe: does v_mfma_scale_f32_32x32x64_f8f6f4 with fp4 (e2m1) operands and
// unit E8M0 scales compute exact +/-1 dot products when lane l feeds row/col
// (l & 31) with 32 values in dwords 0..3 (8 nibbles each), the same k-slot map
// for A and B?  Prints max |error| over random trials (expect 0).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void k(const uint32_t* abits, const uint32_t* bbits, float* out) {
    const int l = threadIdx.x;
    // row (l&31) of A / col (l&31) of B; 32 dims [32*(l>>5), +32) as one 32-bit word
    uint32_t wa = abits[(l & 31) * 2 + (l >> 5)];
    uint32_t wb = bbits[(l & 31) * 2 + (l >> 5)];
    v8i a = {0}, b = {0};
    for (int d = 0; d < 4; ++d) {
        uint32_t xa = 0, xb = 0;
        for (int j = 0; j < 8; ++j) {
            uint32_t ba = (wa >> (8 * d + j)) & 1u, bb = (wb >> (8 * d + j)) & 1u;
            xa |= (0x2u | (ba << 3)) << (4 * j);   // +1.0 = 0b0010, -1.0 = 0b1010
            xb |= (0x2u | (bb << 3)) << (4 * j);
        }
        a[d] = (int)xa;
        b[d] = (int)xb;
    }
    v16f acc = {0};
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
    for (int r = 0; r < 16; ++r) {
        const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
        out[row * 32 + col] = acc[r];
    }
}

int main() {
    std::vector<uint32_t> A(64), Bv(64);
    float* dout;
    uint32_t *da, *db;
    hipMalloc(&dout, 32 * 32 * 4);
    hipMalloc(&da, 256);
    hipMalloc(&db, 256);
    double maxerr = 0;
    srand(7);
    for (int trial = 0; trial < 20; ++trial) {
        for (auto& x : A) x = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
        for (auto& x : Bv) x = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
        hipMemcpy(da, A.data(), 256, hipMemcpyHostToDevice);
        hipMemcpy(db, Bv.data(), 256, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dout);
        std::vector<float> o(1024);
        hipMemcpy(o.data(), dout, 4096, hipMemcpyDeviceToHost);
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) {
                int ham = __builtin_popcount(A[i * 2] ^ Bv[j * 2]) + __builtin_popcount(A[i * 2 + 1] ^ Bv[j * 2 + 1]);
                double ref = 64 - 2 * ham;
                double e = o[i * 32 + j] - ref;
                if (e < 0) e = -e;
                if (e > maxerr) maxerr = e;
            }
    }
    printf("mx_fp4_probe max_abs_err=%g (%s)\n", maxerr, maxerr == 0 ? "EXACT" : "MISMATCH");
    return maxerr == 0 ? 0 : 1;
}
