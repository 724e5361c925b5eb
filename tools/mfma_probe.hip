// mfma_probe.hip — gfx950 int8 MFMA facts the prefill kernel relies on, measured:
//   1. the lane map of v_mfma_i32_16x16x64_i8 with exact integer data (A[16][64], B[64][16]),
//      candidate: lane l holds A[row l&15][k 16(l>>4)+j], B[k 16(l>>4)+j][col l&15], j < 16;
//      C[row 4(l>>4)+i][col l&15] (the 16x16 C map of every dtype);
//   2. cycles per instruction, back-to-back on one SIMD (one wave per SIMD, 4 independent
//      accumulators) for v_mfma_i32_16x16x32_i8 and v_mfma_i32_16x16x64_i8.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v4x __attribute__((ext_vector_type(4)));   // 16 int8 per lane

__global__ void k_layout64(const signed char * A, const signed char * B, int * C) {
    const int l = threadIdx.x;
    int a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    for (int j = 0; j < 16; ++j) {
        a[j / 4] |= (int) (unsigned char) A[(l & 15) * 64 + 16 * (l >> 4) + j] << (8 * (j % 4));
        b[j / 4] |= (int) (unsigned char) B[(16 * (l >> 4) + j) * 16 + (l & 15)] << (8 * (j % 4));
    }
    v4x av = {a[0], a[1], a[2], a[3]}, bv = {b[0], b[1], b[2], b[3]};
    v4i acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

template <int X64>
__global__ void k_rate(int iters, int * out, long long * cyc) {
    const int l = threadIdx.x;
    v4i c0 = {l, 0, 0, 0}, c1 = {0, l, 0, 0}, c2 = {0, 0, l, 0}, c3 = {0, 0, 0, l};
    const long a = 0x0102030405060708L + l, b = 0x0807060504030201L - l;
    const v4x av = {l, 2 * l, 3, 4}, bv = {5, l, 7, 8};
    const long long t0 = clock64();
    for (int i = 0; i < iters; ++i) {
        if constexpr (X64) {
            c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c3, 0, 0, 0);
        } else {
            c0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, c3, 0, 0, 0);
        }
    }
    const long long t1 = clock64();
    out[blockIdx.x * 64 + l] = c0[0] + c1[1] + c2[2] + c3[3];
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    signed char hA[1024], hB[1024];
    int ref[256], hC[256];
    srand(1);
    for (int i = 0; i < 1024; ++i) { hA[i] = (signed char) (rand() % 255 - 127); hB[i] = (signed char) (rand() % 255 - 127); }
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            int s = 0;
            for (int kk = 0; kk < 64; ++kk) s += hA[r * 64 + kk] * hB[kk * 16 + c];
            ref[r * 16 + c] = s;
        }
    signed char *dA, *dB; int * dC;
    hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dC, 1024);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_layout64, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += hC[i] != ref[i];
    printf("mfma_i32_16x16x64_i8 layout (k = 16(l>>4)+j): %d / 256 mismatches\n", bad);

    int * dout; long long * dcyc;
    hipMalloc(&dout, 4 * 64 * 4); hipMalloc(&dcyc, 4 * 8);
    const int iters = 4096;
    for (int x64 = 0; x64 < 2; ++x64) {
        for (int rep = 0; rep < 2; ++rep) {
            if (x64) hipLaunchKernelGGL(k_rate<1>, dim3(1), dim3(64), 0, 0, iters, dout, dcyc);
            else hipLaunchKernelGGL(k_rate<0>, dim3(1), dim3(64), 0, 0, iters, dout, dcyc);
        }
        long long cyc = 0;
        hipMemcpy(&cyc, dcyc, 8, hipMemcpyDeviceToHost);
        printf("v_mfma_i32_16x16x%d_i8: %.2f clock64 ticks per MFMA (one wave, 4 accumulators)\n", x64 ? 64 : 32,
               (double) cyc / (4.0 * iters));
    }
    return bad != 0;
}
