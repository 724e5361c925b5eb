// mfma_layout.hip — checks the lane maps of v_mfma_i32_16x16x32_i8 on gfx950 with exact
// integer data: A[16][32], B[32][16] (int8), C = A.B (int32), assuming
//   lane l: A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15], C[row 4(l>>4)+i][col l&15]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k(const signed char * A, const signed char * B, int * C) {
    const int l = threadIdx.x;
    long a = 0, b = 0;
    for (int j = 0; j < 8; ++j) {
        a |= (long) (unsigned char) A[(l & 15) * 32 + 8 * (l >> 4) + j] << (8 * j);
        b |= (long) (unsigned char) B[(8 * (l >> 4) + j) * 16 + (l & 15)] << (8 * j);
    }
    v4i acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, b, acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

int main() {
    signed char hA[512], hB[512];
    int ref[256], hC[256];
    srand(1);
    for (int i = 0; i < 512; ++i) { hA[i] = (signed char) (rand() % 255 - 127); hB[i] = (signed char) (rand() % 255 - 127); }
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            int s = 0;
            for (int kk = 0; kk < 32; ++kk) s += hA[r * 32 + kk] * hB[kk * 16 + c];
            ref[r * 16 + c] = s;
        }
    signed char *dA, *dB; int * dC;
    hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dC, 1024);
    hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += hC[i] != ref[i];
    printf("mfma_i32_16x16x32_i8 layout check: %d / 256 mismatches\n", bad);
    return bad != 0;
}
