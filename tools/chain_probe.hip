// Cycles per step of the f16 VKQ recurrence on one wave (s_memtime): (a) registers only:
// y = f16(fma_mix(v, vs, y)); (b) + S += vs; (c) + V and vs read from LDS 8 steps ahead (the dsh
// chain's fast batch); (d) two dims per lane (packed cvt).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mad(uint32_t vbits, float vs, uint32_t ybits) {
    float t;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(vbits), "v"(vs), "v"(ybits));
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}
template <int MODE>
__global__ void probe(const uint16_t * vg, const float * sg, unsigned long long * out, uint32_t * sink, int n) {
    __shared__ uint16_t vl[1024 * 64];
    __shared__ float sl[4096 + 16];
    const int lane = threadIdx.x;
    for (int j = lane; j < 1024 * 64; j += 64) vl[j] = vg[j];
    for (int j = lane; j < 4096; j += 64) sl[j] = sg[j];
    __syncthreads();
    uint32_t y = 0, y2 = 0;
    float S = 0.f;
    const uint32_t v0 = vg[lane];
    const float s0 = sg[lane];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0) {
        for (int j = 0; j < n; ++j) y = mad(v0, s0, y);
    } else if (MODE == 1) {
        for (int j = 0; j < n; ++j) { y = mad(v0, s0, y); S = __fadd_rn(S, s0); }
    } else if (MODE == 2) {
        for (int j0 = 0; j0 < n; j0 += 8) {
            uint32_t vv[8]; float vs[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) { vv[u] = vl[((j0 + u) & 1023) * 64 + lane]; vs[u] = sl[j0 + u]; }
#pragma unroll
            for (int u = 0; u < 8; ++u) { y = mad(vv[u], vs[u], y); S = __fadd_rn(S, vs[u]); }
        }
    } else {
        for (int j = 0; j < n; ++j) { y = mad(v0, s0, y); y2 = mad(v0 >> 16, s0, y2); S = __fadd_rn(S, s0); }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[MODE] = t1 - t0;
    sink[lane] = y ^ y2 ^ __float_as_uint(S);
}
int main() {
    const int n = 4096;
    uint16_t * vg; float * sg; unsigned long long * out; uint32_t * sink;
    hipMalloc(&vg, 4096 * 64 * 2); hipMalloc(&sg, 4096 * 4); hipMalloc(&out, 64); hipMalloc(&sink, 256);
    hipMemset(vg, 0x3c, 4096 * 64 * 2); hipMemset(sg, 0, 4096 * 4);
    unsigned long long h[4];
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, vg, sg, out, sink, n);
        hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, vg, sg, out, sink, n);
        hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, vg, sg, out, sink, n);
        hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, vg, sg, out, sink, n);
        hipDeviceSynchronize();
        hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
    }
    printf("cycles per step: mad only %.1f | mad + S %.1f | LDS batch of 8 + mad + S %.1f | two dims + S %.1f\n",
           h[0] / (double) n, h[1] / (double) n, h[2] / (double) n, h[3] / (double) n);
    return 0;
}
