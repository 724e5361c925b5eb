// Dependent latency of single VALU ops on one wave (s_memtime cycles per op, chains unrolled by 8):
// which ops an exact f16 recurrence step could be built from.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ void probe(const float * g, unsigned long long * out, uint32_t * sink, int n) {
    const int lane = threadIdx.x;
    float x = g[lane], a = g[lane + 64], b = g[lane + 128];
    uint32_t u = __float_as_uint(x), ua = __float_as_uint(a);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
    for (int j = 0; j < n; ++j) {
        if (MODE == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b));
        else if (MODE == 1) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(ua), "v"(b));
        else if (MODE == 2) asm volatile("v_cvt_f16_f32 %0, %0" : "+v"(u));
        else if (MODE == 3) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(u));
        else if (MODE == 4) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u) : "v"(ua));
        else if (MODE == 5) asm volatile("v_bfe_u32 %0, %0, 13, 1" : "+v"(u));
        else if (MODE == 6) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u) : "v"(ua));
        else if (MODE == 7) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(u) : "v"(ua));
        else if (MODE == 8) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(u) : "v"(ua), "v"(b));
        else asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[MODE] = t1 - t0;
    sink[lane] = u ^ __float_as_uint(x);
}
int main() {
    const int n = 8192;
    float * g; unsigned long long * out; uint32_t * sink;
    hipMalloc(&g, 192 * 4); hipMalloc(&out, 16 * 8); hipMalloc(&sink, 256);
    hipMemset(g, 0, 192 * 4);
    unsigned long long h[10];
    const char * names[10] = {"v_fma_f32", "v_fma_mix_f32 (f32 acc)", "v_cvt_f16_f32", "v_cvt_f32_f16", "v_add_u32", "v_bfe_u32",
                              "v_and_b32", "v_add3_u32", "v_fma_mix_f32 (f16 acc)", "v_mul_f32"};
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<4>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<5>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<6>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<7>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<8>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<9>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipDeviceSynchronize();
        hipMemcpy(h, out, 80, hipMemcpyDeviceToHost);
    }
    for (int m = 0; m < 10; ++m) printf("%-26s %.1f cycles per dependent op\n", names[m], h[m] / (double) n);
    return 0;
}
