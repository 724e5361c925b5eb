// Dependent latency on one wave, 32 dependent ops per loop iteration (the loop's own branch and
// scalar ops amortized): single ops, and the exact f16 recurrence step y = f16(f32 fma(v, vs, y))
// as v_fma_mix_f32 + v_cvt_f16_f32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define R4(x) x x x x
#define R32(x) R4(R4(x)) R4(R4(x))   // 32 copies

template <int MODE>
__global__ void probe(const float * g, unsigned long long * out, uint32_t * sink, int n) {
    const int lane = threadIdx.x;
    float x = g[lane], a = g[lane + 64], b = g[lane + 128];
    uint32_t u = __float_as_uint(x), ua = __float_as_uint(a);
    float t = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < n; ++j) {
        if (MODE == 0) asm volatile(R32("v_fma_f32 %0, %1, %2, %0\n") : "+v"(x) : "v"(a), "v"(b));
        else if (MODE == 1) asm volatile(R32("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]\n") : "+v"(x) : "v"(ua), "v"(b));
        else if (MODE == 2) asm volatile(R32("v_cvt_f16_f32 %0, %0\n") : "+v"(u));
        else if (MODE == 3) asm volatile(R32("v_add_u32 %0, %0, %1\n") : "+v"(u) : "v"(ua));
        else if (MODE == 4) asm volatile(R32("v_fma_mix_f32 %1, %2, %3, %0 op_sel_hi:[1,0,1]\nv_cvt_f16_f32 %0, %1\n") : "+v"(u), "+v"(t) : "v"(ua), "v"(b));
        else if (MODE == 5) asm volatile(R32("v_cvt_f32_f16 %1, %0\nv_fma_f32 %1, %2, %3, %1\nv_cvt_f16_f32 %0, %1\n") : "+v"(u), "+v"(t) : "v"(a), "v"(b));
        else asm volatile(R32("v_mul_f32 %0, %0, %1\n") : "+v"(x) : "v"(a));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[MODE] = t1 - t0;
    sink[lane] = u ^ __float_as_uint(x) ^ __float_as_uint(t);
}
int main() {
    const int n = 512;
    float * g; unsigned long long * out; uint32_t * sink;
    hipMalloc(&g, 192 * 4); hipMalloc(&out, 16 * 8); hipMalloc(&sink, 256);
    hipMemset(g, 0, 192 * 4);
    unsigned long long h[7];
    const char * names[7] = {"v_fma_f32", "v_fma_mix_f32 (f32 acc)", "v_cvt_f16_f32", "v_add_u32",
                             "STEP fma_mix + cvt_f16", "STEP cvt_f32 + fma + cvt_f16", "v_mul_f32"};
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<4>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<5>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<6>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipDeviceSynchronize();
        hipMemcpy(h, out, 56, hipMemcpyDeviceToHost);
    }
    for (int m = 0; m < 7; ++m) printf("%-32s %.1f cycles per dependent op / step\n", names[m], h[m] / (double) (n * 32));
    return 0;
}
