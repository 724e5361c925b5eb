// Dependent-chain cycles per step of exact forms of y = f16(f32(fma(v, vs, y))) on one wave
// (s_memtime, loops unrolled by 8): which instruction sequence is shortest.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t step_mix(uint32_t vbits, float vs, uint32_t ybits) {
    float t;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(vbits), "v"(vs), "v"(ybits));
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}
// y held as f16 bits: widen, f32 fma, narrow
__device__ __forceinline__ uint32_t step_f32(float vf, float vs, uint32_t ybits) {
    float yf, t;
    asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(yf) : "v"(ybits));
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(t) : "v"(vf), "v"(vs), "v"(yf));
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}
// y held as f32 (always an f16 value): f32 fma, narrow, widen
__device__ __forceinline__ float step_f32b(float vf, float vs, float yf) {
    float t;
    asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(t) : "v"(vf), "v"(vs), "v"(yf));
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    float o;
    asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(o) : "v"(r));
    return o;
}
// v_fma_mix with y as f32 operand
__device__ __forceinline__ float step_mixf(uint32_t vbits, float vs, float yf) {
    float t;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(t) : "v"(vbits), "v"(vs), "v"(yf));
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    float o;
    asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(o) : "v"(r));
    return o;
}
template <int MODE>
__global__ void probe(const float * g, unsigned long long * out, uint32_t * sink, int n) {
    const int lane = threadIdx.x;
    const float vs = g[lane], vf = g[lane + 64];
    const uint32_t vb = __float_as_uint(g[lane + 128]) & 0xffff;
    uint32_t y = 0;
    float yf = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
    for (int j = 0; j < n; ++j) {
        if (MODE == 0) y = step_mix(vb, vs, y);
        else if (MODE == 1) y = step_f32(vf, vs, y);
        else if (MODE == 2) yf = step_f32b(vf, vs, yf);
        else yf = step_mixf(vb, vs, yf);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[MODE] = t1 - t0;
    sink[lane] = y ^ __float_as_uint(yf);
}
int main() {
    const int n = 8192;
    float * g; unsigned long long * out; uint32_t * sink;
    hipMalloc(&g, 192 * 4); hipMalloc(&out, 64); hipMalloc(&sink, 256);
    hipMemset(g, 0, 192 * 4);
    unsigned long long h[4];
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(probe<0>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipLaunchKernelGGL(probe<3>, dim3(1), dim3(64), 0, 0, g, out, sink, n);
        hipDeviceSynchronize();
        hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
    }
    printf("cycles per step: mix+cvt %.1f | cvt32+fma+cvt16 %.1f | fma+cvt16+cvt32 %.1f | mix(f32 y)+cvt16+cvt32 %.1f\n",
           h[0] / (double) n, h[1] / (double) n, h[2] / (double) n, h[3] / (double) n);
    return 0;
}
