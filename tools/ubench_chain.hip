// Latency of dependent VALU chains on gfx950 (s_memtime cycles per step, one wave).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ uint32_t f16_mad(uint32_t vbits, float vs, uint32_t ybits) {
    float t;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(vbits), "v"(vs), "v"(ybits));
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}

template <int MODE>
__global__ void k_chain(const uint32_t * in, float * out, unsigned long long * cyc, int n) {
    uint32_t v = in[threadIdx.x], y = 0, y2 = 0;
    float vs = 0.001f * threadIdx.x, f = 1.0f, S = 0.f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if constexpr (MODE == 0) { y = f16_mad(v, vs, y); }
            if constexpr (MODE == 1) { y = f16_mad(v, vs, y); S += vs; }
            if constexpr (MODE == 2) { y = f16_mad(v, vs, y); y2 = f16_mad(v + 1, vs, y2); }
            if constexpr (MODE == 3) { asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f) : "v"(vs), "v"(vs)); }
            if constexpr (MODE == 4) { asm volatile("v_cvt_f16_f32 %0, %0" : "+v"(y)); }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = (float) y + (float) y2 + f + S;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    uint32_t * in; float * out; unsigned long long * cyc;
    hipMalloc(&in, 1024 * 4); hipMemset(in, 0x3c, 1024 * 4);
    hipMalloc(&out, 1024 * 4); hipMalloc(&cyc, 8);
    const int n = 4096;
    const char * names[] = {"fma_mix+cvt", "fma_mix+cvt + add", "2 chains fma_mix+cvt", "v_fma_f32", "v_cvt_f16_f32"};
    for (int threads : {64, 256}) {
        for (int m = 0; m < 5; ++m) {
            for (int rep = 0; rep < 2; ++rep) {
                switch (m) {
                    case 0: hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(threads), 0, 0, in, out, cyc, n); break;
                    case 1: hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(threads), 0, 0, in, out, cyc, n); break;
                    case 2: hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(threads), 0, 0, in, out, cyc, n); break;
                    case 3: hipLaunchKernelGGL(k_chain<3>, dim3(1), dim3(threads), 0, 0, in, out, cyc, n); break;
                    case 4: hipLaunchKernelGGL(k_chain<4>, dim3(1), dim3(threads), 0, 0, in, out, cyc, n); break;
                }
                hipDeviceSynchronize();
            }
            unsigned long long c;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("threads %3d  %-24s %.2f ticks/step\n", threads, names[m], (double) c / n);
        }
    }
    return 0;
}
