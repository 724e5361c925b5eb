// Is v_fma_mixlo_f16 (f16 result of a mixed-precision fma) bit-identical to the exact FA's
// two-step y = cvt_f16(fma_f32(v, vs, y)) (v_fma_mix_f32 + v_cvt_f16_f32, the CPU's
// ggml_vec_mad_f16 order: f32 fma, then round to f16)?  The two differ only if the hardware
// rounds the exact result straight to f16 (single rounding): the cases that tell them apart are
// fma results within half an f32 ulp of an f16 rounding midpoint.  The host builds such cases
// (y + v*vs aimed at a midpoint) plus uniformly random ones; the kernel evaluates both forms and
// counts mismatches.  Then the dependent-chain latency of one mixlo per step vs the two-step form.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

__device__ __forceinline__ uint32_t mad2(uint32_t v, float vs, uint32_t y) {
    float t;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(v), "v"(vs), "v"(y));
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r & 0xffff;
}
__device__ __forceinline__ uint32_t mad1(uint32_t v, float vs, uint32_t y) {
    uint32_t r = 0;
    asm volatile("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "+v"(r) : "v"(v), "v"(vs), "v"(y));
    return r & 0xffff;
}
// the rescale step y' = f16(y * ms): v_mul_f32 + cvt vs mixlo fma(y, ms, -0)
__device__ __forceinline__ uint32_t scl2(uint32_t y, float ms) {
    float t;
    asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(t) : "v"(y), "v"(ms), "v"(0x80000000u));
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r & 0xffff;
}
__device__ __forceinline__ uint32_t scl1(uint32_t y, float ms) {
    uint32_t r = 0;
    asm volatile("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "+v"(r) : "v"(y), "v"(ms), "v"(0x80000000u));
    return r & 0xffff;
}

__global__ void k_cmp(const uint32_t * v, const float * vs, const uint32_t * y, int n, unsigned long long * bad,
                      uint32_t * ex) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = mad2(v[i], vs[i], y[i]), b = mad1(v[i], vs[i], y[i]);
    const uint32_t c = scl2(y[i], vs[i]), d = scl1(y[i], vs[i]);
    if (a != b) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k < 8) { ex[4 * k] = v[i]; ex[4 * k + 1] = __float_as_uint(vs[i]); ex[4 * k + 2] = y[i]; ex[4 * k + 3] = (a << 16) | b; }
    }
    if (c != d) atomicAdd(bad + 1, 1ull);
}

template <int MODE>
__global__ void k_chain(const uint32_t * in, float * out, unsigned long long * cyc, int n) {
    uint32_t v = in[threadIdx.x] & 0xffff, y = 0x3c00;
    const float vs = 1e-3f * (threadIdx.x + 1);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) y = MODE ? mad1(v, vs, y) : mad2(v, vs, y);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = (float) y;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

static float h2f_host(uint16_t h) {
    const uint32_t s = (h >> 15) & 1, e = (h >> 10) & 31, m = h & 1023;
    float f;
    if (e == 0) f = std::ldexp((float) m, -24);
    else if (e == 31) f = m ? NAN : INFINITY;
    else f = std::ldexp((float) (m | 1024), (int) e - 25);
    return s ? -f : f;
}

int main() {
    const int n = 1 << 24;
    std::vector<uint32_t> v(n), y(n);
    std::vector<float> vs(n);
    std::mt19937_64 rng(1234);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (int i = 0; i < n; ++i) {
        // finite f16 values with exponents in a useful range (|x| in ~[2^-14, 2^8])
        auto rf16 = [&]() {
            const uint32_t e = 1 + (uint32_t) (rng() % 23), m = (uint32_t) (rng() % 1024), s = (uint32_t) (rng() & 1);
            return (s << 15) | (e << 10) | m;
        };
        v[i] = rf16();
        y[i] = rf16();
        if (i & 1) {   // aimed at an f16 midpoint: y + v*vs = mid (+ tiny), mid halfway between y and its neighbour
            const float yf = h2f_host((uint16_t) y[i]);
            const int ey = (int) ((y[i] >> 10) & 31) - 15;
            const double ulp = std::ldexp(1.0, ey - 10);
            const int k = 1 + (int) (rng() % 64);
            const double mid = (double) yf + (k + 0.5) * ulp * ((rng() & 1) ? 1 : -1);
            const double vf = (double) h2f_host((uint16_t) v[i]);
            const double jitter = (U(rng) - 0.5) * std::ldexp(ulp, -14);
            vs[i] = (float) ((mid + jitter - (double) yf) / vf);
        } else {
            vs[i] = (float) (std::exp((U(rng) - 0.5) * 20.0) * ((rng() & 1) ? 1 : -1));
        }
    }
    uint32_t *dv, *dy, *dex;
    float * dvs;
    unsigned long long * dbad;
    hipMalloc(&dv, n * 4); hipMalloc(&dy, n * 4); hipMalloc(&dvs, n * 4); hipMalloc(&dbad, 16); hipMalloc(&dex, 32 * 4);
    hipMemcpy(dv, v.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dy, y.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dvs, vs.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 16);
    hipLaunchKernelGGL(k_cmp, dim3(n / 256), dim3(256), 0, 0, dv, dvs, dy, n, dbad, dex);
    unsigned long long bad[2];
    uint32_t ex[32];
    hipMemcpy(bad, dbad, 16, hipMemcpyDeviceToHost);
    hipMemcpy(ex, dex, sizeof ex, hipMemcpyDeviceToHost);
    printf("mad: %llu of %d differ (half of the cases aimed at f16 midpoints); scale: %llu differ\n", bad[0], n, bad[1]);
    for (int k = 0; k < (int) std::min<unsigned long long>(bad[0], 8); ++k) {
        float f;
        memcpy(&f, &ex[4 * k + 1], 4);
        printf("  v %04x vs %.9g y %04x: two-step %04x mixlo %04x\n", ex[4 * k], f, ex[4 * k + 2], ex[4 * k + 3] >> 16, ex[4 * k + 3] & 0xffff);
    }
    float * out;
    unsigned long long * cyc;
    hipMalloc(&out, 1024 * 4); hipMalloc(&cyc, 8);
    for (int m = 0; m < 2; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            if (m) hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, dv, out, cyc, 4096);
            else hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, dv, out, cyc, 4096);
            hipDeviceSynchronize();
        }
        unsigned long long c;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("chain %-20s %.2f ticks/step\n", m ? "v_fma_mixlo_f16" : "fma_mix + cvt", (double) c / 4096);
    }
    return 0;
}
