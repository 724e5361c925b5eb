// The dec2 chain's fast batch (fa_chain.h dc_fast_batch) in isolation: s_memtime ticks per
// position for a D = 128 head on two waves, four heads-halves on four waves, with idle waves
// beside them, against the plain C++ batch.  hipcc --offload-arch=gfx950 -O3 -I llamacog_amd/csrc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <hip/hip_fp16.h>
#include "fa_chain.h"
using namespace mi355x;

__device__ __forceinline__ uint32_t f16_mad(uint32_t vbits, float vs, uint32_t ybits) {
    float t;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(vbits), "v"(vs), "v"(ybits));
    uint32_t r;
    asm("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}
constexpr int D = 128, CH = 128, U = 8;
typedef __attribute__((address_space(3))) const void * lds_cptr;

// MODE 0: C++ batches; 1: dc_fast_batch.  NCH: chain waves (2 or 4); threads: NT
// HI: V and the coefficients at the top of a 139 KB LDS allocation (as in k_fattn_dec2);
// REG: 160 extra VGPRs live across the loop
template <int MODE, int NCH, int NT, bool HI = false, bool REG = false>
__global__ __launch_bounds__(NT) void k(const uint16_t * vg, const float * sg, float * out, unsigned long long * cyc, int reps, uint32_t flags) {
    __shared__ __attribute__((aligned(16))) uint16_t pad[HI ? 36000 : 8];
    __shared__ __attribute__((aligned(16))) uint16_t vl[2][CH * D];
    __shared__ __attribute__((aligned(16))) float sc[CH + 2 * U];
    float big[REG ? 160 : 1];
#pragma unroll
    for (int i = 0; i < (REG ? 160 : 1); ++i) big[i] = vg[i + threadIdx.x] * 1.5f;
    if (HI && threadIdx.x == 0) pad[threadIdx.x] = 1;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int i = tid; i < CH * D; i += NT) { vl[0][i] = vg[i]; vl[1][i] = vg[i]; }
    for (int i = tid; i < CH + 2 * U; i += NT) sc[i] = i < CH ? sg[i] : 0.0f;
    __syncthreads();
    uint32_t y = 0;
    float S = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave < NCH) {
        const uint16_t * vrow = vl[wave >> 1] + (wave & 1) * 64 + lane;
        const uint32_t va0 = (uint32_t) (uintptr_t) (lds_cptr) vrow, sa0 = (uint32_t) (uintptr_t) (lds_cptr) sc;
        for (int rep = 0; rep < reps; ++rep) {
            uint32_t va[U], vb[U];
            float sa[U], sb[U];
            auto ldb = [&](int j, uint32_t (&vv)[U], float (&vs)[U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) vv[u] = vrow[(j + u) * D];
#pragma unroll
                for (int u = 0; u < U; u += 4) {
                    const float4 t = *(const float4 *) (sc + j + u);
                    vs[u] = t.x; vs[u + 1] = t.y; vs[u + 2] = t.z; vs[u + 3] = t.w;
                }
            };
            auto step = [&](int j, const uint32_t (&vv)[U], const float (&vs)[U], uint32_t (&vn)[U], float (&sn)[U]) {
                if constexpr (MODE == 1) {
                    float4 s0, s1;
                    dc_fast_batch(y, S, vv, vs, vn, s0, s1, va0 + (uint32_t) (j * D * 2), sa0 + (uint32_t) (j * 4));
                    sn[0] = s0.x; sn[1] = s0.y; sn[2] = s0.z; sn[3] = s0.w;
                    sn[4] = s1.x; sn[5] = s1.y; sn[6] = s1.z; sn[7] = s1.w;
                } else if constexpr (MODE == 2) {
                    // the kernel's structure: a per-batch flag picks the fast or the general step
                    ldb(j + U, vn, sn);
                    if (((flags >> (j / U)) & 1u) == 0) {
#pragma unroll
                        for (int u = 0; u < U; ++u) { y = f16_mad(vv[u], vs[u], y); S = __fadd_rn(S, vs[u]); }
                    } else {
                        float ms[U], mv[U];
#pragma unroll
                        for (int u = 0; u < U; ++u) { ms[u] = sc[j + u + 1]; mv[u] = sc[j + u + 2]; }
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const bool live = __float_as_uint(mv[u]) != 0xff800000u;
                            const bool upd = __float_as_uint(ms[u]) != 0x3f800000u;
                            float t = __fmul_rn(__half2float(__ushort_as_half((uint16_t) y)), ms[u]);
                            asm("" : "+v"(t));
                            const uint32_t ys = upd ? (uint32_t) __half_as_ushort(__float2half_rn(t)) : y;
                            const float Ss = upd ? __fmul_rn(S, ms[u]) : S;
                            const uint32_t yn = f16_mad(vv[u], vs[u], ys);
                            const float Sn = __fadd_rn(Ss, vs[u]);
                            y = live ? yn : y;
                            S = live ? Sn : S;
                        }
                    }
                } else {
                    ldb(j + U, vn, sn);
#pragma unroll
                    for (int u = 0; u < U; ++u) { y = f16_mad(vv[u], vs[u], y); S = __fadd_rn(S, vs[u]); }
                }
            };
            ldb(0, va, sa);
            for (int j = 0; j < CH; j += 2 * U) {
                step(j, va, sa, vb, sb);
                step(j + U, vb, sb, va, sa);
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    float bs = 0.0f;
#pragma unroll
    for (int i = 0; i < (REG ? 160 : 1); ++i) bs += big[i];
    if (wave < NCH) out[tid] = __uint_as_float(y) + S + bs + (HI ? (float) pad[tid & 7] : 0.0f);
    if (tid == 0) cyc[0] = t1 - t0;
}

template <int MODE, int NCH, int NT, bool HI = false, bool REG = false>
static void run(const char * name, const uint16_t * vg, const float * sg, float * out, unsigned long long * cyc) {
    const int reps = 200;
    hipLaunchKernelGGL((k<MODE, NCH, NT, HI, REG>), dim3(1), dim3(NT), 0, 0, vg, sg, out, cyc, reps, 0u);
    hipLaunchKernelGGL((k<MODE, NCH, NT, HI, REG>), dim3(1), dim3(NT), 0, 0, vg, sg, out, cyc, reps, 0u);
    unsigned long long h;
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-40s %6.2f ticks/position\n", name, (double) h / (reps * CH));
}

int main() {
    uint16_t * vg; float * sg, * out; unsigned long long * cyc;
    hipMalloc(&vg, CH * D * 2 + 4096); hipMalloc(&sg, CH * 4); hipMalloc(&out, 4096); hipMalloc(&cyc, 8);
    hipMemset(vg, 0x20, CH * D * 2); hipMemset(sg, 0x30, CH * 4);
    run<0, 2, 256>("C++ batch, 2 chain waves / 4", vg, sg, out, cyc);
    run<1, 2, 256>("asm batch, 2 chain waves / 4", vg, sg, out, cyc);
    run<0, 4, 512>("C++ batch, 4 chain waves / 8", vg, sg, out, cyc);
    run<1, 4, 512>("asm batch, 4 chain waves / 8", vg, sg, out, cyc);
    run<1, 4, 256>("asm batch, 4 chain waves / 4", vg, sg, out, cyc);
    run<1, 1, 64>("asm batch, 1 chain wave / 1", vg, sg, out, cyc);
    run<0, 4, 512, true>("C++ batch, 4/8, LDS top", vg, sg, out, cyc);
    run<0, 4, 512, false, true>("C++ batch, 4/8, +160 VGPRs", vg, sg, out, cyc);
    run<0, 4, 512, true, true>("C++ batch, 4/8, LDS top +160 VGPRs", vg, sg, out, cyc);
    run<0, 2, 256, false, true>("C++ batch, 2/4, +160 VGPRs", vg, sg, out, cyc);
    run<2, 2, 256>("C++ batch + flag/general, 2/4", vg, sg, out, cyc);
    run<2, 4, 512>("C++ batch + flag/general, 4/8", vg, sg, out, cyc);
    run<2, 4, 512, true>("C++ batch + flag/general, 4/8, LDS top", vg, sg, out, cyc);
    return 0;
}
