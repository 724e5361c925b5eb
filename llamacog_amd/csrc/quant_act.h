// quant_act.h — device-side activation quantizers shared by the stand-alone quantize
// kernels (k_mmv.hip) and the fused producers (k_fused.hip), so a fused and an unfused
// graph produce the same bytes.  Both work on one wavefront holding 256 consecutive
// elements, lane l owning x[4l .. 4l+3].
#pragma once

#include "common.h"

namespace mi355x {

// Q8_K block (bit-exact quantize_row_q8_K_ref, ggml-quants.c:2471-2508): the first index of
// max |x| wins, iscale = -127/max, q = min(127, nearest_int(iscale*x)), d = 1/iscale,
// bsums over 16.  q -> the block's 256 int8, bsum -> its 16 sums, d -> its scale.
__device__ __forceinline__ void q8K_wave(const float (&vv)[4], int lane, int8_t * q, int16_t * bsum, float * d) {
    float amax = 0.0f, vmax = 0.0f;
    int   imax = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float ax = fabsf(vv[k]);
        if (ax > amax) { amax = ax; vmax = vv[k]; imax = 4 * lane + k; }
    }
    // wave argmax with lowest-index tie break (== sequential strict '>' scan)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float oa = __shfl_xor(amax, o, WAVE);
        const float ov = __shfl_xor(vmax, o, WAVE);
        const int   oi = __shfl_xor(imax, o, WAVE);
        if (oa > amax || (oa == amax && oi < imax)) { amax = oa; vmax = ov; imax = oi; }
    }
    if (amax == 0.0f) {
        *(uint32_t *) (q + 4 * lane) = 0;
        if (lane < 16) bsum[lane] = 0;
        if (lane == 0) *d = 0.0f;
        return;
    }
    const float iscale = -127.0f / vmax;
    int s = 0;
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int iv = (int) rintf(__fmul_rn(iscale, vv[k]));   // nearest_int: round-half-even
        iv = iv < 127 ? iv : 127;
        s += iv;
        packed |= (uint32_t) (iv & 0xff) << (8 * k);
    }
    *(uint32_t *) (q + 4 * lane) = packed;
    s += __shfl_xor(s, 1, WAVE);
    s += __shfl_xor(s, 2, WAVE);
    if ((lane & 3) == 0) bsum[lane >> 2] = (int16_t) s;
    if (lane == 0) *d = 1.0f / iscale;
}

// eight Q8_0 blocks with the x86 AVX rounding (ggml-cpu/arch/x86/quants.c:278-372):
// d = amax/127, id = 127/amax, q = round-half-even(x*id); d is stored as fp16 by the CPU,
// so the fp16-rounded value is kept.  Eight lanes per 32-block.  `valid` = lane's
// elements exist (rows that are not a multiple of 256).
__device__ __forceinline__ void q8_0_wave(const float (&vv)[4], int lane, bool valid, int8_t * q, float * d, int16_t * s8) {
    float amax = fmaxf(fmaxf(fabsf(vv[0]), fabsf(vv[1])), fmaxf(fabsf(vv[2]), fabsf(vv[3])));
    amax = fmaxf(amax, __shfl_xor(amax, 1, WAVE));
    amax = fmaxf(amax, __shfl_xor(amax, 2, WAVE));
    amax = fmaxf(amax, __shfl_xor(amax, 4, WAVE));
    const float dd = amax / 127.0f;
    const float id = amax != 0.0f ? 127.0f / amax : 0.0f;
    int s = 0;
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int iv = (int) rintf(__fmul_rn(vv[k], id));
        iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
        s += iv;
        packed |= (uint32_t) (iv & 0xff) << (8 * k);
    }
    s += __shfl_xor(s, 1, WAVE);
    s += __shfl_xor(s, 2, WAVE);
    s += __shfl_xor(s, 4, WAVE);
    if (valid) {
        *(uint32_t *) (q + 4 * lane) = packed;
        if ((lane & 7) == 0) {
            d[lane >> 3]  = h2f(f2h(dd));
            s8[lane >> 3] = (int16_t) s;
        }
    }
}

// canonical RMS-norm sum of squares of x = a (+ b) [K], as every wave and the stand-alone
// norm kernel (k_fused.hip) compute it: lane l sums elements [l*K/64, (l+1)*K/64) in double,
// in order, then the 64 partials are combined by the xor-butterfly of wave_sum
__device__ __forceinline__ double norm_sumsq(const float * a, const float * b, int64_t K, int lane) {
    const int64_t n = K / 64;
    const float * pa = a + lane * n;
    const float * pb = b ? b + lane * n : nullptr;
    double s = 0.0;
    // batches of 8 float4 loads in flight (one L2 round trip per 32 elements, not per 4)
    for (int64_t k0 = 0; k0 < n; k0 += 32) {
        float4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = min(k0 + 4 * u, n - 4);
            x[u] = *(const float4 *) (pa + k);
            if (pb) {
                const float4 y = *(const float4 *) (pb + k);
                x[u].x = __fadd_rn(x[u].x, y.x); x[u].y = __fadd_rn(x[u].y, y.y);
                x[u].z = __fadd_rn(x[u].z, y.z); x[u].w = __fadd_rn(x[u].w, y.w);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (k0 + 4 * u >= n) break;
            s += (double) __fmul_rn(x[u].x, x[u].x);
            s += (double) __fmul_rn(x[u].y, x[u].y);
            s += (double) __fmul_rn(x[u].z, x[u].z);
            s += (double) __fmul_rn(x[u].w, x[u].w);
        }
    }
    return wave_sum(s);
}

}  // namespace mi355x
