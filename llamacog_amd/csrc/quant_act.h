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

// canonical RMS-norm sum of squares of x = a (+ b) [K] (K % 256 == 0), as every wave, the
// stand-alone norm kernel and the fused norm kernel (k_fused.hip) compute it:
//   q(j, l) = ((x[e]^2 + x[e+1]^2) + x[e+2]^2) + x[e+3]^2 in double, e = 256 j + 4 l
//   s(l)    = q(0, l) + q(1, l) + ... in j order          (lane l of a wave)
//   sum     = xor-butterfly of wave_sum over the 64 s(l)
// Each float4 load of a wave covers 1 KiB of contiguous memory, and the (j, l) partials
// can be formed by any thread holding that float4 (norm_q4), so a workgroup computes the
// same value cooperatively.
__device__ __forceinline__ double norm_q4(const float4 x) {
    double q = (double) __fmul_rn(x.x, x.x);
    q += (double) __fmul_rn(x.y, x.y);
    q += (double) __fmul_rn(x.z, x.z);
    q += (double) __fmul_rn(x.w, x.w);
    return q;
}

__device__ __forceinline__ double norm_sumsq(const float * a, const float * b, int64_t K, int lane) {
    const int64_t n = K / 256;
    double s = 0.0;
    // batches of 8 float4 loads in flight
    for (int64_t j0 = 0; j0 < n; j0 += 8) {
        float4 x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t e = 256 * min(j0 + u, n - 1) + 4 * lane;
            x[u] = *(const float4 *) (a + e);
            if (b) {
                const float4 y = *(const float4 *) (b + e);
                x[u].x = __fadd_rn(x[u].x, y.x); x[u].y = __fadd_rn(x[u].y, y.y);
                x[u].z = __fadd_rn(x[u].z, y.z); x[u].w = __fadd_rn(x[u].w, y.w);
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (j0 + u >= n) break;
            s += norm_q4(x[u]);
        }
    }
    return wave_sum(s);
}

}  // namespace mi355x
