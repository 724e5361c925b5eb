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

// ---- RMS-norm mean, exactly as the CPU forms it -----------------------------------------------
// rms_norm_f32 (ggml-cpu/ops.cpp:3270-3316) sums (double)(x*x) over the row SEQUENTIALLY in
// double, then mean = (float)(sum / ne0).  A parallel sum rounds differently, and on rare rows
// that difference flips the float mean.  Here every thread sums its terms in double-double
// (error ~2^-106 of the sum), the partials are combined the same way, and the float mean is
// taken from that near-exact sum when the rounding is decided: the sequential double sum of n
// non-negative terms lies within (n-1)·2^-53 of the exact one (relative), so when both ends of
// [m(1 - tol), m(1 + tol)] round to the same float the CPU's mean is that float.  Otherwise (a
// fraction ~1e-5 of rows) one thread replays the CPU's sequential loop.
struct ddv { double hi, lo; };

__device__ __forceinline__ ddv dd_add(ddv a, double b) {   // a + b (TwoSum, then renormalise)
    const double s = __dadd_rn(a.hi, b);
    const double bb = __dsub_rn(s, a.hi);
    const double e = __dadd_rn(__dsub_rn(a.hi, __dsub_rn(s, bb)), __dsub_rn(b, bb));
    const double lo = __dadd_rn(a.lo, e);
    const double hi = __dadd_rn(s, lo);
    return ddv{hi, __dsub_rn(lo, __dsub_rn(hi, s))};
}
__device__ __forceinline__ ddv dd_add(ddv a, ddv b) { return dd_add(dd_add(a, b.hi), b.lo); }

__device__ __forceinline__ ddv dd_wave_sum(ddv v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = dd_add(v, ddv{__shfl_xor(v.hi, o, WAVE), __shfl_xor(v.lo, o, WAVE)});
    return v;
}

__device__ __forceinline__ ddv dd_sq4(ddv acc, const float4 x) {   // + the four terms (double)(x*x)
    acc = dd_add(acc, (double) __fmul_rn(x.x, x.x));
    acc = dd_add(acc, (double) __fmul_rn(x.y, x.y));
    acc = dd_add(acc, (double) __fmul_rn(x.z, x.z));
    return dd_add(acc, (double) __fmul_rn(x.w, x.w));
}

// the float mean from the near-exact sum; false when the rounding is not decided
__device__ __forceinline__ bool rms_mean_decided(ddv s, int64_t n, float & mean) {
    const double m = __ddiv_rn(__dadd_rn(s.hi, s.lo), (double) n);
    const double tol = (double) (n + 8) * 0x1p-53;
    const float f0 = (float) __dmul_rn(m, 1.0 - tol), f1 = (float) __dmul_rn(m, 1.0 + tol);
    mean = (float) m;
    return f0 == f1;
}

// the CPU's own loop: x = a (+ b) elementwise, sum += (double)(x*x) in order
__device__ __noinline__ float rms_mean_sequential(const float * a, const float * b, int64_t n) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        const float x = b ? __fadd_rn(a[i], b[i]) : a[i];
        s = __dadd_rn(s, (double) __fmul_rn(x, x));
    }
    return (float) __ddiv_rn(s, (double) n);
}

}  // namespace mi355x
