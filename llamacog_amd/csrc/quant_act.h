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
// The reductions run on DPP / readlane (common.h): max |x| as the unsigned order of the
// non-negative floats' bits, then the lowest index holding it (== the sequential strict '>'
// scan), whose value is read from its lane.  All 64 lanes must be active.
// WT: every store write-through (agent-scope relaxed atomics), for a reader in the same launch
// that waits on a counter; bsums then go two to a dword
template <bool WT = false>
__device__ __forceinline__ void q8K_wave(const float (&vv)[4], int lane, int8_t * q, int16_t * bsum, float * d) {
    auto st32 = [](void * p, uint32_t v) {
        if constexpr (WT) __hip_atomic_store((uint32_t *) p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *(uint32_t *) p = v;
    };
    auto stbs = [&](int s) {   // bsum[lane / 4] = s for lanes 4k
        if constexpr (WT) {
            const int hi = __shfl_down(s, 4, WAVE);
            if ((lane & 7) == 0) st32(bsum + (lane >> 2), ((uint32_t) (uint16_t) (int16_t) s) | ((uint32_t) (uint16_t) (int16_t) hi << 16));
        } else {
            if ((lane & 3) == 0) bsum[lane >> 2] = (int16_t) s;
        }
    };
    float la = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) la = fmaxf(la, fabsf(vv[k]));
    const uint32_t abits = wave_umax(__float_as_uint(la));
    const float amax = __uint_as_float(abits);
    if (amax == 0.0f) {
        st32(q + 4 * lane, 0);
        stbs(0);
        if (lane == 0) st32(d, 0u);
        return;
    }
    uint32_t cand = 0xffffffffu;
#pragma unroll
    for (int k = 3; k >= 0; --k) cand = fabsf(vv[k]) == amax ? (uint32_t) (4 * lane + k) : cand;
    const uint32_t imax = wave_umin(cand);
    const int kk = (int) (imax & 3);
    const float vsel = kk == 0 ? vv[0] : (kk == 1 ? vv[1] : (kk == 2 ? vv[2] : vv[3]));
    const float vmax = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(vsel), (int) (imax >> 2)));
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
    st32(q + 4 * lane, packed);
    s = quad_sum(s);
    stbs(s);
    if (lane == 0) st32(d, __float_as_uint(1.0f / iscale));
}

// The same Q8_K block over 16 lanes (a DPP row), lane j = lane & 15 holding elements
// 16j .. 16j+15: four blocks per wave, reductions within the row only (no readlane), and the
// lane's 16 quantized values are exactly its 16-sum.  Bits as q8K_wave.
__device__ __forceinline__ void q8K_row16(const float (&v)[16], int lane, int8_t * q, int16_t * bsum, float * d) {
    const int j = lane & 15;
    float la = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) la = fmaxf(la, fabsf(v[i]));
    uint32_t ab = __float_as_uint(la);
    ab = max(ab, (uint32_t) dpp<DPP_XOR1>((int) ab));
    ab = max(ab, (uint32_t) dpp<DPP_XOR2>((int) ab));
    ab = max(ab, (uint32_t) dpp<DPP_HMIRROR>((int) ab));
    ab = max(ab, (uint32_t) dpp<DPP_MIRROR>((int) ab));
    const float amax = __uint_as_float(ab);
    if (amax == 0.0f) {
        *(uint4 *) (q + 16 * j) = make_uint4(0, 0, 0, 0);
        bsum[j] = 0;
        if (j == 0) *d = 0.0f;
        return;
    }
    // the first index holding max |x| (the CPU's strict '>' scan) and its value
    uint32_t cand = 0xffffffffu;
    float mine = 0.0f;
#pragma unroll
    for (int i = 15; i >= 0; --i) {
        if (fabsf(v[i]) == amax) { cand = (uint32_t) (16 * j + i); mine = v[i]; }
    }
    uint32_t im = cand;
    im = min(im, (uint32_t) dpp<DPP_XOR1>((int) im));
    im = min(im, (uint32_t) dpp<DPP_XOR2>((int) im));
    im = min(im, (uint32_t) dpp<DPP_HMIRROR>((int) im));
    im = min(im, (uint32_t) dpp<DPP_MIRROR>((int) im));
    int vb = (int) (im >> 4) == j ? __float_as_int(mine) : 0;   // one lane of the row holds it
    vb |= dpp<DPP_XOR1>(vb);
    vb |= dpp<DPP_XOR2>(vb);
    vb |= dpp<DPP_HMIRROR>(vb);
    vb |= dpp<DPP_MIRROR>(vb);
    const float iscale = -127.0f / __int_as_float(vb);
    int s = 0;
    uint32_t pk[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int iv = (int) rintf(__fmul_rn(iscale, v[i]));   // nearest_int: round-half-even
        iv = iv < 127 ? iv : 127;
        s += iv;
        pk[i >> 2] |= (uint32_t) (iv & 0xff) << (8 * (i & 3));
    }
    *(uint4 *) (q + 16 * j) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    bsum[j] = (int16_t) s;
    if (j == 0) *d = 1.0f / iscale;
}

// Eight Q8_0 blocks of 256 elements over 16 lanes, lane j holding elements 16j .. 16j+15 (half
// of block j >> 1, the partner half in lane j ^ 1).  Bits as q8_0_wave.
__device__ __forceinline__ void q8_0_row16(const float (&v)[16], int lane, int8_t * q, float * d, int16_t * s8) {
    const int j = lane & 15;
    float la = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) la = fmaxf(la, fabsf(v[i]));
    uint32_t ab = __float_as_uint(la);
    ab = max(ab, (uint32_t) dpp<DPP_XOR1>((int) ab));
    const float amax = __uint_as_float(ab);
    const float dd = amax / 127.0f;
    const float id = amax != 0.0f ? 127.0f / amax : 0.0f;
    int s = 0;
    uint32_t pk[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int iv = (int) rintf(__fmul_rn(v[i], id));
        iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
        s += iv;
        pk[i >> 2] |= (uint32_t) (iv & 0xff) << (8 * (i & 3));
    }
    s += dpp<DPP_XOR1>(s);
    *(uint4 *) (q + 16 * j) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    if ((j & 1) == 0) {
        d[j >> 1]  = h2f(f2h(dd));
        s8[j >> 1] = (int16_t) s;
    }
}

// eight Q8_0 blocks with the x86 AVX rounding (ggml-cpu/arch/x86/quants.c:278-372):
// d = amax/127, id = 127/amax, q = round-half-even(x*id); d is stored as fp16 by the CPU,
// so the fp16-rounded value is kept.  Eight lanes per 32-block (DPP within the 8).  `valid` =
// lane's elements exist (rows that are not a multiple of 256).  All 64 lanes must be active.
__device__ __forceinline__ void q8_0_wave(const float (&vv)[4], int lane, bool valid, int8_t * q, float * d, int16_t * s8) {
    uint32_t ab = __float_as_uint(fmaxf(fmaxf(fabsf(vv[0]), fabsf(vv[1])), fmaxf(fabsf(vv[2]), fabsf(vv[3]))));
    ab = max(ab, (uint32_t) dpp<DPP_XOR1>((int) ab));
    ab = max(ab, (uint32_t) dpp<DPP_XOR2>((int) ab));
    ab = max(ab, (uint32_t) dpp<DPP_HMIRROR>((int) ab));
    const float amax = __uint_as_float(ab);
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
    s = oct_sum(s);
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
// that difference flips the float mean.  Both sums are of n non-negative terms, so each lies
// within (additions a term passes through)·2^-53 of the exact sum, relatively: (n-1)·2^-53 for
// the CPU's loop, a few dozen ulps for the parallel tree here.  When both ends of
// [m(1 - tol), m(1 + tol)], tol covering the two, round to the same float, that float is the
// CPU's mean; otherwise (a fraction ~1e-5 of rows) one thread replays the CPU's loop.
__device__ __forceinline__ double sq4(const float4 x) {   // (double)(x*x) of four elements, summed
    double q = (double) __fmul_rn(x.x, x.x);
    q = __dadd_rn(q, (double) __fmul_rn(x.y, x.y));
    q = __dadd_rn(q, (double) __fmul_rn(x.z, x.z));
    return __dadd_rn(q, (double) __fmul_rn(x.w, x.w));
}

// the float mean from a parallel double sum s of n terms; false when the rounding is not decided
__device__ __forceinline__ bool rms_mean_decided(double s, int64_t n, float & mean) {
    const double m = __ddiv_rn(s, (double) n);
    const double tol = (double) (2 * n + 64) * 0x1p-53;   // CPU loop (n - 1) + this tree (<= n + 16) + 3 roundings
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

// the same with x = (e0 * w0 + e1 * w1) + b: the MoE combine (MUL by the routing weights, ADD of
// the two slots) feeding the residual ADD
__device__ __noinline__ float rms_mean_sequential_moe(const float * e0, const float * e1, float w0, float w1,
                                                      const float * b, int64_t n) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        const float x = __fadd_rn(__fadd_rn(__fmul_rn(e0[i], w0), __fmul_rn(e1[i], w1)), b[i]);
        s = __dadd_rn(s, (double) __fmul_rn(x, x));
    }
    return (float) __ddiv_rn(s, (double) n);
}

}  // namespace mi355x
