// libm_exact.h — the CPU reference's libm expf / sinf / cosf, restated so that device code
// produces the same bits.
//
// The reference CPU backend calls glibc's scalar expf (flash attention's online softmax,
// ggml-cpu/ops.cpp:7015-7232; the SiLU tail, vec.h:637) and cosf / sinf (the RoPE cache,
// rope_yarn, ggml-cpu/ops.cpp:5087-5102).  glibc 2.35 on x86-64 picks the FMA builds of these
// functions (sysdeps/x86_64/fpu/multiarch/e_expf-fma.c, s_sinf-fma.c, s_cosf-fma.c) on every
// CPU with FMA + AVX2, i.e. on both the build container and the GPU box.  They are not
// correctly rounded (≈0.5 ulp), so a correctly rounded device function differs from them on a
// small fraction of inputs.  This file restates their published algorithm (glibc
// sysdeps/ieee754/flt-32/e_expf.c, s_sinf.c, s_cosf.c, sincosf.h, math_config.h) with the
// FMA contractions of the FMA build made explicit; the constants are the algorithm's published
// tables (e_exp2f_data.c, sincosf_data.c, s_sincosf.h __inv_pio4).
//
// tests/test_libm_exact.py checks these functions against the host libm bit for bit over
// ranges that cover every use (compiled through oracle/, -ffp-contract=off).
//
// Usable from C (gcc, host), C++ and HIP device code: every operation that must not be fused
// is written as a separate statement under `fp contract(off)`, every fused one with fma().
#pragma once

#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#define LX_FN __device__ static inline
#define LX_TABLE __device__ static const
#else
#define LX_FN static inline
#define LX_TABLE static const
#endif

#if defined(__clang__)
#define LX_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define LX_NOCONTRACT
#endif

LX_FN uint32_t lx_asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
LX_FN uint64_t lx_asuint64(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
LX_FN double lx_asdouble(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }

// ---- expf (e_expf.c, EXP2F_TABLE_BITS = 5, TOINT_INTRINSICS = 0) ----------------------------
// tab[i] = asuint64(2^(i/32)) - (i << 47)
#define LX_EXP2F_TAB { \
    0x3ff0000000000000ULL, 0x3fefd9b0d3158574ULL, 0x3fefb5586cf9890fULL, 0x3fef9301d0125b51ULL, \
    0x3fef72b83c7d517bULL, 0x3fef54873168b9aaULL, 0x3fef387a6e756238ULL, 0x3fef1e9df51fdee1ULL, \
    0x3fef06fe0a31b715ULL, 0x3feef1a7373aa9cbULL, 0x3feedea64c123422ULL, 0x3feece086061892dULL, \
    0x3feebfdad5362a27ULL, 0x3feeb42b569d4f82ULL, 0x3feeab07dd485429ULL, 0x3feea47eb03a5585ULL, \
    0x3feea09e667f3bcdULL, 0x3fee9f75e8ec5f74ULL, 0x3feea11473eb0187ULL, 0x3feea589994cce13ULL, \
    0x3feeace5422aa0dbULL, 0x3feeb737b0cdc5e5ULL, 0x3feec49182a3f090ULL, 0x3feed503b23e255dULL, \
    0x3feee89f995ad3adULL, 0x3feeff76f2fb5e47ULL, 0x3fef199bdd85529cULL, 0x3fef3720dcef9069ULL, \
    0x3fef5818dcfba487ULL, 0x3fef7c97337b9b5fULL, 0x3fefa4afa2a490daULL, 0x3fefd0765b6e4540ULL }

LX_TABLE uint64_t lx_exp2f_tab[32] = LX_EXP2F_TAB;

// T: the 32-entry table (lx_exp2f_tab, or a copy of it in LDS)
LX_FN float lx_expf_t(float x, const uint64_t * T) {
    LX_NOCONTRACT
    const double invln2N = 0x1.71547652b82fep+0 * 32;
    const double SHIFT = 0x1.8p+52;
    const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32;
    const double C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32;
    const double C2 = 0x1.62e42ff0c52d6p-1 / 32;
    const double xd = (double) x;
    const uint32_t abstop = (lx_asuint(x) >> 20) & 0x7ff;
    if (abstop >= (lx_asuint(88.0f) >> 20)) {
        if (lx_asuint(x) == lx_asuint(-INFINITY)) return 0.0f;
        if (abstop >= (lx_asuint(INFINITY) >> 20)) return x + x;
        if (x > 0x1.62e42ep6f) return INFINITY;     // __math_oflowf
        if (x < -0x1.9fe368p6f) return 0.0f;        // __math_uflowf
    }
    // the FMA build contracts both uses of z = InvLn2N * xd (z + SHIFT and z - kd)
#ifndef LX_EXPF_KD_FMA
#define LX_EXPF_KD_FMA 1
#endif
    double kd = LX_EXPF_KD_FMA ? fma(invln2N, xd, SHIFT) : invln2N * xd + SHIFT;
    const uint64_t ki = lx_asuint64(kd);
    kd = kd - SHIFT;
    const double r = fma(invln2N, xd, -kd);
    double z;
    uint64_t t = T[ki % 32];
    t += ki << 47;
    const double s = lx_asdouble(t);
    z = fma(C0, r, C1);
    const double r2 = r * r;
    double y = fma(C2, r, 1.0);
    y = fma(z, r2, y);
    y = y * s;
    return (float) y;
}
LX_FN float lx_expf(float x) { return lx_expf_t(x, lx_exp2f_tab); }

// ---- sinf / cosf (s_sinf.c, s_cosf.c, sincosf.h; TOINT_INTRINSICS = 0) ----------------------
struct lx_sincos_t { double sign[4], hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3; };

LX_FN double lx_sinf_poly(double x, double x2, const struct lx_sincos_t * p, int n) {
    LX_NOCONTRACT
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = fma(x2, p->s3, p->s2);
        const double x7 = x3 * x2;
        const double s = fma(x3, p->s1, x);
        return fma(x7, s1, s);
    }
    const double x4 = x2 * x2;
    const double c2 = fma(x2, p->c4, p->c3);
    const double c1 = fma(x2, p->c1, p->c0);
    const double x6 = x4 * x2;
    const double c = fma(x4, p->c2, c1);
    return fma(x6, c2, c);
}

LX_FN double lx_reduce_fast(double x, const struct lx_sincos_t * p, int * np) {
    LX_NOCONTRACT
    const double r = x * p->hpi_inv;
    const int n = ((int32_t) r + 0x800000) >> 24;
    *np = n;
    return fma(-(double) n, p->hpi, x);
}

// 2/pi in 32-bit windows (the published __inv_pio4 of s_sincosf.h)
LX_TABLE uint32_t lx_inv_pio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

LX_FN double lx_reduce_large(uint32_t xi, int * np) {
    LX_NOCONTRACT
    const uint32_t * arr = &lx_inv_pio4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = (uint32_t) (xi * arr[0]);
    const uint64_t res1 = (uint64_t) xi * arr[4];
    const uint64_t res2 = (uint64_t) xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double) (int64_t) res0;
    *np = (int) n;
    return x * 0x1.921FB54442D18p-62;
}

LX_TABLE struct lx_sincos_t lx_sincos_table[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0,
     0x1p0, -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,
         -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
        {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0,
         -0x1p0, 0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16,
         -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};

LX_FN const struct lx_sincos_t * lx_sincos_tab(int k) { return &lx_sincos_table[k]; }

LX_FN uint32_t lx_abstop12(float x) { return (lx_asuint(x) >> 20) & 0x7ff; }

// cos (cos_not_sin = 1) or sin (0) of y
LX_FN float lx_sincosf1(float y, int cos_not_sin) {
    LX_NOCONTRACT
    double x = y;
    int n;
    const struct lx_sincos_t * p = lx_sincos_tab(0);
    if (lx_abstop12(y) < lx_abstop12(0x1.921FB6p-1f)) {
        const double x2 = x * x;
        if (lx_abstop12(y) < lx_abstop12(0x1p-12f)) return cos_not_sin ? 1.0f : y;
        return (float) lx_sinf_poly(x, x2, p, cos_not_sin);
    }
    if (lx_abstop12(y) < lx_abstop12(120.0f)) {
        x = lx_reduce_fast(x, p, &n);
        const double s = p->sign[n & 3];
        if (n & 2) p = lx_sincos_tab(1);
        const double xs = x * s;
        const double x2 = x * x;
        return (float) lx_sinf_poly(xs, x2, p, n ^ cos_not_sin);
    }
    if (lx_abstop12(y) < lx_abstop12(INFINITY)) {
        const uint32_t xi = lx_asuint(y);
        const int sign = xi >> 31;
        x = lx_reduce_large(xi, &n);
        const double s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = lx_sincos_tab(1);
        const double xs = x * s;
        const double x2 = x * x;
        return (float) lx_sinf_poly(xs, x2, p, n ^ cos_not_sin);
    }
    return y - y;   // nan
}

LX_FN float lx_sinf(float y) { return lx_sincosf1(y, 0); }
LX_FN float lx_cosf(float y) { return lx_sincosf1(y, 1); }
