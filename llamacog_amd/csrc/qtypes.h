// qtypes.h — quantized-weight "tasks" of the mat-vec kernels and the CPU backend's float
// combination order for their results.
//
// Every quantized mul_mat result on the reference CPU backend is a set of integer sums per
// weight block (exact in any order) combined in fp32 in a fixed order.  That order is what
// decides the bits, and it is restated here exactly (pinned by oracle/ggml_oracle.c
// orc_dot_cpu against tests/golden/mul_mat_cpu.npz, which the reference produced):
//
//   * Q4_K weights with M % 8 == 0 sit in the CPU_REPACK buffer libllama uses by default
//     (ggml-cpu/repack.cpp:1443-1448): one token runs ggml_gemv_q4_K_8x8_q8_K
//     (arch/x86/repack.cpp:718): A = fma(I_b, d·dy, A), B = fma(Imin_b, dmin·dy, B) over the
//     256-blocks b in order, result A - B ("R1").  Groups of four tokens run
//     ggml_gemm_q4_K_8x8_q8_K (:1771), which accumulates once per PAIR of sub-blocks ("R2").
//   * Q4_0 with M % 8 == 0, repacked likewise (arch/x86/repack.cpp:579, 992): A = fma(I_b, dx·dy, A).
//   * every other case is a vec_dot kernel (arch/x86/quants.c): the integer sum of a block is
//     kept per 32-bit SIMD lane, and lane c of a 256-bit register holds "class" c, the 4-byte
//     group (e % 32) / 4 of every 32-element chunk.  acc[c] = fma(d, cls_b[c], acc[c]) over the
//     blocks, then hsum_float_8 ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7)) ("C"):
//       Q8_0 :965, Q4_0 :531 (d = dx·dy per 32-block), Q6_K :2324, Q5_K :2062 (+ a summs
//       chain of the mins), Q4_K :1837 (+ four chains of the pair mins).
//
// A task is the slice of one weight block that one lane owns.  fetch() loads its weight bytes
// (so the pipelined kernel can prefetch them), load() its activation slice, rec() forms the
// task's integers and, after any cross-lane reduction inside the block, stores the block's
// RECORD (RS dwords: integers, then the fp32 scale products) for one (row, column).  walk()
// then runs the CPU's fp32 chain over a row's records: LPR lanes cooperate (one per class).
// rec() and walk() contain cross-lane shuffles: every lane of the wave must call them.
#pragma once

#include "common.h"

namespace mi355x {

__device__ __forceinline__ float asf(uint32_t u) { return __uint_as_float(u); }
// a * b for operands that fit 24 signed bits (6-bit / int8 scales times block dot products, at
// most 16 * 63 * 127 in magnitude): v_mul_i32_i24 / v_mad_i32_i24 run at full rate where the
// generic 32-bit v_mul_lo_u32 is quarter rate (15 of them per Q6_K task dominated its rec)
__device__ __forceinline__ int m24(int a, int b) { return __mul24(a, b); }
__device__ __forceinline__ uint32_t asu(float f) { return __float_as_uint(f); }

// hsum_float_8 over the 8 lanes s = 0..7 of a class group (lane s holds acc[s]); every lane of
// the group ends with ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7))
__device__ __forceinline__ float hsum8_lanes(float v) {
    v = __fadd_rn(v, dppf_xor4(v));
    v = __fadd_rn(v, dppf_xor2(v));
    return __fadd_rn(v, dppf_xor1(v));
}

// class chains: lane s of the group walks acc = fma(f, cls[s], acc) over nb records of RS
// dwords (classes at dwords 0..7, the scale product at dword fo)
// (records are read eight blocks at a time ahead of their FMAs: the chain then waits on one LDS
// round trip per eight blocks, not per block)
__device__ __forceinline__ float class_chain(const uint32_t * rr, int nb, int RS, int fo, int s) {
    float acc = 0.0f;
    int b = 0;
    for (; b + 8 <= nb; b += 8) {
        float f[8];
        int c[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { f[k] = asf(rr[(b + k) * RS + fo]); c[k] = (int) rr[(b + k) * RS + s]; }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = fmaf(f[k], (float) c[k], acc);
    }
    for (; b < nb; ++b) acc = fmaf(asf(rr[b * RS + fo]), (float) (int) rr[b * RS + s], acc);
    return acc;
}

__device__ __forceinline__ void k4_scales_g(uint32_t s0, uint32_t s1, uint32_t s2, int j,
                                            int & sc_lo, int & sc_hi, int & m_lo, int & m_hi) {
    // get_scale_min_k4 (ggml-quants.c:625) of sub-blocks 2j, 2j+1, as a word shuffle
    const uint32_t km1 = 0x3f3f3f3f, km2 = 0x0f0f0f0f, km3 = 0x03030303;
    const uint32_t u0 = s0 & km1;
    const uint32_t u1 = (s2 & km2) | (((s0 >> 6) & km3) << 4);
    const uint32_t u2 = s1 & km1;
    const uint32_t u3 = ((s2 >> 4) & km2) | (((s1 >> 6) & km3) << 4);
    const uint32_t sw = j < 2 ? u0 : u1;
    const uint32_t mw = j < 2 ? u2 : u3;
    const int sh = 16 * (j & 1);
    sc_lo = (sw >> sh) & 0xff; sc_hi = (sw >> (sh + 8)) & 0xff;
    m_lo  = (mw >> sh) & 0xff; m_hi  = (mw >> (sh + 8)) & 0xff;
}

// weight loads: streamed once per token
typedef unsigned int gv4u __attribute__((ext_vector_type(4)));
// Weight loads.  Decode reads every weight byte once per token, so the loads can be
// non-temporal (MI355X_MICROARCH.md nt-weights row: -5..10 % per decode layer); MI_WNT=0 builds
// the default-policy loads for A/B.
#ifndef MI_WNT
#define MI_WNT 1
#endif
#if MI_WNT
typedef gv4u gv4u_u __attribute__((aligned(1)));
typedef unsigned int gv2u __attribute__((ext_vector_type(2)));
typedef gv2u gv2u_u __attribute__((aligned(1)));
typedef uint16_t u16_u __attribute__((aligned(1)));
__device__ __forceinline__ uint4 wld16(const uint8_t * p) {
    const gv4u v = __builtin_nontemporal_load((const gv4u_u *) p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 wld8(const uint8_t * p) {
    const gv2u v = __builtin_nontemporal_load((const gv2u_u *) p);
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t wld2(const uint8_t * p) { return __builtin_nontemporal_load((const u16_u *) p); }
#else
__device__ __forceinline__ uint4 wld16(const uint8_t * p) { return ld16(p); }
__device__ __forceinline__ uint2 wld8(const uint8_t * p) { return ld8(p); }
__device__ __forceinline__ uint32_t wld2(const uint8_t * p) { return ld2(p); }
#endif

// where a task's weight bytes come from: HBM (non-temporal, streamed once) or the LDS copy the
// one-shot GEMV's LDS-DMA staged (k_gemv.hip); the byte offsets are the same either way
struct ld_glb {
    __device__ static uint4 l16(const uint8_t * p) { return wld16(p); }
    __device__ static uint2 l8(const uint8_t * p) { return wld8(p); }
    __device__ static uint32_t l2(const uint8_t * p) { return wld2(p); }
};
struct ld_lds {
    __device__ static uint4 l16(const uint8_t * p) { return ld16(p); }
    __device__ static uint2 l8(const uint8_t * p) { return ld8(p); }
    __device__ static uint32_t l2(const uint8_t * p) { return ld2(p); }
};
// the same from LDS when a block may start 2 bytes off a dword (Q6_K 210-B, Q8_0 34-B, Q4_0
// 18-B blocks): dword-aligned reads re-aligned by v_alignbyte.  Misaligned ds_reads are split
// by the LDS unit; on the 6-bit K-quant they made the one-shot GEMV's record stage cost as much
// as its weight stream (output head 63 -> 105 us, tools/gemv_lab.hip LAB_EXACT)
struct ld_lds_u {
    __device__ static uint32_t al(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }
    __device__ static uint4 l16(const uint8_t * p) {
        const uint32_t s = (uint32_t) (uintptr_t) p & 3;
        const uint32_t * q = (const uint32_t *) (p - s);
        const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
        return make_uint4(al(w1, w0, s), al(w2, w1, s), al(w3, w2, s), al(w4, w3, s));
    }
    __device__ static uint2 l8(const uint8_t * p) {
        const uint32_t s = (uint32_t) (uintptr_t) p & 3;
        const uint32_t * q = (const uint32_t *) (p - s);
        const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
        return make_uint2(al(w1, w0, s), al(w2, w1, s));
    }
    __device__ static uint32_t l2(const uint8_t * p) { return ld2(p); }
};
// the LDS loader for a weight type: plain where every block starts 16-B aligned
template <class T> struct lds_loader { using type = typename std::conditional<T::blk_bytes % 16 == 0, ld_lds, ld_lds_u>::type; };

// the Q8_K / Q8_0 activation (quant_act.h layout): qs, d, and the 16-sums (Q8_K) / 32-sums (Q8_0)
struct gemv_act { const int8_t * qs; const float * d; const int16_t * s; };

// ---- Q4_K / Q5_K: task (b, j) = sub-blocks 2j, 2j+1 of block b (64 weights) ------------------------
struct k4_act { int a[16]; int bs0, bs1; float dy; };

__device__ __forceinline__ void k4_load(const gemv_act & A, int t, k4_act & x) {
    const int b = t >> 2, j = t & 3;
    const int4 * v = (const int4 *) (A.qs + b * 256 + 64 * j);
    const int4 v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3];
    x.a[0] = v0.x; x.a[1] = v0.y; x.a[2] = v0.z; x.a[3] = v0.w;
    x.a[4] = v1.x; x.a[5] = v1.y; x.a[6] = v1.z; x.a[7] = v1.w;
    x.a[8] = v2.x; x.a[9] = v2.y; x.a[10] = v2.z; x.a[11] = v2.w;
    x.a[12] = v3.x; x.a[13] = v3.y; x.a[14] = v3.z; x.a[15] = v3.w;
    const int16_t * bs = A.s + b * 16 + 4 * j;
    x.bs0 = bs[0] + bs[1];
    x.bs1 = bs[2] + bs[3];
    x.dy = A.d[b];
}

struct q4k_raw { uint4 hdr, qa, qb; };
template <class L = ld_glb>
__device__ __forceinline__ void q4k_fetch(const uint8_t * wrow, int t, q4k_raw & w) {
    const int b = t >> 2, j = t & 3;
    const uint8_t * blk = wrow + (int64_t) b * 144;
    w.hdr = L::l16(blk);
    w.qa  = L::l16(blk + 16 + 32 * j);
    w.qb  = L::l16(blk + 32 + 32 * j);
}
// sumi = sc_lo·<q_lo, y> + sc_hi·<q_hi, y> and the pair's min integer
__device__ __forceinline__ void q4k_ints(const q4k_raw & w, int t, const k4_act & x, int & sumi, int & summ) {
    const int j = t & 3;
    int sc_lo, sc_hi, m_lo, m_hi;
    k4_scales_g(w.hdr.y, w.hdr.z, w.hdr.w, j, sc_lo, sc_hi, m_lo, m_hi);
    const uint32_t q[8] = {w.qa.x, w.qa.y, w.qa.z, w.qa.w, w.qb.x, w.qb.y, w.qb.z, w.qb.w};
    int dl = 0, dh = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        dl = dot4((int) (q[i] & 0x0f0f0f0f), x.a[i], dl);
        dh = dot4((int) ((q[i] >> 4) & 0x0f0f0f0f), x.a[8 + i], dh);
    }
    sumi = m24(sc_lo, dl) + m24(sc_hi, dh);
    summ = m24(m_lo, x.bs0) + m24(m_hi, x.bs1);
}

// Q4_K, repacked gemv order R1.  Record: I, Imin, d·dy, dmin·dy (the quad of a block reduced by
// shuffles).  One lane per row walks A and B.
struct g_q4_K {
    static constexpr int per_block = 4, blk_bytes = 144, RS = 4, LPR = 1;
    using act = k4_act;
    using raw = q4k_raw;
    __device__ static void load(const gemv_act & A, int t, act & x) { k4_load(A, t, x); }
    template <class L = ld_glb> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) { q4k_fetch<L>(wrow, t, w); }
    __device__ static void rec(const raw & w, int t, const act & x, bool active, uint32_t * rr) {
        int sumi, summ;
        q4k_ints(w, t, x, sumi, summ);
        if (!active) sumi = summ = 0;
        sumi = quad_sum(sumi);
        summ = quad_sum(summ);
        if (active && (t & 3) == 0) {
            const float d = h2f(w.hdr.x & 0xffff), dmin = h2f(w.hdr.x >> 16);
            *(uint4 *) (rr + (t >> 2) * RS) = make_uint4((uint32_t) sumi, (uint32_t) summ, asu(d * x.dy), asu(dmin * x.dy));
        }
    }
    __device__ static float walk(const uint32_t * rr, int nb, int) {
        float A = 0.0f, B = 0.0f;
        int b = 0;
        for (; b + 8 <= nb; b += 8) {   // eight records in flight ahead of their FMAs
            uint4 r[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) r[k] = *(const uint4 *) (rr + (b + k) * RS);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                A = fmaf((float) (int) r[k].x, asf(r[k].z), A);
                B = fmaf((float) (int) r[k].y, asf(r[k].w), B);
            }
        }
        for (; b < nb; ++b) {
            const uint4 r = *(const uint4 *) (rr + b * RS);
            A = fmaf((float) (int) r.x, asf(r.z), A);
            B = fmaf((float) (int) r.y, asf(r.w), B);
        }
        return __fsub_rn(A, B);
    }
};

// Q4_K with per-pair records, for batches: the caller picks R2 (ggml_gemm_q4_K_8x8_q8_K, one
// fma per sub-block pair) for tokens in whole groups of four and R1 for the rest.
// Record: I_pair[4], Imin_pair[4], d·dy, dmin·dy — each lane of the quad writes its own pair.
struct g_q4_K_p {
    static constexpr int per_block = 4, blk_bytes = 144, RS = 10, LPR = 1;
    using act = k4_act;
    using raw = q4k_raw;
    __device__ static void load(const gemv_act & A, int t, act & x) { k4_load(A, t, x); }
    template <class L = ld_glb> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) { q4k_fetch<L>(wrow, t, w); }
    __device__ static void rec(const raw & w, int t, const act & x, bool active, uint32_t * rr) {
        int sumi, summ;
        q4k_ints(w, t, x, sumi, summ);
        if (!active) return;
        uint32_t * r = rr + (t >> 2) * RS;
        const int j = t & 3;
        r[j] = (uint32_t) sumi;
        r[4 + j] = (uint32_t) summ;
        if (j == 0) {
            r[8] = asu(h2f(w.hdr.x & 0xffff) * x.dy);
            r[9] = asu(h2f(w.hdr.x >> 16) * x.dy);
        }
    }
    // gemm: true = R2, false = R1
    __device__ static float walk_m(const uint32_t * rr, int nb, bool gemm) {
        float A = 0.0f, B = 0.0f;
        for (int b = 0; b < nb; ++b) {
            const uint32_t * r = rr + b * RS;
            const float dd = asf(r[8]), dm = asf(r[9]);
            if (gemm) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    A = fmaf((float) (int) r[k], dd, A);
                    B = fmaf((float) (int) r[4 + k], dm, B);
                }
            } else {
                const int I = (int) r[0] + (int) r[1] + (int) r[2] + (int) r[3];
                const int Im = (int) r[4] + (int) r[5] + (int) r[6] + (int) r[7];
                A = fmaf((float) I, dd, A);
                B = fmaf((float) Im, dm, B);
            }
        }
        return __fsub_rn(A, B);
    }
    __device__ static float walk(const uint32_t * rr, int nb, int) { return walk_m(rr, nb, false); }
};

// Q4_K in the vec_dot order (M % 8 != 0: not repacked): ggml_vec_dot_q4_K_q8_K, AVX2
// (arch/x86/quants.c:1837).  acc[c] = fma(dy·d, cls[c], acc[c]); acc_m[k] = fma(-dy·dmin, P[k],
// acc_m[k]) with P[k] the mins of pair k; hsum8(acc) + ((m0+m2)+(m1+m3)).
// Record: cls[8], P[4], dy·d, -dy·dmin.
struct g_q4_K_c {
    static constexpr int per_block = 4, blk_bytes = 144, RS = 16, LPR = 8;   // 16-B aligned records
    using act = k4_act;
    using raw = q4k_raw;
    __device__ static void load(const gemv_act & A, int t, act & x) { k4_load(A, t, x); }
    template <class L = ld_glb> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) { q4k_fetch<L>(wrow, t, w); }
    __device__ static void rec(const raw & w, int t, const act & x, bool active, uint32_t * rr) {
        const int j = t & 3;
        int sc_lo, sc_hi, m_lo, m_hi;
        k4_scales_g(w.hdr.y, w.hdr.z, w.hdr.w, j, sc_lo, sc_hi, m_lo, m_hi);
        const uint32_t q[8] = {w.qa.x, w.qa.y, w.qa.z, w.qa.w, w.qb.x, w.qb.y, w.qb.z, w.qb.w};
        int c[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            c[i] = m24(sc_lo, dot4((int) (q[i] & 0x0f0f0f0f), x.a[i], 0)) + m24(sc_hi, dot4((int) ((q[i] >> 4) & 0x0f0f0f0f), x.a[8 + i], 0));
            if (!active) c[i] = 0;
            c[i] = quad_sum(c[i]);
        }
        if (!active) return;
        uint32_t * r = rr + (t >> 2) * RS;
        r[8 + j] = (uint32_t) (m24(m_lo, x.bs0) + m24(m_hi, x.bs1));
        if (j == 0) {
            *(uint4 *) r = make_uint4((uint32_t) c[0], (uint32_t) c[1], (uint32_t) c[2], (uint32_t) c[3]);
            *(uint4 *) (r + 4) = make_uint4((uint32_t) c[4], (uint32_t) c[5], (uint32_t) c[6], (uint32_t) c[7]);
            *(uint2 *) (r + 12) = make_uint2(asu(x.dy * h2f(w.hdr.x & 0xffff)), asu(-x.dy * h2f(w.hdr.x >> 16)));
        }
    }
    __device__ static float walk(const uint32_t * rr, int nb, int s) {
        const float acc = class_chain(rr, nb, RS, 12, s);
        float m = 0.0f;
        for (int b = 0; b < nb; ++b) m = fmaf(asf(rr[b * RS + 13]), (float) (int) rr[b * RS + 8 + (s & 3)], m);
        float mm = __fadd_rn(m, dppf_xor2(m));   // (m0+m2), (m1+m3)
        mm = __fadd_rn(mm, dppf_xor1(mm));
        return __fadd_rn(hsum8_lanes(acc), mm);
    }
};

// Q5_K, vec_dot order (arch/x86/quants.c:2062): acc[c] = fma(dy·d, cls[c], acc[c]);
// summs = fma(Imin, -dy·dmin, summs); hsum8(acc) + summs.  Record: cls[8], Imin, dy·d, -dy·dmin.
struct g_q5_K {
    static constexpr int per_block = 4, blk_bytes = 176, RS = 12, LPR = 8;   // 16-B aligned records
    using act = k4_act;
    struct raw { uint4 hdr, ha, hb, qa, qb; };
    __device__ static void load(const gemv_act & A, int t, act & x) { k4_load(A, t, x); }
    template <class L = ld_glb> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const int b = t >> 2, j = t & 3;
        const uint8_t * blk = wrow + (int64_t) b * 176;
        w.hdr = L::l16(blk);
        w.ha  = L::l16(blk + 16);
        w.hb  = L::l16(blk + 32);
        w.qa  = L::l16(blk + 48 + 32 * j);
        w.qb  = L::l16(blk + 64 + 32 * j);
    }
    __device__ static void rec(const raw & w, int t, const act & x, bool active, uint32_t * rr) {
        const int j = t & 3;
        int sc_lo, sc_hi, m_lo, m_hi;
        k4_scales_g(w.hdr.y, w.hdr.z, w.hdr.w, j, sc_lo, sc_hi, m_lo, m_hi);
        const uint32_t q[8]  = {w.qa.x, w.qa.y, w.qa.z, w.qa.w, w.qb.x, w.qb.y, w.qb.z, w.qb.w};
        const uint32_t qh[8] = {w.ha.x, w.ha.y, w.ha.z, w.ha.w, w.hb.x, w.hb.y, w.hb.z, w.hb.w};
        int c[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t lo = (q[i] & 0x0f0f0f0f) | (((qh[i] >> (2 * j)) & 0x01010101) << 4);
            const uint32_t hi = ((q[i] >> 4) & 0x0f0f0f0f) | (((qh[i] >> (2 * j + 1)) & 0x01010101) << 4);
            c[i] = m24(sc_lo, dot4((int) lo, x.a[i], 0)) + m24(sc_hi, dot4((int) hi, x.a[8 + i], 0));
            if (!active) c[i] = 0;
            c[i] = quad_sum(c[i]);
        }
        int mn = active ? m24(m_lo, x.bs0) + m24(m_hi, x.bs1) : 0;
        mn = quad_sum(mn);
        if (active && j == 0) {
            uint32_t * r = rr + (t >> 2) * RS;
            *(uint4 *) r = make_uint4((uint32_t) c[0], (uint32_t) c[1], (uint32_t) c[2], (uint32_t) c[3]);
            *(uint4 *) (r + 4) = make_uint4((uint32_t) c[4], (uint32_t) c[5], (uint32_t) c[6], (uint32_t) c[7]);
            *(uint4 *) (r + 8) = make_uint4((uint32_t) mn, asu(x.dy * h2f(w.hdr.x & 0xffff)), asu(-x.dy * h2f(w.hdr.x >> 16)), 0u);
        }
    }
    __device__ static float walk(const uint32_t * rr, int nb, int s) {
        const float acc = class_chain(rr, nb, RS, 9, s);
        float summs = 0.0f;
        for (int b = 0; b < nb; ++b) summs = fmaf((float) (int) rr[b * RS + 8], asf(rr[b * RS + 10]), summs);
        return __fadd_rn(hsum8_lanes(acc), summs);
    }
};

// Q6_K, vec_dot order (arch/x86/quants.c:2324).  Task (b, h, lr): four groups of 16 weights at
// 256b + 128h + 32g + 16lr; its dot4 pieces i = 0..3 are classes 4lr + i.  The activation carries
// -32·(sum of each 4-byte piece), so dot4(q6, y, -32Σy) = <q6 - 32, y>.  Record: cls[8], dy·d.
struct g_q6_K {
    // RS = 12 (not 9): a record starts 16-B aligned, so its uint4 stores are single aligned
    // ds_write_b128s (a 36-B stride split them; the one-shot GEMV's rec stage ran 1.8x longer)
    static constexpr int per_block = 4, blk_bytes = 210, RS = 12, LPR = 8;
    struct act { int4 a0, a1, a2, a3; int4 n0, n1, n2, n3; float dy; };
    __device__ static void load(const gemv_act & A, int t, act & x) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        const int8_t * ap = A.qs + b * 256 + 128 * h + 16 * lr;
        x.a0 = *(const int4 *) (ap);
        x.a1 = *(const int4 *) (ap + 32);
        x.a2 = *(const int4 *) (ap + 64);
        x.a3 = *(const int4 *) (ap + 96);
        const int m32 = (int) 0xe0e0e0e0;   // -32 in every byte
        auto neg = [&](const int4 & v) {
            return make_int4(dot4(m32, v.x, 0), dot4(m32, v.y, 0), dot4(m32, v.z, 0), dot4(m32, v.w, 0));
        };
        x.n0 = neg(x.a0); x.n1 = neg(x.a1); x.n2 = neg(x.a2); x.n3 = neg(x.a3);
        x.dy = A.d[b];
    }
    struct raw { uint4 la, lb, hh; uint2 sc8; uint32_t d16; };
    template <class L = ld_glb> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        const uint8_t * blk = wrow + (int64_t) b * 210;
        w.la = L::l16(blk + 64 * h + 16 * lr);
        w.lb = L::l16(blk + 64 * h + 32 + 16 * lr);
        w.hh = L::l16(blk + 128 + 32 * h + 16 * lr);
        w.sc8 = L::l8(blk + 192 + 8 * h);
        w.d16 = L::l2(blk + 208);
    }
    __device__ static void rec(const raw & w, int t, const act & x, bool active, uint32_t * rr) {
        const int lr = t & 1;
        const int sc0 = (int8_t) ((w.sc8.x >> (8 * lr)) & 0xff);
        const int sc1 = (int8_t) ((w.sc8.x >> (8 * lr + 16)) & 0xff);
        const int sc2 = (int8_t) ((w.sc8.y >> (8 * lr)) & 0xff);
        const int sc3 = (int8_t) ((w.sc8.y >> (8 * lr + 16)) & 0xff);
        const uint32_t L[4] = {w.la.x, w.la.y, w.la.z, w.la.w};
        const uint32_t M[4] = {w.lb.x, w.lb.y, w.lb.z, w.lb.w};
        const uint32_t H[4] = {w.hh.x, w.hh.y, w.hh.z, w.hh.w};
        const int A0[4] = {x.a0.x, x.a0.y, x.a0.z, x.a0.w}, N0[4] = {x.n0.x, x.n0.y, x.n0.z, x.n0.w};
        const int A1[4] = {x.a1.x, x.a1.y, x.a1.z, x.a1.w}, N1[4] = {x.n1.x, x.n1.y, x.n1.z, x.n1.w};
        const int A2[4] = {x.a2.x, x.a2.y, x.a2.z, x.a2.w}, N2[4] = {x.n2.x, x.n2.y, x.n2.z, x.n2.w};
        const int A3[4] = {x.a3.x, x.a3.y, x.a3.z, x.a3.w}, N3[4] = {x.n3.x, x.n3.y, x.n3.z, x.n3.w};
        int c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s0 = dot4((int) ((L[i] & 0x0f0f0f0f)        | ((H[i] & 0x03030303) << 4)), A0[i], N0[i]);
            const int s1 = dot4((int) ((M[i] & 0x0f0f0f0f)        | (((H[i] >> 2) & 0x03030303) << 4)), A1[i], N1[i]);
            const int s2 = dot4((int) (((L[i] >> 4) & 0x0f0f0f0f) | (((H[i] >> 4) & 0x03030303) << 4)), A2[i], N2[i]);
            const int s3 = dot4((int) (((M[i] >> 4) & 0x0f0f0f0f) | (((H[i] >> 6) & 0x03030303) << 4)), A3[i], N3[i]);
            c[i] = active ? m24(sc0, s0) + m24(sc1, s1) + m24(sc2, s2) + m24(sc3, s3) : 0;
            c[i] += dpp<DPP_XOR2>(c[i]);   // the other half h of the block
        }
        if (active && (t & 2) == 0) {
            uint32_t * r = rr + (t >> 2) * RS;
            *(uint4 *) (r + 4 * lr) = make_uint4((uint32_t) c[0], (uint32_t) c[1], (uint32_t) c[2], (uint32_t) c[3]);
            if (lr == 0) r[8] = asu(x.dy * h2f((uint16_t) w.d16));
        }
    }
    __device__ static float walk(const uint32_t * rr, int nb, int s) { return hsum8_lanes(class_chain(rr, nb, RS, 8, s)); }
};

// Q8_0, vec_dot order (arch/x86/quants.c:965; tinyBLAS_Q0_AVX, llamafile/sgemm.cpp:914-961, has
// the same for batches).  Task = one 32-block; its eight dot4 are the eight classes.
// Record: cls[8], dx·dy — nine dwords, stored one by one (padded to 12 for 16-B stores it held
// Mixtral's Q8_0 K / V launches to 6 workgroups per CU by LDS)
struct g_q8_0 {
    static constexpr int per_block = 1, blk_bytes = 34, RS = 9, LPR = 8;
    struct act { int4 a0, a1; float dy; };
    __device__ static void load(const gemv_act & A, int t, act & x) {
        const int4 * ap = (const int4 *) (A.qs + (int64_t) t * 32);
        x.a0 = ap[0]; x.a1 = ap[1];
        x.dy = A.d[t];
    }
    struct raw { uint4 qa, qb; uint32_t d16; };
    template <class L = ld_glb> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const uint8_t * blk = wrow + (int64_t) t * 34;
        w.d16 = L::l2(blk);
        w.qa = L::l16(blk + 2);
        w.qb = L::l16(blk + 18);
    }
    __device__ static void rec(const raw & w, int t, const act & x, bool active, uint32_t * rr) {
        if (!active) return;
        uint32_t * r = rr + t * RS;
        r[0] = (uint32_t) dot4(w.qa.x, x.a0.x, 0); r[1] = (uint32_t) dot4(w.qa.y, x.a0.y, 0);
        r[2] = (uint32_t) dot4(w.qa.z, x.a0.z, 0); r[3] = (uint32_t) dot4(w.qa.w, x.a0.w, 0);
        r[4] = (uint32_t) dot4(w.qb.x, x.a1.x, 0); r[5] = (uint32_t) dot4(w.qb.y, x.a1.y, 0);
        r[6] = (uint32_t) dot4(w.qb.z, x.a1.z, 0); r[7] = (uint32_t) dot4(w.qb.w, x.a1.w, 0);
        r[8] = asu(h2f((uint16_t) w.d16) * x.dy);
    }
    __device__ static float walk(const uint32_t * rr, int nb, int s) { return hsum8_lanes(class_chain(rr, nb, RS, 8, s)); }
};

// Q4_0 repacked (M % 8 == 0, arch/x86/repack.cpp:579 / 992): A = fma(I_b, dx·dy, A).
// Record: I, dx·dy.
struct g_q4_0 {
    static constexpr int per_block = 1, blk_bytes = 18, RS = 2, LPR = 1;
    struct act { int4 a0, a1; int s8; float dy; };
    __device__ static void load(const gemv_act & A, int t, act & x) {
        const int4 * ap = (const int4 *) (A.qs + (int64_t) t * 32);
        x.a0 = ap[0]; x.a1 = ap[1];
        x.s8 = 8 * A.s[t];
        x.dy = A.d[t];
    }
    struct raw { uint4 q; uint32_t d16; };
    template <class L = ld_glb> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const uint8_t * blk = wrow + (int64_t) t * 18;
        w.d16 = L::l2(blk);
        w.q = L::l16(blk + 2);
    }
    __device__ static void rec(const raw & w, int t, const act & x, bool active, uint32_t * rr) {
        if (!active) return;
        const uint32_t q[4] = {w.q.x, w.q.y, w.q.z, w.q.w};
        const int al[4] = {x.a0.x, x.a0.y, x.a0.z, x.a0.w};
        const int ah[4] = {x.a1.x, x.a1.y, x.a1.z, x.a1.w};
        int s = -x.s8;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s = dot4((int) (q[i] & 0x0f0f0f0f), al[i], s);
            s = dot4((int) ((q[i] >> 4) & 0x0f0f0f0f), ah[i], s);
        }
        *(uint2 *) (rr + t * RS) = make_uint2((uint32_t) s, asu(h2f((uint16_t) w.d16) * x.dy));
    }
    __device__ static float walk(const uint32_t * rr, int nb, int) {
        float A = 0.0f;
        for (int b = 0; b < nb; ++b) {
            const uint2 r = *(const uint2 *) (rr + b * RS);
            A = fmaf((float) (int) r.x, asf(r.y), A);
        }
        return A;
    }
};

// Q4_0 in the vec_dot order (M % 8 != 0, arch/x86/quants.c:531): classes j/4 (low nibbles,
// elements j < 16) and 4 + j/4 (high nibbles).  Record: cls[8], dx·dy.
struct g_q4_0_c {
    static constexpr int per_block = 1, blk_bytes = 18, RS = 12, LPR = 8;   // 16-B aligned records
    using act = g_q8_0::act;
    using raw = g_q4_0::raw;
    __device__ static void load(const gemv_act & A, int t, act & x) { g_q8_0::load(A, t, x); }
    template <class L = ld_glb> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) { g_q4_0::template fetch<L>(wrow, t, w); }
    __device__ static void rec(const raw & w, int t, const act & x, bool active, uint32_t * rr) {
        if (!active) return;
        const uint32_t q[4] = {w.q.x, w.q.y, w.q.z, w.q.w};
        const int al[4] = {x.a0.x, x.a0.y, x.a0.z, x.a0.w};
        const int ah[4] = {x.a1.x, x.a1.y, x.a1.z, x.a1.w};
        const int m8 = 0x08080808;
        uint32_t * r = rr + t * RS;
        uint32_t lo[4], hi[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            // <q - 8, y> = <q, y> - <8, y>
            lo[i] = (uint32_t) (dot4((int) (q[i] & 0x0f0f0f0f), al[i], 0) - dot4(m8, al[i], 0));
            hi[i] = (uint32_t) (dot4((int) ((q[i] >> 4) & 0x0f0f0f0f), ah[i], 0) - dot4(m8, ah[i], 0));
        }
        *(uint4 *) r = make_uint4(lo[0], lo[1], lo[2], lo[3]);
        *(uint4 *) (r + 4) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
        *(uint4 *) (r + 8) = make_uint4(asu(h2f((uint16_t) w.d16) * x.dy), 0u, 0u, 0u);
    }
    __device__ static float walk(const uint32_t * rr, int nb, int s) { return hsum8_lanes(class_chain(rr, nb, RS, 8, s)); }
};

// within-wave LDS hand-off between lanes: DS operations of one wave execute in program order,
// so only the compiler must not move the reads above the writes
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace mi355x
