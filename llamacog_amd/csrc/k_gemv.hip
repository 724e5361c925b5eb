// k_gemv.hip — decode mat-vec (one activation column) over quantized weights, with
// grouped launches and fused epilogues.
//
// Arithmetic is the one of k_mmv.hip (integer sub-block sums against the CPU-exact Q8_K /
// Q8_0 activation, fp32 combination per task), so results are those of the general
// mat-vec kernel.  The layout is built for HBM latency on MI355X:
//   * a wavefront owns R consecutive weight rows; every lane keeps the activation slice of
//     its task in VGPRs and walks the R rows, so the activation is read once per R rows
//     (not once per row) and each lane has R independent 48..64-byte weight loads in
//     flight;
//   * for short matrices WPR waves split a row's K range (LDS reduction) so that the grid
//     keeps >= 2048 waves in flight;
//   * one launch covers up to three matrices that share src1 (Q/K/V, gate/up): the grid
//     walks the concatenated row space, each workgroup inside one matrix;
//   * optional SiLU epilogue: the gate projection also writes silu(gate) — the UNARY node
//     that follows it — with ggml_vec_silu_f32's arithmetic (vec.cpp:233: AVX-512 ggml_v_silu
//     on 16-element chunks, x/(1+expf(-x)) on the tail);
//   * optional f16 epilogue: the V projection also performs the CPY of its output into the
//     f16 KV cache (destination read from the dynamic-pointer table, exec_ctx::dyn_slot).
#include "ops.h"
#include <hip/hip_ext.h>
#include "rope.h"
#include "quant_act.h"

namespace mi355x {

struct gemv_act { const int8_t * qs; const float * d; const int16_t * s; };

// weight loads: streamed once per token, so non-temporal (MI355X_MICROARCH.md, nt-weights:
// once-read decode weights land sooner with the nt policy)
#ifndef GEMV_NT
#define GEMV_NT 0
#endif
typedef unsigned int gv4u __attribute__((ext_vector_type(4)));
typedef unsigned int gv2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 wld16(const uint8_t * p) {
#if GEMV_NT
    const gv4u v = __builtin_nontemporal_load((const gv4u *) p);
    return make_uint4(v.x, v.y, v.z, v.w);
#else
    return ld16(p);
#endif
}
__device__ __forceinline__ uint2 wld8(const uint8_t * p) {
#if GEMV_NT
    const gv2u v = __builtin_nontemporal_load((const gv2u *) p);
    return make_uint2(v.x, v.y);
#else
    return ld8(p);
#endif
}
__device__ __forceinline__ uint32_t wld2(const uint8_t * p) {
#if GEMV_NT
    return __builtin_nontemporal_load((const unsigned short *) p);
#else
    return ld2(p);
#endif
}

// ---- per-type tasks: load(): activation slice of task t; dot(): that task's weight slice of
// one row -> fp32 contribution (same formula as k_mmv.hip's tasks) ------------------------------
__device__ __forceinline__ void k4_scales_g(uint32_t s0, uint32_t s1, uint32_t s2, int j,
                                            int & sc_lo, int & sc_hi, int & m_lo, int & m_hi) {
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

struct g_q4_K {
    static constexpr int per_block = 4, blk_bytes = 144;
    struct act { int a[16]; int bs0, bs1; float dy; };
    // activation element of the k-th (0..63) value of task t, in act.a order
    __device__ static int elem(int t, int k) { return 64 * t + k; }
    // act from the task's 64 quantized values (4 per int, act order), its 16-sums, block scale
    __device__ static void pack(act & x, const int (&q4)[16], const int (&g16)[4], float d) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x.a[i] = q4[i];
        x.bs0 = g16[0] + g16[1];
        x.bs1 = g16[2] + g16[3];
        x.dy = d;
    }
    __device__ static void load(const gemv_act & A, int t, act & x) {
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
    struct raw { uint4 hdr, qa, qb; };
    __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const int b = t >> 2, j = t & 3;
        const uint8_t * blk = wrow + (int64_t) b * 144;
        w.hdr = wld16(blk);
        w.qa  = wld16(blk + 16 + 32 * j);
        w.qb  = wld16(blk + 32 + 32 * j);
    }
    __device__ static float dot(const uint8_t * wrow, int t, const act & x) {
        raw w;
        fetch(wrow, t, w);
        return dotr(w, t, x);
    }
    __device__ static float dotr(const raw & w, int t, const act & x) {
        const int j = t & 3;
        const uint4 hdr = w.hdr, qa = w.qa, qb = w.qb;
        const float d    = h2f(hdr.x & 0xffff);
        const float dmin = h2f(hdr.x >> 16);
        int sc_lo, sc_hi, m_lo, m_hi;
        k4_scales_g(hdr.y, hdr.z, hdr.w, j, sc_lo, sc_hi, m_lo, m_hi);
        const uint32_t q[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        int dl = 0, dh = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            dl = dot4((int) (q[i] & 0x0f0f0f0f), x.a[i], dl);
            dh = dot4((int) ((q[i] >> 4) & 0x0f0f0f0f), x.a[8 + i], dh);
        }
        const int sumi = sc_lo * dl + sc_hi * dh;
        const int summ = m_lo * x.bs0 + m_hi * x.bs1;
        return (d * x.dy) * (float) sumi - (dmin * x.dy) * (float) summ;
    }
};

struct g_q5_K {
    static constexpr int per_block = 4, blk_bytes = 176;
    using act = g_q4_K::act;
    __device__ static int elem(int t, int k) { return g_q4_K::elem(t, k); }
    __device__ static void pack(act & x, const int (&q4)[16], const int (&g16)[4], float d) { g_q4_K::pack(x, q4, g16, d); }
    __device__ static void load(const gemv_act & A, int t, act & x) { g_q4_K::load(A, t, x); }
    struct raw { uint4 hdr, ha, hb, qa, qb; };
    __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const int b = t >> 2, j = t & 3;
        const uint8_t * blk = wrow + (int64_t) b * 176;
        w.hdr = wld16(blk);
        w.ha  = wld16(blk + 16);
        w.hb  = wld16(blk + 32);
        w.qa  = wld16(blk + 48 + 32 * j);
        w.qb  = wld16(blk + 64 + 32 * j);
    }
    __device__ static float dot(const uint8_t * wrow, int t, const act & x) {
        raw w;
        fetch(wrow, t, w);
        return dotr(w, t, x);
    }
    __device__ static float dotr(const raw & w, int t, const act & x) {
        const int j = t & 3;
        const uint4 hdr = w.hdr, ha = w.ha, hb = w.hb, qa = w.qa, qb = w.qb;
        const float d    = h2f(hdr.x & 0xffff);
        const float dmin = h2f(hdr.x >> 16);
        int sc_lo, sc_hi, m_lo, m_hi;
        k4_scales_g(hdr.y, hdr.z, hdr.w, j, sc_lo, sc_hi, m_lo, m_hi);
        const uint32_t q[8]  = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        const uint32_t qh[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
        int dl = 0, dh = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t lo = (q[i] & 0x0f0f0f0f) | (((qh[i] >> (2 * j)) & 0x01010101) << 4);
            const uint32_t hi = ((q[i] >> 4) & 0x0f0f0f0f) | (((qh[i] >> (2 * j + 1)) & 0x01010101) << 4);
            dl = dot4((int) lo, x.a[i], dl);
            dh = dot4((int) hi, x.a[8 + i], dh);
        }
        const int sumi = sc_lo * dl + sc_hi * dh;
        const int summ = m_lo * x.bs0 + m_hi * x.bs1;
        return (d * x.dy) * (float) sumi - (dmin * x.dy) * (float) summ;
    }
};

struct g_q6_K {
    static constexpr int per_block = 4, blk_bytes = 210;
    struct act { int4 a0, a1, a2, a3; int b0, b1, b2, b3; float dy; };
    // task (b, h, lr): four groups of 16 at 256b + 128h + 16lr + 32g
    __device__ static int elem(int t, int k) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        return 256 * b + 128 * h + 16 * lr + 32 * (k >> 4) + (k & 15);
    }
    __device__ static void pack(act & x, const int (&q4)[16], const int (&g16)[4], float d) {
        x.a0 = make_int4(q4[0], q4[1], q4[2], q4[3]);
        x.a1 = make_int4(q4[4], q4[5], q4[6], q4[7]);
        x.a2 = make_int4(q4[8], q4[9], q4[10], q4[11]);
        x.a3 = make_int4(q4[12], q4[13], q4[14], q4[15]);
        x.b0 = 32 * g16[0]; x.b1 = 32 * g16[1]; x.b2 = 32 * g16[2]; x.b3 = 32 * g16[3];
        x.dy = d;
    }
    __device__ static void load(const gemv_act & A, int t, act & x) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        const int8_t * ap = A.qs + b * 256 + 128 * h + 16 * lr;
        x.a0 = *(const int4 *) (ap);
        x.a1 = *(const int4 *) (ap + 32);
        x.a2 = *(const int4 *) (ap + 64);
        x.a3 = *(const int4 *) (ap + 96);
        const int16_t * bs = A.s + b * 16 + 8 * h + lr;
        x.b0 = 32 * bs[0]; x.b1 = 32 * bs[2]; x.b2 = 32 * bs[4]; x.b3 = 32 * bs[6];
        x.dy = A.d[b];
    }
    struct raw { uint4 la, lb, hh; uint2 sc8; uint32_t d16; };
    __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        const uint8_t * blk = wrow + (int64_t) b * 210;
        w.la = wld16(blk + 64 * h + 16 * lr);
        w.lb = wld16(blk + 64 * h + 32 + 16 * lr);
        w.hh = wld16(blk + 128 + 32 * h + 16 * lr);
        w.sc8 = wld8(blk + 192 + 8 * h);
        w.d16 = wld2(blk + 208);
    }
    __device__ static float dot(const uint8_t * wrow, int t, const act & x) {
        raw w;
        fetch(wrow, t, w);
        return dotr(w, t, x);
    }
    __device__ static float dotr(const raw & w, int t, const act & x) {
        const int lr = t & 1;
        const uint4 la = w.la, lb = w.lb, hh = w.hh;
        const uint2 sc8 = w.sc8;
        const float d = h2f((uint16_t) w.d16);
        const int sc0 = (int8_t) ((sc8.x >> (8 * lr)) & 0xff);
        const int sc1 = (int8_t) ((sc8.x >> (8 * lr + 16)) & 0xff);
        const int sc2 = (int8_t) ((sc8.y >> (8 * lr)) & 0xff);
        const int sc3 = (int8_t) ((sc8.y >> (8 * lr + 16)) & 0xff);
        const uint32_t L[4] = {la.x, la.y, la.z, la.w};
        const uint32_t M[4] = {lb.x, lb.y, lb.z, lb.w};
        const uint32_t H[4] = {hh.x, hh.y, hh.z, hh.w};
        const int A0[4] = {x.a0.x, x.a0.y, x.a0.z, x.a0.w};
        const int A1[4] = {x.a1.x, x.a1.y, x.a1.z, x.a1.w};
        const int A2[4] = {x.a2.x, x.a2.y, x.a2.z, x.a2.w};
        const int A3[4] = {x.a3.x, x.a3.y, x.a3.z, x.a3.w};
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s0 = dot4((int) ((L[i] & 0x0f0f0f0f)        | ((H[i] & 0x03030303) << 4)), A0[i], s0);
            s1 = dot4((int) ((M[i] & 0x0f0f0f0f)        | (((H[i] >> 2) & 0x03030303) << 4)), A1[i], s1);
            s2 = dot4((int) (((L[i] >> 4) & 0x0f0f0f0f) | (((H[i] >> 4) & 0x03030303) << 4)), A2[i], s2);
            s3 = dot4((int) (((M[i] >> 4) & 0x0f0f0f0f) | (((H[i] >> 6) & 0x03030303) << 4)), A3[i], s3);
        }
        s0 -= x.b0; s1 -= x.b1; s2 -= x.b2; s3 -= x.b3;
        const int sumi = sc0 * s0 + sc1 * s1 + sc2 * s2 + sc3 * s3;
        return (d * x.dy) * (float) sumi;
    }
};

struct g_q8_0 {
    static constexpr int per_block = 1, blk_bytes = 34;
    struct act { int4 a0, a1; float dy; };
    static constexpr bool no_prologue = true;
    __device__ static int elem(int, int) { return 0; }
    __device__ static void pack(act &, const int (&)[16], const int (&)[4], float) {}
    __device__ static void load(const gemv_act & A, int t, act & x) {
        const int4 * ap = (const int4 *) (A.qs + (int64_t) t * 32);
        x.a0 = ap[0]; x.a1 = ap[1];
        x.dy = A.d[t];
    }
    struct raw { uint4 qa, qb; uint32_t d16; };
    __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const uint8_t * blk = wrow + (int64_t) t * 34;
        w.d16 = wld2(blk);
        w.qa = wld16(blk + 2);
        w.qb = wld16(blk + 18);
    }
    __device__ static float dot(const uint8_t * wrow, int t, const act & x) {
        raw w;
        fetch(wrow, t, w);
        return dotr(w, t, x);
    }
    __device__ static float dotr(const raw & w, int t, const act & x) {
        const float d = h2f((uint16_t) w.d16);
        const uint4 qa = w.qa, qb = w.qb;
        int s = 0;
        s = dot4(qa.x, x.a0.x, s); s = dot4(qa.y, x.a0.y, s); s = dot4(qa.z, x.a0.z, s); s = dot4(qa.w, x.a0.w, s);
        s = dot4(qb.x, x.a1.x, s); s = dot4(qb.y, x.a1.y, s); s = dot4(qb.z, x.a1.z, s); s = dot4(qb.w, x.a1.w, s);
        return (float) s * (d * x.dy);
    }
};

struct g_q4_0 {
    static constexpr int per_block = 1, blk_bytes = 18;
    struct act { int4 a0, a1; int s8; float dy; };
    static constexpr bool no_prologue = true;
    __device__ static int elem(int, int) { return 0; }
    __device__ static void pack(act &, const int (&)[16], const int (&)[4], float) {}
    __device__ static void load(const gemv_act & A, int t, act & x) {
        const int4 * ap = (const int4 *) (A.qs + (int64_t) t * 32);
        x.a0 = ap[0]; x.a1 = ap[1];
        x.s8 = 8 * A.s[t];
        x.dy = A.d[t];
    }
    struct raw { uint4 q; uint32_t d16; };
    __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const uint8_t * blk = wrow + (int64_t) t * 18;
        w.d16 = wld2(blk);
        w.q = wld16(blk + 2);
    }
    __device__ static float dot(const uint8_t * wrow, int t, const act & x) {
        raw r;
        fetch(wrow, t, r);
        return dotr(r, t, x);
    }
    __device__ static float dotr(const raw & r, int t, const act & x) {
        const float d = h2f((uint16_t) r.d16);
        const uint4 q = r.q;
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
        const int al[4] = {x.a0.x, x.a0.y, x.a0.z, x.a0.w};
        const int ah[4] = {x.a1.x, x.a1.y, x.a1.z, x.a1.w};
        int s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s = dot4((int) (w[i] & 0x0f0f0f0f), al[i], s);
            s = dot4((int) ((w[i] >> 4) & 0x0f0f0f0f), ah[i], s);
        }
        s -= x.s8;
        return (float) s * (d * x.dy);
    }
};

// ---- kernel ------------------------------------------------------------------------------------
constexpr int GEMV_MAXMAT = 3;
constexpr int GEMV_ROPE_MAXPAIRS = 256;
constexpr int GEMV_MAXG = 16;             // row groups per workgroup of the pipelined kernel with epilogues   // rope table of the fused epilogue: n_dims <= 512

struct gemv_args {
    const uint8_t * W[GEMV_MAXMAT]; int64_t nb01[GEMV_MAXMAT]; int64_t M[GEMV_MAXMAT];
    float * dst[GEMV_MAXMAT];
    float * silu[GEMV_MAXMAT];            // SiLU epilogue output (nullable)
    uint16_t * const * f16out[GEMV_MAXMAT];   // fused f32->f16 CPY (KV-cache store) slot (nullable)
    int64_t blk0[GEMV_MAXMAT + 1];        // first workgroup of each matrix
    gemv_act A;
    int ntasks;
    // fused ROPE (NORM mode, one token) of the projection output: adjacent rows (2i, 2i+1)
    // of a head are rotated in the epilogue; optional f16 copy of the result (KV-cache store)
    float * rope_out[GEMV_MAXMAT];
    uint16_t * const * rope_f16[GEMV_MAXMAT];
    rope_params rp;
    const int32_t * rope_pos; const float * rope_ff; int64_t rope_d;
    int need_pairs;
    const float2 * rtab_g;                // the graph's cos/sin table of the position (rope_table)
    // activation prologue (instead of a separate producer kernel), K-quant weights, one wave
    // covering a row's tasks per WPR group:
    //   pro 1: x = pa (+ pb); y = rms_norm(x) (eps); yw = y * pw; act = Q8_K(yw)
    //   pro 2: yw = pa * pb; act = Q8_K(yw)
    // workgroup 0 also stores the graph nodes' outputs (o_add, o_norm, o_mul) and the Q8_K
    // activation (cq, cd, cs) for later launches that share the input
    int pro;
    const float * pa; const float * pb; const float * pw; float eps; int64_t pk;
    float * o_add; float * o_norm; float * o_mul;
    int8_t * cq; float * cd; int16_t * cs;
    // a deferred in-place ADD stored by workgroup 0 (x[i] = x[i] + y[i], n elements)
    float * post_add; const float * post_b; int64_t post_n;
    // MUL_MAT_ID decode (gemv_mul_mat_id): matrix m is expert ids[ids_e[m]] of the stack at
    // W[0] (stride nb02), read on the device so routing needs no host round trip
    const int32_t * ids; int64_t nb02; int64_t ids_e[GEMV_MAXMAT];
};

// the activation prologue, once per workgroup (4 waves): wave w owns the Q8_K blocks
// j = w, w+4, ... (256 consecutive elements each, lane l holding 4l..4l+3).
//   pro 1: x = pa (+ pb); the canonical RMS-norm sum of squares (quant_act.h norm_sumsq:
//          q(j, l) partials in LDS, summed in j order per lane, then the wave butterfly);
//          y = x * scale; yw = y * pw
//   pro 2: yw = pa * pb
// then yw is quantized block by block with q8K_wave (the quantizer of the stand-alone and
// fused producer kernels, so the bytes are theirs) into LDS, where the mat-vec's
// task loads read it.  Workgroup 0 also stores the chain's node outputs and the quantized
// activation for later launches that share it.  Returns the LDS activation.
constexpr int GEMV_PRO_XREG = 4;   // blocks per wave kept in registers between the two passes

template <int NWV>
__device__ __forceinline__ gemv_act prologue_wg(const gemv_args & p, uint8_t * lds) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nb = (int) (p.pk / 256);
    const bool writer = blockIdx.x == 0;
    int8_t * qs = (int8_t *) lds;
    int16_t * bs = (int16_t *) (lds + p.pk);
    float * dd = (float *) (lds + p.pk + p.pk / 8);
    double * qp = (double *) (lds + ((p.pk + p.pk / 8 + 4 * nb + 15) & ~(int64_t) 15));   // [nb][64], pro 1 only
    float scale = 1.0f;
    float4 xr[GEMV_PRO_XREG], wr[GEMV_PRO_XREG];
    auto load_x = [&](int j) {
        const int64_t e = 256 * (int64_t) j + 4 * lane;
        float4 x = *(const float4 *) (p.pa + e);
        if (p.pb) {
            const float4 y = *(const float4 *) (p.pb + e);
            if (p.pro == 1) {
                x.x = __fadd_rn(x.x, y.x); x.y = __fadd_rn(x.y, y.y); x.z = __fadd_rn(x.z, y.z); x.w = __fadd_rn(x.w, y.w);
            } else {
                x.x = __fmul_rn(x.x, y.x); x.y = __fmul_rn(x.y, y.y); x.z = __fmul_rn(x.z, y.z); x.w = __fmul_rn(x.w, y.w);
            }
        }
        return x;
    };
    if (p.pro == 1) {
#pragma unroll
        for (int i = 0; i < GEMV_PRO_XREG; ++i) {
            const int j = wave + NWV * i;
            if (j < nb) {
                xr[i] = load_x(j);
                if (p.pw) wr[i] = *(const float4 *) (p.pw + 256 * (int64_t) j + 4 * lane);
            }
        }
        for (int j = wave; j < nb; j += NWV) {
            const int i = (j - wave) / NWV;
            float4 x;
            if (i < GEMV_PRO_XREG) {
                x = xr[0];
#pragma unroll
                for (int k = 1; k < GEMV_PRO_XREG; ++k) x = i == k ? xr[k] : x;
            } else {
                x = load_x(j);
            }
            qp[j * 64 + lane] = norm_q4(x);
            if (writer && p.o_add) *(float4 *) (p.o_add + 256 * (int64_t) j + 4 * lane) = x;
        }
        __syncthreads();
        double sq = 0.0;
        for (int j = 0; j < nb; ++j) sq += qp[j * 64 + lane];
        sq = wave_sum(sq);
        const float mean = (float) (sq / (double) p.pk);
        scale = 1.0f / sqrtf(mean + p.eps);
    }
    for (int j = wave; j < nb; j += NWV) {
        const int i = (j - wave) / NWV;
        const int64_t e = 256 * (int64_t) j + 4 * lane;
        float4 x;
        if (p.pro == 1 && i < GEMV_PRO_XREG) {
            x = xr[0];
#pragma unroll
            for (int k = 1; k < GEMV_PRO_XREG; ++k) x = i == k ? xr[k] : x;
        } else {
            x = load_x(j);
        }
        float v[4] = {x.x, x.y, x.z, x.w};
        if (p.pro == 1) {
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = __fmul_rn(v[k], scale);
            if (writer && p.o_norm) *(float4 *) (p.o_norm + e) = make_float4(v[0], v[1], v[2], v[3]);
            if (p.pw) {
                float4 w4;
                if (i < GEMV_PRO_XREG) {
                    w4 = wr[0];
#pragma unroll
                    for (int k = 1; k < GEMV_PRO_XREG; ++k) w4 = i == k ? wr[k] : w4;
                } else {
                    w4 = *(const float4 *) (p.pw + e);
                }
                v[0] = __fmul_rn(v[0], w4.x); v[1] = __fmul_rn(v[1], w4.y);
                v[2] = __fmul_rn(v[2], w4.z); v[3] = __fmul_rn(v[3], w4.w);
            }
        }
        if (writer && p.o_mul) *(float4 *) (p.o_mul + e) = make_float4(v[0], v[1], v[2], v[3]);
        q8K_wave(v, lane, qs + 256 * j, bs + 16 * j, dd + j);
    }
    __syncthreads();
    if (writer) {
        for (int i = threadIdx.x; i < p.pk / 16; i += 64 * NWV) {
            *(int4 *) (p.cq + 16 * i) = *(const int4 *) (qs + 16 * i);
            p.cs[i] = bs[i];
        }
        for (int i = threadIdx.x; i < nb; i += 64 * NWV) p.cd[i] = dd[i];
    }
    return gemv_act{qs, dd, bs};
}

// LDS bytes of the prologue: Q8_K activation (qs, bsums, d) + the norm partials
static inline size_t prologue_lds_bytes(int pro, int64_t K) {
    const int64_t nb = K / 256;
    return (size_t) ((K + K / 8 + 4 * nb + 15) & ~(int64_t) 15) + (pro == 1 ? (size_t) nb * 64 * 8 : 0);
}

// epilogue of one output row; v = this row's sum, vp = the sum of its rope partner row^1
__device__ __forceinline__ void gemv_store(const gemv_args & p, int mi, int64_t M, int64_t row, float v, float vp,
                                           const float2 * rtab = nullptr, uint16_t * const * f16p = nullptr) {
    if (p.dst[mi]) p.dst[mi][row] = v;
    if (p.f16out[mi]) (f16p ? f16p[2 * mi] : *p.f16out[mi])[row] = f2h(v);
    if (p.silu[mi]) {
        const int64_t nvec = (M / 16) * 16;
        p.silu[mi][row] = row < nvec ? v / (1.0f + v_expf_avx512(-v)) : v / (1.0f + expf_cr(-v));
    }
    if (p.rope_out[mi] || p.rope_f16[mi]) {
        const int64_t i0 = row % p.rope_d;
        float o = v;
        if (i0 < p.rp.n_dims) {
            float c, sn, o0, o1;
            if (rtab) { c = rtab[i0 / 2].x; sn = rtab[i0 / 2].y; }
            else rope_cs(p.rp, (float) p.rope_pos[0], i0 / 2, p.rope_ff, c, sn);
            const bool odd = row & 1;
            rope_rotate(odd ? vp : v, odd ? v : vp, c, sn, o0, o1);
            o = odd ? o1 : o0;
        }
        if (p.rope_out[mi]) p.rope_out[mi][row] = o;
        if (p.rope_f16[mi]) (f16p ? f16p[2 * mi + 1] : *p.rope_f16[mi])[row] = f2h(o);
    }
}

typedef __attribute__((address_space(3))) void * lds_vptr;

template <class T, int R, int WPR, bool LDS>
__global__ __launch_bounds__(256) void k_gemv(const gemv_args p) {
    constexpr int RB = (4 / WPR) * R;   // rows per workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wsub = wave % WPR;
    int mi = 0;
#pragma unroll
    for (int k = 1; k < GEMV_MAXMAT; ++k) mi += blockIdx.x >= p.blk0[k] ? 1 : 0;
    const int64_t M = p.M[mi];
    const int64_t rowg = (blockIdx.x - p.blk0[mi]) * RB;     // first row of the workgroup
    const int64_t row0 = rowg + (wave / WPR) * R;            // first row of this wave
    const uint8_t * W = p.W[mi];
    const int64_t nb01 = p.nb01[mi];

    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0f;
    const uint8_t * wrow[R];
    if constexpr (LDS) {
        // stream the workgroup's RB contiguous rows HBM -> LDS (global_load_lds, 16 B per
        // lane, 1 KiB per wave instruction, no VGPRs), then compute out of LDS
        extern __shared__ __attribute__((aligned(16))) uint8_t slab[];
        const int64_t nrow = min((int64_t) RB, M - rowg);
        const int64_t nchunk = nrow * nb01 / 16;
        const int64_t last = nchunk - 1;
        const uint8_t * src = W + rowg * nb01;
        for (int64_t c0 = (int64_t) wave * 64; c0 < nchunk; c0 += 256) {
            const int64_t c = min(c0 + lane, last);
            __builtin_amdgcn_global_load_lds((const void *) (src + 16 * c), (lds_vptr) (slab + 16 * c0), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) wrow[r] = slab + min((int64_t) ((wave / WPR) * R + r), nrow - 1) * nb01;
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) wrow[r] = W + min(row0 + r, M - 1) * nb01;
    }

    if (row0 < M) {
        for (int t = wsub * WAVE + lane; t < p.ntasks; t += WAVE * WPR) {
            typename T::act x;
            T::load(p.A, t, x);
#pragma unroll
            for (int r = 0; r < R; ++r) acc[r] += T::dot(wrow[r], t, x);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
    if constexpr (WPR > 1) {
        __shared__ float red[4][R];
        if (lane == 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) red[wave][r] = acc[r];
        }
        __syncthreads();
        if (wsub == 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                float s = red[wave][r];
#pragma unroll
                for (int w = 1; w < WPR; ++w) s += red[wave + w][r];
                acc[r] = s;
            }
        }
    }
    if (wsub == 0 && lane < R) {
        float v = acc[0], vp = acc[R > 1 ? 1 : 0];
#pragma unroll
        for (int r = 1; r < R; ++r) v = lane == r ? acc[r] : v;
#pragma unroll
        for (int r = 0; r < R; ++r) vp = (lane ^ 1) == r ? acc[r] : vp;
        const int64_t row = row0 + lane;
        if (row < M) gemv_store(p, mi, M, row, v, vp);
    }
}

// ---- persistent, software-pipelined variant ------------------------------------------------------
// A grid of ~2 workgroups per CU walks the row groups; each wave fetches the next group's
// weight slices into registers before computing the current one, so dequantization and the
// dot products overlap the HBM stream instead of following it (a one-shot grid computes
// only after its last load lands).  Needs ntasks <= 64*WPR (one pass over K per wave).
// MODE: 0 = plain stores (no prologue, no epilogue), 1 = epilogues, 2 = activation prologue +
// epilogues.  The lean modes keep the register footprint (and so the number of resident
// workgroups) of the plain mat-vec: 90 VGPRs at R = 2 against 134 with the prologue compiled in.
// The body runs as workgroup wg0 of nwg over the launch's ngroups row groups, so one launch can
// hold two bodies of different weight types (k_gemv_pipe2).
template <class T, int R, int WPR, int MODE, int NWV, bool ID = false>
__device__ __forceinline__ void gemv_pipe_body(const gemv_args & p, const int64_t ngroups, const int64_t wg0, const int64_t nwg) {
    constexpr int NT = 64 * NWV;
    constexpr int RPG = (NWV / WPR) * R;   // rows per group
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wsub = wave % WPR;
    const int t = wsub * WAVE + lane;
    const bool active = t < p.ntasks;
    const int tt = active ? t : 0;
    auto locate = [&](int64_t g, int & mi, int64_t & row0) {
        mi = 0;
#pragma unroll
        for (int k = 1; k < GEMV_MAXMAT; ++k) mi += g >= p.blk0[k] ? 1 : 0;
        row0 = (g - p.blk0[mi]) * RPG + (wave / WPR) * R;
    };
    // ID: matrix k is the expert ids[ids_e[k]] of the stack at W[0] (MUL_MAT_ID decode), its
    // base read once per workgroup
    const uint8_t * Wb[GEMV_MAXMAT];
    if constexpr (ID) {
#pragma unroll
        for (int k = 0; k < GEMV_MAXMAT; ++k) Wb[k] = p.W[0] + (int64_t) p.ids[p.ids_e[k]] * p.nb02;
    }
    auto fetch = [&](int64_t g, typename T::raw (&w)[R]) {
        int mi;
        int64_t row0;
        locate(g, mi, row0);
        const int64_t M = p.M[mi];
        const uint8_t * Wm = p.W[mi];
        if constexpr (ID) {
            Wm = Wb[0];
#pragma unroll
            for (int k = 1; k < GEMV_MAXMAT; ++k) Wm = mi == k ? Wb[k] : Wm;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) T::fetch(Wm + min(row0 + r, M - 1) * p.nb01[mi], tt, w[r]);
    };

    // the first group's weight loads leave before anything else, so the activation prologue,
    // the rope table and the activation loads below overlap that HBM latency
    typename T::raw cur[R], nxt[R];
    int64_t g = wg0;
    if (g < ngroups) fetch(g, cur);
    // cos/sin of every rope pair at this token's position, one pair per thread (rope_cs, the
    // same arithmetic the stand-alone ROPE kernel uses), instead of per output row in the
    // epilogue's few active lanes
    typename T::act x;
    if constexpr (MODE != 2) T::load(p.A, tt, x);   // in flight with the first weight loads
    __shared__ float2 rtab[MODE ? GEMV_ROPE_MAXPAIRS : 1];
    // KV-cache destinations of the f16 epilogues, read from the dynamic-pointer table now
    // rather than as a dependent load in the epilogue
    __shared__ uint16_t * f16p[2 * GEMV_MAXMAT];
    if (MODE) {
        if (threadIdx.x < 2 * GEMV_MAXMAT) {
            const int mi = threadIdx.x >> 1;
            uint16_t * const * slot = (threadIdx.x & 1) ? p.rope_f16[mi] : p.f16out[mi];
            f16p[threadIdx.x] = slot ? *slot : nullptr;
        }
        if (p.need_pairs) {
            for (int ip = threadIdx.x; ip < p.rp.n_dims / 2; ip += NT) {
                if (p.rtab_g) {
                    rtab[ip] = p.rtab_g[ip];
                } else {
                    float c, sn;
                    rope_cs(p.rp, (float) p.rope_pos[0], ip, p.rope_ff, c, sn);
                    rtab[ip] = make_float2(c, sn);
                }
            }
        }
        __syncthreads();
    }
    if constexpr (MODE == 2) {
        extern __shared__ __attribute__((aligned(16))) uint8_t pro_lds[];
        const gemv_act A = prologue_wg<NWV>(p, pro_lds);
        T::load(A, tt, x);
    }
    if (MODE && p.post_add && wg0 == 0) {
        for (int64_t i = threadIdx.x; i < p.post_n; i += NT) p.post_add[i] = __fadd_rn(p.post_add[i], p.post_b[i]);
    }
    __shared__ float red[2][NWV][R];
    // MODE >= 1: row sums are parked in LDS and the epilogues run after the loop on all 256
    // threads (not on the R lanes holding the sums, with the next group's loads live)
    __shared__ float res[MODE ? GEMV_MAXG * RPG : 1];
    int par = 0, kg = 0;
    for (; g < ngroups; g += nwg, par ^= 1, ++kg) {
        const int64_t gn = g + nwg;
        if (gn < ngroups) fetch(gn, nxt);
        float acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = active ? T::dotr(cur[r], tt, x) : 0.0f;
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
        if constexpr (WPR > 1) {
            if (lane == 0) {
#pragma unroll
                for (int r = 0; r < R; ++r) red[par][wave][r] = acc[r];
            }
            __syncthreads();
            if (wsub == 0) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    float s = red[par][wave][r];
#pragma unroll
                    for (int w = 1; w < WPR; ++w) s += red[par][wave + w][r];
                    acc[r] = s;
                }
            }
        }
        if (wsub == 0 && lane < R) {
            float v = acc[0];
#pragma unroll
            for (int r = 1; r < R; ++r) v = lane == r ? acc[r] : v;
            if constexpr (MODE == 0) {
                int mi;
                int64_t row0;
                locate(g, mi, row0);
                if (row0 + lane < p.M[mi]) p.dst[mi][row0 + lane] = v;
            } else {
                res[kg * RPG + (wave / WPR) * R + lane] = v;
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) cur[r] = nxt[r];
    }
    if constexpr (MODE >= 1) {
        __syncthreads();
        for (int i = threadIdx.x; i < kg * RPG; i += NT) {
            const int64_t gg = wg0 + (int64_t) (i / RPG) * nwg;
            int mi = 0;
#pragma unroll
            for (int k = 1; k < GEMV_MAXMAT; ++k) mi += gg >= p.blk0[k] ? 1 : 0;
            const int64_t row = (gg - p.blk0[mi]) * RPG + i % RPG;
            // rope partner row ^ 1 lies in the same group (RPG is even whenever rope is fused)
            if (row < p.M[mi]) gemv_store(p, mi, p.M[mi], row, res[i], res[RPG > 1 ? i ^ 1 : i], rtab, f16p);
        }
    }
}

template <class T, int R, int WPR, int MODE, int NWV, bool ID = false>
__global__ __launch_bounds__(64 * NWV) void k_gemv_pipe(const gemv_args p, const int64_t ngroups) {
    gemv_pipe_body<T, R, WPR, MODE, NWV, ID>(p, ngroups, blockIdx.x, gridDim.x);
}

// Q/K of one K-quant and V of another (Llama-3 Q4_K_M: Q4_K and Q6_K on 16 of 32 layers) in
// one launch with epilogues: workgroups [0, nwg1) run p1's matrices, the rest p2's.  Each
// row's arithmetic is its type's own (WPR depends on K only), so the bits are those of two
// separate launches.
template <class T1, class T2, int R2, int WPR>
__global__ __launch_bounds__(256) void k_gemv_pipe2(const gemv_args p1, const int64_t ng1, const int64_t nwg1,
                                                    const gemv_args p2, const int64_t ng2) {
    if ((int64_t) blockIdx.x < nwg1) gemv_pipe_body<T1, 2, WPR, 1, 4>(p1, ng1, blockIdx.x, nwg1);
    else gemv_pipe_body<T2, R2, WPR, 1, 4>(p2, ng2, (int64_t) blockIdx.x - nwg1, (int64_t) gridDim.x - nwg1);
}

// cos/sin of every rope pair at the token's position (one token), once per graph: rope_cs,
// the arithmetic of the stand-alone ROPE kernel, so the fused epilogue's bits do not change.
// Built per pair by a chain of up to n_dims/2 dependent multiplies (theta *= theta_scale, as
// ggml_rope_cache_init) plus double-precision cos/sin — ~4 us of latency that every
// workgroup of every Q/K projection paid before the table was shared.
__global__ __launch_bounds__(256) void k_rope_table(const rope_params rp, const int32_t * __restrict__ pos,
                                                    const float * __restrict__ ff, float2 * __restrict__ tab) {
    for (int ip = threadIdx.x; ip < rp.n_dims / 2; ip += blockDim.x) {
        float c, sn;
        rope_cs(rp, (float) pos[0], ip, ff, c, sn);
        tab[ip] = make_float2(c, sn);
    }
}

// the table for a ROPE node's parameters and position tensor, launched on first use in the
// graph (run_nodes clears the key: positions change every graph, the capture replays the
// launch); slot 3 of the scratch arena holds it
static const float2 * rope_table(exec_ctx & ctx, const ggml_tensor * r, const rope_params & rp, const int32_t * pos,
                                 const float * ff) {
    if (ctx.rt_table && ctx.rt_pos == pos && ctx.rt_ff == ff && memcmp(ctx.rt_params, r->op_params, sizeof(ctx.rt_params)) == 0) {
        return ctx.rt_table;
    }
    float2 * tab = (float2 *) ctx.scratch(3, sizeof(float2) * GEMV_ROPE_MAXPAIRS);
    hipLaunchKernelGGL(k_rope_table, dim3(1), dim3(256), 0, ctx.stream, rp, pos, ff, tab);
    ctx.rt_table = tab;
    ctx.rt_pos = pos;
    ctx.rt_ff = ff;
    memcpy(ctx.rt_params, r->op_params, sizeof(ctx.rt_params));
    return tab;
}

// ---- host ----------------------------------------------------------------------------------------
// kernel-timing mode: the GEMV kernel itself is launched with start/stop events
// (hipExtLaunchKernel records them at the dispatch's start and completion, without extra
// marker packets around it), so bench.py's per-launch time is the kernel's own duration
static thread_local hipEvent_t t_ev_beg = nullptr, t_ev_end = nullptr;

static int g_gemv_lds = -1;   // GGML_MI355X_GEMV_LDS: 1 = stage weights through LDS

template <class T, int R, int WPR>
static void launch_g(hipStream_t st, gemv_args & a, int nmat) {
    constexpr int RB = (4 / WPR) * R;
    a.blk0[0] = 0;
    for (int i = 0; i < GEMV_MAXMAT; ++i) {
        a.blk0[i + 1] = a.blk0[i] + (i < nmat ? ceil_div(a.M[i], RB) : 0);
    }
    for (int i = nmat; i < GEMV_MAXMAT; ++i) a.blk0[i] = a.blk0[nmat];   // never selected
    if (g_gemv_lds < 0) g_gemv_lds = getenv("GGML_MI355X_GEMV_LDS") ? atoi(getenv("GGML_MI355X_GEMV_LDS")) : 0;
    int64_t maxrow = 0;
    bool rows16 = true;
    for (int i = 0; i < nmat; ++i) {
        maxrow = std::max<int64_t>(maxrow, a.nb01[i]);
        rows16 = rows16 && a.nb01[i] % 16 == 0 && ((uintptr_t) a.W[i]) % 16 == 0;
    }
    const size_t slab = (size_t) RB * maxrow;
    if (g_gemv_lds && rows16 && slab <= 64 * 1024) {
        hipExtLaunchKernelGGL((k_gemv<T, R, WPR, true>), dim3((unsigned) a.blk0[nmat]), dim3(256), (uint32_t) slab, st,
                              t_ev_beg, t_ev_end, 0, a);
    } else {
        hipExtLaunchKernelGGL((k_gemv<T, R, WPR, false>), dim3((unsigned) a.blk0[nmat]), dim3(256), 0, st,
                              t_ev_beg, t_ev_end, 0, a);
    }
}

template <class T> struct is_kq_t { static constexpr bool value = false; };
template <> struct is_kq_t<g_q4_K> { static constexpr bool value = true; };
template <> struct is_kq_t<g_q5_K> { static constexpr bool value = true; };
template <> struct is_kq_t<g_q6_K> { static constexpr bool value = true; };

static int g_gemv_pipe = -1;   // GGML_MI355X_GEMV_PIPE: 0 disables the pipelined kernel
static int g_gemv_wgs = -1;    // GGML_MI355X_GEMV_WGS: persistent grid size
static int g_gemv_bal = -1;    // GGML_MI355X_GEMV_BAL: 1 = balanced resident grid (k rounds: k + 1)

static int g_num_cu = 0;

template <class T, int R, int WPR, int MODE>
static void launch_pipe_m(hipStream_t st, gemv_args & a, int nmat) {
    // the prologue is computed once per workgroup: 16-wave workgroups, one per CU
    constexpr int NWV = MODE == 2 ? 16 : 4;
    constexpr int RPG = (NWV / WPR) * R;
    a.blk0[0] = 0;
    for (int i = 0; i < GEMV_MAXMAT; ++i) a.blk0[i + 1] = a.blk0[i] + (i < nmat ? ceil_div(a.M[i], RPG) : 0);
    for (int i = nmat; i < GEMV_MAXMAT; ++i) a.blk0[i] = a.blk0[nmat];
    const int64_t ng = a.blk0[nmat];
    if (!g_num_cu) {
        int dev = 0;
        hipDeviceProp_t prop;
        MI_CHECK(hipGetDevice(&dev));
        MI_CHECK(hipGetDeviceProperties(&prop, dev));
        g_num_cu = prop.multiProcessorCount;
    }
    int64_t grid = std::min<int64_t>(ng, MODE == 2 ? g_num_cu : g_gemv_wgs);
    if constexpr (WPR == 4 && !std::is_same<T, g_q6_K>::value) {
        // four waves per row (K = 14336, the FFN down projection): one resident round of
        // workgroups (5 per CU at <= 96 VGPRs) beats 2048 single-group workgroups in two
        // rounds (Q4_K 4096 x 14336: 12.0 -> 11.2 us, scripts/probe_geom.py)
        static const int wgs4 = getenv("GGML_MI355X_GEMV_WGS4") ? atoi(getenv("GGML_MI355X_GEMV_WGS4")) : 5 * g_num_cu;
        if (MODE != 2 && wgs4 > 0) grid = std::min<int64_t>(ng, wgs4);
    }
    if (g_gemv_bal && MODE != 2) {
        // balanced resident grid: every workgroup resident at once and the same number of
        // groups (+-1 only when ng does not divide) per workgroup, so no second round of
        // workgroups and no tail of single-group waves
        static int occ = -1;
        if (occ < 0) {
            MI_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void *>(&k_gemv_pipe<T, R, WPR, MODE, NWV>), 64 * NWV, 0));
            occ = std::max(occ, 1);
        }
        const int64_t cap = (int64_t) occ * g_num_cu * (g_gemv_bal >= 2 ? g_gemv_bal - 1 : 1);
        const int64_t per = ceil_div(ng, cap);
        grid = ceil_div(ng, per);
    }
    if (MODE >= 1) grid = std::max<int64_t>(grid, ceil_div(ng, GEMV_MAXG));   // LDS-parked row sums
    const size_t lds = MODE == 2 ? prologue_lds_bytes(a.pro, a.pk) : 0;
    if (MODE == 0 && a.ids) {
        hipLaunchKernelGGL((k_gemv_pipe<T, R, WPR, 0, NWV, true>), dim3((unsigned) grid), dim3(64 * NWV), lds, st, a, ng);
    } else if (t_ev_beg) {
        hipExtLaunchKernelGGL((k_gemv_pipe<T, R, WPR, MODE, NWV>), dim3((unsigned) grid), dim3(64 * NWV), lds, st, t_ev_beg, t_ev_end, 0, a, ng);
    } else {
        hipLaunchKernelGGL((k_gemv_pipe<T, R, WPR, MODE, NWV>), dim3((unsigned) grid), dim3(64 * NWV), lds, st, a, ng);
    }
}

template <class T, int R, int WPR>
static void launch_pipe(hipStream_t st, gemv_args & a, int nmat) {
    bool epi = a.post_add != nullptr || a.need_pairs;
    for (int i = 0; i < nmat; ++i) {
        epi = epi || !a.dst[i] || a.silu[i] || a.f16out[i] || a.rope_out[i] || a.rope_f16[i];
    }
    if (a.pro) {
        if constexpr (is_kq_t<T>::value) launch_pipe_m<T, R, WPR, 2>(st, a, nmat);
        else GGML_ABORT("mi355x: GEMV prologue on a non-K-quant");
    } else if (epi) {
        launch_pipe_m<T, R, WPR, 1>(st, a, nmat);
    } else {
        launch_pipe_m<T, R, WPR, 0>(st, a, nmat);
    }
}

template <class T>
static bool launch_pipe_t(hipStream_t st, gemv_args & a, int nmat, int64_t Mt) {
    if (g_gemv_pipe < 0) g_gemv_pipe = getenv("GGML_MI355X_GEMV_PIPE") ? atoi(getenv("GGML_MI355X_GEMV_PIPE")) : 1;
    if (g_gemv_wgs < 0) g_gemv_wgs = getenv("GGML_MI355X_GEMV_WGS") ? atoi(getenv("GGML_MI355X_GEMV_WGS")) : 2048;
    if (g_gemv_bal < 0) g_gemv_bal = getenv("GGML_MI355X_GEMV_BAL") ? atoi(getenv("GGML_MI355X_GEMV_BAL")) : 0;
    if (!g_gemv_pipe || a.ntasks > 4 * WAVE) return false;
    if (a.need_pairs && a.rp.n_dims > 2 * GEMV_ROPE_MAXPAIRS) return false;
    const int wpr = a.ntasks <= WAVE ? 1 : (a.ntasks <= 2 * WAVE ? 2 : 4);
    // geometry measured on MI355X (tools/gemv_lab.hip, back-to-back launches over cold
    // weights): two rows per wave and a grid of up to 2048 workgroups is the fastest or within
    // 5 % of it on every Llama-3-8B shape; the 6-bit K-quant at K = 14336 prefers four rows;
    // a matrix too short to give 256 workgroups at two rows per wave takes one
    int R = 2;
    if (std::is_same<T, g_q6_K>::value && wpr == 4) R = 4;
    static const int r_wpr4 = getenv("GGML_MI355X_GEMV_R4W") ? atoi(getenv("GGML_MI355X_GEMV_R4W")) : 0;   // lab knob
    if (wpr == 4 && (r_wpr4 == 1 || r_wpr4 == 2 || r_wpr4 == 4)) R = r_wpr4;
    // a matrix too short to give 256 workgroups at two rows per wave takes one (the rope
    // epilogue reads its partner row from the LDS-parked sums of the same group)
    if (ceil_div(Mt * wpr, a.pro ? 32 : 8) < 256) R = 1;
    if (a.pro && R > 2) R = 2;   // 16-wave workgroups: four rows per wave would spill
    switch (R * 8 + wpr) {
        case 4 * 8 + 1: launch_pipe<T, 4, 1>(st, a, nmat); break;
        case 4 * 8 + 2: launch_pipe<T, 4, 2>(st, a, nmat); break;
        case 4 * 8 + 4: launch_pipe<T, 4, 4>(st, a, nmat); break;
        case 2 * 8 + 1: launch_pipe<T, 2, 1>(st, a, nmat); break;
        case 2 * 8 + 2: launch_pipe<T, 2, 2>(st, a, nmat); break;
        case 2 * 8 + 4: launch_pipe<T, 2, 4>(st, a, nmat); break;
        case 1 * 8 + 1: launch_pipe<T, 1, 1>(st, a, nmat); break;
        case 1 * 8 + 2: launch_pipe<T, 1, 2>(st, a, nmat); break;
        default:        launch_pipe<T, 1, 4>(st, a, nmat); break;
    }
    return true;
}

// two weight types in one launch (k_gemv_pipe2): p1's matrices at two rows per wave, p2's at
// R2 by the single-type rule; false when the shapes fall outside the compiled variants
template <class T1, class T2, int R2, int WPR>
static void launch_pipe2_v(hipStream_t st, gemv_args & a1, int n1, gemv_args & a2, int n2) {
    constexpr int NWV = 4;
    auto blocks = [](gemv_args & a, int nmat, int rpg) {
        a.blk0[0] = 0;
        for (int i = 0; i < GEMV_MAXMAT; ++i) a.blk0[i + 1] = a.blk0[i] + (i < nmat ? ceil_div(a.M[i], rpg) : 0);
        for (int i = nmat; i < GEMV_MAXMAT; ++i) a.blk0[i] = a.blk0[nmat];
        return a.blk0[nmat];
    };
    const int64_t ng1 = blocks(a1, n1, (NWV / WPR) * 2), ng2 = blocks(a2, n2, (NWV / WPR) * R2);
    auto grid_of = [](int64_t ng) {
        return std::max<int64_t>(std::min<int64_t>(ng, g_gemv_wgs), ceil_div(ng, GEMV_MAXG));   // LDS-parked row sums
    };
    const int64_t w1 = grid_of(ng1), w2 = grid_of(ng2);
    if (t_ev_beg) {
        hipExtLaunchKernelGGL((k_gemv_pipe2<T1, T2, R2, WPR>), dim3((unsigned) (w1 + w2)), dim3(64 * NWV), 0, st, t_ev_beg, t_ev_end,
                              0, a1, ng1, w1, a2, ng2);
    } else {
        hipLaunchKernelGGL((k_gemv_pipe2<T1, T2, R2, WPR>), dim3((unsigned) (w1 + w2)), dim3(64 * NWV), 0, st, a1, ng1, w1, a2, ng2);
    }
}

template <class T1, class T2>
static bool launch_pipe2_t(hipStream_t st, gemv_args & a1, int n1, gemv_args & a2, int n2) {
    if (g_gemv_pipe < 0) g_gemv_pipe = getenv("GGML_MI355X_GEMV_PIPE") ? atoi(getenv("GGML_MI355X_GEMV_PIPE")) : 1;
    if (g_gemv_wgs < 0) g_gemv_wgs = getenv("GGML_MI355X_GEMV_WGS") ? atoi(getenv("GGML_MI355X_GEMV_WGS")) : 2048;
    if (!g_gemv_pipe || a1.ntasks != a2.ntasks || a1.ntasks > 2 * WAVE) return false;
    if ((a1.need_pairs || a2.need_pairs) && a1.rp.n_dims > 2 * GEMV_ROPE_MAXPAIRS) return false;
    const int wpr = a1.ntasks <= WAVE ? 1 : 2;
    int64_t m1 = 0, m2 = 0;
    for (int i = 0; i < n1; ++i) m1 += a1.M[i];
    for (int i = 0; i < n2; ++i) m2 += a2.M[i];
    // the single-type launch's rows-per-wave rule (launch_pipe_t), per part
    if (ceil_div(m1 * wpr, 8) < 256) return false;
    const int r2 = ceil_div(m2 * wpr, 8) < 256 ? 1 : 2;
    switch (r2 * 8 + wpr) {
        case 1 * 8 + 1: launch_pipe2_v<T1, T2, 1, 1>(st, a1, n1, a2, n2); break;
        case 1 * 8 + 2: launch_pipe2_v<T1, T2, 1, 2>(st, a1, n1, a2, n2); break;
        case 2 * 8 + 1: launch_pipe2_v<T1, T2, 2, 1>(st, a1, n1, a2, n2); break;
        default:        launch_pipe2_v<T1, T2, 2, 2>(st, a1, n1, a2, n2); break;
    }
    return true;
}

// Q/K/V of two K-quant types (gemv_group); false: launch the parts separately
static bool launch_mixed(hipStream_t st, ggml_type t1, gemv_args & a1, int n1, ggml_type t2, gemv_args & a2, int n2) {
    if (t1 == GGML_TYPE_Q4_K && t2 == GGML_TYPE_Q6_K) return launch_pipe2_t<g_q4_K, g_q6_K>(st, a1, n1, a2, n2);
    if (t1 == GGML_TYPE_Q4_K && t2 == GGML_TYPE_Q5_K) return launch_pipe2_t<g_q4_K, g_q5_K>(st, a1, n1, a2, n2);
    if (t1 == GGML_TYPE_Q5_K && t2 == GGML_TYPE_Q6_K) return launch_pipe2_t<g_q5_K, g_q6_K>(st, a1, n1, a2, n2);
    return false;
}

bool gemv_mixed_ok(const ggml_tensor * mm0, const ggml_tensor * c) {
    static const int on = getenv("GGML_MI355X_GEMV_MIXED") ? atoi(getenv("GGML_MI355X_GEMV_MIXED")) : 1;
    const ggml_type t1 = mm0->src[0]->type, t2 = c->src[0]->type;
    return on && ((t1 == GGML_TYPE_Q4_K && (t2 == GGML_TYPE_Q6_K || t2 == GGML_TYPE_Q5_K)) ||
                  (t1 == GGML_TYPE_Q5_K && t2 == GGML_TYPE_Q6_K));
}

template <class T>
static void launch_t(hipStream_t st, gemv_args & a, int nmat) {
    int64_t Mt = 0;
    for (int i = 0; i < nmat; ++i) Mt += a.M[i];
    if (launch_pipe_t<T>(st, a, nmat, Mt)) return;
    GGML_ASSERT(!a.pro && "mi355x: GEMV prologue needs the pipelined kernel");
    // WPR depends on K only, so a row's summation order (and its bits) is the same whether
    // the matrix is launched alone or grouped; R (rows per wave: activation reuse, loads in
    // flight) is then the largest that keeps >= 2048 waves on the chip
    const int wpr = a.ntasks >= 8 * WAVE ? 4 : (a.ntasks >= 3 * WAVE ? 2 : 1);
    int R = ceil_div(Mt, 4) * wpr >= 2048 ? 4 : (ceil_div(Mt, 2) * wpr >= 2048 ? 2 : 1);
    if (R == 1 && a.need_pairs) R = 2;
    switch (R * 8 + wpr) {
        case 4 * 8 + 1: launch_g<T, 4, 1>(st, a, nmat); break;
        case 4 * 8 + 2: launch_g<T, 4, 2>(st, a, nmat); break;
        case 4 * 8 + 4: launch_g<T, 4, 4>(st, a, nmat); break;
        case 2 * 8 + 1: launch_g<T, 2, 1>(st, a, nmat); break;
        case 2 * 8 + 2: launch_g<T, 2, 2>(st, a, nmat); break;
        case 2 * 8 + 4: launch_g<T, 2, 4>(st, a, nmat); break;
        case 1 * 8 + 2: launch_g<T, 1, 2>(st, a, nmat); break;
        case 1 * 8 + 4: launch_g<T, 1, 4>(st, a, nmat); break;
        default:        launch_g<T, 1, 1>(st, a, nmat); break;
    }
}


static bool is_kq(ggml_type t) { return t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K; }

bool gemv_supported(const ggml_tensor * mm) {
    const ggml_tensor * w = mm->src[0];
    const ggml_tensor * x = mm->src[1];
    switch (w->type) {
        case GGML_TYPE_Q4_0: case GGML_TYPE_Q8_0: case GGML_TYPE_Q4_K: case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K: break;
        default: return false;
    }
    return x->type == GGML_TYPE_F32 && x->ne[1] == 1 && x->ne[2] == 1 && x->ne[3] == 1 && w->ne[2] == 1 && w->ne[3] == 1 &&
           mm->type == GGML_TYPE_F32 && ggml_is_contiguous(mm) && x->nb[0] == 4 &&
           w->ne[0] % ggml_blck_size(w->type) == 0;
}

bool gemv_epilogue_ok(const ggml_tensor * mm) { return gemv_supported(mm); }

// prologue: K-quant weights, K a multiple of 256 with ntasks = K/64 <= 256 (the pipelined
// kernel), every activation aligned for 16-byte loads
bool gemv_prologue_ok(const ggml_tensor * mm) {
    if (!gemv_supported(mm) || !is_kq(mm->src[0]->type)) return false;
    const int64_t K = mm->src[0]->ne[0];
    if (K % 256 != 0 || K / 64 > 4 * WAVE || prologue_lds_bytes(1, K) > 48 * 1024) return false;
    static int pipe = -1;
    if (pipe < 0) pipe = getenv("GGML_MI355X_GEMV_PIPE") ? atoi(getenv("GGML_MI355X_GEMV_PIPE")) : 1;
    return pipe != 0;
}

// one launch for up to three MUL_MATs sharing src1 (all gemv_supported, same weight type
// and K); silu[i] = optional SiLU output for matrix i
void gemv_group(exec_ctx & ctx, ggml_tensor * const * mms, int nmat, const gemv_epi * epi) {
    GGML_ASSERT(nmat >= 1 && nmat <= GEMV_MAXMAT);
    const ggml_tensor * src1 = mms[0]->src[1];
    const ggml_type wt = mms[0]->src[0]->type;
    const bool kq = is_kq(wt);
    double bytes = 0;
    for (int i = 0; i < nmat; ++i) bytes += (double) ggml_nbytes(mms[i]->src[0]) + (double) ggml_nbytes(mms[i]);
    bytes += (double) src1->ne[0] * (kq ? 1.14 : 1.0);

    q8_act act;
    gemv_args a = {};
    const int pro = epi ? epi->pro : 0;
    if (pro) {
        GGML_ASSERT(kq && gemv_prologue_ok(mms[0]));
        const int64_t K = src1->ne[0];
        carve_act(act, ctx.scratch(exec_ctx::QSLOT, q8_act::bytes(K, 1, true)), K, 1, true);
        a.pro = pro;
        a.pk = K;
        a.cq = act.qs; a.cd = act.d; a.cs = act.s;
        if (pro == 1) {
            const ggml_tensor * add = epi->pro_add;
            const ggml_tensor * nrm = epi->pro_norm;
            a.pa = add ? (const float *) add->src[0]->data : (const float *) nrm->src[0]->data;
            a.pb = add ? (const float *) add->src[1]->data : nullptr;
            a.o_add = add && !epi->pro_add_later ? (float *) add->data : nullptr;
            a.o_norm = epi->elide_norm ? nullptr : (float *) nrm->data;
            memcpy(&a.eps, nrm->op_params, sizeof(float));
            a.pw = epi->pro_mul ? (const float *) epi->pro_mul->src[1]->data : nullptr;
            a.o_mul = epi->pro_mul && !epi->elide_mul ? (float *) epi->pro_mul->data : nullptr;
        } else {
            a.pa = (const float *) epi->pro_mul->src[0]->data;
            a.pb = (const float *) epi->pro_mul->src[1]->data;
            a.o_mul = epi->elide_mul ? nullptr : (float *) epi->pro_mul->data;
        }
    } else if (!ctx.qcache_get(src1, kq, act)) {
        quantize_act(ctx, src1, kq, act, exec_ctx::QSLOT);
        ctx.qcache_put(src1, kq, act);
    }
    for (int i = 0; i < nmat; ++i) {
        const ggml_tensor * w = mms[i]->src[0];
        a.W[i] = (const uint8_t *) w->data;
        a.nb01[i] = w->nb[1];
        a.M[i] = w->ne[1];
        a.dst[i] = epi && epi->elide_dst[i] ? nullptr : (float *) mms[i]->data;
        a.silu[i] = epi && epi->silu[i] ? (float *) epi->silu[i]->data : nullptr;
        a.f16out[i] = epi ? (uint16_t * const *) epi->f16out[i] : nullptr;
        a.rope_out[i] = epi && epi->rope[i] && !epi->elide_rope[i] ? (float *) epi->rope[i]->data : nullptr;
        a.rope_f16[i] = epi ? (uint16_t * const *) epi->rope_f16[i] : nullptr;
        if (epi && epi->rope[i]) {
            const ggml_tensor * r = epi->rope[i];
            rope_params_of(r, a.rp);
            a.rope_pos = (const int32_t *) r->src[1]->data;
            a.rope_ff = r->src[2] ? (const float *) r->src[2]->data : nullptr;
            a.rope_d = r->src[0]->ne[0];
            a.need_pairs = 1;
        }
    }
    a.rtab_g = nullptr;
    if (a.need_pairs && a.rp.n_dims <= 2 * GEMV_ROPE_MAXPAIRS) {
        static const bool shared_tab = !getenv("GGML_MI355X_ROPE_TABLE") || atoi(getenv("GGML_MI355X_ROPE_TABLE")) != 0;
        if (shared_tab) {
            for (int i = 0; i < nmat; ++i) {
                if (epi && epi->rope[i]) { a.rtab_g = rope_table(ctx, epi->rope[i], a.rp, a.rope_pos, a.rope_ff); break; }
            }
        }
    }
    a.A = {act.qs, act.d, act.s};
    if (ctx.post_add) {
        ggml_tensor * ad = ctx.post_add;
        // in place over src[0] or src[1]: x = out (aliasing one input), y = the other input
        a.post_add = (float *) ad->data;
        a.post_b = (const float *) (ad->src[0]->data == ad->data ? ad->src[1]->data : ad->src[0]->data);
        a.post_n = ggml_nelements(ad);
        ctx.post_add = nullptr;
    }
    const int64_t nblk = src1->ne[0] / ggml_blck_size(wt);
    if (ctx.timing) {
        t_ev_beg = ctx.get_event();
        t_ev_end = ctx.get_event();
    }
    // matrices of a second K-quant type (V beside Q/K, gemv_mixed_ok): one two-body launch
    int ia[GEMV_MAXMAT], ib[GEMV_MAXMAT], n1 = 0, n2 = 0;
    ggml_type wt2 = wt;
    for (int i = 0; i < nmat; ++i) {
        const ggml_type ti = mms[i]->src[0]->type;
        if (ti == wt) ia[n1++] = i;
        else { GGML_ASSERT((wt2 == wt || wt2 == ti) && is_kq(ti) && kq && !pro); wt2 = ti; ib[n2++] = i; }
    }
    if (n2) {
        auto part = [&](gemv_args & d, const int * idx, int cnt) {
            d.need_pairs = 0;
            for (int k = 0; k < GEMV_MAXMAT; ++k) {
                const int s = idx[k < cnt ? k : 0];
                d.W[k] = a.W[s]; d.nb01[k] = a.nb01[s]; d.M[k] = a.M[s];
                d.dst[k] = a.dst[s]; d.silu[k] = a.silu[s]; d.f16out[k] = a.f16out[s];
                d.rope_out[k] = a.rope_out[s]; d.rope_f16[k] = a.rope_f16[s];
                if (k < cnt && epi && epi->rope[s]) d.need_pairs = 1;
            }
            d.ntasks = (int) (nblk * 4);
        };
        gemv_args a1 = a, a2 = a;
        part(a1, ia, n1);
        part(a2, ib, n2);
        a2.post_add = nullptr;   // stored by workgroup 0 of the first body
        if (!launch_mixed(ctx.stream, wt, a1, n1, wt2, a2, n2)) {
            auto one = [&](ggml_type t, gemv_args & d, int cnt) {
                switch (t) {
                    case GGML_TYPE_Q4_K: launch_t<g_q4_K>(ctx.stream, d, cnt); break;
                    case GGML_TYPE_Q5_K: launch_t<g_q5_K>(ctx.stream, d, cnt); break;
                    default:             launch_t<g_q6_K>(ctx.stream, d, cnt); break;
                }
            };
            one(wt, a1, n1);
            if (ctx.timing) {   // the second launch is timed as its own mat-vec
                ctx.pending.push_back({t_ev_beg, t_ev_end, bytes, TK_MMV});
                t_ev_beg = ctx.get_event();
                t_ev_end = ctx.get_event();
                bytes = 0;
            }
            one(wt2, a2, n2);
        }
    } else switch (wt) {
        case GGML_TYPE_Q4_K: a.ntasks = (int) (nblk * 4); launch_t<g_q4_K>(ctx.stream, a, nmat); break;
        case GGML_TYPE_Q5_K: a.ntasks = (int) (nblk * 4); launch_t<g_q5_K>(ctx.stream, a, nmat); break;
        case GGML_TYPE_Q6_K: a.ntasks = (int) (nblk * 4); launch_t<g_q6_K>(ctx.stream, a, nmat); break;
        case GGML_TYPE_Q8_0: a.ntasks = (int) nblk;       launch_t<g_q8_0>(ctx.stream, a, nmat); break;
        case GGML_TYPE_Q4_0: a.ntasks = (int) nblk;       launch_t<g_q4_0>(ctx.stream, a, nmat); break;
        default: GGML_ABORT("mi355x: gemv type");
    }
    if (pro) ctx.qcache_put(src1, true, act);   // written by workgroup 0 of this launch
    if (ctx.timing) {
        ctx.pending.push_back({t_ev_beg, t_ev_end, bytes, TK_MMV});
        t_ev_beg = t_ev_end = nullptr;
    }
}

// MUL_MAT_ID of one token (decode) on the pipelined mat-vec: the routed experts are the
// matrices of a grouped launch, their bases read from ids on the device.  A shared activation
// (b->ne[1] == 1: up / gate) makes one launch over the n_used experts; per-slot activations
// (down) one launch per slot.  Returns false when the pipelined kernel does not apply.
bool gemv_mul_mat_id(exec_ctx & ctx, ggml_tensor * dst, const q8_act & act) {
    const ggml_tensor * as = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const ggml_tensor * ids = dst->src[2];
    const ggml_type wt = as->type;
    const int64_t n_used = ids->ne[0], K = as->ne[0];
    if (ids->ne[1] != 1 || n_used > GEMV_MAXMAT || (b->ne[1] != 1 && b->ne[1] != n_used)) return false;
    if (wt != GGML_TYPE_Q4_K && wt != GGML_TYPE_Q5_K && wt != GGML_TYPE_Q6_K && wt != GGML_TYPE_Q8_0 && wt != GGML_TYPE_Q4_0) return false;
    if (ids->nb[0] % sizeof(int32_t) != 0) return false;
    const int64_t nblk = K / ggml_blck_size(wt);
    const int per = (wt == GGML_TYPE_Q8_0 || wt == GGML_TYPE_Q4_0) ? 1 : 4;
    if (nblk * per > 4 * WAVE) return false;   // the pipelined kernel covers K in one pass per wave
    const bool shared = b->ne[1] == 1;
    const int nlaunch = shared ? 1 : (int) n_used;
    for (int l = 0; l < nlaunch; ++l) {
        gemv_args a = {};
        const int nmat = shared ? (int) n_used : 1;
        a.ids = (const int32_t *) ids->data;
        a.nb02 = as->nb[2];
        for (int m = 0; m < nmat; ++m) {
            const int e = shared ? m : l;
            a.W[m] = (const uint8_t *) as->data;
            a.nb01[m] = as->nb[1];
            a.M[m] = as->ne[1];
            a.dst[m] = (float *) ((char *) dst->data + e * dst->nb[1]);
            a.ids_e[m] = e * (int64_t) (ids->nb[0] / sizeof(int32_t));
        }
        for (int m = nmat; m < GEMV_MAXMAT; ++m) a.ids_e[m] = a.ids_e[0];
        const int64_t col = shared ? 0 : l;
        a.A = {act.qs + col * act.qs_stride(), act.d + col * act.d_stride(), act.s + col * act.s_stride()};
        a.ntasks = (int) (nblk * per);
        int64_t Mt = a.M[0] * nmat;
        bool ok = false;
        switch (wt) {
            case GGML_TYPE_Q4_K: ok = launch_pipe_t<g_q4_K>(ctx.stream, a, nmat, Mt); break;
            case GGML_TYPE_Q5_K: ok = launch_pipe_t<g_q5_K>(ctx.stream, a, nmat, Mt); break;
            case GGML_TYPE_Q6_K: ok = launch_pipe_t<g_q6_K>(ctx.stream, a, nmat, Mt); break;
            case GGML_TYPE_Q8_0: ok = launch_pipe_t<g_q8_0>(ctx.stream, a, nmat, Mt); break;
            default:             ok = launch_pipe_t<g_q4_0>(ctx.stream, a, nmat, Mt); break;
        }
        if (!ok) {
            GGML_ASSERT(l == 0 && "mi355x: pipelined MUL_MAT_ID launch refused after the first slot");
            return false;
        }
    }
    return true;
}

}  // namespace mi355x
