// k_mmv.hip — activation quantization and the decode mat-vec (GEMV) path.
//
// Parity design (SURVEY.md finding 6): the CPU backend never multiplies quantized
// weights with f32 activations.  It first quantizes each activation row to the weight
// type's vec_dot_type (ggml-cpu/ggml-cpu.c:193-282, quantize loop ggml-cpu.c:1254-1289):
//   * K-quants (Q4_K/Q5_K/Q6_K) -> Q8_K  : quantize_row_q8_K_ref  (ggml-quants.c:2471-2508)
//   * Q4_0/Q8_0                 -> Q8_0  : x86 quantize_row_q8_0 (ggml-cpu/arch/x86/quants.c:278-372)
// and then takes integer dot products per sub-block (ggml-cpu/quants.c:110-297, 514-722).
// We reproduce the quantizers bit-exactly (so every integer partial sum equals the
// CPU's) and differ only in the order of the fp32 combination of block results.
//
// Kernel shape (MI355X-first, not the CUDA mmvq layout): one wavefront walks one weight
// row; each lane owns a "task" = a 32..64-weight slice of one quant block, loads it with
// 16-byte (unaligned-tolerant) vector loads straight into VGPRs, unpacks nibbles with
// bit ops and issues v_dot4_i32_i8 against the pre-quantized activation slice (L1/L2
// resident).  Partial sums reduce across the wave with DPP shuffles; for short matrices
// (M small) WPR waves split one row's K range and reduce through LDS so the grid still
// fills 256 CUs.
#include "ops.h"
#include "quant_act.h"

#include <algorithm>

namespace mi355x {

// ------------------------------------------------------------------------------------------
// activation quantizers
// ------------------------------------------------------------------------------------------

// Q8_K, one wave per 256-element block; lane l holds x[4l..4l+3] (quant_act.h).
__global__ __launch_bounds__(64) void k_quantize_q8_K(const char * __restrict__ x, int64_t K,
                                                      int64_t ne1, int64_t ne2,
                                                      int64_t nb1, int64_t nb2, int64_t nb3,
                                                      int8_t * __restrict__ qs, float * __restrict__ dd,
                                                      int16_t * __restrict__ bs) {
    const int lane = threadIdx.x;
    const int64_t b   = blockIdx.x;
    const int64_t col = blockIdx.y;
    const int64_t i1 = col % ne1, i2 = (col / ne1) % ne2, i3 = col / (ne1 * ne2);
    const float * row = (const float *) (x + i1 * nb1 + i2 * nb2 + i3 * nb3);
    const uint4 v = ld16(row + b * 256 + 4 * lane);
    const float vv[4] = {__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
    q8K_wave(vv, lane, qs + col * K + b * 256, bs + col * (K / 16) + b * 16, dd + col * (K / 256) + b);
}

// Q8_0 (x86 rounding), eight 32-blocks per wave (quant_act.h).
__global__ __launch_bounds__(64) void k_quantize_q8_0(const char * __restrict__ x, int64_t K,
                                                      int64_t ne1, int64_t ne2,
                                                      int64_t nb1, int64_t nb2, int64_t nb3,
                                                      int8_t * __restrict__ qs, float * __restrict__ dd,
                                                      int16_t * __restrict__ bs) {
    const int lane = threadIdx.x;
    const int64_t col = blockIdx.y;
    const int64_t c0 = (int64_t) blockIdx.x * 256;
    const int64_t e0 = c0 + 4 * lane;
    const int64_t i1 = col % ne1, i2 = (col / ne1) % ne2, i3 = col / (ne1 * ne2);
    const float * row = (const float *) (x + i1 * nb1 + i2 * nb2 + i3 * nb3);
    const bool valid = e0 < K;
    float vv[4] = {0.f, 0.f, 0.f, 0.f};
    if (valid) {
        const uint4 v = ld16(row + e0);
        vv[0] = __uint_as_float(v.x); vv[1] = __uint_as_float(v.y); vv[2] = __uint_as_float(v.z); vv[3] = __uint_as_float(v.w);
    }
    q8_0_wave(vv, lane, valid, qs + col * K + c0, dd + col * (K / 32) + c0 / 32, bs + col * (K / 32) + c0 / 32);
}

size_t q8_act::bytes(int64_t K, int64_t ncols, bool k_quant) {
    const int64_t nd = k_quant ? K / 256 : K / 32;
    const int64_t ns = k_quant ? K / 16 : K / 32;
    auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
    return al(K * ncols) + al(nd * ncols * 4) + al(ns * ncols * 2);
}

void carve_act(q8_act & act, void * base, int64_t K, int64_t ncols, bool k_quant) {
    auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
    const int64_t nd = k_quant ? K / 256 : K / 32;
    char * p = (char *) base;
    act.qs = (int8_t *) p;  p += al(K * ncols);
    act.d  = (float *) p;   p += al(nd * ncols * 4);
    act.s  = (int16_t *) p;
    act.K = K; act.ncols = ncols; act.k_quant = k_quant;
}

void quantize_act(exec_ctx & ctx, const ggml_tensor * src, bool k_quant, q8_act & act, int slot) {
    const int64_t K = src->ne[0];
    const int64_t ncols = src->ne[1] * src->ne[2] * src->ne[3];
    GGML_ASSERT(src->type == GGML_TYPE_F32 && src->nb[0] == 4);
    GGML_ASSERT(K % (k_quant ? 256 : 32) == 0);
    carve_act(act, ctx.scratch(slot, q8_act::bytes(K, ncols, k_quant)), K, ncols, k_quant);
    dim3 grid((unsigned) ceil_div(K, 256), (unsigned) ncols);
    if (k_quant) {
        hipLaunchKernelGGL(k_quantize_q8_K, grid, dim3(64), 0, ctx.stream, (const char *) src->data, K,
                           src->ne[1], src->ne[2], (int64_t) src->nb[1], (int64_t) src->nb[2], (int64_t) src->nb[3],
                           act.qs, act.d, act.s);
    } else {
        hipLaunchKernelGGL(k_quantize_q8_0, grid, dim3(64), 0, ctx.stream, (const char *) src->data, K,
                           src->ne[1], src->ne[2], (int64_t) src->nb[1], (int64_t) src->nb[2], (int64_t) src->nb[3],
                           act.qs, act.d, act.s);
    }
}

void quantize_act_raw(hipStream_t stream, const float * x, int64_t K, int64_t ncols, int64_t row_stride_elems,
                      bool k_quant, q8_act & act) {
    dim3 grid((unsigned) ceil_div(K, 256), (unsigned) ncols);
    const int64_t nb1 = row_stride_elems * 4;
    if (k_quant) {
        hipLaunchKernelGGL(k_quantize_q8_K, grid, dim3(64), 0, stream, (const char *) x, K, ncols, (int64_t) 1,
                           nb1, nb1 * ncols, nb1 * ncols, act.qs, act.d, act.s);
    } else {
        hipLaunchKernelGGL(k_quantize_q8_0, grid, dim3(64), 0, stream, (const char *) x, K, ncols, (int64_t) 1,
                           nb1, nb1 * ncols, nb1 * ncols, act.qs, act.d, act.s);
    }
}

// ------------------------------------------------------------------------------------------
// per-type tasks: acc[c] += <weight slice, activation slice of column c>
// ------------------------------------------------------------------------------------------
struct act_view {
    const int8_t * qs; const float * d; const int16_t * s;
    int64_t qs_st, d_st, s_st;  // per-column strides (elements)
};

__device__ __forceinline__ void ld_act64(const int8_t * p, int (&a)[16]) {
    const int4 * v = (const int4 *) p;
    int4 v0 = v[0], v1 = v[1], v2 = v[2], v3 = v[3];
    a[0] = v0.x; a[1] = v0.y; a[2]  = v0.z; a[3]  = v0.w;
    a[4] = v1.x; a[5] = v1.y; a[6]  = v1.z; a[7]  = v1.w;
    a[8] = v2.x; a[9] = v2.y; a[10] = v2.z; a[11] = v2.w;
    a[12] = v3.x; a[13] = v3.y; a[14] = v3.z; a[15] = v3.w;
}

// Q4_K/Q5_K packed 6-bit scales -> (scale, min) of sub-blocks 2j and 2j+1, using the
// same word shuffle as ggml_vec_dot_q4_K_q8_K (ggml-cpu/quants.c:539-545).
__device__ __forceinline__ void k4_scales(uint32_t s0, uint32_t s1, uint32_t s2, int j,
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

template <int NC>
struct task_q4_K {
    static constexpr int per_block = 4;      // 64 weights per task
    static constexpr int blk_bytes = 144;
    __device__ static void run(const uint8_t * wrow, int t, const act_view & A, int nc, float (&acc)[NC]) {
        const int b = t >> 2, j = t & 3;
        const uint8_t * blk = wrow + (int64_t) b * 144;
        const uint4 hdr = ld16(blk);
        const uint4 qa  = ld16(blk + 16 + 32 * j);
        const uint4 qb  = ld16(blk + 32 + 32 * j);
        const float d    = h2f(hdr.x & 0xffff);
        const float dmin = h2f(hdr.x >> 16);
        int sc_lo, sc_hi, m_lo, m_hi;
        k4_scales(hdr.y, hdr.z, hdr.w, j, sc_lo, sc_hi, m_lo, m_hi);
        const uint32_t q[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= nc) break;
            int a[16];
            ld_act64(A.qs + c * A.qs_st + b * 256 + 64 * j, a);
            int dl = 0, dh = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                dl = dot4((int) (q[i] & 0x0f0f0f0f), a[i], dl);
                dh = dot4((int) ((q[i] >> 4) & 0x0f0f0f0f), a[8 + i], dh);
            }
            const int16_t * bs = A.s + c * A.s_st + b * 16 + 4 * j;
            const int sumi = sc_lo * dl + sc_hi * dh;
            const int summ = m_lo * (bs[0] + bs[1]) + m_hi * (bs[2] + bs[3]);
            const float dy = A.d[c * A.d_st + b];
            acc[c] += (d * dy) * (float) sumi - (dmin * dy) * (float) summ;
        }
    }
};

template <int NC>
struct task_q5_K {
    static constexpr int per_block = 4;
    static constexpr int blk_bytes = 176;
    __device__ static void run(const uint8_t * wrow, int t, const act_view & A, int nc, float (&acc)[NC]) {
        const int b = t >> 2, j = t & 3;
        const uint8_t * blk = wrow + (int64_t) b * 176;
        const uint4 hdr = ld16(blk);
        const uint4 ha  = ld16(blk + 16);
        const uint4 hb  = ld16(blk + 32);
        const uint4 qa  = ld16(blk + 48 + 32 * j);
        const uint4 qb  = ld16(blk + 64 + 32 * j);
        const float d    = h2f(hdr.x & 0xffff);
        const float dmin = h2f(hdr.x >> 16);
        int sc_lo, sc_hi, m_lo, m_hi;
        k4_scales(hdr.y, hdr.z, hdr.w, j, sc_lo, sc_hi, m_lo, m_hi);
        const uint32_t q[8]  = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        const uint32_t qh[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
        uint32_t lo[8], hi[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            lo[i] = (q[i] & 0x0f0f0f0f) | (((qh[i] >> (2 * j)) & 0x01010101) << 4);
            hi[i] = ((q[i] >> 4) & 0x0f0f0f0f) | (((qh[i] >> (2 * j + 1)) & 0x01010101) << 4);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= nc) break;
            int a[16];
            ld_act64(A.qs + c * A.qs_st + b * 256 + 64 * j, a);
            int dl = 0, dh = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                dl = dot4((int) lo[i], a[i], dl);
                dh = dot4((int) hi[i], a[8 + i], dh);
            }
            const int16_t * bs = A.s + c * A.s_st + b * 16 + 4 * j;
            const int sumi = sc_lo * dl + sc_hi * dh;
            const int summ = m_lo * (bs[0] + bs[1]) + m_hi * (bs[2] + bs[3]);
            const float dy = A.d[c * A.d_st + b];
            acc[c] += (d * dy) * (float) sumi - (dmin * dy) * (float) summ;
        }
    }
};

// Q6_K task (b, half h, lr): ql[l], ql[l+32], qh[l] for l in 16*lr .. 16*lr+15 of half h,
// i.e. 4 groups of 16 weights at offsets 0/32/64/96 (dequantize_row_q6_K, ggml-quants.c:1684).
template <int NC>
struct task_q6_K {
    static constexpr int per_block = 4;
    static constexpr int blk_bytes = 210;
    __device__ static void run(const uint8_t * wrow, int t, const act_view & A, int nc, float (&acc)[NC]) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        const uint8_t * blk = wrow + (int64_t) b * 210;
        const uint4 la = ld16(blk + 64 * h + 16 * lr);
        const uint4 lb = ld16(blk + 64 * h + 32 + 16 * lr);
        const uint4 hh = ld16(blk + 128 + 32 * h + 16 * lr);
        const uint2 sc8 = ld8(blk + 192 + 8 * h);
        const float d = h2f(ld2(blk + 208));
        // scales for groups g=0..3 are sc[8h + lr + 2g]
        const int sc0 = (int8_t) ((sc8.x >> (8 * lr)) & 0xff);
        const int sc1 = (int8_t) ((sc8.x >> (8 * lr + 16)) & 0xff);
        const int sc2 = (int8_t) ((sc8.y >> (8 * lr)) & 0xff);
        const int sc3 = (int8_t) ((sc8.y >> (8 * lr + 16)) & 0xff);
        const uint32_t L[4] = {la.x, la.y, la.z, la.w};
        const uint32_t M[4] = {lb.x, lb.y, lb.z, lb.w};
        const uint32_t H[4] = {hh.x, hh.y, hh.z, hh.w};
        uint32_t g0[4], g1[4], g2[4], g3[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            g0[i] = (L[i] & 0x0f0f0f0f)        | ((H[i] & 0x03030303) << 4);
            g1[i] = (M[i] & 0x0f0f0f0f)        | (((H[i] >> 2) & 0x03030303) << 4);
            g2[i] = ((L[i] >> 4) & 0x0f0f0f0f) | (((H[i] >> 4) & 0x03030303) << 4);
            g3[i] = ((M[i] >> 4) & 0x0f0f0f0f) | (((H[i] >> 6) & 0x03030303) << 4);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= nc) break;
            const int8_t * ap = A.qs + c * A.qs_st + b * 256 + 128 * h + 16 * lr;
            const int4 a0 = *(const int4 *) (ap);
            const int4 a1 = *(const int4 *) (ap + 32);
            const int4 a2 = *(const int4 *) (ap + 64);
            const int4 a3 = *(const int4 *) (ap + 96);
            int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
            s0 = dot4(g0[0], a0.x, s0); s0 = dot4(g0[1], a0.y, s0); s0 = dot4(g0[2], a0.z, s0); s0 = dot4(g0[3], a0.w, s0);
            s1 = dot4(g1[0], a1.x, s1); s1 = dot4(g1[1], a1.y, s1); s1 = dot4(g1[2], a1.z, s1); s1 = dot4(g1[3], a1.w, s1);
            s2 = dot4(g2[0], a2.x, s2); s2 = dot4(g2[1], a2.y, s2); s2 = dot4(g2[2], a2.z, s2); s2 = dot4(g2[3], a2.w, s2);
            s3 = dot4(g3[0], a3.x, s3); s3 = dot4(g3[1], a3.y, s3); s3 = dot4(g3[2], a3.z, s3); s3 = dot4(g3[3], a3.w, s3);
            // (q - 32) * a  ==  q*a - 32*a ; the 16-sums of a are the Q8_K bsums
            const int16_t * bs = A.s + c * A.s_st + b * 16 + 8 * h + lr;
            s0 -= 32 * bs[0]; s1 -= 32 * bs[2]; s2 -= 32 * bs[4]; s3 -= 32 * bs[6];
            const int sumi = sc0 * s0 + sc1 * s1 + sc2 * s2 + sc3 * s3;
            const float dy = A.d[c * A.d_st + b];
            acc[c] += (d * dy) * (float) sumi;
        }
    }
};

template <int NC>
struct task_q8_0 {
    static constexpr int per_block = 1;   // 32 weights per task
    static constexpr int blk_bytes = 34;
    __device__ static void run(const uint8_t * wrow, int t, const act_view & A, int nc, float (&acc)[NC]) {
        const uint8_t * blk = wrow + (int64_t) t * 34;
        const float d = h2f(ld2(blk));
        const uint4 qa = ld16(blk + 2);
        const uint4 qb = ld16(blk + 18);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= nc) break;
            const int4 * ap = (const int4 *) (A.qs + c * A.qs_st + (int64_t) t * 32);
            const int4 a0 = ap[0], a1 = ap[1];
            int s = 0;
            s = dot4(qa.x, a0.x, s); s = dot4(qa.y, a0.y, s); s = dot4(qa.z, a0.z, s); s = dot4(qa.w, a0.w, s);
            s = dot4(qb.x, a1.x, s); s = dot4(qb.y, a1.y, s); s = dot4(qb.z, a1.z, s); s = dot4(qb.w, a1.w, s);
            acc[c] += (float) s * (d * A.d[c * A.d_st + t]);
        }
    }
};

template <int NC>
struct task_q4_0 {
    static constexpr int per_block = 1;
    static constexpr int blk_bytes = 18;
    __device__ static void run(const uint8_t * wrow, int t, const act_view & A, int nc, float (&acc)[NC]) {
        const uint8_t * blk = wrow + (int64_t) t * 18;
        const float d = h2f(ld2(blk));
        const uint4 q = ld16(blk + 2);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= nc) break;
            const int4 * ap = (const int4 *) (A.qs + c * A.qs_st + (int64_t) t * 32);
            const int4 a0 = ap[0], a1 = ap[1];
            const int al[4] = {a0.x, a0.y, a0.z, a0.w};
            const int ah[4] = {a1.x, a1.y, a1.z, a1.w};
            int s = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                s = dot4((int) (w[i] & 0x0f0f0f0f), al[i], s);
                s = dot4((int) ((w[i] >> 4) & 0x0f0f0f0f), ah[i], s);
            }
            s -= 8 * A.s[c * A.s_st + t];   // (q-8)*a
            acc[c] += (float) s * (d * A.d[c * A.d_st + t]);
        }
    }
};

// ------------------------------------------------------------------------------------------
// GEMV kernel: grid (row groups, column groups, i12*i13), 256 threads = 4 waves.
// WPR waves cooperate on one row.
// ------------------------------------------------------------------------------------------
struct mmv_args {
    const uint8_t * W; int64_t nb01, nb02, nb03; int64_t M; int64_t nblk;
    act_view A; int64_t ne11, ne12, r2, r3;
    float * dst; int64_t nb1, nb2, nb3;   // in bytes
};

template <template <int> class TASK, int NC, int WPR>
__global__ __launch_bounds__(256) void k_mmv_q(const mmv_args p) {
    using T = TASK<NC>;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int RPB = 4 / WPR;
    const int64_t row = (int64_t) blockIdx.x * RPB + wave / WPR;
    const int wsub = wave % WPR;
    const int64_t c0 = (int64_t) blockIdx.y * NC;
    const int64_t i12 = blockIdx.z % p.ne12, i13 = blockIdx.z / p.ne12;
    const int nc = (int) min((int64_t) NC, p.ne11 - c0);

    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0f;

    if (row < p.M) {
        const uint8_t * wrow = p.W + (i12 / p.r2) * p.nb02 + (i13 / p.r3) * p.nb03 + row * p.nb01;
        const int64_t colbase = c0 + p.ne11 * (i12 + p.ne12 * i13);
        act_view A = p.A;
        A.qs += colbase * A.qs_st; A.d += colbase * A.d_st; A.s += colbase * A.s_st;
        const int ntasks = (int) (p.nblk * T::per_block);
        for (int t = wsub * WAVE + lane; t < ntasks; t += WAVE * WPR) {
            T::run(wrow, t, A, nc, acc);
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = wave_sum(acc[c]);

    if constexpr (WPR > 1) {
        __shared__ float red[4][NC];
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < NC; ++c) red[wave][c] = acc[c];
        }
        __syncthreads();
        if (wsub == 0 && lane == 0) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                float s = red[wave][c];
#pragma unroll
                for (int w = 1; w < WPR; ++w) s += red[wave + w][c];
                acc[c] = s;
            }
        }
    }
    if (row < p.M && wsub == 0 && lane == 0) {
        char * d = (char *) p.dst + i12 * p.nb2 + i13 * p.nb3 + row * 4;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < nc) *(float *) (d + (c0 + c) * p.nb1) = acc[c];
        }
    }
}

// ------------------------------------------------------------------------------------------
// f16 / f32 weights (FA-off KQ / KQV, f16/f32 projections): float dot, 8 elements per task
// ------------------------------------------------------------------------------------------
struct mmv_f_args {
    const char * W; int64_t nb01, nb02, nb03; int64_t M; int64_t K;
    const char * X; int64_t nb11, nb12, nb13; int64_t ne11, ne12, r2, r3;
    float * dst; int64_t nb1, nb2, nb3;
};

template <typename WT, int NC, int WPR>
__global__ __launch_bounds__(256) void k_mmv_f(const mmv_f_args p) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int RPB = 4 / WPR;
    const int64_t row = (int64_t) blockIdx.x * RPB + wave / WPR;
    const int wsub = wave % WPR;
    const int64_t c0 = (int64_t) blockIdx.y * NC;
    const int64_t i12 = blockIdx.z % p.ne12, i13 = blockIdx.z / p.ne12;
    const int nc = (int) min((int64_t) NC, p.ne11 - c0);

    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0f;

    if (row < p.M) {
        const char * wrow = p.W + (i12 / p.r2) * p.nb02 + (i13 / p.r3) * p.nb03 + row * p.nb01;
        const char * xb = p.X + i12 * p.nb12 + i13 * p.nb13 + c0 * p.nb11;
        const int64_t nvec = p.K / 8;
        for (int64_t t = wsub * WAVE + lane; t < nvec; t += WAVE * WPR) {
            float w[8];
            if constexpr (sizeof(WT) == 2) {
                const uint4 v = ld16(wrow + t * 16);
                const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) { w[2 * i] = h2f(u[i] & 0xffff); w[2 * i + 1] = h2f(u[i] >> 16); }
            } else {
                const uint4 v0 = ld16(wrow + t * 32), v1 = ld16(wrow + t * 32 + 16);
                w[0] = __uint_as_float(v0.x); w[1] = __uint_as_float(v0.y); w[2] = __uint_as_float(v0.z); w[3] = __uint_as_float(v0.w);
                w[4] = __uint_as_float(v1.x); w[5] = __uint_as_float(v1.y); w[6] = __uint_as_float(v1.z); w[7] = __uint_as_float(v1.w);
            }
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (c >= nc) break;
                const char * xr = xb + c * p.nb11 + t * 32;
                const uint4 x0 = ld16(xr), x1 = ld16(xr + 16);
                float s = acc[c];
                s = fmaf(w[0], __uint_as_float(x0.x), s); s = fmaf(w[1], __uint_as_float(x0.y), s);
                s = fmaf(w[2], __uint_as_float(x0.z), s); s = fmaf(w[3], __uint_as_float(x0.w), s);
                s = fmaf(w[4], __uint_as_float(x1.x), s); s = fmaf(w[5], __uint_as_float(x1.y), s);
                s = fmaf(w[6], __uint_as_float(x1.z), s); s = fmaf(w[7], __uint_as_float(x1.w), s);
                acc[c] = s;
            }
        }
        // tail elements (K % 8)
        for (int64_t k = nvec * 8 + wsub * WAVE + lane; k < p.K; k += WAVE * WPR) {
            float w;
            if constexpr (sizeof(WT) == 2) w = h2f(ld2(wrow + k * 2));
            else w = __uint_as_float(ld4(wrow + k * 4));
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if (c >= nc) break;
                acc[c] = fmaf(w, *(const float *) (xb + c * p.nb11 + k * 4), acc[c]);
            }
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = wave_sum(acc[c]);
    if constexpr (WPR > 1) {
        __shared__ float red[4][NC];
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < NC; ++c) red[wave][c] = acc[c];
        }
        __syncthreads();
        if (wsub == 0 && lane == 0) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                float s = red[wave][c];
#pragma unroll
                for (int w = 1; w < WPR; ++w) s += red[wave + w][c];
                acc[c] = s;
            }
        }
    }
    if (row < p.M && wsub == 0 && lane == 0) {
        char * d = (char *) p.dst + i12 * p.nb2 + i13 * p.nb3 + row * 4;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < nc) *(float *) (d + (c0 + c) * p.nb1) = acc[c];
        }
    }
}

// ------------------------------------------------------------------------------------------
// f16 / f32 weights, CPU-exact order: the CPU converts src1 to the weight's vec_dot_type
// (f16 for f16 weights) and takes ggml_vec_dot_f16 / ggml_vec_dot_f32 (vec.cpp:191-231,
// AVX-512: 16 lanes x 4 f32 accumulators, REDUCE tree, double leftovers).  One thread per
// (row, column) reproduces that order exactly.  Used for the FA-off KQ / KQV products and
// for f16/f32 weight matrices (not on the FA decode hot path).
// ------------------------------------------------------------------------------------------
template <typename WT>
__global__ __launch_bounds__(256) void k_mmv_f_exact(const mmv_f_args p) {
    // one wave per row: lane s keeps the AVX-512 partial acc[s] of ggml_vec_dot_f32 (4
    // accumulators x 16 lanes, FMA'd over the row in steps of 64), so the loads are coalesced
    // 256-B rows and the sum order is the CPU's; lane 0 then forms REDUCE + the
    // _mm512_reduce_add_ps tree and the scalar tail in double
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row = (int64_t) blockIdx.x * 4 + wave;
    const int64_t c = blockIdx.y;
    const int64_t i12 = blockIdx.z % p.ne12, i13 = blockIdx.z / p.ne12;
    const bool ok = row < p.M;
    const char * wrow = p.W + (i12 / p.r2) * p.nb02 + (i13 / p.r3) * p.nb03 + (ok ? row : 0) * p.nb01;
    const float * x = (const float *) (p.X + i12 * p.nb12 + i13 * p.nb13 + c * p.nb11);
    auto wv = [&](int64_t k) -> float {
        if constexpr (sizeof(WT) == 2) return h2f(ld2(wrow + 2 * k));
        else return __uint_as_float(ld4(wrow + 4 * k));
    };
    auto xv = [&](int64_t k) -> float {
        if constexpr (sizeof(WT) == 2) return h2f(f2h(x[k]));  // src1 -> f16 (vec_dot_type)
        else return x[k];
    };
    const int64_t np = p.K & ~int64_t(63);
    float acc = 0.0f;
#pragma unroll 8
    for (int64_t i = 0; i < np; i += 64) acc = fmaf(wv(i + lane), xv(i + lane), acc);
    __shared__ float part[4][64];
    part[wave][lane] = acc;
    __syncthreads();
    if (ok && lane == 0) {
        const float * a = part[wave];
        float w[16];
#pragma unroll
        for (int l = 0; l < 16; ++l) w[l] = __fadd_rn(__fadd_rn(a[l], a[32 + l]), __fadd_rn(a[16 + l], a[48 + l]));
        double sumf = (double) reduce16_avx512(w);
        for (int64_t k = np; k < p.K; ++k) sumf += (double) __fmul_rn(wv(k), xv(k));
        *(float *) ((char *) p.dst + i12 * p.nb2 + i13 * p.nb3 + c * p.nb1 + row * 4) = (float) sumf;
    }
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
static int64_t total_rows_waves(int64_t M, int64_t ncolgroups, int64_t nbatch) { return M * ncolgroups * nbatch; }

template <template <int> class TASK, int NC>
static void launch_mmv_q_nc(hipStream_t st, const mmv_args & a, int64_t ncg, int64_t nbatch, int wpr) {
    if (wpr == 4) {
        dim3 grid((unsigned) a.M, (unsigned) ncg, (unsigned) nbatch);
        hipLaunchKernelGGL((k_mmv_q<TASK, NC, 4>), grid, dim3(256), 0, st, a);
    } else if (wpr == 2) {
        dim3 grid((unsigned) ceil_div(a.M, 2), (unsigned) ncg, (unsigned) nbatch);
        hipLaunchKernelGGL((k_mmv_q<TASK, NC, 2>), grid, dim3(256), 0, st, a);
    } else {
        dim3 grid((unsigned) ceil_div(a.M, 4), (unsigned) ncg, (unsigned) nbatch);
        hipLaunchKernelGGL((k_mmv_q<TASK, NC, 1>), grid, dim3(256), 0, st, a);
    }
}

template <template <int> class TASK>
static void launch_mmv_q(hipStream_t st, mmv_args & a, int64_t ne11, int64_t nbatch) {
    // columns per launch group: up to 8 activation columns share one weight pass
    const int nc = ne11 >= 8 ? 8 : (ne11 >= 4 ? 4 : (ne11 >= 2 ? 2 : 1));
    const int64_t ncg = ceil_div(ne11, nc);
    const int64_t waves = total_rows_waves(a.M, ncg, nbatch);
    const int wpr = waves >= 8192 ? 1 : (waves >= 2048 ? 2 : 4);
    switch (nc) {
        case 1: launch_mmv_q_nc<TASK, 1>(st, a, ncg, nbatch, wpr); break;
        case 2: launch_mmv_q_nc<TASK, 2>(st, a, ncg, nbatch, wpr); break;
        case 4: launch_mmv_q_nc<TASK, 4>(st, a, ncg, nbatch, wpr); break;
        default: launch_mmv_q_nc<TASK, 8>(st, a, ncg, nbatch, wpr); break;
    }
}

template <typename WT, int NC>
static void launch_mmv_f_nc(hipStream_t st, const mmv_f_args & a, int64_t ncg, int64_t nbatch, int wpr) {
    if (wpr == 4) {
        dim3 grid((unsigned) a.M, (unsigned) ncg, (unsigned) nbatch);
        hipLaunchKernelGGL((k_mmv_f<WT, NC, 4>), grid, dim3(256), 0, st, a);
    } else {
        dim3 grid((unsigned) ceil_div(a.M, 4), (unsigned) ncg, (unsigned) nbatch);
        hipLaunchKernelGGL((k_mmv_f<WT, NC, 1>), grid, dim3(256), 0, st, a);
    }
}

template <typename WT>
static void launch_mmv_f(hipStream_t st, mmv_f_args & a, int64_t ne11, int64_t nbatch) {
    const int nc = ne11 >= 8 ? 8 : (ne11 >= 4 ? 4 : (ne11 >= 2 ? 2 : 1));
    const int64_t ncg = ceil_div(ne11, nc);
    const int wpr = (a.M * ncg * nbatch >= 4096 || a.K < 1024) ? 1 : 4;
    switch (nc) {
        case 1: launch_mmv_f_nc<WT, 1>(st, a, ncg, nbatch, wpr); break;
        case 2: launch_mmv_f_nc<WT, 2>(st, a, ncg, nbatch, wpr); break;
        case 4: launch_mmv_f_nc<WT, 4>(st, a, ncg, nbatch, wpr); break;
        default: launch_mmv_f_nc<WT, 8>(st, a, ncg, nbatch, wpr); break;
    }
}

bool mmv_q_supported_type(ggml_type t) {
    return t == GGML_TYPE_Q4_0 || t == GGML_TYPE_Q8_0 || t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K ||
           t == GGML_TYPE_Q6_K;
}

static bool is_k_quant(ggml_type t) { return t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K; }

// weight bytes + activation bytes + output bytes moved by one mat-vec launch
static double mmv_bytes(const ggml_tensor * src0, const ggml_tensor * src1, const ggml_tensor * dst) {
    return (double) ggml_nbytes(src0) + (double) ggml_nelements(src1) * (is_k_quant(src0->type) ? 1.14 : 1.0) +
           (double) ggml_nbytes(dst);
}

// mat-vec entry: quantized or float weights, any number of columns (columns are
// processed in groups of up to 8 per weight pass).
void mul_mat_vec(exec_ctx & ctx, ggml_tensor * dst, const q8_act * pre) {
    const ggml_tensor * src0 = dst->src[0];
    const ggml_tensor * src1 = dst->src[1];
    const int64_t nbatch = src1->ne[2] * src1->ne[3];

    hipEvent_t ev_beg = nullptr;
    const double bytes = mmv_bytes(src0, src1, dst);
    if (ctx.timing) ctx.time_begin(TK_MMV, bytes, ev_beg);

    if (mmv_q_supported_type(src0->type)) {
        q8_act act;
        const bool kq = is_k_quant(src0->type);
        if (pre) {
            act = *pre;
        } else if (!ctx.qcache_get(src1, kq, act)) {
            quantize_act(ctx, src1, kq, act, exec_ctx::QSLOT);
            ctx.qcache_put(src1, kq, act);
        }
        mmv_args a;
        a.W = (const uint8_t *) src0->data;
        a.nb01 = src0->nb[1]; a.nb02 = src0->nb[2]; a.nb03 = src0->nb[3];
        a.M = src0->ne[1];
        a.nblk = src0->ne[0] / ggml_blck_size(src0->type);
        a.A = {act.qs, act.d, act.s, act.qs_stride(), act.d_stride(), act.s_stride()};
        a.ne11 = src1->ne[1]; a.ne12 = src1->ne[2];
        a.r2 = src1->ne[2] / src0->ne[2]; a.r3 = src1->ne[3] / src0->ne[3];
        a.dst = (float *) dst->data; a.nb1 = dst->nb[1]; a.nb2 = dst->nb[2]; a.nb3 = dst->nb[3];
        switch (src0->type) {
            case GGML_TYPE_Q4_K: launch_mmv_q<task_q4_K>(ctx.stream, a, a.ne11, nbatch); break;
            case GGML_TYPE_Q5_K: launch_mmv_q<task_q5_K>(ctx.stream, a, a.ne11, nbatch); break;
            case GGML_TYPE_Q6_K: launch_mmv_q<task_q6_K>(ctx.stream, a, a.ne11, nbatch); break;
            case GGML_TYPE_Q8_0: launch_mmv_q<task_q8_0>(ctx.stream, a, a.ne11, nbatch); break;
            case GGML_TYPE_Q4_0: launch_mmv_q<task_q4_0>(ctx.stream, a, a.ne11, nbatch); break;
            default: GGML_ABORT("mi355x: unsupported mmv type");
        }
    } else {
        mmv_f_args a;
        a.W = (const char *) src0->data;
        a.nb01 = src0->nb[1]; a.nb02 = src0->nb[2]; a.nb03 = src0->nb[3];
        a.M = src0->ne[1]; a.K = src0->ne[0];
        a.X = (const char *) src1->data;
        a.nb11 = src1->nb[1]; a.nb12 = src1->nb[2]; a.nb13 = src1->nb[3];
        a.ne11 = src1->ne[1]; a.ne12 = src1->ne[2];
        a.r2 = src1->ne[2] / src0->ne[2]; a.r3 = src1->ne[3] / src0->ne[3];
        a.dst = (float *) dst->data; a.nb1 = dst->nb[1]; a.nb2 = dst->nb[2]; a.nb3 = dst->nb[3];
        static const bool fast = getenv("GGML_MI355X_MMF_FAST") != nullptr;
        if (fast) {
            if (src0->type == GGML_TYPE_F16) launch_mmv_f<uint16_t>(ctx.stream, a, a.ne11, nbatch);
            else launch_mmv_f<float>(ctx.stream, a, a.ne11, nbatch);
        } else {
            dim3 grid((unsigned) ceil_div(a.M, 4), (unsigned) a.ne11, (unsigned) nbatch);
            if (src0->type == GGML_TYPE_F16) hipLaunchKernelGGL(k_mmv_f_exact<uint16_t>, grid, dim3(256), 0, ctx.stream, a);
            else hipLaunchKernelGGL(k_mmv_f_exact<float>, grid, dim3(256), 0, ctx.stream, a);
        }
    }
    if (ctx.timing) ctx.time_end(TK_MMV, bytes, ev_beg);
}

// ------------------------------------------------------------------------------------------
// MUL_MAT_ID (ggml-cpu/ggml-cpu.c:1466 ggml_compute_forward_mul_mat_id; graph use in
// build_moe_ffn, src/llama-graph.cpp:727-758): for token t and slot e < n_used,
//   dst[:, e, t] = as[ids[e, t]] . b[:, e % ne11, t]
// with the per-row arithmetic of the mat-vec above (same quantized activation, same tasks).
// The routing never leaves the device (the reference's CUDA path copies ids to the host,
// ggml-cuda.cu:2061-2084):
//   * few (slot, token) pairs (decode): one mat-vec per pair, the expert read from ids by
//     the kernel (k_mmv_q_id);
//   * many pairs (prefill): a one-workgroup counting sort groups the pairs by expert
//     (k_moe_sort), the activations are quantized straight into that order
//     (k_quant_gather), and each expert's rows are streamed once per 8 of its pairs
//     (k_mmv_q_idg); workgroups past an expert's pair count exit at once.
// ------------------------------------------------------------------------------------------
struct mmv_id_args {
    const uint8_t * W; int64_t nb01, nb02; int64_t M; int64_t nblk; int64_t n_as;
    act_view A;
    const char * ids; int64_t ids_nb0, ids_nb1; int64_t n_used; int64_t ne11;
    float * dst; int64_t nb1, nb2;   // bytes
    const int32_t * cnt; const int32_t * off; const int32_t * list;   // grouped mode
};

template <template <int> class TASK, int WPR>
__global__ __launch_bounds__(256) void k_mmv_q_id(const mmv_id_args p) {
    using T = TASK<1>;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int RPB = 4 / WPR;
    const int64_t row = (int64_t) blockIdx.x * RPB + wave / WPR;
    const int wsub = wave % WPR;
    const int64_t e = blockIdx.y % p.n_used, t = blockIdx.y / p.n_used;
    const int32_t ex = *(const int32_t *) (p.ids + e * p.ids_nb0 + t * p.ids_nb1);
    const bool ok = row < p.M && ex >= 0 && ex < p.n_as;
    float acc[1] = {0.0f};
    if (ok) {
        const uint8_t * wrow = p.W + (int64_t) ex * p.nb02 + row * p.nb01;
        const int64_t col = e % p.ne11 + p.ne11 * t;
        act_view A = p.A;
        A.qs += col * A.qs_st; A.d += col * A.d_st; A.s += col * A.s_st;
        const int ntasks = (int) (p.nblk * T::per_block);
        for (int tk = wsub * WAVE + lane; tk < ntasks; tk += WAVE * WPR) T::run(wrow, tk, A, 1, acc);
    }
    acc[0] = wave_sum(acc[0]);
    if constexpr (WPR > 1) {
        __shared__ float red[4];
        if (lane == 0) red[wave] = acc[0];
        __syncthreads();
        if (wsub == 0 && lane == 0) {
            float s = red[wave];
#pragma unroll
            for (int w = 1; w < WPR; ++w) s += red[wave + w];
            acc[0] = s;
        }
    }
    if (ok && wsub == 0 && lane == 0) *(float *) ((char *) p.dst + e * p.nb1 + t * p.nb2 + row * 4) = acc[0];
}

template <template <int> class TASK, int NC, int WPR>
__global__ __launch_bounds__(256) void k_mmv_q_idg(const mmv_id_args p) {
    using T = TASK<NC>;
    const int ex = blockIdx.z;
    const int n = p.cnt[ex];
    const int c0 = blockIdx.y * NC;
    if (c0 >= n) return;   // uniform over the workgroup, before any barrier
    const int nc = min(NC, n - c0);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int RPB = 4 / WPR;
    const int64_t row = (int64_t) blockIdx.x * RPB + wave / WPR;
    const int wsub = wave % WPR;
    const int64_t pos0 = p.off[ex] + c0;   // first expert-ordered activation column
    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0f;
    if (row < p.M) {
        const uint8_t * wrow = p.W + (int64_t) ex * p.nb02 + row * p.nb01;
        act_view A = p.A;
        A.qs += pos0 * A.qs_st; A.d += pos0 * A.d_st; A.s += pos0 * A.s_st;
        const int ntasks = (int) (p.nblk * T::per_block);
        for (int tk = wsub * WAVE + lane; tk < ntasks; tk += WAVE * WPR) T::run(wrow, tk, A, nc, acc);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = wave_sum(acc[c]);
    if constexpr (WPR > 1) {
        __shared__ float red[4][NC];
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < NC; ++c) red[wave][c] = acc[c];
        }
        __syncthreads();
        if (wsub == 0 && lane == 0) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                float s = red[wave][c];
#pragma unroll
                for (int w = 1; w < WPR; ++w) s += red[wave + w][c];
                acc[c] = s;
            }
        }
    }
    if (row < p.M && wsub == 0 && lane == 0) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= nc) break;
            const int pair = p.list[pos0 + c];
            const int64_t e = pair % p.n_used, t = pair / p.n_used;
            *(float *) ((char *) p.dst + e * p.nb1 + t * p.nb2 + row * 4) = acc[c];
        }
    }
}

// counting sort of the (slot, token) pairs by expert, one workgroup: cnt[x] pairs routed to
// expert x, off[x] their first position (exclusive prefix), list[off[x] + k] = pair index
// e + n_used * t.  The order inside an expert is immaterial: every pair's output depends
// only on its own activation column.  Out-of-range ids (the CPU asserts on them) route nowhere.
__global__ __launch_bounds__(256) void k_moe_sort(const char * __restrict__ ids, int64_t nb0, int64_t nb1, int64_t n_used,
                                                  int64_t n_pairs, int n_as, int32_t * __restrict__ cnt,
                                                  int32_t * __restrict__ off, int32_t * __restrict__ list) {
    extern __shared__ int cur[];   // [n_as]
    for (int x = threadIdx.x; x < n_as; x += blockDim.x) cur[x] = 0;
    __syncthreads();
    for (int64_t q = threadIdx.x; q < n_pairs; q += blockDim.x) {
        const int32_t ex = *(const int32_t *) (ids + (q % n_used) * nb0 + (q / n_used) * nb1);
        if (ex >= 0 && ex < n_as) atomicAdd(&cur[ex], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int x = 0; x < n_as; ++x) {
            const int c = cur[x];
            cnt[x] = c;
            off[x] = acc;
            cur[x] = acc;
            acc += c;
        }
    }
    __syncthreads();
    for (int64_t q = threadIdx.x; q < n_pairs; q += blockDim.x) {
        const int32_t ex = *(const int32_t *) (ids + (q % n_used) * nb0 + (q / n_used) * nb1);
        if (ex >= 0 && ex < n_as) list[atomicAdd(&cur[ex], 1)] = (int32_t) q;
    }
}

// quantization of the activation column of each sorted pair into position order (the
// quantizers of quant_act.h, so the bytes equal the unsorted quantization's)
template <int QMODE>
__global__ __launch_bounds__(64) void k_quant_gather(const char * __restrict__ x, int64_t K, int64_t nb11, int64_t nb12,
                                                     int64_t ne11, int64_t n_used, const int32_t * __restrict__ list,
                                                     const int32_t * __restrict__ cnt, const int32_t * __restrict__ off,
                                                     int n_as, int8_t * __restrict__ qs, float * __restrict__ qd,
                                                     int16_t * __restrict__ qsum) {
    const int lane = threadIdx.x;
    const int64_t j = blockIdx.y;
    if (j >= off[n_as - 1] + cnt[n_as - 1]) return;
    const int pair = list[j];
    const int64_t e = pair % n_used, t = pair / n_used;
    const float * row = (const float *) (x + (e % ne11) * nb11 + t * nb12);
    const int64_t c0 = (int64_t) blockIdx.x * 256, e0 = c0 + 4 * lane;
    const bool valid = e0 < K;
    float q[4] = {0.f, 0.f, 0.f, 0.f};
    if (valid) {
        const uint4 v = ld16(row + e0);
        q[0] = __uint_as_float(v.x); q[1] = __uint_as_float(v.y); q[2] = __uint_as_float(v.z); q[3] = __uint_as_float(v.w);
    }
    if constexpr (QMODE == 1) {
        q8K_wave(q, lane, qs + j * K + c0, qsum + j * (K / 16) + c0 / 16, qd + j * (K / 256) + c0 / 256);
    } else {
        q8_0_wave(q, lane, valid, qs + j * K + c0, qd + j * (K / 32) + c0 / 32, qsum + j * (K / 32) + c0 / 32);
    }
}

bool mul_mat_id_supported(const ggml_tensor * op) {
    const ggml_tensor * as = op->src[0];
    const ggml_tensor * b = op->src[1];
    const ggml_tensor * ids = op->src[2];
    if (!as || !b || !ids) return false;
    if (!mmv_q_supported_type(as->type) || as->nb[0] != ggml_type_size(as->type)) return false;
    if (b->type != GGML_TYPE_F32 || b->nb[0] != sizeof(float) || op->type != GGML_TYPE_F32 || op->nb[0] != sizeof(float)) return false;
    if (ids->type != GGML_TYPE_I32) return false;
    if (as->ne[0] % (is_k_quant(as->type) ? 256 : 32) != 0 || b->ne[0] != as->ne[0]) return false;
    if (as->ne[3] != 1 || b->ne[3] != 1 || ids->ne[2] != 1 || ids->ne[3] != 1) return false;
    return b->ne[2] == ids->ne[1] && op->ne[1] == ids->ne[0] && op->ne[2] == ids->ne[1] && as->ne[2] <= 4096;
}

template <template <int> class TASK>
static void launch_mmv_id(hipStream_t st, const mmv_id_args & a, int64_t n_pairs, bool grouped) {
    const int64_t waves = a.M * (grouped ? ceil_div(n_pairs, 8 * a.n_as) : n_pairs);
    const int wpr = waves >= 8192 ? 1 : (waves >= 2048 ? 2 : 4);
    const unsigned rb = (unsigned) ceil_div(a.M, 4 / wpr);
    if (!grouped) {
        const dim3 grid(rb, (unsigned) n_pairs);
        if (wpr == 1) hipLaunchKernelGGL((k_mmv_q_id<TASK, 1>), grid, dim3(256), 0, st, a);
        else if (wpr == 2) hipLaunchKernelGGL((k_mmv_q_id<TASK, 2>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((k_mmv_q_id<TASK, 4>), grid, dim3(256), 0, st, a);
        return;
    }
    const dim3 grid(rb, (unsigned) ceil_div(n_pairs, 8), (unsigned) a.n_as);
    if (wpr == 1) hipLaunchKernelGGL((k_mmv_q_idg<TASK, 8, 1>), grid, dim3(256), 0, st, a);
    else if (wpr == 2) hipLaunchKernelGGL((k_mmv_q_idg<TASK, 8, 2>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_mmv_q_idg<TASK, 8, 4>), grid, dim3(256), 0, st, a);
}

bool gemv_mul_mat_id(exec_ctx & ctx, ggml_tensor * dst, const q8_act & act);
bool mmq_id_supported(const ggml_tensor * dst);
void mul_mat_q_id(exec_ctx & ctx, ggml_tensor * dst, const q8_act & act, const int32_t * cnt, const int32_t * off,
                  const int32_t * list, int64_t n_pairs);

void op_mul_mat_id(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * as = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const ggml_tensor * ids = dst->src[2];
    const bool kq = is_k_quant(as->type);
    const int64_t K = as->ne[0];
    const int64_t n_used = ids->ne[0], T = ids->ne[1], n_pairs = n_used * T;
    const int n_as = (int) as->ne[2];
    if (n_pairs == 0) return;

    hipEvent_t ev_beg = nullptr;
    // algorithmic bytes: one pass over the rows of every routed expert (at most n_pairs of them)
    const double bytes = (double) as->nb[2] * (double) std::min<int64_t>(n_pairs, n_as) +
                         (double) ggml_nelements(b) * (kq ? 1.14 : 1.0) + (double) ggml_nbytes(dst);
    if (ctx.timing) ctx.time_begin(TK_MMV, bytes, ev_beg);

    mmv_id_args a;
    a.W = (const uint8_t *) as->data;
    a.nb01 = as->nb[1]; a.nb02 = as->nb[2];
    a.M = as->ne[1];
    a.nblk = K / ggml_blck_size(as->type);
    a.n_as = n_as;
    a.ids = (const char *) ids->data; a.ids_nb0 = ids->nb[0]; a.ids_nb1 = ids->nb[1];
    a.n_used = n_used; a.ne11 = b->ne[1];
    a.dst = (float *) dst->data; a.nb1 = dst->nb[1]; a.nb2 = dst->nb[2];
    a.cnt = a.off = a.list = nullptr;

    const bool grouped = n_pairs > 8;
    q8_act act;
    if (!grouped) {
        if (!ctx.qcache_get(b, kq, act)) {
            quantize_act(ctx, b, kq, act, exec_ctx::QSLOT);
            ctx.qcache_put(b, kq, act);
        }
        // GGML_MI355X_MMID_PIPE=1: the routed experts on the pipelined decode mat-vec (k_gemv.hip).
        // Off by default: one row per wave (k_mmv_q_id) measured faster on the Mixtral shapes —
        // up/gate 2 x 40 MB Q5_K 23.4 vs 31.6 us, down 40 MB 11.4 vs 24.4 us (scripts/probe_mmid.py)
        static const bool pipe_id = getenv("GGML_MI355X_MMID_PIPE") && atoi(getenv("GGML_MI355X_MMID_PIPE")) != 0;
        if (pipe_id && T == 1 && gemv_mul_mat_id(ctx, dst, act)) {
            if (ctx.timing) ctx.time_end(TK_MMV, bytes, ev_beg);
            return;
        }
    } else {
        auto al = [](size_t v) { return (v + 255) & ~size_t(255); };
        const size_t ib = al(sizeof(int32_t) * (size_t) (2 * n_as + n_pairs));
        char * base = (char *) ctx.scratch(2, ib + q8_act::bytes(K, n_pairs, kq));
        int32_t * cnt = (int32_t *) base;
        int32_t * off = cnt + n_as;
        int32_t * list = off + n_as;
        carve_act(act, base + ib, K, n_pairs, kq);
        hipLaunchKernelGGL(k_moe_sort, dim3(1), dim3(256), sizeof(int) * n_as, ctx.stream, (const char *) ids->data,
                           (int64_t) ids->nb[0], (int64_t) ids->nb[1], n_used, n_pairs, n_as, cnt, off, list);
        const dim3 qg((unsigned) ceil_div(K, 256), (unsigned) n_pairs);
        if (kq) {
            hipLaunchKernelGGL(k_quant_gather<1>, qg, dim3(64), 0, ctx.stream, (const char *) b->data, K, (int64_t) b->nb[1],
                               (int64_t) b->nb[2], (int64_t) b->ne[1], n_used, list, cnt, off, n_as, act.qs, act.d, act.s);
        } else {
            hipLaunchKernelGGL(k_quant_gather<2>, qg, dim3(64), 0, ctx.stream, (const char *) b->data, K, (int64_t) b->nb[1],
                               (int64_t) b->nb[2], (int64_t) b->ne[1], n_used, list, cnt, off, n_as, act.qs, act.d, act.s);
        }
        a.cnt = cnt; a.off = off; a.list = list;
        // enough tokens per expert for the 64-token MFMA tile
        if (n_pairs >= 64 && mmq_id_supported(dst)) {
            mul_mat_q_id(ctx, dst, act, cnt, off, list, n_pairs);
            if (ctx.timing) ctx.time_end(TK_MMV, bytes, ev_beg);
            return;
        }
    }
    a.A = {act.qs, act.d, act.s, act.qs_stride(), act.d_stride(), act.s_stride()};
    switch (as->type) {
        case GGML_TYPE_Q4_K: launch_mmv_id<task_q4_K>(ctx.stream, a, n_pairs, grouped); break;
        case GGML_TYPE_Q5_K: launch_mmv_id<task_q5_K>(ctx.stream, a, n_pairs, grouped); break;
        case GGML_TYPE_Q6_K: launch_mmv_id<task_q6_K>(ctx.stream, a, n_pairs, grouped); break;
        case GGML_TYPE_Q8_0: launch_mmv_id<task_q8_0>(ctx.stream, a, n_pairs, grouped); break;
        case GGML_TYPE_Q4_0: launch_mmv_id<task_q4_0>(ctx.stream, a, n_pairs, grouped); break;
        default: GGML_ABORT("mi355x: unsupported mul_mat_id type");
    }
    if (ctx.timing) ctx.time_end(TK_MMV, bytes, ev_beg);
}

}  // namespace mi355x
