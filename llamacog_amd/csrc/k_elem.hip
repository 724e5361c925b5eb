// k_elem.hip — the small ops of the LLaMA graph: broadcast binary ops, scale, unary
// (SiLU/GELU/...), copies/casts (incl. the f32 -> f16 / q8_0 KV-cache store), get_rows,
// RMS norm (optionally fused with the following norm-weight MUL), RoPE and soft_max.
//
// Each op follows the CPU backend's arithmetic (ggml/src/ggml-cpu/ops.cpp,
// binary-ops.cpp, unary-ops.cpp, vec.h) — operation order per element is kept, reductions
// use wider accumulators where the CPU does (rms_norm sums in ggml_float = double).
// They are HBM/latency-bound; rows are split over several 256-thread workgroups when
// there are few of them (decode).
#include "ops.h"
#include "rope.h"
#include "quant_act.h"

#include <cmath>

namespace mi355x {

struct t4 { int64_t ne[4]; int64_t nb[4]; };
__device__ __forceinline__ int64_t nrows_all(const t4 & t) { return t.ne[1] * t.ne[2] * t.ne[3]; }
static t4 mk(const ggml_tensor * t) {
    t4 r;
    for (int i = 0; i < 4; ++i) { r.ne[i] = t->ne[i]; r.nb[i] = (int64_t) t->nb[i]; }
    return r;
}

// column slices per row: few rows (decode) spread one row over many workgroups, many rows
// (prefill) keep one workgroup per row
static unsigned col_blocks(int64_t ne0, int64_t nrows, unsigned thr) {
    const int64_t want = std::max<int64_t>(1, 1024 / std::max<int64_t>(nrows, 1));
    return (unsigned) std::min<int64_t>(ceil_div(ne0, thr), want);
}

// ------------------------------------------------------------------------------------------
// binary broadcast: dst = op(src0, src1), src1 repeats across dims (ggml-cpu/binary-ops.cpp)
// ------------------------------------------------------------------------------------------
enum bin_op { BIN_ADD = 0, BIN_SUB, BIN_MUL, BIN_DIV };

template <int OP>
__device__ __forceinline__ float bin_apply(float a, float b) {
    if constexpr (OP == BIN_ADD) return a + b;
    else if constexpr (OP == BIN_SUB) return a - b;
    else if constexpr (OP == BIN_MUL) return a * b;
    else return a / b;
}

template <int OP>
__global__ __launch_bounds__(256) void k_binary(const char * __restrict__ a, t4 ta, const char * __restrict__ b, t4 tb,
                                                char * __restrict__ d, t4 td) {
    const int64_t cb = gridDim.x / nrows_all(td);   // column slices per row
    const int64_t r = blockIdx.x / cb;              // row over (i1, i2, i3) of dst
    const int64_t i1 = r % td.ne[1], i2 = (r / td.ne[1]) % td.ne[2], i3 = r / (td.ne[1] * td.ne[2]);
    const char * ar = a + i1 * ta.nb[1] + i2 * ta.nb[2] + i3 * ta.nb[3];
    const char * br = b + (i1 % tb.ne[1]) * tb.nb[1] + (i2 % tb.ne[2]) * tb.nb[2] + (i3 % tb.ne[3]) * tb.nb[3];
    char * dr = d + i1 * td.nb[1] + i2 * td.nb[2] + i3 * td.nb[3];
    const int64_t ne0 = td.ne[0], ne10 = tb.ne[0];
    for (int64_t i0 = (blockIdx.x % cb) * blockDim.x + threadIdx.x; i0 < ne0; i0 += cb * blockDim.x) {
        const float x = *(const float *) (ar + i0 * ta.nb[0]);
        const float y = *(const float *) (br + (i0 % ne10) * tb.nb[0]);
        *(float *) (dr + i0 * td.nb[0]) = bin_apply<OP>(x, y);
    }
}

void op_binary(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * s0 = dst->src[0];
    const ggml_tensor * s1 = dst->src[1];
    const int64_t nrows = dst->ne[1] * dst->ne[2] * dst->ne[3];
    if (nrows == 0 || dst->ne[0] == 0) return;
    const unsigned thr = dst->ne[0] >= 256 ? 256 : 64;
    const dim3 grid((unsigned) (col_blocks(dst->ne[0], nrows, thr) * nrows));
    auto A = mk(s0), B = mk(s1), D = mk(dst);
    switch (dst->op) {
        case GGML_OP_ADD: hipLaunchKernelGGL(k_binary<BIN_ADD>, grid, dim3(thr), 0, ctx.stream, (const char *) s0->data, A, (const char *) s1->data, B, (char *) dst->data, D); break;
        case GGML_OP_SUB: hipLaunchKernelGGL(k_binary<BIN_SUB>, grid, dim3(thr), 0, ctx.stream, (const char *) s0->data, A, (const char *) s1->data, B, (char *) dst->data, D); break;
        case GGML_OP_MUL: hipLaunchKernelGGL(k_binary<BIN_MUL>, grid, dim3(thr), 0, ctx.stream, (const char *) s0->data, A, (const char *) s1->data, B, (char *) dst->data, D); break;
        case GGML_OP_DIV: hipLaunchKernelGGL(k_binary<BIN_DIV>, grid, dim3(thr), 0, ctx.stream, (const char *) s0->data, A, (const char *) s1->data, B, (char *) dst->data, D); break;
        default: GGML_ABORT("mi355x: bad binary op");
    }
}

// ------------------------------------------------------------------------------------------
// scale (ops.cpp ggml_compute_forward_scale_f32: y = x*s) and unary ops
// ------------------------------------------------------------------------------------------
enum un_op { UN_SILU = 0, UN_GELU, UN_RELU, UN_NEG, UN_TANH, UN_SIGMOID, UN_SCALE, UN_GELU_QUICK, UN_EXP, UN_ABS, UN_SGN, UN_STEP, UN_GELU_ERF };

template <int OP>
__device__ __forceinline__ float un_apply(float x, float s) {
    if constexpr (OP == UN_SILU) return x / (1.0f + v_expf_avx512(-x));              // vec.h:759 ggml_v_silu
    else if constexpr (OP == UN_RELU) return x > 0.0f ? x : 0.0f;
    else if constexpr (OP == UN_NEG) return -x;
    else if constexpr (OP == UN_TANH) return tanhf(x);
    else if constexpr (OP == UN_SIGMOID) return 1.0f / (1.0f + expf(-x));
    else if constexpr (OP == UN_SCALE) return x * s;
    else if constexpr (OP == UN_EXP) return expf(x);
    else if constexpr (OP == UN_ABS) return fabsf(x);
    else if constexpr (OP == UN_SGN) return (x > 0.f) ? 1.f : ((x < 0.f) ? -1.f : 0.f);
    else if constexpr (OP == UN_STEP) return (x > 0.f) ? 1.f : 0.f;
    else if constexpr (OP == UN_GELU_QUICK) return x * (1.0f / (1.0f + expf(-1.702f * x)));
    else if constexpr (OP == UN_GELU_ERF) return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
    else {  // GELU tanh approximation (vec.h ggml_gelu_f32)
        const float GELU_COEF_A = 0.044715f, SQRT_2_OVER_PI = 0.79788456080286535587989211986876f;
        return 0.5f * x * (1.0f + tanhf(SQRT_2_OVER_PI * x * (1.0f + GELU_COEF_A * x * x)));
    }
}

template <int OP>
__global__ __launch_bounds__(256) void k_unary(const char * __restrict__ a, t4 ta, char * __restrict__ d, t4 td, float s) {
    const int64_t cb = gridDim.x / nrows_all(td);
    const int64_t r = blockIdx.x / cb;
    const int64_t i1 = r % td.ne[1], i2 = (r / td.ne[1]) % td.ne[2], i3 = r / (td.ne[1] * td.ne[2]);
    const char * ar = a + i1 * ta.nb[1] + i2 * ta.nb[2] + i3 * ta.nb[3];
    char * dr = d + i1 * td.nb[1] + i2 * td.nb[2] + i3 * td.nb[3];
    const int64_t nvec = (td.ne[0] / 16) * 16;  // ggml_vec_silu_f32: 16-wide SIMD body, scalar tail
    for (int64_t i0 = (blockIdx.x % cb) * blockDim.x + threadIdx.x; i0 < td.ne[0]; i0 += cb * blockDim.x) {
        const float x = *(const float *) (ar + i0 * ta.nb[0]);
        float yv;
        if constexpr (OP == UN_SILU) yv = i0 < nvec ? un_apply<OP>(x, s) : x / (1.0f + expf_cr(-x));
        else yv = un_apply<OP>(x, s);
        *(float *) (dr + i0 * td.nb[0]) = yv;
    }
}

template <int OP>
static void launch_unary(exec_ctx & ctx, const ggml_tensor * src, ggml_tensor * dst, float s) {
    const int64_t nrows = dst->ne[1] * dst->ne[2] * dst->ne[3];
    if (nrows == 0 || dst->ne[0] == 0) return;
    const unsigned thr = dst->ne[0] >= 256 ? 256 : 64;
    hipLaunchKernelGGL(k_unary<OP>, dim3((unsigned) (col_blocks(dst->ne[0], nrows, thr) * nrows)), dim3(thr), 0, ctx.stream, (const char *) src->data, mk(src),
                       (char *) dst->data, mk(dst), s);
}

void op_scale(exec_ctx & ctx, ggml_tensor * dst) {
    float s;
    memcpy(&s, dst->op_params, sizeof(float));
    launch_unary<UN_SCALE>(ctx, dst->src[0], dst, s);
}

void op_unary(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * src = dst->src[0];
    switch (ggml_get_unary_op(dst)) {
        case GGML_UNARY_OP_SILU:       launch_unary<UN_SILU>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_GELU:       launch_unary<UN_GELU>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_GELU_ERF:   launch_unary<UN_GELU_ERF>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_GELU_QUICK: launch_unary<UN_GELU_QUICK>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_RELU:       launch_unary<UN_RELU>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_NEG:        launch_unary<UN_NEG>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_TANH:       launch_unary<UN_TANH>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_SIGMOID:    launch_unary<UN_SIGMOID>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_EXP:        launch_unary<UN_EXP>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_ABS:        launch_unary<UN_ABS>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_SGN:        launch_unary<UN_SGN>(ctx, src, dst, 0.f); break;
        case GGML_UNARY_OP_STEP:       launch_unary<UN_STEP>(ctx, src, dst, 0.f); break;
        default: GGML_ABORT("mi355x: unsupported unary op");
    }
}

// ------------------------------------------------------------------------------------------
// copies / casts: element i of src (row-major order) -> element i of dst (row-major order),
// the semantics of ggml_compute_forward_dup for non-quantized types.
// ------------------------------------------------------------------------------------------
template <typename TS, typename TD>
__device__ __forceinline__ TD cvt(TS v);
template <> __device__ __forceinline__ float    cvt<float, float>(float v) { return v; }
template <> __device__ __forceinline__ uint16_t cvt<float, uint16_t>(float v) { return f2h(v); }
template <> __device__ __forceinline__ float    cvt<uint16_t, float>(uint16_t v) { return h2f(v); }
template <> __device__ __forceinline__ uint16_t cvt<uint16_t, uint16_t>(uint16_t v) { return v; }
template <> __device__ __forceinline__ int32_t  cvt<int32_t, int32_t>(int32_t v) { return v; }

template <typename TS, typename TD>
__global__ __launch_bounds__(256) void k_cpy(const char * __restrict__ s, t4 ts, char * __restrict__ d, t4 td, int64_t n,
                                             char * const * dslot) {
    if (dslot) d = *dslot;
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        int64_t r = i;
        const int64_t s0 = r % ts.ne[0]; r /= ts.ne[0];
        const int64_t s1 = r % ts.ne[1]; r /= ts.ne[1];
        const int64_t s2 = r % ts.ne[2]; const int64_t s3 = r / ts.ne[2];
        r = i;
        const int64_t d0 = r % td.ne[0]; r /= td.ne[0];
        const int64_t d1 = r % td.ne[1]; r /= td.ne[1];
        const int64_t d2 = r % td.ne[2]; const int64_t d3 = r / td.ne[2];
        const TS v = *(const TS *) (s + s0 * ts.nb[0] + s1 * ts.nb[1] + s2 * ts.nb[2] + s3 * ts.nb[3]);
        *(TD *) (d + d0 * td.nb[0] + d1 * td.nb[1] + d2 * td.nb[2] + d3 * td.nb[3]) = cvt<TS, TD>(v);
    }
}

// contiguous f32 -> f16 fast path (KV store of K/V rows, mask cast)
__global__ __launch_bounds__(256) void k_cpy_f32_f16_contig(const float * __restrict__ s, uint16_t * __restrict__ d, int64_t n,
                                                            uint16_t * const * dslot) {
    if (dslot) d = *dslot;
    for (int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t) gridDim.x * blockDim.x) {
        d[i] = f2h(s[i]);
    }
}

// f32 rows -> q8_0 blocks (x86 quantize_row_q8_0 semantics, see k_mmv.hip); one wave per 8 blocks
__global__ __launch_bounds__(64) void k_cpy_f32_q8_0(const char * __restrict__ s, t4 ts, char * __restrict__ d, t4 td,
                                                     char * const * dslot) {
    if (dslot) d = *dslot;
    const int lane = threadIdx.x;
    const int64_t r = blockIdx.y;  // source row
    const int64_t i1 = r % ts.ne[1], i2 = (r / ts.ne[1]) % ts.ne[2], i3 = r / (ts.ne[1] * ts.ne[2]);
    const char * srow = s + i1 * ts.nb[1] + i2 * ts.nb[2] + i3 * ts.nb[3];
    // destination row with the same flat row index
    const int64_t j1 = r % td.ne[1], j2 = (r / td.ne[1]) % td.ne[2], j3 = r / (td.ne[1] * td.ne[2]);
    char * drow = d + j1 * td.nb[1] + j2 * td.nb[2] + j3 * td.nb[3];
    const int64_t e0 = (int64_t) blockIdx.x * 256 + 4 * lane;
    const bool valid = e0 < ts.ne[0];
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (valid) {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = *(const float *) (srow + (e0 + k) * ts.nb[0]);
    }
    float amax = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
    amax = fmaxf(amax, __shfl_xor(amax, 1, WAVE));
    amax = fmaxf(amax, __shfl_xor(amax, 2, WAVE));
    amax = fmaxf(amax, __shfl_xor(amax, 4, WAVE));
    const float dd = amax / 127.0f;
    const float id = amax != 0.0f ? 127.0f / amax : 0.0f;
    if (!valid) return;
    blk_q8_0 * blk = (blk_q8_0 *) (drow + (e0 / 32) * sizeof(blk_q8_0));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int iv = (int) rintf(__fmul_rn(v[k], id));
        iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
        blk->qs[(e0 % 32) + k] = (int8_t) iv;
    }
    if ((lane & 7) == 0) blk->d = f2h(dd);
}

// f32 rows -> q4_0 blocks, quantize_row_q4_0_ref (ggml-quants.c, the CPU backend's from_float
// for Q4_0, ggml-cpu/quants.c:24): the first element of largest |x| gives max, d = max / -8,
// id = 1/d, q = min(15, (int8_t)(x*id + 8.5)) with separate f32 roundings (the reference builds
// ggml-quants.c without FMA), elements j and j + 16 share byte j.  One thread per block.
__global__ __launch_bounds__(64) void k_cpy_f32_q4_0(const char * __restrict__ s, t4 ts, char * __restrict__ d, t4 td,
                                                     char * const * dslot) {
    if (dslot) d = *dslot;
    const int64_t r = blockIdx.y;
    const int64_t b = (int64_t) blockIdx.x * 64 + threadIdx.x;
    if (32 * b >= ts.ne[0]) return;
    const int64_t i1 = r % ts.ne[1], i2 = (r / ts.ne[1]) % ts.ne[2], i3 = r / (ts.ne[1] * ts.ne[2]);
    const char * srow = s + i1 * ts.nb[1] + i2 * ts.nb[2] + i3 * ts.nb[3];
    const int64_t j1 = r % td.ne[1], j2 = (r / td.ne[1]) % td.ne[2], j3 = r / (td.ne[1] * td.ne[2]);
    char * drow = d + j1 * td.nb[1] + j2 * td.nb[2] + j3 * td.nb[3];
    float x[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) x[j] = *(const float *) (srow + (32 * b + j) * ts.nb[0]);
    float amax = 0.0f, mx = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        if (amax < fabsf(x[j])) { amax = fabsf(x[j]); mx = x[j]; }
    }
    const float dd = mx / -8.0f;
    const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
    uint8_t * blk = (uint8_t *) (drow + b * 18);
    const uint16_t dh = f2h(dd);
    blk[0] = (uint8_t) (dh & 0xff);
    blk[1] = (uint8_t) (dh >> 8);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int q0 = min(15, (int) (int8_t) (int) __fadd_rn(__fmul_rn(x[j], id), 8.5f));
        const int q1 = min(15, (int) (int8_t) (int) __fadd_rn(__fmul_rn(x[j + 16], id), 8.5f));
        blk[2 + j] = (uint8_t) (q0 | (q1 << 4));
    }
}

void op_cpy(exec_ctx & ctx, const ggml_tensor * src, ggml_tensor * dst, const ggml_tensor * node) {
    const int64_t n = ggml_nelements(src);
    if (n == 0) return;
    char * const * dslot = node ? (char * const *) ctx.dyn_slot(node) : nullptr;
    const t4 S = mk(src), D = mk(dst);
    const unsigned grid = (unsigned) std::min<int64_t>(ceil_div(n, 256), 8192);
    if (src->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_F16 && ggml_is_contiguous(src) && ggml_is_contiguous(dst)) {
        hipLaunchKernelGGL(k_cpy_f32_f16_contig, dim3(grid), dim3(256), 0, ctx.stream, (const float *) src->data, (uint16_t *) dst->data, n,
                           (uint16_t * const *) dslot);
        return;
    }
    if (src->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_Q8_0 && ggml_is_contiguous(src) && ggml_is_contiguous(dst) &&
        src->ne[0] != dst->ne[0]) {
        // contiguous both sides (the KV-cache store of a [D, H, T] Kcur): the same 32-blocks as
        // quantizing src row by row (dup_to_q, ops.cpp), as one flat row
        t4 S1 = S, D1 = D;
        S1.ne[0] = D1.ne[0] = n;
        for (int k = 1; k < 4; ++k) { S1.ne[k] = D1.ne[k] = 1; S1.nb[k] = S.nb[0] * n; D1.nb[k] = ggml_row_size(GGML_TYPE_Q8_0, n); }
        dim3 g((unsigned) ceil_div(n, 256), 1u);
        hipLaunchKernelGGL(k_cpy_f32_q8_0, g, dim3(64), 0, ctx.stream, (const char *) src->data, S1, (char *) dst->data, D1, dslot);
        return;
    }
    if (src->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_Q4_0) {
        // contiguous both sides: one flat row (the KV-cache store); else row by row
        t4 S1 = S, D1 = D;
        int64_t ne0 = src->ne[0], nrows = src->ne[1] * src->ne[2] * src->ne[3];
        if (ggml_is_contiguous(src) && ggml_is_contiguous(dst) && src->ne[0] != dst->ne[0]) {
            ne0 = n;
            nrows = 1;
            S1.ne[0] = D1.ne[0] = n;
            for (int k = 1; k < 4; ++k) { S1.ne[k] = D1.ne[k] = 1; S1.nb[k] = S.nb[0] * n; D1.nb[k] = ggml_row_size(GGML_TYPE_Q4_0, n); }
        }
        dim3 g((unsigned) ceil_div(ne0 / 32, 64), (unsigned) nrows);
        hipLaunchKernelGGL(k_cpy_f32_q4_0, g, dim3(64), 0, ctx.stream, (const char *) src->data, S1, (char *) dst->data, D1, dslot);
        return;
    }
    if (src->type == GGML_TYPE_F32 && dst->type == GGML_TYPE_Q8_0) {
        const int64_t nrows = src->ne[1] * src->ne[2] * src->ne[3];
        dim3 g((unsigned) ceil_div(src->ne[0], 256), (unsigned) nrows);
        hipLaunchKernelGGL(k_cpy_f32_q8_0, g, dim3(64), 0, ctx.stream, (const char *) src->data, S, (char *) dst->data, D, dslot);
        return;
    }
#define CPY_CASE(TS_, TD_, ts, td) \
    if (src->type == TS_ && dst->type == TD_) { hipLaunchKernelGGL((k_cpy<ts, td>), dim3(grid), dim3(256), 0, ctx.stream, (const char *) src->data, S, (char *) dst->data, D, n, dslot); return; }
    CPY_CASE(GGML_TYPE_F32, GGML_TYPE_F32, float, float)
    CPY_CASE(GGML_TYPE_F32, GGML_TYPE_F16, float, uint16_t)
    CPY_CASE(GGML_TYPE_F16, GGML_TYPE_F32, uint16_t, float)
    CPY_CASE(GGML_TYPE_F16, GGML_TYPE_F16, uint16_t, uint16_t)
    CPY_CASE(GGML_TYPE_I32, GGML_TYPE_I32, int32_t, int32_t)
#undef CPY_CASE
    GGML_ABORT("mi355x: unsupported cpy %s -> %s", ggml_type_name(src->type), ggml_type_name(dst->type));
}

// ------------------------------------------------------------------------------------------
// get_rows: dst[:, i10, i11, i12] = dequant(src0[:, rows[i10,i11,i12], i11, i12])
// ------------------------------------------------------------------------------------------
__device__ float dequant_elem(int type, const char * row, int64_t i) {
    switch (type) {
        case GGML_TYPE_F32: return *(const float *) (row + 4 * i);
        case GGML_TYPE_F16: return h2f(*(const uint16_t *) (row + 2 * i));
        case GGML_TYPE_Q8_0: {
            const blk_q8_0 * b = (const blk_q8_0 *) (row) + i / 32;
            return h2f(ld2(&b->d)) * b->qs[i % 32];
        }
        case GGML_TYPE_Q4_0: {
            const blk_q4_0 * b = (const blk_q4_0 *) (row) + i / 32;
            const int j = i % 32;
            const int q = j < 16 ? (b->qs[j] & 0xF) : (b->qs[j - 16] >> 4);
            return (q - 8) * h2f(ld2(&b->d));
        }
        case GGML_TYPE_Q4_K: {
            const blk_q4_K * b = (const blk_q4_K *) (row) + i / 256;
            const int j = i % 256, g = j / 64, l = j % 32, hi = (j % 64) >= 32;
            int sc, m;
            scale_min_k4(2 * g + hi, b->scales, sc, m);
            const int q = hi ? (b->qs[32 * g + l] >> 4) : (b->qs[32 * g + l] & 0xF);
            return h2f(ld2(&b->d)) * sc * q - h2f(ld2(&b->dmin)) * m;
        }
        case GGML_TYPE_Q5_K: {
            const blk_q5_K * b = (const blk_q5_K *) (row) + i / 256;
            const int j = i % 256, g = j / 64, l = j % 32, hi = (j % 64) >= 32;
            int sc, m;
            scale_min_k4(2 * g + hi, b->scales, sc, m);
            int q = hi ? (b->qs[32 * g + l] >> 4) : (b->qs[32 * g + l] & 0xF);
            q += ((b->qh[l] >> (2 * g + hi)) & 1) << 4;
            return h2f(ld2(&b->d)) * sc * q - h2f(ld2(&b->dmin)) * m;
        }
        case GGML_TYPE_Q6_K: {
            const blk_q6_K * b = (const blk_q6_K *) (row) + i / 256;
            const int j = i % 256, n = j / 128, jj = j % 128, grp = jj / 32, l = jj % 32;
            const uint8_t * ql = b->ql + 64 * n;
            const uint8_t * qh = b->qh + 32 * n;
            int q;
            switch (grp) {
                case 0: q = (ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4); break;
                case 1: q = (ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4); break;
                case 2: q = (ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4); break;
                default: q = (ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4); break;
            }
            const int is = 8 * n + l / 16 + 2 * grp;
            return h2f(ld2(&b->d)) * b->scales[is] * (q - 32);
        }
        default: return 0.0f;
    }
}

__global__ __launch_bounds__(256) void k_get_rows(const char * __restrict__ s0, t4 t0, int type,
                                                  const char * __restrict__ s1, t4 t1, char * __restrict__ d, t4 td) {
    const int64_t r = blockIdx.x;  // over (i10, i11, i12)
    const int64_t i10 = r % t1.ne[0], i11 = (r / t1.ne[0]) % t1.ne[1], i12 = r / (t1.ne[0] * t1.ne[1]);
    const int32_t row = *(const int32_t *) (s1 + i10 * t1.nb[0] + i11 * t1.nb[1] + i12 * t1.nb[2]);
    const char * srow = s0 + row * t0.nb[1] + i11 * t0.nb[2] + i12 * t0.nb[3];
    char * drow = d + i10 * td.nb[1] + i11 * td.nb[2] + i12 * td.nb[3];
    for (int64_t i = threadIdx.x; i < t0.ne[0]; i += blockDim.x) {
        *(float *) (drow + i * td.nb[0]) = dequant_elem(type, srow, i);
    }
}

void op_get_rows(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * s0 = dst->src[0];
    const ggml_tensor * s1 = dst->src[1];
    const int64_t n = s1->ne[0] * s1->ne[1] * s1->ne[2];
    if (n == 0) return;
    hipLaunchKernelGGL(k_get_rows, dim3((unsigned) n), dim3(256), 0, ctx.stream, (const char *) s0->data, mk(s0),
                       (int) s0->type, (const char *) s1->data, mk(s1), (char *) dst->data, mk(dst));
}

// ------------------------------------------------------------------------------------------
// RMS norm (ops.cpp:3270-3316): sum of x*x in double, mean = sum/ne0 (rounded to float),
// scale = 1/sqrtf(mean+eps), y = x*scale; optionally y *= w (the following MUL node).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_rms_norm(const char * __restrict__ x, t4 tx, char * __restrict__ y, t4 ty,
                                                  const char * __restrict__ w, t4 tw, char * __restrict__ y2, t4 ty2,
                                                  float eps) {
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % tx.ne[1], i2 = (r / tx.ne[1]) % tx.ne[2], i3 = r / (tx.ne[1] * tx.ne[2]);
    const float * xr = (const float *) (x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3]);
    float * yr = (float *) (y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3]);
    const int64_t ne0 = tx.ne[0];
    // the CPU's sequential double sum, decided from a parallel one (quant_act.h)
    double acc = 0.0;
    for (int64_t i = threadIdx.x; i < ne0; i += 256) {
        const float v = *(const float *) ((const char *) xr + i * tx.nb[0]);
        acc = __dadd_rn(acc, (double) __fmul_rn(v, v));
    }
    acc = wave_sum(acc);
    __shared__ double part[4];
    __shared__ float smean;
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double s = __dadd_rn(__dadd_rn(part[0], part[1]), __dadd_rn(part[2], part[3]));
        float m;
        if (!rms_mean_decided(s, ne0, m)) {
            double q = 0.0;
            for (int64_t i = 0; i < ne0; ++i) {
                const float v = *(const float *) ((const char *) xr + i * tx.nb[0]);
                q = __dadd_rn(q, (double) __fmul_rn(v, v));
            }
            m = (float) __ddiv_rn(q, (double) ne0);
        }
        smean = m;
    }
    __syncthreads();
    const float mean = smean;
    const float scale = 1.0f / sqrtf(mean + eps);
    if (y2) {
        // fused norm-weight MUL: the norm output is still stored (other readers stay
        // correct, and an in-place MUL sees the same thread write y then y*w in order)
        float * y2r = (float *) (y2 + i1 * ty2.nb[1] + i2 * ty2.nb[2] + i3 * ty2.nb[3]);
        const char * wr = w + (i1 % tw.ne[1]) * tw.nb[1] + (i2 % tw.ne[2]) * tw.nb[2] + (i3 % tw.ne[3]) * tw.nb[3];
        const int64_t nw = tw.ne[0];
        for (int64_t i = threadIdx.x; i < ne0; i += 256) {
            const float v = __fmul_rn(xr[i], scale);
            yr[i] = v;
            y2r[i] = __fmul_rn(v, *(const float *) (wr + (i % nw) * tw.nb[0]));
        }
    } else {
        for (int64_t i = threadIdx.x; i < ne0; i += 256) yr[i] = __fmul_rn(*(const float *) ((const char *) xr + i * tx.nb[0]), scale);
    }
}

void op_rms_norm(exec_ctx & ctx, ggml_tensor * dst, const ggml_tensor * mul_w, ggml_tensor * out) {
    const ggml_tensor * src = dst->src[0];
    float eps;
    memcpy(&eps, dst->op_params, sizeof(float));
    const int64_t nrows = src->ne[1] * src->ne[2] * src->ne[3];
    if (nrows == 0) return;
    t4 tw = {}, t2 = {};
    for (int i = 0; i < 4; ++i) { tw.ne[i] = 1; t2.ne[i] = 1; }
    if (mul_w) { tw = mk(mul_w); t2 = mk(out); }
    hipLaunchKernelGGL(k_rms_norm, dim3((unsigned) nrows), dim3(256), 0, ctx.stream, (const char *) src->data, mk(src),
                       (char *) dst->data, mk(dst), mul_w ? (const char *) mul_w->data : nullptr, tw,
                       mul_w ? (char *) out->data : nullptr, t2, eps);
}

// layer norm (ops.cpp ggml_compute_forward_norm_f32): mean/variance in double
__global__ __launch_bounds__(256) void k_norm(const char * __restrict__ x, t4 tx, char * __restrict__ y, t4 ty, float eps) {
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % tx.ne[1], i2 = (r / tx.ne[1]) % tx.ne[2], i3 = r / (tx.ne[1] * tx.ne[2]);
    const float * xr = (const float *) (x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3]);
    float * yr = (float *) (y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3]);
    const int64_t ne0 = tx.ne[0];
    __shared__ double part[4];
    double sum = 0.0;
    for (int64_t i = threadIdx.x; i < ne0; i += 256) sum += (double) xr[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, WAVE);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = sum;
    __syncthreads();
    const float mean = (float) ((part[0] + part[1] + part[2] + part[3]) / (double) ne0);
    __syncthreads();
    double s2 = 0.0;
    for (int64_t i = threadIdx.x; i < ne0; i += 256) {
        const float v = xr[i] - mean;
        s2 += (double) (v * v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, WAVE);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s2;
    __syncthreads();
    const float variance = (float) ((part[0] + part[1] + part[2] + part[3]) / (double) ne0);
    const float scale = 1.0f / sqrtf(variance + eps);
    for (int64_t i = threadIdx.x; i < ne0; i += 256) yr[i] = (xr[i] - mean) * scale;
}

void op_norm(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * src = dst->src[0];
    float eps;
    memcpy(&eps, dst->op_params, sizeof(float));
    const int64_t nrows = src->ne[1] * src->ne[2] * src->ne[3];
    if (nrows == 0) return;
    hipLaunchKernelGGL(k_norm, dim3((unsigned) nrows), dim3(256), 0, ctx.stream, (const char *) src->data, mk(src),
                       (char *) dst->data, mk(dst), eps);
}

// ------------------------------------------------------------------------------------------
// RoPE (ops.cpp:5080-5362).  theta for pair i is built exactly like ggml_rope_cache_init:
// theta_0 = p, theta_{i+1} = theta_i * theta_scale (fp32, sequential), then rope_yarn.
// ------------------------------------------------------------------------------------------
// one ROPE node: x -> y, optionally also stored as f16 into a KV-cache view (the CPY that
// follows K's rope, fused; its destination comes from the dynamic-pointer table)
struct rope_job {
    const char * x; t4 tx; char * y; t4 ty;
    uint16_t * const * cache;   // nullable: f16 copy of y (y contiguous, flat element order)
    int64_t nrows;
};

struct rope_jobs { rope_job j[2]; int njobs; };

// cos/sin of every rope pair at the positions of ntok tokens ([token][pair]), once per graph:
// rope_cs, the arithmetic of the ROPE kernel, so fused (k_gemv.hip epilogue) and table-driven
// ROPE kernels produce the same bits; every layer's ROPE nodes read it (the sinf / cosf of the
// CPU's libm are ~100 instructions each)
__global__ __launch_bounds__(256) void k_rope_table(const rope_params rp, const int32_t * __restrict__ pos,
                                                    const float * __restrict__ ff, int64_t ntok, float2 * __restrict__ tab) {
    const int np = rp.n_dims / 2;
    for (int64_t e = (int64_t) blockIdx.x * 256 + threadIdx.x; e < ntok * np; e += (int64_t) gridDim.x * 256) {
        const int64_t t = e / np;
        const int ip = (int) (e % np);
        float c, sn;
        rope_cs(rp, (float) pos[t], ip, ff, c, sn);
        tab[e] = make_float2(c, sn);
    }
}

// the table for a ROPE node's parameters and position tensor, launched on first use in the
// graph (run_nodes clears the key: positions change every graph, a capture replays the
// launch); slot 3 of the scratch arena holds it
const float2 * rope_table(exec_ctx & ctx, const ggml_tensor * r, const rope_params & rp, const int32_t * pos,
                          const float * ff, int64_t ntok) {
    if (ctx.rt_table && ctx.rt_pos == pos && ctx.rt_ff == ff && ctx.rt_ntok == ntok &&
        memcmp(ctx.rt_params, r->op_params, sizeof(ctx.rt_params)) == 0) {
        return ctx.rt_table;
    }
    const int64_t n = ntok * (rp.n_dims / 2);
    float2 * tab = (float2 *) ctx.scratch(3, sizeof(float2) * std::max<int64_t>(n, 256));
    hipLaunchKernelGGL(k_rope_table, dim3((unsigned) std::min<int64_t>(ceil_div(n, 256), 1024)), dim3(256), 0, ctx.stream,
                       rp, pos, ff, ntok, tab);
    ctx.rt_table = tab;
    ctx.rt_ntok = ntok;
    ctx.rt_pos = pos;
    ctx.rt_ff = ff;
    memcpy(ctx.rt_params, r->op_params, sizeof(ctx.rt_params));
    return tab;
}

__global__ __launch_bounds__(256) void k_rope(const rope_jobs J, const int32_t * __restrict__ pos,
                                              const float * __restrict__ ff, rope_params rp, const float2 * __restrict__ tab) {
    int64_t r = blockIdx.x;  // row over (i1 head, i2 token, i3) of job 0, then job 1
    const int jb = (J.njobs > 1 && r >= J.j[0].nrows) ? 1 : 0;
    if (jb) r -= J.j[0].nrows;
    const rope_job & jo = J.j[jb];
    const t4 & tx = jo.tx;
    const t4 & ty = jo.ty;
    const int64_t i1 = r % tx.ne[1], i2 = (r / tx.ne[1]) % tx.ne[2], i3 = r / (tx.ne[1] * tx.ne[2]);
    const char * xr = jo.x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3];
    char * yr = jo.y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3];
    uint16_t * cr = jo.cache ? *jo.cache + (yr - jo.y) / 4 : nullptr;
    const int64_t ne0 = tx.ne[0];
    const float p = (float) pos[i2];
    const bool neox = rp.mode & 2;
    for (int64_t ip = threadIdx.x; ip < ne0 / 2; ip += blockDim.x) {
        const int64_t i0 = 2 * ip;
        int64_t a0, a1;
        float o0, o1;
        if (i0 < rp.n_dims) {
            float c, s;
            if (tab) {
                const float2 cs = tab[i2 * (rp.n_dims / 2) + ip];
                c = cs.x; s = cs.y;
            } else {
                rope_cs(rp, p, ip, ff, c, s);
            }
            if (neox) { a0 = ip; a1 = ip + rp.n_dims / 2; }
            else      { a0 = i0; a1 = i0 + 1; }
            const float x0 = *(const float *) (xr + a0 * tx.nb[0]);
            const float x1 = *(const float *) (xr + a1 * tx.nb[0]);
            rope_rotate(x0, x1, c, s, o0, o1);
        } else {
            a0 = i0; a1 = i0 + 1;
            o0 = *(const float *) (xr + i0 * tx.nb[0]);
            o1 = *(const float *) (xr + (i0 + 1) * tx.nb[0]);
        }
        *(float *) (yr + a0 * ty.nb[0]) = o0;
        *(float *) (yr + a1 * ty.nb[0]) = o1;
        if (cr) { cr[a0] = f2h(o0); cr[a1] = f2h(o1); }
    }
}

bool rope_params_of(const ggml_tensor * dst, rope_params & rp) {
    const int32_t * op = dst->op_params;
    rp.n_dims = op[1];
    rp.mode = op[2];
    const int n_ctx_orig = op[4];
    float freq_base, beta_fast, beta_slow;
    memcpy(&freq_base, op + 5, 4);
    memcpy(&rp.freq_scale, op + 6, 4);
    memcpy(&rp.ext_factor, op + 7, 4);
    memcpy(&rp.attn_factor, op + 8, 4);
    memcpy(&beta_fast, op + 9, 4);
    memcpy(&beta_slow, op + 10, 4);
    rp.theta_scale = powf(freq_base, -2.0f / rp.n_dims);
    float corr[2];
    ggml_rope_yarn_corr_dims(rp.n_dims, n_ctx_orig, freq_base, beta_fast, beta_slow, corr);
    rp.corr0 = corr[0]; rp.corr1 = corr[1];
    rp.has_ff = dst->src[2] != nullptr;
    return true;
}

static rope_job make_rope_job(const ggml_tensor * dst, uint16_t * const * cache) {
    const ggml_tensor * src = dst->src[0];
    rope_job j;
    j.x = (const char *) src->data; j.tx = mk(src);
    j.y = (char *) dst->data; j.ty = mk(dst);
    j.cache = cache;
    j.nrows = src->ne[1] * src->ne[2] * src->ne[3];
    return j;
}

// one or two ROPE nodes with identical parameters / positions in one launch;
// cache[i] = dynamic-table slot of a fused f16 KV-cache store for node i (nullable)
void op_rope_multi(exec_ctx & ctx, ggml_tensor * const * nodes, int n, void * const * const * cache) {
    rope_params rp;
    rope_params_of(nodes[0], rp);
    rope_jobs J;
    J.njobs = n;
    int64_t rows = 0;
    for (int i = 0; i < n; ++i) {
        J.j[i] = make_rope_job(nodes[i], cache ? (uint16_t * const *) cache[i] : nullptr);
        rows += J.j[i].nrows;
    }
    if (rows == 0) return;
    const ggml_tensor * pos = nodes[0]->src[1];
    const ggml_tensor * ff  = nodes[0]->src[2];
    const unsigned thr = nodes[0]->src[0]->ne[0] / 2 >= 256 ? 256 : 64;
    // positions indexed by i2 only (the llama layout: [dims, heads, tokens]); a table of
    // pos->ne[0] tokens shared by every ROPE node of the graph
    const bool tabbed = pos->ne[0] == nodes[0]->src[0]->ne[2] && nodes[0]->src[0]->ne[3] == 1;
    const float2 * tab = tabbed ? rope_table(ctx, nodes[0], rp, (const int32_t *) pos->data, ff ? (const float *) ff->data : nullptr,
                                             pos->ne[0]) : nullptr;
    hipLaunchKernelGGL(k_rope, dim3((unsigned) rows), dim3(thr), 0, ctx.stream, J, (const int32_t *) pos->data,
                       ff ? (const float *) ff->data : nullptr, rp, tab);
}

void op_rope(exec_ctx & ctx, ggml_tensor * dst) {
    ggml_tensor * nodes[1] = {dst};
    op_rope_multi(ctx, nodes, 1, nullptr);
}

// ------------------------------------------------------------------------------------------
// soft_max (ops.cpp:4731-4827): w = x*scale + slope*mask; y = exp(w-max)/sum (sum in double)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_soft_max(const char * __restrict__ x, t4 tx, char * __restrict__ y, t4 ty,
                                                  const char * __restrict__ mask, t4 tm, int mask_f16,
                                                  float scale, float max_bias, float m0, float m1, uint32_t n_head_log2) {
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % tx.ne[1], i2 = (r / tx.ne[1]) % tx.ne[2], i3 = r / (tx.ne[1] * tx.ne[2]);
    const float * xr = (const float *) (x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3]);
    float * yr = (float *) (y + i1 * ty.nb[1] + i2 * ty.nb[2] + i3 * ty.nb[3]);
    const int64_t nc = tx.ne[0];
    const uint32_t h = (uint32_t) i2;  // head index = (flat_row / ne01) % ne02
    const float slope = max_bias > 0.0f ? (h < n_head_log2 ? powf(m0, h + 1) : powf(m1, 2 * (h - n_head_log2) + 1)) : 1.0f;
    const char * mr = mask ? mask + (i1 % tm.ne[1]) * tm.nb[1] : nullptr;

    __shared__ float redf[4];
    __shared__ double redd[4];
    float mx = -INFINITY;
    for (int64_t i = threadIdx.x; i < nc; i += 256) {
        float w = __fmul_rn(xr[i], scale);
        if (mr) w = __fadd_rn(w, __fmul_rn(slope, mask_f16 ? h2f(*(const uint16_t *) (mr + 2 * i)) : *(const float *) (mr + 4 * i)));
        yr[i] = w;
        mx = fmaxf(mx, w);
    }
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) redf[threadIdx.x >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
    // ggml_vec_soft_max_f32 (vec.cpp:257-300, AVX-512): 16-wide chunks of ggml_v_expf, each
    // chunk reduced by _mm512_reduce_add_ps and accumulated in double in chunk order; the
    // n % 16 tail uses libm expf.  Chunk sums go to LDS and one thread adds them in order.
    constexpr int MAXCH = 4096;
    __shared__ float csum[MAXCH];
    const int64_t nch = nc / 16;
    double sum = 0.0;
    for (int64_t c = threadIdx.x; c < nch; c += 256) {
        float w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            w[k] = v_expf_avx512(__fsub_rn(yr[16 * c + k], mx));
            yr[16 * c + k] = w[k];
        }
        const float cs = reduce16_avx512(w);
        if (c < MAXCH) csum[c] = cs;
        else sum += (double) cs;  // beyond MAXCH chunks: order-approximate double sum
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, WAVE);
    if ((threadIdx.x & 63) == 0) redd[threadIdx.x >> 6] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int64_t c = 0; c < min(nch, (int64_t) MAXCH); ++c) s += (double) csum[c];
        s += redd[0] + redd[1] + redd[2] + redd[3];
        for (int64_t i = 16 * nch; i < nc; ++i) {
            const float e = expf_cr(__fsub_rn(yr[i], mx));
            yr[i] = e;
            s += (double) e;
        }
        redd[0] = s;
    }
    __syncthreads();
    const float inv = (float) (1.0 / redd[0]);
    for (int64_t i = threadIdx.x; i < nc; i += 256) yr[i] = __fmul_rn(yr[i], inv);
}

void op_soft_max(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * src = dst->src[0];
    const ggml_tensor * mask = dst->src[1];
    float scale, max_bias;
    memcpy(&scale, (const float *) dst->op_params + 0, 4);
    memcpy(&max_bias, (const float *) dst->op_params + 1, 4);
    const uint32_t n_head = (uint32_t) src->ne[2];
    const uint32_t n_head_log2 = 1u << (uint32_t) floor(log2((double) n_head));
    const float m0 = powf(2.0f, -(max_bias) / n_head_log2);
    const float m1 = powf(2.0f, -(max_bias / 2.0f) / n_head_log2);
    const int64_t nrows = src->ne[1] * src->ne[2] * src->ne[3];
    if (nrows == 0) return;
    t4 tm = {};
    for (int i = 0; i < 4; ++i) tm.ne[i] = 1;
    if (mask) tm = mk(mask);
    hipLaunchKernelGGL(k_soft_max, dim3((unsigned) nrows), dim3(256), 0, ctx.stream, (const char *) src->data, mk(src),
                       (char *) dst->data, mk(dst), mask ? (const char *) mask->data : nullptr, tm,
                       mask && mask->type == GGML_TYPE_F16 ? 1 : 0, scale, max_bias, m0, m1, n_head_log2);
}

// ------------------------------------------------------------------------------------------
// ARGSORT (ops.cpp:6956-6993; ggml_top_k of the MoE router, src/llama-graph.cpp:694): the
// CPU's exchange sort restated per row — for j, every later k whose value orders before
// position j's swaps with it — so ties resolve exactly as on the CPU.  One workgroup per
// row, the row and its index permutation in LDS, the exchange loop on one lane (router
// rows are n_expert long; supports_op caps ne0).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_argsort(const char * __restrict__ x, t4 tx, char * __restrict__ d, t4 td, int order) {
    extern __shared__ __attribute__((aligned(16))) char sm[];
    const int n = (int) tx.ne[0];
    float * v = (float *) sm;
    int * ix = (int *) (v + n);
    const int64_t r = blockIdx.x;
    const int64_t i1 = r % tx.ne[1], i2 = (r / tx.ne[1]) % tx.ne[2], i3 = r / (tx.ne[1] * tx.ne[2]);
    const char * xr = x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3];
    char * dr = d + i1 * td.nb[1] + i2 * td.nb[2] + i3 * td.nb[3];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        v[i] = *(const float *) (xr + i * tx.nb[0]);
        ix[i] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int j = 0; j < n; ++j) {
            for (int k = j + 1; k < n; ++k) {
                const float a = v[ix[j]], b = v[ix[k]];
                if ((order == GGML_SORT_ORDER_ASC && a > b) || (order == GGML_SORT_ORDER_DESC && a < b)) {
                    const int tmp = ix[j];
                    ix[j] = ix[k];
                    ix[k] = tmp;
                }
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) *(int32_t *) (dr + i * td.nb[0]) = ix[i];
}

void op_argsort(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * src = dst->src[0];
    const int64_t nrows = ggml_nrows(src);
    if (nrows == 0 || src->ne[0] == 0) return;
    const int order = dst->op_params[0];
    const size_t lds = (size_t) src->ne[0] * (sizeof(float) + sizeof(int));
    hipLaunchKernelGGL(k_argsort, dim3((unsigned) nrows), dim3(64), lds, ctx.stream, (const char *) src->data, mk(src),
                       (char *) dst->data, mk(dst), order);
}

// ------------------------------------------------------------------------------------------
// SUM_ROWS (ops.cpp:1956-1986 with ggml_vec_sum_f32, vec.h:908: sequential double sum,
// rounded once): one lane per row, the CPU's order
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_sum_rows(const char * __restrict__ x, t4 tx, char * __restrict__ d, t4 td, int64_t nrows) {
    const int64_t r = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    const int64_t i1 = r % tx.ne[1], i2 = (r / tx.ne[1]) % tx.ne[2], i3 = r / (tx.ne[1] * tx.ne[2]);
    const char * xr = x + i1 * tx.nb[1] + i2 * tx.nb[2] + i3 * tx.nb[3];
    double s = 0.0;
    for (int64_t i = 0; i < tx.ne[0]; ++i) s += (double) *(const float *) (xr + i * tx.nb[0]);
    *(float *) (d + i1 * td.nb[1] + i2 * td.nb[2] + i3 * td.nb[3]) = (float) s;
}

void op_sum_rows(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * src = dst->src[0];
    const int64_t nrows = ggml_nrows(src);
    if (nrows == 0) return;
    hipLaunchKernelGGL(k_sum_rows, dim3((unsigned) ceil_div(nrows, 64)), dim3(64), 0, ctx.stream, (const char *) src->data,
                       mk(src), (char *) dst->data, mk(dst), nrows);
}

// ------------------------------------------------------------------------------------------
// MoE router chain in one launch (build_moe_ffn, src/llama-graph.cpp:661-712, softmax gating
// with norm_w): probs = SOFT_MAX(logits * scale), order = ARGSORT(probs, DESC) (ggml_top_k's
// view keeps its first n_used), w = GET_ROWS(probs, top-k), sum = SUM_ROWS(w), wn = w / sum.
// One lane per token; every output node is written with the arithmetic of its stand-alone
// kernel above (k_soft_max's chunked AVX-512 exp + double sum for n >= 16, libm expf tail;
// the exchange sort; the double row sum; the broadcast DIV), so fused and unfused graphs agree
// bit for bit.  Replaces five small launches per MoE layer.
// ------------------------------------------------------------------------------------------
struct moe_route_args {
    const char * logits; int64_t nb_l;
    char * probs; int64_t nb_p;
    char * order; int64_t nb_o;
    char * w; int64_t nb_w;           // GET_ROWS output rows ([1, n_used, T]: row t at t * nb_w)
    char * wsum; int64_t nb_s;        // SUM_ROWS output (nullable)
    char * wn; int64_t nb_n;          // DIV output rows (nullable)
    int n_exp, n_used;
    int64_t T;
    float scale;
    int stage;                        // bit 0: SOFT_MAX + ARGSORT; bit 1: GET_ROWS [+ SUM_ROWS + DIV]
};

// stage 1 [+ 2] of token t for up to 16 experts, the logits at x (global or LDS)
__device__ __forceinline__ void moe_route16(const moe_route_args & a, int64_t t, const float * x) {
    float * p = (float *) (a.probs + t * a.nb_p);
    int32_t * o = (int32_t *) (a.order + t * a.nb_o);
    const int n = a.n_exp;
    {
        // up to 16 experts (Mixtral: 8): the same arithmetic in registers. The global
        // probabilities / order are written once at the end instead of being re-read through every
        // pass (the exchange sort's p[o[j]] was a chain of dependent global loads: 7.3 us a launch)
        float pv[16];
        int32_t ov[16];
        float mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            pv[i] = i < n ? __fmul_rn(x[i], a.scale) : 0.0f;
            if (i < n) mx = fmaxf(mx, pv[i]);
        }
        double s = 0.0;
        if (n == 16) {
            float e[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) e[k] = pv[k] = v_expf_avx512(__fsub_rn(pv[k], mx));
            s += (double) reduce16_avx512(e);
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                if (i < n) {
                    pv[i] = expf_cr(__fsub_rn(pv[i], mx));
                    s += (double) pv[i];
                }
            }
        }
        const float inv = (float) (1.0 / s);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            pv[i] = __fmul_rn(pv[i], inv);
            ov[i] = i;
            if (i < n) p[i] = pv[i];
        }
        // the exchange sort on (value, index) pairs: sv[j] is always p[o[j]]
        float sv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) sv[i] = pv[i];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
#pragma unroll
            for (int k = j + 1; k < 16; ++k) {
                if (k < n && sv[j] < sv[k]) {   // GGML_SORT_ORDER_DESC
                    const float tv = sv[j]; sv[j] = sv[k]; sv[k] = tv;
                    const int32_t ti = ov[j]; ov[j] = ov[k]; ov[k] = ti;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) if (i < n) o[i] = ov[i];
        if (a.stage & 2) {
            float * wr = (float *) (a.w + t * a.nb_w);
            double ws = 0.0;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k < a.n_used) {
                    wr[k] = sv[k];
                    ws += (double) sv[k];
                }
            }
            if (a.wsum) {
                const float sf = (float) ws;
                *(float *) (a.wsum + t * a.nb_s) = sf;
                if (a.wn) {
                    float * nr = (float *) (a.wn + t * a.nb_n);
#pragma unroll
                    for (int k = 0; k < 16; ++k) if (k < a.n_used) nr[k] = sv[k] / sf;
                }
            }
        }
    }
}

// the exchange sort (DESC) of the first N (value, index) pairs, as ggml's argsort loop
template <int N>
__device__ __forceinline__ void xsort_desc(float (&sv)[16], int32_t (&ov)[16]) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
#pragma unroll
        for (int k = j + 1; k < N; ++k) {   // selects, not branches
            const bool c = sv[j] < sv[k];
            const float a = sv[j], b = sv[k];
            const int32_t ia = ov[j], ib = ov[k];
            sv[j] = c ? b : a; sv[k] = c ? a : b;
            ov[j] = c ? ib : ia; ov[k] = c ? ia : ib;
        }
    }
}

// moe_route16's arithmetic for n < 16 experts with lane i holding expert i's logit (a whole wave
// calls it): the exps of every expert at once (expf's table loads in flight together, where the
// one-lane loop waited for each), the double sum, the stores and the exchange sort in order
__device__ void moe_route_wave(const moe_route_args & a, int64_t t, float lgt, const uint64_t * etab) {
    const int lane = threadIdx.x & 63;
    const int n = a.n_exp;
    const float v = lane < n ? __fmul_rn(lgt, a.scale) : -INFINITY;
    // the max of lanes 0..15 (n < 16) by DPP within row 0, then broadcast (the shuffle tree was
    // six ds_bpermute round trips)
    float m = v;
    m = fmaxf(m, dppf_xor1(m));
    m = fmaxf(m, dppf_xor2(m));
    m = fmaxf(m, __int_as_float(dpp<DPP_HMIRROR>(__float_as_int(m))));
    m = fmaxf(m, __int_as_float(dpp<DPP_MIRROR>(__float_as_int(m))));
    const float mx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(m), 0));
    const float e = lane < n ? lx_expf_t(__fsub_rn(v, mx), etab) : 0.0f;   // expf_cr, its table from LDS
    // uniform values by v_readlane (a shuffle per step was a ds_bpermute round trip each)
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) if (i < n) s += (double) __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e), i));
    const float inv = (float) (1.0 / s);
    const float pl = __fmul_rn(e, inv);
    float * p = (float *) (a.probs + t * a.nb_p);
    int32_t * o = (int32_t *) (a.order + t * a.nb_o);
    if (lane < n) p[lane] = pl;
    // distinct probabilities: the exchange sort's result is the descending order, so each lane
    // forms its own rank and every output is stored in parallel; a tie (or a NaN) takes the
    // exchange sort below, whose order among equal values is its own
    {
        const float me = lane < n ? pl : -INFINITY;
        int rank = 0;
        bool tie = !(me == me);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float pj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(me), j));
            rank += pj > me ? 1 : 0;
            tie = tie || (pj == me && j != lane);
        }
        if (__ballot(lane < n && tie) == 0 && a.n_used <= n) {
            if (lane < n) o[rank] = lane;
            if (a.stage & 2) {
                const bool top = lane < n && rank < a.n_used;
                if (top) ((float *) (a.w + t * a.nb_w))[rank] = pl;
                if (a.wsum) {
                    double ws = 0.0;   // in rank order, as the CPU's SUM_ROWS
                    for (int k = 0; k < a.n_used; ++k) {
                        const int src = __builtin_ctzll(__ballot(lane < n && rank == k));
                        ws += (double) __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pl), src));
                    }
                    const float sf = (float) ws;
                    if (lane == 0) *(float *) (a.wsum + t * a.nb_s) = sf;
                    if (a.wn && top) ((float *) (a.wn + t * a.nb_n))[rank] = pl / sf;
                }
            }
            return;
        }
    }
    float sv[16];
    int32_t ov[16];
    // the sort on per-lane copies (a shuffle keeps them in VGPRs: branch-free selects, where the
    // scalar copies became a branch per compare-exchange)
#pragma unroll
    for (int i = 0; i < 16; ++i) { sv[i] = __shfl(pl, i, WAVE); ov[i] = i; }
    switch (n) {
        case 8: xsort_desc<8>(sv, ov); break;
        case 4: xsort_desc<4>(sv, ov); break;
        default:
#pragma unroll
            for (int j = 0; j < 16; ++j) {
#pragma unroll
                for (int k = j + 1; k < 16; ++k) {
                    if (k < n && sv[j] < sv[k]) {
                        const float tv = sv[j]; sv[j] = sv[k]; sv[k] = tv;
                        const int32_t ti = ov[j]; ov[j] = ov[k]; ov[k] = ti;
                    }
                }
            }
    }
    if (lane != 0) return;
#pragma unroll
    for (int i = 0; i < 16; ++i) if (i < n) o[i] = ov[i];
    if (a.stage & 2) {
        float * wr = (float *) (a.w + t * a.nb_w);
        double ws = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (k < a.n_used) {
                wr[k] = sv[k];
                ws += (double) sv[k];
            }
        }
        if (a.wsum) {
            const float sf = (float) ws;
            *(float *) (a.wsum + t * a.nb_s) = sf;
            if (a.wn) {
                float * nr = (float *) (a.wn + t * a.nb_n);
#pragma unroll
                for (int k = 0; k < 16; ++k) if (k < a.n_used) nr[k] = sv[k] / sf;
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_moe_route(const moe_route_args a) {
    const int64_t t = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.T) return;
    const float * x = (const float *) (a.logits + t * a.nb_l);
    float * p = (float *) (a.probs + t * a.nb_p);
    int32_t * o = (int32_t *) (a.order + t * a.nb_o);
    const int n = a.n_exp;
    if ((a.stage & 1) && n <= 16) {
        moe_route16(a, t, x);
        return;
    }
    if ((a.stage & 2) && !(a.stage & 1) && a.n_used <= 8) {
        // stage 2 alone: the routed ids, then their probabilities, each as one batch of loads
        int32_t oi[8];
        float wv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) oi[k] = k < a.n_used ? o[k] : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) wv[k] = k < a.n_used ? p[oi[k]] : 0.0f;
        float * wr = (float *) (a.w + t * a.nb_w);
        double ws = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k < a.n_used) {
                wr[k] = wv[k];
                ws += (double) wv[k];
            }
        }
        if (a.wsum) {
            const float sf = (float) ws;
            *(float *) (a.wsum + t * a.nb_s) = sf;
            if (a.wn) {
                float * nr = (float *) (a.wn + t * a.nb_n);
#pragma unroll
                for (int k = 0; k < 8; ++k) if (k < a.n_used) nr[k] = wv[k] / sf;
            }
        }
        return;
    }
    if (a.stage & 1) {
    float mx = -INFINITY;
    for (int i = 0; i < n; ++i) {
        const float v = __fmul_rn(x[i], a.scale);
        p[i] = v;
        mx = fmaxf(mx, v);
    }
    const int nch = n / 16;
    double s = 0.0;
    for (int c = 0; c < nch; ++c) {
        float e[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            e[k] = v_expf_avx512(__fsub_rn(p[16 * c + k], mx));
            p[16 * c + k] = e[k];
        }
        s += (double) reduce16_avx512(e);
    }
    for (int i = 16 * nch; i < n; ++i) {
        const float e = expf_cr(__fsub_rn(p[i], mx));
        p[i] = e;
        s += (double) e;
    }
    const float inv = (float) (1.0 / s);
    for (int i = 0; i < n; ++i) p[i] = __fmul_rn(p[i], inv);
    for (int j = 0; j < n; ++j) o[j] = j;
    for (int j = 0; j < n; ++j) {
        for (int k = j + 1; k < n; ++k) {
            if (p[o[j]] < p[o[k]]) {   // GGML_SORT_ORDER_DESC
                const int32_t tmp = o[j];
                o[j] = o[k];
                o[k] = tmp;
            }
        }
    }
    }
    if (!(a.stage & 2)) return;
    float * wr = (float *) (a.w + t * a.nb_w);
    double ws = 0.0;
    for (int k = 0; k < a.n_used; ++k) {
        wr[k] = p[o[k]];
        ws += (double) wr[k];
    }
    if (a.wsum) {
        const float sf = (float) ws;
        *(float *) (a.wsum + t * a.nb_s) = sf;
        if (a.wn) {
            float * nr = (float *) (a.wn + t * a.nb_n);
            for (int k = 0; k < a.n_used; ++k) nr[k] = wr[k] / sf;
        }
    }
}

// The router logits (MUL_MAT of the f32 gate_inp [K, n_exp] by the norm output,
// build_moe_ffn :661) and the route chain in one launch, one workgroup per token: wave e forms
// logit e in the order the CPU's mat-vec takes for this shape (k_mmv_f_exact: for one token
// ggml_vec_dot_f32's 4 x 16 AVX-512 accumulators, REDUCE, double tail; for two or more
// llamafile's 16-lane FMA chain), then thread 0 runs moe_route16 on them from LDS.  With wscr
// the routed weights, their sum and the normalised weights (GET_ROWS, SUM_ROWS, DIV) go to a
// private scratch [3][T][n_used] the combine reads.
struct moe_router_args {
    const char * W; int64_t nb01; int64_t K;
    const char * X; int64_t nb11;
    char * logits; int64_t nb_lo;   // MUL_MAT output row t at t * nb_lo
    moe_route_args r;
    // norm prologue (one token, k_moe_router_mw): X = RMS_NORM(px) * pw formed by every workgroup
    // with k_norm_fused's arithmetic; workgroup 0 stores it (to X) and its Q8_K quantization
    const float * px; const float * pw; float eps;
    int8_t * qs; float * qd; int16_t * qsum;
    unsigned long long * kt;        // in-graph kernel timeline region (nullable)
};

template <bool TINY>
__global__ __launch_bounds__(1024) void k_moe_router(const moe_router_args a) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t t = blockIdx.x;
    __shared__ float part[16][64];
    __shared__ float lg[16];
    const float * w = (const float *) (a.W + wave * a.nb01);
    const float * x = (const float *) (a.X + t * a.nb11);
    if constexpr (TINY) {
        float acc = 0.0f;
        const int s = lane & 15;
        if (lane < 16) {
            int64_t k = 0;
            for (; k + 32 * 16 <= a.K; k += 32 * 16) {
                float wv[32], xv[32];
#pragma unroll
                for (int u = 0; u < 32; ++u) { wv[u] = w[k + 16 * u + s]; xv[u] = x[k + 16 * u + s]; }
#pragma unroll
                for (int u = 0; u < 32; ++u) acc = fmaf(wv[u], xv[u], acc);
            }
            for (; k < a.K; k += 16) acc = fmaf(w[k + s], x[k + s], acc);
        }
        acc = __fadd_rn(acc, __shfl_xor(acc, 8, WAVE));
        acc = __fadd_rn(acc, __shfl_xor(acc, 4, WAVE));
        acc = __fadd_rn(acc, __shfl_xor(acc, 2, WAVE));
        acc = __fadd_rn(acc, __shfl_xor(acc, 1, WAVE));
        if (lane == 0) lg[wave] = acc;
    } else {
        const int64_t np = a.K & ~int64_t(63);
        float acc = 0.0f;
        int64_t i = 0;
        // 32 steps of the chain per batch: every load of a batch in flight before its FMAs (a
        // chain that waits on each load pays the memory latency per step: 10 us a launch)
        for (; i + 32 * 64 <= np; i += 32 * 64) {
            float wv[32], xv[32];
#pragma unroll
            for (int u = 0; u < 32; ++u) { wv[u] = w[i + 64 * u + lane]; xv[u] = x[i + 64 * u + lane]; }
#pragma unroll
            for (int u = 0; u < 32; ++u) acc = fmaf(wv[u], xv[u], acc);
        }
        for (; i < np; i += 64) acc = fmaf(w[i + lane], x[i + lane], acc);
        part[wave][lane] = acc;
        __syncthreads();
        if (lane == 0) {
            const float * pa = part[wave];
            float v[16];
#pragma unroll
            for (int l = 0; l < 16; ++l) v[l] = __fadd_rn(__fadd_rn(pa[l], pa[32 + l]), __fadd_rn(pa[16 + l], pa[48 + l]));
            double sumf = (double) reduce16_avx512(v);
            for (int64_t k = np; k < a.K; ++k) sumf += (double) __fmul_rn(w[k], x[k]);
            lg[wave] = (float) sumf;
        }
    }
    __syncthreads();
    if (wave == 0) {
        float * lo = (float *) (a.logits + t * a.nb_lo);
        if (lane < a.r.n_exp) lo[lane] = lg[lane];
        if (a.r.n_exp < 16) moe_route_wave(a.r, t, lane < a.r.n_exp ? lg[lane] : 0.0f, lx_exp2f_tab);
        else if (lane == 0) moe_route16(a.r, t, lg);
    }
}

// The same over n_exp workgroups per token (grid n_exp x T): workgroup e stages x and router row
// e in LDS with every load in flight at once (one CU streaming all 8 rows took ~10 us a launch),
// wave 0 forms logit e in the same order, and the last workgroup of the token to store its logit
// (arrival counter, self-resetting) runs the route on the logits read back past L1.
template <bool TINY>
__global__ __launch_bounds__(256) void k_moe_router_mw(const moe_router_args a, int * cnt) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    kt_enter(a.kt, 5);
    __shared__ uint64_t etab[32];   // expf's table, fetched with the first loads
    const uint64_t et = lx_exp2f_tab[tid & 31];
    const int e = blockIdx.x;
    const int64_t t = blockIdx.y;
    extern __shared__ __attribute__((aligned(16))) float xs[];   // [K] x, [K] w
    float * ws = xs + a.K;
    const float * w = (const float *) (a.W + e * a.nb01);
    const float * x = (const float *) (a.X + t * a.nb11);
    // every load in flight before the first LDS store (K <= 8192; the launcher checks)
    if (a.px) {
        // x = RMS_NORM(px) * pw: thread t owns the float4s at 4 (t + 256 u); the double sum in
        // any order is decided against the CPU's sequential one (quant_act.h rms_mean_decided)
        __shared__ double wpart[4];
        __shared__ float smean;
        float4 pv[4], nw[4], wv[4];
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = 4 * (tid + 256 * u);
            if (k < a.K) { pv[u] = *(const float4 *) (a.px + k); nw[u] = *(const float4 *) (a.pw + k); wv[u] = *(const float4 *) (w + k); }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (4 * (tid + 256 * u) < a.K) acc = __dadd_rn(acc, sq4(pv[u]));
        }
        acc = wave_sum(acc);
        if (lane == 0) wpart[wave] = acc;
        __syncthreads();
        if (tid == 0) {
            const double sum = __dadd_rn(__dadd_rn(wpart[0], wpart[1]), __dadd_rn(wpart[2], wpart[3]));
            float mean;
            if (!rms_mean_decided(sum, a.K, mean)) mean = rms_mean_sequential(a.px, nullptr, a.K);
            smean = mean;
        }
        __syncthreads();
        const float scale = 1.0f / sqrtf(smean + a.eps);
        float * yo = e == 0 ? (float *) (a.X + t * a.nb11) : nullptr;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t k = 4 * (tid + 256 * u);
            if (k >= a.K) continue;
            float4 y;
            y.x = __fmul_rn(__fmul_rn(pv[u].x, scale), nw[u].x); y.y = __fmul_rn(__fmul_rn(pv[u].y, scale), nw[u].y);
            y.z = __fmul_rn(__fmul_rn(pv[u].z, scale), nw[u].z); y.w = __fmul_rn(__fmul_rn(pv[u].w, scale), nw[u].w);
            *(float4 *) (xs + k) = y;
            *(float4 *) (ws + k) = wv[u];
            if (yo) {
                *(float4 *) (yo + k) = y;
                if (a.qs) {   // wave w's 256 elements of pass u: Q8_K block w + 4 u
                    const float q[4] = {y.x, y.y, y.z, y.w};
                    const int64_t c0 = 256 * (wave + 4 * u);
                    q8K_wave(q, lane, a.qs + c0, a.qsum + c0 / 16, a.qd + c0 / 256);
                }
            }
        }
    } else {
        float4 xv[8], wv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = 4 * (tid + 256 * u);
            if (k < a.K) { xv[u] = *(const float4 *) (x + k); wv[u] = *(const float4 *) (w + k); }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t k = 4 * (tid + 256 * u);
            if (k < a.K) { *(float4 *) (xs + k) = xv[u]; *(float4 *) (ws + k) = wv[u]; }
        }
    }
    if (tid < 32) etab[tid] = et;
    __syncthreads();
    __shared__ int is_last;
    if (wave == 0) {
        float lgt;
        if constexpr (TINY) {
            float acc = 0.0f;
            const int s = lane & 15;
            if (lane < 16) {
                int64_t k = 0;
                for (; k + 16 * 16 <= a.K; k += 16 * 16) {   // LDS reads of a batch ahead of its FMAs
                    float wv[16], xv[16];
#pragma unroll
                    for (int u = 0; u < 16; ++u) { wv[u] = ws[k + 16 * u + s]; xv[u] = xs[k + 16 * u + s]; }
#pragma unroll
                    for (int u = 0; u < 16; ++u) acc = fmaf(wv[u], xv[u], acc);
                }
                for (; k < a.K; k += 16) acc = fmaf(ws[k + s], xs[k + s], acc);
            }
            acc = __fadd_rn(acc, __shfl_xor(acc, 8, WAVE));
            acc = __fadd_rn(acc, __shfl_xor(acc, 4, WAVE));
            acc = __fadd_rn(acc, __shfl_xor(acc, 2, WAVE));
            acc = __fadd_rn(acc, __shfl_xor(acc, 1, WAVE));
            lgt = acc;
        } else {
            const int64_t np = a.K & ~int64_t(63);
            float acc = 0.0f;
            int64_t i = 0;
            for (; i + 16 * 64 <= np; i += 16 * 64) {   // LDS reads of a batch ahead of its FMAs
                float wv[16], xv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) { wv[u] = ws[i + 64 * u + lane]; xv[u] = xs[i + 64 * u + lane]; }
#pragma unroll
                for (int u = 0; u < 16; ++u) acc = fmaf(wv[u], xv[u], acc);
            }
            for (; i < np; i += 64) acc = fmaf(ws[i + lane], xs[i + lane], acc);
            // the AVX-512 REDUCE of the 4 x 16 accumulators, then _mm512_reduce_add_ps, as
            // lane-parallel halvings (k_moe_router1)
            float r = __fadd_rn(acc, __shfl_down(acc, 32, WAVE));
            r = __fadd_rn(r, __shfl_down(r, 16, WAVE));
            r = __fadd_rn(__shfl_down(r, 8, WAVE), r);
            r = __fadd_rn(__shfl_down(r, 4, WAVE), r);
            r = __fadd_rn(r, __shfl_down(r, 2, WAVE));
            r = __fadd_rn(r, __shfl_down(r, 1, WAVE));
            double sumf = (double) r;
            for (int64_t k = np; k < a.K; ++k) sumf += (double) __fmul_rn(ws[k], xs[k]);
            lgt = (float) sumf;
        }
        if (lane == 0) {
            // the logit written through to the coherent level and drained before the counter add;
            // the last workgroup reads them back with agent-scope (L1-bypassing) loads
            __hip_atomic_store((float *) (a.logits + t * a.nb_lo) + e, lgt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int prev = __hip_atomic_fetch_add(cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            is_last = prev == a.r.n_exp - 1;
            if (is_last) __hip_atomic_store(cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (is_last && wave == 0) {
        const float * lo = (const float *) (a.logits + t * a.nb_lo);
        if (a.r.n_exp < 16) {
            const float l = lane < a.r.n_exp ? __hip_atomic_load(lo + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
            moe_route_wave(a.r, t, l, etab);
        } else if (lane == 0) {
            float lg[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) lg[i] = __hip_atomic_load(lo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            moe_route16(a.r, t, lg);
        }
    }
    kt_exit(a.kt, 5);   // waves 1-3: the hand-off; wave 0 of the last workgroup: after the route
}

// One token, K = 64 KS, in ONE workgroup of 64 n_exp threads with no hand-off: wave e holds its
// router row's 64-step slice of every AVX-512 accumulator lane in registers (all KS loads in
// flight at once), the input (or its norm prologue) is staged once in LDS, the waves' chains run
// side by side, and wave 0 routes from the logits in LDS.
template <int KS>
__global__ __launch_bounds__(1024) void k_moe_router1(const moe_router_args a) {
    constexpr int K = 64 * KS;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int NT = blockDim.x, n = a.r.n_exp;
    kt_enter(a.kt, 1 + (unsigned) n);
    __shared__ uint64_t etab[32];
    __shared__ __attribute__((aligned(16))) float xs[K];
    __shared__ double wpart[16];
    __shared__ float smean, lg[16];
    const float * w = (const float *) (a.W + wave * a.nb01);
    const int NV = K / 4;   // float4s of the row
    // x and the norm weight first, then the router rows: the loads return in order, so the norm
    // runs while the 128 KiB of rows are still arriving (issued behind the rows, the norm waited
    // for all of them: 2.3 us to its first sum); NV <= 4 NT (the launcher checks)
    float4 x4[4], w4[4];
    if (a.px) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int v = tid + NT * u;
            if (v < NV) { x4[u] = *(const float4 *) (a.px + 4 * v); w4[u] = *(const float4 *) (a.pw + 4 * v); }
        }
    }
    float wv[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) wv[s] = w[64 * s + lane];
    const uint64_t et = lx_exp2f_tab[tid & 31];   // stored to LDS once the loads are all issued
    // phase stamps (GGML_MI355X_KTRACE_RAW=moe_router): slot 2 + i, written by thread 0
    auto stamp = [&](int i) { if (a.kt && tid == 0) a.kt[2 + i] = __builtin_amdgcn_s_memrealtime(); };
    if (a.px) {
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < 4; ++u) if (tid + NT * u < NV) acc = __dadd_rn(acc, sq4(x4[u]));
        acc = wave_sum_rows_f64(acc);   // any order: the mean is decided against the CPU's below
        if (lane == 0) wpart[wave] = acc;
        __syncthreads();
        stamp(0);
        if (tid == 0) {
            double sum = 0.0;
            for (int i = 0; i < NT / 64; ++i) sum = __dadd_rn(sum, wpart[i]);
            float mean;
            if (!rms_mean_decided(sum, K, mean)) mean = rms_mean_sequential(a.px, nullptr, K);
            smean = mean;
        }
        __syncthreads();
        const float scale = 1.0f / sqrtf(smean + a.eps);
        float * yo = (float *) a.X;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int v = tid + NT * u;
            if (v >= NV) continue;
            float4 y;
            y.x = __fmul_rn(__fmul_rn(x4[u].x, scale), w4[u].x); y.y = __fmul_rn(__fmul_rn(x4[u].y, scale), w4[u].y);
            y.z = __fmul_rn(__fmul_rn(x4[u].z, scale), w4[u].z); y.w = __fmul_rn(__fmul_rn(x4[u].w, scale), w4[u].w);
            *(float4 *) (xs + 4 * v) = y;
            *(float4 *) (yo + 4 * v) = y;
        }
        // (its Q8_K quantization runs after the logits, on the waves the route leaves idle)
    } else {
        for (int v = tid; v < NV; v += NT) *(float4 *) (xs + 4 * v) = *(const float4 *) ((const float *) a.X + 4 * v);
    }
    if (tid < 32) etab[tid] = et;
    stamp(1);
    __syncthreads();
    stamp(2);
    float acc = 0.0f;
#pragma unroll
    for (int s0 = 0; s0 < KS; s0 += 16) {   // LDS reads of a batch ahead of its FMAs
        float xv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) xv[u] = s0 + u < KS ? xs[64 * (s0 + u) + lane] : 0.0f;
#pragma unroll
        for (int u = 0; u < 16; ++u) if (s0 + u < KS) acc = fmaf(wv[s0 + u], xv[u], acc);
    }
    // REDUCE of the 4 x 16 accumulators, (a[l] + a[32 + l]) + (a[16 + l] + a[48 + l]), then the
    // _mm512_reduce_add_ps tree (k_mmv_f_exact's order) as lane-parallel halvings
    // (lane i + 32 / i + 16 by gfx950's cross-row permlane swaps, i + 8 .. i + 1 by DPP row shifts:
    // the shuffles were six ds_bpermute round trips)
    const auto h32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc), __float_as_uint(acc), false, false);
    float r = __fadd_rn(acc, __uint_as_float(h32[1]));   // lanes 0..31: + lane i + 32
    const auto h16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(r), __float_as_uint(r), false, false);
    r = __fadd_rn(r, __uint_as_float(h16[1]));           // lanes 0..15: + lane i + 16
    r = __fadd_rn(__int_as_float(dpp<0x108>(__float_as_int(r))), r);   // row_shl:8
    r = __fadd_rn(__int_as_float(dpp<0x104>(__float_as_int(r))), r);
    r = __fadd_rn(r, __int_as_float(dpp<0x102>(__float_as_int(r))));
    r = __fadd_rn(r, __int_as_float(dpp<0x101>(__float_as_int(r))));
    if (lane == 0) {
        const float l = r;   // (float) of the double sum of one float
        lg[wave] = l;
        ((float *) a.logits)[wave] = l;
    }
    stamp(3);
    __syncthreads();
    stamp(4);
    if (wave == 0) {
        moe_route_wave(a.r, 0, lane < n ? lg[lane] : 0.0f, etab);
    } else if (a.px && a.qs) {
        // the normalized row's Q8_K blocks from LDS, by waves 1.. while wave 0 routes (formed
        // before the logits, they cost 0.5 us on the path to the route): lane l quantizes
        // elements 4l .. 4l + 3 of its block, as the norm's own wave did
        for (int b = wave - 1; b < K / 256; b += NT / 64 - 1) {
            const float4 y = *(const float4 *) (xs + 256 * b + 4 * lane);
            const float q[4] = {y.x, y.y, y.z, y.w};
            q8K_wave(q, lane, a.qs + 256 * b, a.qsum + 16 * b, a.qd + b);
        }
    }
    if (a.kt && tid == 0) a.kt[1] = __builtin_amdgcn_s_memrealtime();
}

// which router kernel takes MUL_MAT node mm: MOE_R1 the one-workgroup kernel (one token, K = 4096),
// MOE_RMW the multi-workgroup counter kernel, MOE_RPLAIN the per-token fallback, MOE_RNONE none.
// With the norm prologue (pro) only the first two form the FFN norm; plan_resid (dispatch.cpp)
// asks this same predicate before it hands the norm to the router launch
int moe_router_path(const ggml_tensor * mm, bool pro) {
    const ggml_tensor * W = mm->src[0], * X = mm->src[1];
    const int64_t n = W->ne[1], K = W->ne[0], T = X->ne[1];
    if (W->type != GGML_TYPE_F32 || X->type != GGML_TYPE_F32 || n > 16 || n < 1 || W->ne[2] != 1 || W->ne[3] != 1 ||
        X->ne[2] != 1 || X->ne[3] != 1 || X->nb[0] != 4 || W->nb[0] != 4 || mm->nb[0] != 4 || mm->ne[1] != T) return MOE_RNONE;
    static const bool one = !getenv("GGML_MI355X_ROUTER1") || atoi(getenv("GGML_MI355X_ROUTER1")) != 0;
    if (one && T == 1 && K == 4096 && ggml_is_contiguous(X) && n >= 4 && n < 16 && (uintptr_t) X->data % 16 == 0) return MOE_R1;
    // the norm prologue of the counter kernel: one token, K <= 4096 (four float4s per thread), X contiguous
    if (pro && (T != 1 || K % 1024 != 0 || K > 4096 || !ggml_is_contiguous(X))) return MOE_RNONE;
    const size_t lds = 2 * K * sizeof(float);
    if (T <= exec_ctx::MOE_CNT && K % 4 == 0 && K <= 8192 && lds <= 64 * 1024 && X->nb[1] % 16 == 0 && W->nb[1] % 16 == 0 &&
        ((uintptr_t) X->data % 16) == 0 && ((uintptr_t) W->data % 16) == 0) return MOE_RMW;
    return pro ? MOE_RNONE : MOE_RPLAIN;
}

// the multi-workgroup router's arrival counters, allocated once per context (not during capture)
bool moe_router_counters(exec_ctx & ctx) {
    if (!ctx.moe_cnt && !ctx.capturing) {
        MI_CHECK(hipMalloc(&ctx.moe_cnt, exec_ctx::MOE_CNT * sizeof(int)));
        MI_CHECK(hipMemsetAsync(ctx.moe_cnt, 0, exec_ctx::MOE_CNT * sizeof(int), ctx.stream));
    }
    return ctx.moe_cnt != nullptr;
}

bool moe_router(exec_ctx & ctx, ggml_tensor * mm, const ggml_tensor * sm, ggml_tensor * as, int n_used, float * wscr,
                const moe_router_pro * pro) {
    const ggml_tensor * W = mm->src[0], * X = mm->src[1];
    const int64_t n = W->ne[1], K = W->ne[0], T = X->ne[1];
    if (W->type != GGML_TYPE_F32 || X->type != GGML_TYPE_F32 || n > 16 || n < 1 || W->ne[2] != 1 || W->ne[3] != 1 ||
        X->ne[2] != 1 || X->ne[3] != 1 || X->nb[0] != 4 || W->nb[0] != 4 || mm->nb[0] != 4 || mm->ne[1] != T) return false;
    if (!ggml_is_contiguous(sm) || sm->src[0] != mm || !ggml_is_contiguous(as) || as->ne[0] != n || ggml_nrows(as) != T ||
        sm->ne[0] != n || ggml_nrows(sm) != T) return false;
    moe_router_args a = {};
    a.W = (const char *) W->data; a.nb01 = W->nb[1]; a.K = K;
    a.X = (const char *) X->data; a.nb11 = X->nb[1];
    a.logits = (char *) mm->data; a.nb_lo = mm->nb[1];
    moe_route_args & r = a.r;
    r.probs = (char *) sm->data; r.nb_p = sm->nb[1];
    r.order = (char *) as->data; r.nb_o = as->nb[1];
    r.n_exp = (int) n; r.T = T; r.stage = 1;
    memcpy(&r.scale, sm->op_params, sizeof(float));
    if (wscr) {
        r.stage = 3; r.n_used = n_used;
        r.w = (char *) wscr; r.nb_w = n_used * sizeof(float);
        r.wsum = (char *) (wscr + T * n_used); r.nb_s = n_used * sizeof(float);
        r.wn = (char *) (wscr + 2 * T * n_used); r.nb_n = n_used * sizeof(float);
    }
    // the tinyBLAS order for >= 2 columns, as mul_mat_vec picks it
    const bool tiny = T >= 2 && K % 16 == 0 && n % 4 == 0 && ggml_is_contiguous(X);
    int path = moe_router_path(mm, pro != nullptr);
    if (path == MOE_RMW && !moe_router_counters(ctx)) path = pro ? MOE_RNONE : MOE_RPLAIN;
    if (path == MOE_RNONE) return false;
    if (pro) {
        a.px = pro->x; a.pw = pro->w; a.eps = pro->eps;
        if (pro->q) { a.qs = pro->q->qs; a.qd = pro->q->d; a.qsum = pro->q->s; }
    }
    if (path == MOE_R1) {
        a.kt = ctx.kt_take("moe_router", 1, (unsigned) (64 * n));
        hipLaunchKernelGGL(k_moe_router1<64>, dim3(1), dim3((unsigned) (64 * n)), 0, ctx.stream, a);
        return true;
    }
    if (path == MOE_RMW) {
        const size_t lds = 2 * K * sizeof(float);
        const dim3 grid((unsigned) n, (unsigned) T);
        a.kt = T == 1 ? ctx.kt_take("moe_router", (unsigned) n, 256) : nullptr;
        if (tiny) hipLaunchKernelGGL(k_moe_router_mw<true>, grid, dim3(256), lds, ctx.stream, a, ctx.moe_cnt);
        else hipLaunchKernelGGL(k_moe_router_mw<false>, grid, dim3(256), lds, ctx.stream, a, ctx.moe_cnt);
        return true;
    }
    // the per-token kernel ignores the prologue's sources: never reached with pro (moe_router_path)
    GGML_ASSERT(!pro);
    const dim3 block((unsigned) (64 * n));
    if (tiny) hipLaunchKernelGGL(k_moe_router<true>, dim3((unsigned) T), block, 0, ctx.stream, a);
    else hipLaunchKernelGGL(k_moe_router<false>, dim3((unsigned) T), block, 0, ctx.stream, a);
    return true;
}

// stage 1 (at the SOFT_MAX): probabilities and their descending order; as = the ARGSORT node
bool moe_route_sort(exec_ctx & ctx, const ggml_tensor * sm, ggml_tensor * as) {
    const int64_t n = sm->ne[0], T = ggml_nrows(sm);
    if (n > 256 || !ggml_is_contiguous(sm) || !ggml_is_contiguous(sm->src[0]) || !ggml_is_contiguous(as) ||
        as->ne[0] != n || ggml_nrows(as) != T) return false;
    moe_route_args a = {};
    a.logits = (const char *) sm->src[0]->data; a.nb_l = sm->src[0]->nb[1];
    a.probs = (char *) sm->data; a.nb_p = sm->nb[1];
    a.order = (char *) as->data; a.nb_o = as->nb[1];
    a.n_exp = (int) n; a.T = T; a.stage = 1;
    memcpy(&a.scale, sm->op_params, sizeof(float));
    hipLaunchKernelGGL(k_moe_route, dim3((unsigned) ceil_div(T, 64)), dim3(64), 0, ctx.stream, a);
    return true;
}

// stage 2 (at the GET_ROWS): the routed experts' probabilities, their sum and the normalised
// weights; probabilities and order as stage 1 (or the stand-alone kernels) stored them
bool moe_route_weights(exec_ctx & ctx, ggml_tensor * gr, ggml_tensor * sr, ggml_tensor * dv) {
    const ggml_tensor * pr = gr->src[0];   // [1, n_exp, T] view of the probabilities
    const ggml_tensor * ids = gr->src[1];  // [n_used, T] view of the order
    const int64_t n = pr->ne[1], T = pr->ne[2], n_used = ids->ne[0];
    if (n > 256 || n_used > n || ids->ne[1] != T || pr->nb[1] != sizeof(float) || ids->nb[0] != sizeof(int32_t)) return false;
    if (gr->ne[0] != 1 || gr->ne[1] != n_used || gr->ne[2] != T || !ggml_is_contiguous(gr)) return false;
    if (!sr || !dv || sr->src[0]->data != gr->data || ggml_nelements(sr) != T || !ggml_is_contiguous(sr)) return false;
    if (dv->src[1] != sr || dv->src[0]->data != gr->data || ggml_nelements(dv) != T * n_used || !ggml_is_contiguous(dv)) return false;
    moe_route_args a = {};
    a.probs = (char *) pr->data; a.nb_p = pr->nb[2];
    a.order = (char *) ids->data; a.nb_o = ids->nb[1];
    a.w = (char *) gr->data; a.nb_w = gr->nb[2];
    a.wsum = (char *) sr->data; a.nb_s = sizeof(float);
    a.wn = (char *) dv->data; a.nb_n = sizeof(float) * n_used;
    a.n_exp = (int) n; a.n_used = (int) n_used; a.T = T; a.stage = 2;
    hipLaunchKernelGGL(k_moe_route, dim3((unsigned) ceil_div(T, 64)), dim3(64), 0, ctx.stream, a);
    return true;
}

// MoE output: MUL(experts [ne0, 2, T], weights [1, 2, T]) then ADD of its two slot views, with
// the unfused arithmetic (m_k = e_k * w_k rounded, then m_0 + m_1); one element per lane
__global__ __launch_bounds__(256) void k_moe_combine(const char * __restrict__ e, int64_t nb_e1, int64_t nb_e2,
                                                     const char * __restrict__ w, int64_t nb_w1, int64_t nb_w2,
                                                     char * __restrict__ out, int64_t nb_o1, int64_t ne0) {
    const int64_t t = blockIdx.y;
    const int64_t i = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ne0) return;
    const float w0 = *(const float *) (w + t * nb_w2), w1 = *(const float *) (w + nb_w1 + t * nb_w2);
    const float m0 = __fmul_rn(((const float *) (e + t * nb_e2))[i], w0);
    const float m1 = __fmul_rn(((const float *) (e + nb_e1 + t * nb_e2))[i], w1);
    ((float *) (out + t * nb_o1))[i] = __fadd_rn(m0, m1);
}

void moe_combine(exec_ctx & ctx, const ggml_tensor * mul, ggml_tensor * add, const float * wscr) {
    const ggml_tensor * e = mul->src[0], * w = mul->src[1];
    const dim3 grid((unsigned) ceil_div(mul->ne[0], 256), (unsigned) mul->ne[2]);
    // wscr: the router's private copy of the normalised weights ([T][2], k_moe_router)
    const char * wp = wscr ? (const char *) wscr : (const char *) w->data;
    const int64_t nbw1 = wscr ? (int64_t) sizeof(float) : (int64_t) w->nb[1];
    const int64_t nbw2 = wscr ? (int64_t) (2 * sizeof(float)) : (int64_t) w->nb[2];
    hipLaunchKernelGGL(k_moe_combine, grid, dim3(256), 0, ctx.stream, (const char *) e->data, (int64_t) e->nb[1],
                       (int64_t) e->nb[2], wp, nbw1, nbw2, (char *) add->data, (int64_t) add->nb[1], mul->ne[0]);
}

}  // namespace mi355x
