// k_mmv.hip — activation quantization and the general quantized / float mat-vec.
//
// Parity design: the CPU backend never multiplies quantized weights with f32 activations.
// It first quantizes each activation row to the weight type's vec_dot_type
// (ggml-cpu/ggml-cpu.c:193-282, quantize loop ggml-cpu.c:1254-1289):
//   * K-quants (Q4_K/Q5_K/Q6_K) -> Q8_K  : quantize_row_q8_K_ref  (ggml-quants.c:2471-2508)
//   * Q4_0/Q8_0                 -> Q8_0  : x86 quantize_row_q8_0 (ggml-cpu/arch/x86/quants.c:278-372)
// then takes integer dot products per block and combines them in a fixed fp32 order.  The
// quantizers here are bit-exact, and the combination follows the CPU's order exactly
// (qtypes.h), so every output equals the reference's bit for bit.
#include "ops.h"
#include "quant_act.h"
#include "qtypes.h"

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
    if (debug_ops()) fprintf(stderr, "[ops]   quantize %s %s K=%lld cols=%lld\n", k_quant ? "q8_K" : "q8_0", src->name, (long long) K, (long long) ncols);
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
// General quantized mat-vec in the CPU's exact order (qtypes.h): any shape, 1..8 columns per
// weight pass.  One wave owns one weight row (four rows per workgroup); per pass of 64 tasks
// each lane fetches its weight slice once and forms the integer records of every column of the
// workgroup into the wave's LDS region; the walker lanes (LPR per column) then run the CPU's
// fp32 chain.  Three column sources:
//   KIND 0  plain MUL_MAT: columns c0.. of batch (i12, i13) (ggml-cpu.c:1192-1384 broadcast
//           rules r2 / r3); Q4_K repacked: columns i11 < ne11 - ne11 % 4 take the gemm order
//           (repack.cpp:1261-1274), the rest the gemv order;
//   KIND 1  MUL_MAT_ID, one (slot, token) pair per workgroup row: the expert read from ids on
//           the device (the reference's CUDA path copies ids to the host,
//           ggml-cuda.cu:2061-2084);
//   KIND 2  MUL_MAT_ID over expert-sorted pairs (k_moe_sort): workgroup z = expert, columns =
//           that expert's pairs; workgroups past its pair count exit at once.
// MUL_MAT_ID follows ggml_compute_forward_mul_mat_id (ggml-cpu.c:1466) / the repack
// forward_mul_mat_id (repack.cpp:1277-1405, one gemv per pair).
// ------------------------------------------------------------------------------------------
struct mmx_args {
    const uint8_t * W; int64_t nb01, nb02, nb03; int64_t M; int ntasks; int nb;
    gemv_act A; int64_t qs_st, d_st, s_st;   // per-column strides (elements)
    int64_t ne11, ne12, r2, r3;
    float * dst; int64_t nb1, nb2, nb3;      // bytes
    int64_t gemm_cols;                        // KIND 0, Q4_K repacked: columns below this take R2
    const char * ids; int64_t ids_nb0, ids_nb1; int64_t n_used, n_as, id_ne11;
    const int32_t * cnt; const int32_t * off; const int32_t * list;
};

template <class T, int NC, int KIND>
__global__ __launch_bounds__(256) void k_mmx(const mmx_args p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row = (int64_t) blockIdx.x * 4 + wave;
    const bool rowok = row < p.M;
    const uint8_t * wbase;
    int nc = NC;
    int64_t c0 = 0, pos0 = 0, e1 = 0, t1 = 0, i12 = 0, i13 = 0;
    if constexpr (KIND == 0) {
        i12 = blockIdx.z % p.ne12; i13 = blockIdx.z / p.ne12;
        c0 = (int64_t) blockIdx.y * NC;
        nc = (int) min((int64_t) NC, p.ne11 - c0);
        wbase = p.W + (i12 / p.r2) * p.nb02 + (i13 / p.r3) * p.nb03;
    } else if constexpr (KIND == 1) {
        e1 = blockIdx.y % p.n_used; t1 = blockIdx.y / p.n_used;
        const int32_t ex = *(const int32_t *) (p.ids + e1 * p.ids_nb0 + t1 * p.ids_nb1);
        if (ex < 0 || ex >= p.n_as) return;   // uniform over the workgroup
        nc = 1;
        wbase = p.W + (int64_t) ex * p.nb02;
    } else {
        const int ex = blockIdx.z;
        const int n = p.cnt[ex];
        c0 = (int64_t) blockIdx.y * NC;
        if (c0 >= n) return;   // uniform over the workgroup, before any barrier
        nc = (int) min((int64_t) NC, n - c0);
        pos0 = p.off[ex] + c0;
        wbase = p.W + (int64_t) ex * p.nb02;
    }
    auto col_of = [&](int c) -> int64_t {   // activation column of the c-th column
        if constexpr (KIND == 0) return c0 + c + p.ne11 * (i12 + p.ne12 * i13);
        else if constexpr (KIND == 1) return e1 % p.id_ne11 + p.id_ne11 * t1;
        else return pos0 + c;
    };
    const uint8_t * wrow = wbase + (rowok ? row : p.M - 1) * p.nb01;
    uint32_t * xw = xr + (size_t) wave * NC * p.nb * T::RS;
    for (int t0 = 0; t0 < p.ntasks; t0 += WAVE) {
        const int t = t0 + lane;
        const bool active = t < p.ntasks;
        const int tt = active ? t : 0;
        typename T::raw w;
        T::fetch(wrow, tt, w);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= nc) break;
            const int64_t col = col_of(c);
            const gemv_act A = {p.A.qs + col * p.qs_st, p.A.d + col * p.d_st, p.A.s + col * p.s_st};
            typename T::act x;
            T::load(A, tt, x);
            T::rec(w, tt, x, active, xw + (size_t) c * p.nb * T::RS);
        }
    }
    wave_lds_sync();
    const int cw = lane / T::LPR, ws = lane % T::LPR;
    const int cwc = cw < nc ? cw : 0;
    float v;
    if constexpr (std::is_same<T, g_q4_K_p>::value) {
        v = T::walk_m(xw + (size_t) cwc * p.nb * T::RS, p.nb, KIND == 0 && c0 + cwc < p.gemm_cols);
    } else {
        v = T::walk(xw + (size_t) cwc * p.nb * T::RS, p.nb, ws);
    }
    if (!rowok || cw >= nc || ws != 0) return;
    char * d;
    if constexpr (KIND == 0) {
        d = (char *) p.dst + i12 * p.nb2 + i13 * p.nb3 + (c0 + cw) * p.nb1;
    } else if constexpr (KIND == 1) {
        d = (char *) p.dst + e1 * p.nb1 + t1 * p.nb2;
    } else {
        const int pair = p.list[pos0 + cw];
        d = (char *) p.dst + (pair % p.n_used) * p.nb1 + (pair / p.n_used) * p.nb2;
    }
    *(float *) (d + row * 4) = v;
}

// LDS bytes of one k_mmx workgroup: four waves x NC columns x nb records
template <class T>
static size_t mmx_lds(int nc, int64_t nb) { return (size_t) 4 * nc * nb * T::RS * 4; }

// columns per weight pass: the most (<= 8, <= the columns there are) whose records fit 64 KiB
template <class T>
static int mmx_nc(int64_t ncols, int64_t nb) {
    int nc = 8;
    while (nc > 1 && (nc / 2 >= ncols || mmx_lds<T>(nc, nb) > 64 * 1024)) nc /= 2;
    GGML_ASSERT(mmx_lds<T>(nc, nb) <= 64 * 1024 && "mi355x: mat-vec records exceed LDS");
    return nc;
}

template <class T, int KIND>
static void launch_mmx_nc(hipStream_t st, const mmx_args & a, int nc, dim3 grid) {
    const size_t lds = mmx_lds<T>(nc, a.nb);
    switch (nc) {
        case 1: hipLaunchKernelGGL((k_mmx<T, 1, KIND>), grid, dim3(256), lds, st, a); break;
        case 2: hipLaunchKernelGGL((k_mmx<T, 2, KIND>), grid, dim3(256), lds, st, a); break;
        case 4: hipLaunchKernelGGL((k_mmx<T, 4, KIND>), grid, dim3(256), lds, st, a); break;
        default: hipLaunchKernelGGL((k_mmx<T, 8, KIND>), grid, dim3(256), lds, st, a); break;
    }
}

// KIND 0 over ne11 columns x nbatch batches; KIND 1 over n_pairs; KIND 2 over n_pairs sorted
template <class T>
static void launch_mmx(hipStream_t st, mmx_args & a, int kind, int64_t ncols, int64_t nbatch) {
    a.ntasks = (int) (a.nb * T::per_block);
    const unsigned gx = (unsigned) ceil_div(a.M, 4);
    if (kind == 1) {
        launch_mmx_nc<T, 1>(st, a, 1, dim3(gx, (unsigned) ncols));
        return;
    }
    const int nc = mmx_nc<T>(kind == 0 ? ncols : 8, a.nb);
    if (kind == 0) launch_mmx_nc<T, 0>(st, a, nc, dim3(gx, (unsigned) ceil_div(ncols, nc), (unsigned) nbatch));
    else launch_mmx_nc<T, 2>(st, a, nc, dim3(gx, (unsigned) ceil_div(ncols, nc), (unsigned) a.n_as));
}

// the weight type's CPU order (qtypes.h): repacked Q4_K / Q4_0 when M % 8 == 0
static void launch_mmx_type(hipStream_t st, ggml_type t, mmx_args & a, int kind, int64_t ncols, int64_t nbatch) {
    const bool rep = a.M % 8 == 0;
    switch (t) {
        case GGML_TYPE_Q4_K:
            if (rep) launch_mmx<g_q4_K_p>(st, a, kind, ncols, nbatch);
            else launch_mmx<g_q4_K_c>(st, a, kind, ncols, nbatch);
            break;
        case GGML_TYPE_Q4_0:
            if (rep) launch_mmx<g_q4_0>(st, a, kind, ncols, nbatch);
            else launch_mmx<g_q4_0_c>(st, a, kind, ncols, nbatch);
            break;
        case GGML_TYPE_Q5_K: launch_mmx<g_q5_K>(st, a, kind, ncols, nbatch); break;
        case GGML_TYPE_Q6_K: launch_mmx<g_q6_K>(st, a, kind, ncols, nbatch); break;
        case GGML_TYPE_Q8_0: launch_mmx<g_q8_0>(st, a, kind, ncols, nbatch); break;
        default: GGML_ABORT("mi355x: unsupported mat-vec type");
    }
}

// ------------------------------------------------------------------------------------------
// f16 / f32 weights, CPU-exact order.  The CPU converts src1 to the weight's vec_dot_type (f16
// for f16 weights).  One column (T = 1) or a shape llamafile declines: ggml_vec_dot_f16 /
// ggml_vec_dot_f32 (vec.cpp:191-231, AVX-512: 4 accumulators x 16 lanes, REDUCE,
// _mm512_reduce_add_ps, double leftovers).  Two or more columns with K % 16 == 0 and
// M % 4 == 0: llamafile tinyBLAS<16, __m512> (llamafile/sgemm.cpp:331-427, 3334-3342,
// 3421-3428): one 16-lane FMA chain per output over K in steps of 16, then
// _mm512_reduce_add_ps.  Used by the FA-off KQ / KQV products and f32 / f16 weight matrices
// (the MoE router).
// ------------------------------------------------------------------------------------------
struct mmv_f_args {
    const char * W; int64_t nb01, nb02, nb03; int64_t M; int64_t K;
    const char * X; int64_t nb11, nb12, nb13; int64_t ne11, ne12, r2, r3;
    float * dst; int64_t nb1, nb2, nb3;
};

template <typename WT, bool TINY>
__global__ __launch_bounds__(256) void k_mmv_f_exact(const mmv_f_args p) {
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
    char * out = (char *) p.dst + i12 * p.nb2 + i13 * p.nb3 + c * p.nb1 + row * 4;
    if constexpr (TINY) {
        // lanes 0..15 hold the CPU's 16 accumulators: lane s walks k = s, s + 16, ...; the
        // xor butterfly over 8 / 4 / 2 / 1 is the _mm512_reduce_add_ps tree
        float acc = 0.0f;
        const int s = lane & 15;
        if (lane < 16) {
#pragma unroll 8
            for (int64_t k = 0; k < p.K; k += 16) acc = fmaf(wv(k + s), xv(k + s), acc);
        }
        acc = __fadd_rn(acc, __shfl_xor(acc, 8, WAVE));
        acc = __fadd_rn(acc, __shfl_xor(acc, 4, WAVE));
        acc = __fadd_rn(acc, __shfl_xor(acc, 2, WAVE));
        acc = __fadd_rn(acc, __shfl_xor(acc, 1, WAVE));
        if (ok && lane == 0) *(float *) out = acc;
        return;
    }
    // one wave per row: lane s keeps the AVX-512 partial acc[s] of ggml_vec_dot_f32 (4
    // accumulators x 16 lanes, FMA'd over the row in steps of 64), so the loads are coalesced
    // 256-B rows and the sum order is the CPU's; lane 0 then forms REDUCE + the
    // _mm512_reduce_add_ps tree and the scalar tail in double
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
        *(float *) out = (float) sumf;
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

// mat-vec entry: quantized or float weights, any number of columns
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
        mmx_args a = {};
        a.W = (const uint8_t *) src0->data;
        a.nb01 = src0->nb[1]; a.nb02 = src0->nb[2]; a.nb03 = src0->nb[3];
        a.M = src0->ne[1];
        a.nb = (int) (src0->ne[0] / ggml_blck_size(src0->type));
        a.A = {act.qs, act.d, act.s};
        a.qs_st = act.qs_stride(); a.d_st = act.d_stride(); a.s_st = act.s_stride();
        a.ne11 = src1->ne[1]; a.ne12 = src1->ne[2];
        a.r2 = src1->ne[2] / src0->ne[2]; a.r3 = src1->ne[3] / src0->ne[3];
        a.dst = (float *) dst->data; a.nb1 = dst->nb[1]; a.nb2 = dst->nb[2]; a.nb3 = dst->nb[3];
        a.gemm_cols = a.ne11 > 3 ? a.ne11 - a.ne11 % 4 : 0;
        launch_mmx_type(ctx.stream, src0->type, a, 0, a.ne11, nbatch);
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
        // llamafile_sgemm (ggml-cpu.c:1227-1320) services src1 with >= 2 columns, contiguous
        // rows, K % 16 == 0 and M % 4 == 0 (tinyBLAS::matmul, sgemm.cpp:341-360)
        const bool tiny = a.ne11 >= 2 && a.K % 16 == 0 && a.M % 4 == 0 && ggml_is_contiguous(src1);
        dim3 grid((unsigned) ceil_div(a.M, 4), (unsigned) a.ne11, (unsigned) nbatch);
        if (src0->type == GGML_TYPE_F16) {
            if (tiny) hipLaunchKernelGGL((k_mmv_f_exact<uint16_t, true>), grid, dim3(256), 0, ctx.stream, a);
            else hipLaunchKernelGGL((k_mmv_f_exact<uint16_t, false>), grid, dim3(256), 0, ctx.stream, a);
        } else {
            if (tiny) hipLaunchKernelGGL((k_mmv_f_exact<float, true>), grid, dim3(256), 0, ctx.stream, a);
            else hipLaunchKernelGGL((k_mmv_f_exact<float, false>), grid, dim3(256), 0, ctx.stream, a);
        }
    }
    if (ctx.timing) ctx.time_end(TK_MMV, bytes, ev_beg);
}

// ------------------------------------------------------------------------------------------
// MUL_MAT_ID (ggml-cpu/ggml-cpu.c:1466 ggml_compute_forward_mul_mat_id; graph use in
// build_moe_ffn, src/llama-graph.cpp:727-758): for token t and slot e < n_used,
//   dst[:, e, t] = as[ids[e, t]] . b[:, e % ne11, t]
// with the per-row arithmetic of the mat-vec above (same quantized activation, same order).
//   * few (slot, token) pairs (decode): one mat-vec per pair, the expert read from ids by the
//     kernel (k_mmx KIND 1);
//   * many pairs (prefill): a one-workgroup counting sort groups the pairs by expert
//     (k_moe_sort), the activations are quantized straight into that order
//     (k_quant_gather), and each expert's rows are streamed once per 8 of its pairs
//     (k_mmx KIND 2) or, with enough pairs, by the int8 MFMA tile (k_mmq.hip).
// ------------------------------------------------------------------------------------------
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

bool mmq_id_supported(const ggml_tensor * dst);
void mul_mat_q_id(exec_ctx & ctx, ggml_tensor * dst, const q8_act & act, const int32_t * cnt, const int32_t * off,
                  const int32_t * list, int64_t n_pairs);
bool gemv_mmid(exec_ctx & ctx, ggml_tensor * dst, const q8_act & act, ggml_tensor * dst2 = nullptr);

// the gate and up projections of the same routed slots of one token (dst, dst2: same input and
// ids) as one launch of the one-shot ID instance; false: nothing was launched
bool op_mul_mat_id_pair(exec_ctx & ctx, ggml_tensor * dst, ggml_tensor * dst2) {
    const ggml_tensor * as = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const ggml_tensor * ids = dst->src[2];
    if (ids->ne[1] != 1 || ids->ne[0] > 8 || dst2->src[1] != b || dst2->src[2] != ids) return false;
    const bool kq = is_k_quant(as->type);
    hipEvent_t ev_beg = nullptr;
    const double bytes = 2.0 * ((double) as->nb[2] * (double) std::min<int64_t>(ids->ne[0], as->ne[2]) + (double) ggml_nbytes(dst)) +
                         (double) ggml_nelements(b) * (kq ? 1.14 : 1.0);
    q8_act act;
    if (!ctx.qcache_get(b, kq, act)) {
        quantize_act(ctx, b, kq, act, exec_ctx::QSLOT);
        ctx.qcache_put(b, kq, act);
    }
    if (ctx.timing) ctx.time_begin(TK_MMV, bytes, ev_beg);
    const bool ok = gemv_mmid(ctx, dst, act, dst2);
    // declined: the caller's op_mul_mat_id times the same work, so no sample here
    if (ctx.timing) {
        if (ok) ctx.time_end(TK_MMV, bytes, ev_beg);
        else ctx.time_cancel(ev_beg);
    }
    return ok;
}

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

    mmx_args a = {};
    a.W = (const uint8_t *) as->data;
    a.nb01 = as->nb[1]; a.nb02 = as->nb[2];
    a.M = as->ne[1];
    a.nb = (int) (K / ggml_blck_size(as->type));
    a.n_as = n_as;
    a.ids = (const char *) ids->data; a.ids_nb0 = ids->nb[0]; a.ids_nb1 = ids->nb[1];
    a.n_used = n_used; a.id_ne11 = b->ne[1];
    a.dst = (float *) dst->data; a.nb1 = dst->nb[1]; a.nb2 = dst->nb[2];

    const bool grouped = n_pairs > 8;
    q8_act act;
    if (!grouped) {
        if (!ctx.qcache_get(b, kq, act)) {
            quantize_act(ctx, b, kq, act, exec_ctx::QSLOT);
            ctx.qcache_put(b, kq, act);
        }
        // one token: the routed experts as one one-shot launch (k_gemv.hip, its ID instance)
        if (T == 1 && gemv_mmid(ctx, dst, act)) {
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
    a.A = {act.qs, act.d, act.s};
    a.qs_st = act.qs_stride(); a.d_st = act.d_stride(); a.s_st = act.s_stride();
    launch_mmx_type(ctx.stream, as->type, a, grouped ? 2 : 1, n_pairs, 1);
    if (ctx.timing) ctx.time_end(TK_MMV, bytes, ev_beg);
}

}  // namespace mi355x
