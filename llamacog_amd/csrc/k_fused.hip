// k_fused.hip — fused producers of the decode graph.  Each replaces a chain of ggml nodes
// with ONE kernel that writes every node's output exactly as the unfused kernels would
// (same per-element arithmetic, same reduction), plus the quantized activation of the
// MUL_MAT that consumes the chain (into exec_ctx's quantization cache), so the MUL_MAT does
// not launch its own quantizer:
//
//   [ADD] -> RMS_NORM -> [MUL w] -> (MUL_MAT)     k_norm_fused   (src/llama-graph.cpp:464-497
//                                                 build_norm; residual ADDs :llama.cpp build)
//   MUL (silu(gate) * up) -> (MUL_MAT down)       k_mul_quant    (build_ffn LLM_FFN_PAR)
//
// Arithmetic: ADD/MUL are single f32 ops; RMS_NORM's mean is the CPU's sequential double sum
// of float(x*x) (ops.cpp:3270-3316, quant_act.h rms_mean_decided), scale =
// 1/sqrtf(mean+eps), y = x*scale; quantizers are quant_act.h's (bit-exact with the CPU's).
// All run with rows in registers.
#include "ops.h"
#include "quant_act.h"

namespace mi355x {

struct norm_fused_args {
    const float * a; const float * b;   // x = a (+ b)
    float * xsum;                       // ADD output (nullable)
    float * y;                          // RMS_NORM output
    const float * w; float * yw;        // MUL weight / output (nullable)
    int64_t ne0;
    float eps;
    int qmode;                          // 0 none, 1 Q8_K, 2 Q8_0 (of yw if w else y), 3 both
    int8_t * qs; float * qd; int16_t * qsum;
    int8_t * qs0; float * qd0; int16_t * qsum0;   // qmode 3: the Q8_0 one
    int64_t nrows;
    // MoE combine source instead of a: x = (e[., 0, row] * cw[row, 0] + e[., 1, row] * cw[row, 1]) + b
    const float * e; const float * cw; int nu;
    unsigned long long * kt;            // in-graph kernel timeline region (nullable)
    unsigned kt_stride;                 // its slots per workgroup (1 + threads / 64)
};

// one workgroup of BT threads per row; thread t owns the float4s at element 4 (t + BT k), k < NV,
// so wave w's 256 elements of slice k are one Q8_K block / eight Q8_0 blocks of the quantized
// output.  The mean is the CPU's sequential one (quant_act.h rms_mean_decided).
template <int NV>
__global__ __launch_bounds__(1024) void k_norm_fused(const norm_fused_args p) {
    kt_enter(p.kt, p.kt_stride);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int BT = blockDim.x, NW = BT >> 6;
    const int64_t row = blockIdx.x;
    const int64_t ro = row * p.ne0;
    __shared__ double wpart[16];
    __shared__ float smean;
    float4 v[NV], wv[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        // the norm weight is loaded with the row, not after the reduction
        if (p.w) wv[k] = *(const float4 *) (p.w + 4 * (tid + BT * k));
    }
    double acc = 0.0;
    const float * e0 = p.e ? p.e + 2 * ro : nullptr, * e1 = p.e ? e0 + p.ne0 : nullptr;
    const float cw0 = p.e ? p.cw[row * p.nu] : 0.0f, cw1 = p.e ? p.cw[row * p.nu + 1] : 0.0f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int64_t e = 4 * (tid + BT * k);
        if (p.e) {
            const float4 x0 = *(const float4 *) (e0 + e), x1 = *(const float4 *) (e1 + e);
            v[k].x = __fadd_rn(__fmul_rn(x0.x, cw0), __fmul_rn(x1.x, cw1));
            v[k].y = __fadd_rn(__fmul_rn(x0.y, cw0), __fmul_rn(x1.y, cw1));
            v[k].z = __fadd_rn(__fmul_rn(x0.z, cw0), __fmul_rn(x1.z, cw1));
            v[k].w = __fadd_rn(__fmul_rn(x0.w, cw0), __fmul_rn(x1.w, cw1));
        } else {
            v[k] = *(const float4 *) (p.a + ro + e);
        }
        if (p.b) {
            const float4 bb = *(const float4 *) (p.b + ro + e);
            v[k].x = __fadd_rn(v[k].x, bb.x); v[k].y = __fadd_rn(v[k].y, bb.y);
            v[k].z = __fadd_rn(v[k].z, bb.z); v[k].w = __fadd_rn(v[k].w, bb.w);
        }
        acc = __dadd_rn(acc, sq4(v[k]));
    }
    // (DPP sums in any order — the mean is decided against the CPU's sequential one below; the
    // shuffle trees were ds_bpermute round trips on the path to every consumer of the norm)
    acc = wave_sum_rows_f64(acc);
    if (lane == 0) wpart[wave] = acc;
    __syncthreads();
    if (wave == 0) {
        double t = lane < NW ? wpart[lane] : 0.0;
        t = row_sum16_f64(t);
        if (lane == 0) {
            float mean;
            if (!rms_mean_decided(t, p.ne0, mean))
                mean = p.e ? rms_mean_sequential_moe(e0, e1, cw0, cw1, p.b + ro, p.ne0)
                           : rms_mean_sequential(p.a + ro, p.b ? p.b + ro : nullptr, p.ne0);
            smean = mean;
        }
    }
    __syncthreads();
    // the ADD output is stored only now: the sequential replay above reads a and b, and the
    // ADD may be in place over one of them
    if (p.xsum) {
#pragma unroll
        for (int k = 0; k < NV; ++k) *(float4 *) (p.xsum + ro + 4 * (tid + BT * k)) = v[k];
    }
    const float scale = 1.0f / sqrtf(smean + p.eps);

#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int64_t e = 4 * (tid + BT * k);
        float4 y;
        y.x = __fmul_rn(v[k].x, scale); y.y = __fmul_rn(v[k].y, scale);
        y.z = __fmul_rn(v[k].z, scale); y.w = __fmul_rn(v[k].w, scale);
        if (p.y) *(float4 *) (p.y + ro + e) = y;
        if (p.w) {
            const float4 ww = wv[k];
            y.x = __fmul_rn(y.x, ww.x); y.y = __fmul_rn(y.y, ww.y);
            y.z = __fmul_rn(y.z, ww.z); y.w = __fmul_rn(y.w, ww.w);
            if (p.yw) *(float4 *) (p.yw + ro + e) = y;
        }
        const float q[4] = {y.x, y.y, y.z, y.w};
        const int64_t c0 = 4 * (int64_t) BT * k + 256 * wave;
        if (p.qmode & 1) {
            q8K_wave(q, lane, p.qs + ro + c0, p.qsum + row * (p.ne0 / 16) + c0 / 16, p.qd + row * (p.ne0 / 256) + c0 / 256);
        }
        if (p.qmode == 2) {
            q8_0_wave(q, lane, true, p.qs + ro + c0, p.qd + row * (p.ne0 / 32) + c0 / 32, p.qsum + row * (p.ne0 / 32) + c0 / 32);
        } else if (p.qmode == 3) {
            q8_0_wave(q, lane, true, p.qs0 + ro + c0, p.qd0 + row * (p.ne0 / 32) + c0 / 32, p.qsum0 + row * (p.ne0 / 32) + c0 / 32);
        }
    }
    kt_exit(p.kt, p.kt_stride);
}

// dst = a*b (same shape, contiguous) and its quantization; one wave per 256 elements.
// SILU: a is the gate projection and the kernel first forms s = silu(a) — the UNARY node
// before the MUL, ggml_vec_silu_f32's arithmetic (vec.cpp:233: AVX-512 ggml_v_silu on
// 16-element chunks of the row, x/(1+expf(-x)) on the tail) — storing it only when a later
// node reads it (sdst != nullptr).  dst == nullptr: the product is read by nothing but the
// quantized activation (QMODE 0 keeps no quantization and always stores).
template <int QMODE, bool SILU>
__global__ __launch_bounds__(64) void k_mul_quant(const float * __restrict__ a, const float * __restrict__ b,
                                                  float * __restrict__ dst, int64_t K,
                                                  int8_t * __restrict__ qs, float * __restrict__ qd,
                                                  int16_t * __restrict__ qsum, float * __restrict__ sdst,
                                                  unsigned long long * kt) {
    kt_enter(kt, 2);
    const int lane = threadIdx.x;
    const int64_t row = blockIdx.y;
    const int64_t nblk = (K + 255) / 256;
    const int64_t c0 = (int64_t) blockIdx.x * 256;
    const int64_t e0 = c0 + 4 * lane;
    const bool valid = e0 < K;
    float q[4] = {0.f, 0.f, 0.f, 0.f};
    if (valid) {
        float4 x = *(const float4 *) (a + row * K + e0);
        const float4 y = *(const float4 *) (b + row * K + e0);
        if constexpr (SILU) {
            const int64_t nvec = (K / 16) * 16;
            float v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                v[c] = e0 + c < nvec ? v[c] / (1.0f + v_expf_avx512(-v[c])) : v[c] / (1.0f + expf_cr(-v[c]));
            }
            x = make_float4(v[0], v[1], v[2], v[3]);
            if (sdst) *(float4 *) (sdst + row * K + e0) = x;
        }
        float4 r;
        r.x = __fmul_rn(x.x, y.x); r.y = __fmul_rn(x.y, y.y); r.z = __fmul_rn(x.z, y.z); r.w = __fmul_rn(x.w, y.w);
        if (dst) *(float4 *) (dst + row * K + e0) = r;
        q[0] = r.x; q[1] = r.y; q[2] = r.z; q[3] = r.w;
    }
    if constexpr (QMODE == 1) {
        q8K_wave(q, lane, qs + row * K + c0, qsum + row * (K / 16) + c0 / 16, qd + row * (K / 256) + c0 / 256);
    } else if constexpr (QMODE == 2) {
        q8_0_wave(q, lane, valid, qs + row * K + c0, qd + row * (K / 32) + c0 / 32, qsum + row * (K / 32) + c0 / 32);
    }
    kt_exit(kt, 2);
}

// ---- host side -------------------------------------------------------------------------------
static bool f32_contig(const ggml_tensor * t) { return t && t->type == GGML_TYPE_F32 && ggml_is_contiguous(t); }

bool mmv_q_supported_type(ggml_type t);

// vec_dot_type quantization wanted by a MUL_MAT consumer of `x` (0 = none / not fusable)
static int consumer_qmode(const ggml_tensor * mm, const ggml_tensor * x) {
    // MUL_MAT_ID: the decode path (<= 8 routed pairs) takes the cached activation as well
    if (!mm || (mm->op != GGML_OP_MUL_MAT && mm->op != GGML_OP_MUL_MAT_ID) || mm->src[1] != x) return 0;
    const ggml_type t = mm->src[0]->type;
    if (!mmv_q_supported_type(t)) return 0;
    split_parts sp;
    if (tensor_split_parts(mm->src[0], sp)) return 0;   // row-split weights read the f32 input
    // MUL_MAT_ID: the decode path only (batches gather their own quantization); a MUL_MAT of any
    // width reads the cache (mat-vec and MFMA prefill tiles alike)
    if (mm->op == GGML_OP_MUL_MAT_ID && mm->src[1]->ne[1] * mm->src[1]->ne[2] * mm->src[1]->ne[3] > 8) return 0;
    const bool kq = t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K;
    if (x->ne[0] % (kq ? 256 : 32) != 0) return 0;
    return kq ? 1 : 2;
}

bool fused_norm(exec_ctx & ctx, const ggml_tensor * add, ggml_tensor * norm, ggml_tensor * mul, const ggml_tensor * mm,
                bool store_norm, bool store_mul, const ggml_tensor * qkey, const ggml_tensor * mm0, const norm_combine * comb) {
    const int64_t ne0 = norm->ne[0];
    // ne0 <= 4096: one float4 per thread; above: whole 4096-element slices per 1024 threads
    if (ne0 % 256 != 0 || (ne0 > 4096 && ne0 % 4096 != 0) || ne0 > 16384) return false;
    if (!f32_contig(norm) || !f32_contig(norm->src[0])) return false;
    if (add && (!f32_contig(add->src[0]) || !f32_contig(add->src[1]) || !ggml_are_same_shape(add->src[0], add->src[1]) ||
                !ggml_are_same_shape(add, norm) || norm->src[0] != add)) return false;
    if (mul && (!f32_contig(mul) || !f32_contig(mul->src[1]) || ggml_nelements(mul->src[1]) != ne0)) return false;
    const ggml_tensor * out = mul ? mul : norm;
    const ggml_tensor * key = qkey ? qkey : out;
    const int64_t nrows = ggml_nrows(norm);
    // batches keep the stand-alone quantizer: one 1024-thread workgroup per row quantizing its 16
    // blocks ran pp512's norms at 20 us a launch against 7.3 + 6.8 us for norm + k_quantize_q8_K
    // (GGML_MI355X_NORM_BQ=1: quantize batches here too — with NORM_NV, a geometry probe)
    static const bool bq = getenv("GGML_MI355X_NORM_BQ") && atoi(getenv("GGML_MI355X_NORM_BQ")) != 0;
    int qmode = nrows <= 8 || bq ? consumer_qmode(mm, key) : 0;
    // mm0: a later Q8_0 consumer of the same output beside a K-quant first one
    const bool with0 = qmode == 1 && !qkey && consumer_qmode(mm0, out) == 2;

    norm_fused_args p;
    p.a = add ? (const float *) add->src[0]->data : (const float *) norm->src[0]->data;
    p.b = add ? (const float *) add->src[1]->data : nullptr;
    p.e = nullptr; p.cw = nullptr; p.nu = 0;
    if (comb) {
        // the combine's slot sum is one ADD operand (never stored); the other is the residual
        if (!add || (add->src[0] != comb->sum && add->src[1] != comb->sum) || comb->n_used != 2) return false;
        p.b = (const float *) (add->src[0] == comb->sum ? add->src[1] : add->src[0])->data;
        p.a = nullptr;
        p.e = comb->e; p.cw = comb->w; p.nu = comb->n_used;
    }
    p.xsum = add ? (float *) add->data : nullptr;
    p.w = mul ? (const float *) mul->src[1]->data : nullptr;
    // an output nothing reads is not stored; the last one is kept unless it is quantized here
    const bool last_needed = !qmode || (mul ? store_mul : store_norm);
    p.y = (mul ? store_norm : last_needed) ? (float *) norm->data : nullptr;
    p.yw = mul && last_needed ? (float *) mul->data : nullptr;
    p.ne0 = ne0;
    memcpy(&p.eps, norm->op_params, sizeof(float));
    p.qmode = qmode;
    q8_act act;
    if (qmode) {
        const bool kq = qmode == 1;
        void * base = ctx.scratch(exec_ctx::QSLOT, q8_act::bytes(ne0, nrows, kq));
        carve_act(act, base, ne0, nrows, kq);
        p.qs = act.qs; p.qd = act.d; p.qsum = act.s;
    } else {
        p.qs = nullptr; p.qd = nullptr; p.qsum = nullptr;
    }
    q8_act act0;
    p.qs0 = nullptr; p.qd0 = nullptr; p.qsum0 = nullptr;
    if (with0) {
        carve_act(act0, ctx.scratch(exec_ctx::QSLOT0, q8_act::bytes(ne0, nrows, false)), ne0, nrows, false);
        p.qs0 = act0.qs; p.qd0 = act0.d; p.qsum0 = act0.s;
        p.qmode = qmode = 3;
    }
    // up to 1024 threads per row, one float4 each (512 / 256 threads with several float4 each
    // measured no faster on Llama-3-8B decode, round 2); the canonical slice order j = w + NW k
    // is the same for every split, so the bits would not change
    int nv = ne0 <= 4096 ? 1 : (int) (ne0 / 4096);
    // GGML_MI355X_NORM_NV=<2,4>: batches (more than 8 rows) on ne0 / (4 nv)-thread workgroups, nv
    // float4s per thread (the canonical slice order j = w + NW k is the same, so are the bits)
    static const int nvb = getenv("GGML_MI355X_NORM_NV") ? atoi(getenv("GGML_MI355X_NORM_NV")) : 0;
    if (nrows > 8 && (nvb == 2 || nvb == 4) && ne0 % (1024 * nvb) == 0 && ne0 / (4 * nvb) >= 256) nv = nvb;
    const dim3 block((unsigned) (ne0 / (4 * nv)));
    p.nrows = nrows;
    const dim3 grid((unsigned) nrows);
    p.kt = nrows == 1 ? ctx.kt_take("norm_fused", 1, block.x) : nullptr;
    p.kt_stride = 1 + block.x / 64;
    switch (nv) {
        case 1: hipLaunchKernelGGL(k_norm_fused<1>, grid, block, 0, ctx.stream, p); break;
        case 2: hipLaunchKernelGGL(k_norm_fused<2>, grid, block, 0, ctx.stream, p); break;
        case 3: hipLaunchKernelGGL(k_norm_fused<3>, grid, block, 0, ctx.stream, p); break;
        default: hipLaunchKernelGGL(k_norm_fused<4>, grid, block, 0, ctx.stream, p); break;
    }
    if (qmode) ctx.qcache_put(key, qmode != 2, act);
    if (with0) {
        ctx.qc0_tensor = out; ctx.qc0_data = out->data; ctx.qc0_act = act0;
    }
    return true;
}

bool fused_mul_quant(exec_ctx & ctx, ggml_tensor * mul, const ggml_tensor * mm) {
    return fused_silu_mul_quant(ctx, nullptr, mul, mm, true);
}

// [SILU ->] MUL (a * b) -> quantized activation of the consuming MUL_MAT.  silu: the UNARY SILU
// node that is mul's src[0] (nullptr: mul alone); store_silu / store_mul: whether those outputs
// are read by any later node (dispatch.cpp dead_after), else only the quantization is kept.
bool fused_silu_mul_quant(exec_ctx & ctx, ggml_tensor * silu, ggml_tensor * mul, const ggml_tensor * mm, bool store_silu,
                          bool store_mul) {
    if (!f32_contig(mul) || !f32_contig(mul->src[0]) || !f32_contig(mul->src[1])) return false;
    if (!ggml_are_same_shape(mul->src[0], mul->src[1]) || !ggml_are_same_shape(mul, mul->src[0])) return false;
    if (silu && (mul->src[0] != silu || !f32_contig(silu->src[0]) || !ggml_are_same_shape(silu, silu->src[0]))) return false;
    const int qmode = consumer_qmode(mm, mul);
    if (mul->ne[0] % 4 != 0 || (!qmode && !silu)) return false;
    if (!qmode) store_mul = true;
    const int64_t K = mul->ne[0], nrows = ggml_nrows(mul);
    const bool kq = qmode == 1;
    q8_act act = {};
    if (qmode) carve_act(act, ctx.scratch(exec_ctx::QSLOT, q8_act::bytes(K, nrows, kq)), K, nrows, kq);
    const dim3 grid((unsigned) ceil_div(K, 256), (unsigned) nrows);
    const float * a = (const float *) (silu ? silu->src[0]->data : mul->src[0]->data);
    const float * b = (const float *) mul->src[1]->data;
    float * d = store_mul ? (float *) mul->data : nullptr;
    float * sd = silu && store_silu ? (float *) silu->data : nullptr;
    unsigned long long * kt = nrows == 1 ? ctx.kt_take("mul_quant", grid.x, 64) : nullptr;
#define MQ_LAUNCH(Q, S) hipLaunchKernelGGL((k_mul_quant<Q, S>), grid, dim3(64), 0, ctx.stream, a, b, d, K, act.qs, act.d, act.s, sd, kt)
    if (silu) {
        if (qmode == 1) MQ_LAUNCH(1, true); else if (qmode == 2) MQ_LAUNCH(2, true); else MQ_LAUNCH(0, true);
    } else {
        if (qmode == 1) MQ_LAUNCH(1, false); else MQ_LAUNCH(2, false);
    }
#undef MQ_LAUNCH
    if (qmode) ctx.qcache_put(mul, kq, act);
    return true;
}

}  // namespace mi355x
