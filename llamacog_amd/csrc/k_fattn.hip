// k_fattn.hip — FLASH_ATTN_EXT: the op's support test and its dispatch onto the CPU-exact
// kernels of k_fattn_exact.hip (f16, q8_0 and q4_0 caches; D 64 / 128 / 256).
//
// Semantics of ggml_compute_forward_flash_attn_ext_f16 (ggml-cpu/ops.cpp:7015-7232): Q converted
// to K's vec_dot_type, s = (K·Q)*scale (softcap optional) + slope*mask, masked positions skipped,
// the online softmax with V accumulated in f16 (f32 for a quantized V), output VKQ * (1/S).
// Every case runs the exact kernels; the f32 split-K kernels of rounds 1-2 (opt-in, not
// bit-exact: at 1536 positions the CPU's per-position f16 rounding moved the logits by 1.56
// relative) were removed in round 3.
#include "fattn.h"

#include <cmath>

namespace mi355x {

unsigned long long * g_fa_prof = nullptr;

bool fattn_supported(const ggml_tensor * op) {
    const ggml_tensor * q = op->src[0];
    const ggml_tensor * k = op->src[1];
    const ggml_tensor * v = op->src[2];
    const ggml_tensor * mask = op->src[3];
    if (op->src[4] != nullptr) return false;  // attention sinks not supported
    if (q->type != GGML_TYPE_F32) return false;
    if (k->ne[0] != v->ne[0]) return false;
    const int64_t D = k->ne[0];
    if (D != 64 && D != 128 && D != 256) return false;
    if (k->type != v->type) return false;
    if (k->type != GGML_TYPE_F16 && k->type != GGML_TYPE_Q8_0 && k->type != GGML_TYPE_Q4_0) return false;
    if (mask && mask->type != GGML_TYPE_F16) return false;
    if (mask && (mask->ne[2] != 1 || mask->ne[3] != 1)) return false;
    if (q->ne[2] % k->ne[2] != 0) return false;
    if (k->ne[3] != q->ne[3] || v->ne[3] != q->ne[3]) return false;
    float max_bias;
    memcpy(&max_bias, (const float *) op->op_params + 1, 4);
    return true;
}

bool mmv_q_supported_type(ggml_type t);

void fa_args_of(exec_ctx & ctx, ggml_tensor * dst, const ggml_tensor * mm, fa_args & a, q8_act & act, int64_t & nq3) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const ggml_tensor * mask = dst->src[3];
    a = {};
    a.q = (const char *) q->data; a.nbq1 = q->nb[1]; a.nbq2 = q->nb[2]; a.nbq3 = q->nb[3];
    a.k = (const char *) k->data; a.nbk1 = k->nb[1]; a.nbk2 = k->nb[2]; a.nbk3 = k->nb[3];
    a.v = (const char *) v->data; a.nbv1 = v->nb[1]; a.nbv2 = v->nb[2]; a.nbv3 = v->nb[3];
    a.mask = mask ? (const char *) mask->data : nullptr;
    a.nbm1 = mask ? mask->nb[1] : 0;
    a.mask_ne1 = mask ? mask->ne[1] : 1;
    a.k_type = k->type; a.v_type = v->type;
    a.D = k->ne[0]; a.n_kv = k->ne[1]; a.n_q = q->ne[1]; a.H = q->ne[2]; a.Hkv = k->ne[2];
    memcpy(&a.scale, (const float *) dst->op_params + 0, 4);
    memcpy(&a.max_bias, (const float *) dst->op_params + 1, 4);
    memcpy(&a.softcap, (const float *) dst->op_params + 2, 4);
    if (a.softcap != 0.0f) a.scale /= a.softcap;
    const uint32_t n_head = (uint32_t) a.H;
    a.n_head_log2 = 1u << (uint32_t) floor(log2((double) n_head));
    a.m0 = powf(2.0f, -(a.max_bias) / a.n_head_log2);
    a.m1 = powf(2.0f, -(a.max_bias / 2.0f) / a.n_head_log2);
    a.dst = (float *) dst->data;
    a.nb1_dst = dst->nb[1];
    a.nb2_dst = dst->nb[3];  // batch stride (dst ne = [D, H, n_q, ne3])
    nq3 = q->ne[3];

    a.chunk = a.n_kv;
    a.nchunks = 1;
    a.part = nullptr;
    a.qmode = 0;
    a.prof = g_fa_prof;
    a.kt = nullptr;
    a.qs = nullptr; a.qd = nullptr; a.qsum = nullptr;
    a.cnt = nullptr;
    // fused quantization of the output for the next MUL_MAT (decode: one row)
    if (mm && a.n_q == 1 && nq3 == 1 && mmv_q_supported_type(mm->src[0]->type) &&
        mm->src[1]->ne[0] == a.H * a.D && ggml_nrows(mm->src[1]) == 1 && ggml_is_contiguous(dst)) {
        const ggml_type wt = mm->src[0]->type;
        const bool kq = wt == GGML_TYPE_Q4_K || wt == GGML_TYPE_Q5_K || wt == GGML_TYPE_Q6_K;
        // Q8_K blocks span 256/D whole heads (D divides 256 or equals it); in k_fattn_exact their
        // workgroups meet on a counter (allocated outside any capture, zeroed once)
        if (kq && !ctx.fa_cnt && !ctx.capturing) {
            MI_CHECK(hipMalloc(&ctx.fa_cnt, exec_ctx::FA_CNT * sizeof(int)));
            MI_CHECK(hipMemsetAsync(ctx.fa_cnt, 0, exec_ctx::FA_CNT * sizeof(int), ctx.stream));
        }
        if ((a.H * a.D) % (kq ? 256 : 32) == 0 && (!kq || (ctx.fa_cnt && (a.H * a.D) / 256 <= exec_ctx::FA_CNT))) {
            carve_act(act, ctx.scratch(exec_ctx::QSLOT, q8_act::bytes(a.H * a.D, 1, kq)), a.H * a.D, 1, kq);
            a.qmode = kq ? 1 : 2;
            a.qs = act.qs; a.qd = act.d; a.qsum = act.s;
            a.cnt = ctx.fa_cnt;
        }
    } else if (mm && a.n_q > 1 && nq3 == 1 && fattn_pf_quant_ok(a) && mm->src[1]->ne[0] == a.H * a.D &&
               ggml_nrows(mm->src[1]) == a.n_q && ggml_is_contiguous(dst) &&
               (mm->src[0]->type == GGML_TYPE_Q4_K || mm->src[0]->type == GGML_TYPE_Q5_K || mm->src[0]->type == GGML_TYPE_Q6_K)) {
        // prefill: the batch tile quantizes its rows' output (k_fattn_pf), two Q8_K blocks a wave
        carve_act(act, ctx.scratch(exec_ctx::QSLOT, q8_act::bytes(a.H * a.D, a.n_q, true)), a.H * a.D, a.n_q, true);
        a.qmode = 1;
        a.qs = act.qs; a.qd = act.d; a.qsum = act.s;
    }
}

void op_flash_attn(exec_ctx & ctx, ggml_tensor * dst, const ggml_tensor * mm) {
    fa_args a;
    q8_act act;
    int64_t nq3 = 1;
    fa_args_of(ctx, dst, mm, a, act, nq3);
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    hipEvent_t ev = nullptr;
    const double bytes = (double) (ggml_nbytes(k) + ggml_nbytes(v)) + (double) ggml_nbytes(q) + (double) ggml_nbytes(dst);
    if (ctx.timing) ctx.time_begin(TK_FATTN, bytes, ev);
    // decode (one query row): the short-context kernel (k_fattn_dsh) or the two-heads-per-workgroup
    // one (k_fattn_dec2) where they apply, the long-context pair past FA_LONG_MIN, else
    // k_fattn_exact, one workgroup per head; batches: k_fattn_exact's prefill tiles
    if (fattn_long_ok(a, nq3)) {
        // long cache: scores by a wide grid, then the exact recurrence (k_fattn_exact.hip)
        float * sco = (float *) ctx.scratch(1, (size_t) a.H * a.n_kv * sizeof(float));
        unsigned long long * kts = ctx.kt_take("fa_scores", (unsigned) (ceil_div(a.n_kv, (int64_t) FAL_PB) * a.Hkv), 256);
        a.kt = ctx.kt_take("fa_chain", (unsigned) (a.H * FAL_DSPLIT), FAL_THREADS);
        launch_fattn_long(ctx.stream, a, sco, kts);
    } else if (fattn_dsh_ok(a, nq3)) {
        a.kt = ctx.kt_take("fa_dsh", (unsigned) (a.H / 2 * nq3), 512);
        launch_fattn_dsh(ctx.stream, a, nq3);
    } else if (fattn_dec2_ok(a, nq3)) {
        a.kt = ctx.kt_take("fa_dec2", (unsigned) (a.H / 2 * nq3), (unsigned) fattn_dec2_threads(a));
        launch_fattn_dec2(ctx.stream, a, nq3);
    } else {
        if (a.n_q == 1) a.kt = ctx.kt_take("fa_exact", (unsigned) (a.H * nq3), 256);
        launch_fattn_exact(ctx.stream, a, nq3);
    }
    if (a.qmode) ctx.qcache_put(mm->src[1], a.qmode == 1, act);
    if (ctx.timing) ctx.time_end(TK_FATTN, bytes, ev);
}

}  // namespace mi355x
