/*
 * gen_golden.c — golden-vector generator linked against the REFERENCE's own ggml
 * (libggml-base + the score-selected ggml-cpu variant built from /root/reference sources
 * by refhost/Makefile).  TEST INFRASTRUCTURE ONLY: oracle/make_golden.py calls these
 * functions through ctypes to produce tests/golden/*.npz, which pin oracle/ggml_oracle.c.
 *
 * Every function runs the reference implementation itself: ggml_quantize_chunk
 * (ggml.c, the model-file quantizers), the CPU backend's from_float/vec_dot type traits
 * (ggml-cpu/ggml-cpu.c:193-282) and ggml graphs computed by the CPU backend
 * (ggml_graph_compute_with_ctx, ggml-cpu/ggml-cpu.c).
 */
#include <stdint.h>
#include <string.h>

#include "ggml.h"
#include "ggml-alloc.h"
#include "ggml-backend.h"
#include "ggml-cpu.h"

static struct ggml_context * mk_ctx(size_t mb) {
    struct ggml_init_params ip = {mb * 1024 * 1024, NULL, false};
    return ggml_init(ip);
}

static void run(struct ggml_context * ctx, struct ggml_tensor * out, int nth) {
    struct ggml_cgraph * gf = ggml_new_graph(ctx);
    ggml_build_forward_expand(gf, out);
    ggml_graph_compute_with_ctx(ctx, gf, nth);
}

void gg_init(void) { ggml_cpu_init(); }

/* model-file quantization of nrows rows (ggml_quantize_chunk, ggml.c) */
size_t gg_quantize(int type, const float * src, void * dst, int64_t nrows, int64_t n_per_row) {
    return ggml_quantize_chunk((enum ggml_type) type, src, dst, 0, nrows, n_per_row, NULL);
}

/* the CPU backend's activation quantizer for a vec_dot_type (Q8_K / Q8_0) */
void gg_from_float(int type, const float * x, void * y, int64_t k) {
    ggml_get_type_traits_cpu((enum ggml_type) type)->from_float(x, y, k);
}

void gg_to_float(int type, const void * x, float * y, int64_t k) {
    ggml_get_type_traits((enum ggml_type) type)->to_float(x, y, k);
}

/* the CPU backend's vec_dot of one weight row against one activation row quantized to the
 * weight type's vec_dot_type */
float gg_vec_dot(int type, int64_t n, const void * x, const void * y) {
    float s = 0.0f;
    ggml_get_type_traits_cpu((enum ggml_type) type)->vec_dot((int) n, &s, 0, x, 0, y, 0, 1);
    return s;
}

/* Y[T][M] = mul_mat(W[M][K], X[T][K]) on the CPU backend */
void gg_mul_mat(int type, const void * W, int64_t K, int64_t M, const float * X, int64_t T, float * Y, int nth) {
    struct ggml_context * ctx = mk_ctx(64 + (size_t) ((K * M * 4 + K * T * 4 + M * T * 4) >> 20) * 2);
    struct ggml_tensor * w = ggml_new_tensor_2d(ctx, (enum ggml_type) type, K, M);
    struct ggml_tensor * x = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, T);
    memcpy(w->data, W, ggml_nbytes(w));
    memcpy(x->data, X, ggml_nbytes(x));
    struct ggml_tensor * y = ggml_mul_mat(ctx, w, x);
    run(ctx, y, nth);
    memcpy(Y, y->data, ggml_nbytes(y));
    ggml_free(ctx);
}

/* Y[T][M] = mul_mat(W[M][K], X[T][K]) the way libllama runs it on the CPU backend: the
 * weight in the CPU device's first extra buffer type (CPU_REPACK: set_tensor repacks Q4_K /
 * Q4_0 rows for the 8x8 AVX2 kernels, ggml-cpu/repack.cpp:1416-1480) when use_extra is set,
 * else in the default CPU buffer; the graph computed by ggml_backend_graph_compute. */
int gg_mul_mat_backend(int type, const void * W, int64_t K, int64_t M, const float * X, int64_t T, float * Y, int nth,
                       int use_extra) {
    ggml_backend_t be = ggml_backend_cpu_init();
    ggml_backend_cpu_set_n_threads(be, nth);
    ggml_backend_dev_t dev = ggml_backend_get_device(be);
    ggml_backend_reg_t reg = ggml_backend_dev_backend_reg(dev);
    ggml_backend_buffer_type_t wbuft = ggml_backend_get_default_buffer_type(be);
    if (use_extra) {
        ggml_backend_dev_get_extra_bufts_t get = (ggml_backend_dev_get_extra_bufts_t)
            ggml_backend_reg_get_proc_address(reg, "ggml_backend_dev_get_extra_bufts");
        ggml_backend_buffer_type_t * ex = get ? get(dev) : NULL;
        if (!ex || !ex[0]) { ggml_backend_free(be); return -1; }
        wbuft = ex[0];
    }
    struct ggml_init_params ip = {ggml_tensor_overhead() * 8 + ggml_graph_overhead(), NULL, true};
    struct ggml_context * cw = ggml_init(ip);
    struct ggml_context * cx = ggml_init(ip);
    struct ggml_tensor * w = ggml_new_tensor_2d(cw, (enum ggml_type) type, K, M);
    struct ggml_tensor * x = ggml_new_tensor_2d(cx, GGML_TYPE_F32, K, T);
    struct ggml_tensor * y = ggml_mul_mat(cx, w, x);
    ggml_backend_buffer_t bw = ggml_backend_alloc_ctx_tensors_from_buft(cw, wbuft);
    ggml_backend_buffer_t bx = ggml_backend_alloc_ctx_tensors_from_buft(cx, ggml_backend_get_default_buffer_type(be));
    ggml_backend_tensor_set(w, W, 0, ggml_nbytes(w));
    ggml_backend_tensor_set(x, X, 0, ggml_nbytes(x));
    struct ggml_cgraph * gf = ggml_new_graph(cx);
    ggml_build_forward_expand(gf, y);
    const int st = (int) ggml_backend_graph_compute(be, gf);
    ggml_backend_tensor_get(y, Y, 0, ggml_nbytes(y));
    ggml_backend_buffer_free(bw);
    ggml_backend_buffer_free(bx);
    ggml_free(cw);
    ggml_free(cx);
    ggml_backend_free(be);
    return st;
}

/* Y[T][n_used][M] = mul_mat_id(As [n_as][M][K], X [T][ne11][K], ids [T][n_used]) on the CPU backend */
void gg_mul_mat_id(int type, const void * As, int64_t K, int64_t M, int64_t n_as, const int32_t * ids, int64_t n_used,
                   const float * X, int64_t ne11, int64_t T, float * Y, int nth) {
    struct ggml_context * ctx = mk_ctx(64 + (size_t) ((K * M * n_as * 4 + K * ne11 * T * 4 + M * n_used * T * 4) >> 20) * 2);
    struct ggml_tensor * as = ggml_new_tensor_3d(ctx, (enum ggml_type) type, K, M, n_as);
    struct ggml_tensor * id = ggml_new_tensor_2d(ctx, GGML_TYPE_I32, n_used, T);
    struct ggml_tensor * x = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, K, ne11, T);
    memcpy(as->data, As, ggml_nbytes(as));
    memcpy(id->data, ids, ggml_nbytes(id));
    memcpy(x->data, X, ggml_nbytes(x));
    struct ggml_tensor * y = ggml_mul_mat_id(ctx, as, x, id);
    run(ctx, y, nth);
    memcpy(Y, y->data, ggml_nbytes(y));
    ggml_free(ctx);
}

/* mul_mat_id as libllama runs it: the expert stack in the CPU device's first extra buffer type
 * (CPU_REPACK: Q4_K / Q4_0 stacks with M % 8 == 0 take repack.cpp forward_mul_mat_id, one gemv
 * per routed pair, repack.cpp:1277-1405) when use_extra is set; graph computed by
 * ggml_backend_graph_compute */
int gg_mul_mat_id_backend(int type, const void * As, int64_t K, int64_t M, int64_t n_as, const int32_t * ids,
                          int64_t n_used, const float * X, int64_t ne11, int64_t T, float * Y, int nth, int use_extra) {
    ggml_backend_t be = ggml_backend_cpu_init();
    ggml_backend_cpu_set_n_threads(be, nth);
    ggml_backend_dev_t dev = ggml_backend_get_device(be);
    ggml_backend_reg_t reg = ggml_backend_dev_backend_reg(dev);
    ggml_backend_buffer_type_t wbuft = ggml_backend_get_default_buffer_type(be);
    if (use_extra) {
        ggml_backend_dev_get_extra_bufts_t get = (ggml_backend_dev_get_extra_bufts_t)
            ggml_backend_reg_get_proc_address(reg, "ggml_backend_dev_get_extra_bufts");
        ggml_backend_buffer_type_t * ex = get ? get(dev) : NULL;
        if (!ex || !ex[0]) { ggml_backend_free(be); return -1; }
        wbuft = ex[0];
    }
    struct ggml_init_params ip = {ggml_tensor_overhead() * 8 + ggml_graph_overhead(), NULL, true};
    struct ggml_context * cw = ggml_init(ip);
    struct ggml_context * cx = ggml_init(ip);
    struct ggml_tensor * as = ggml_new_tensor_3d(cw, (enum ggml_type) type, K, M, n_as);
    struct ggml_tensor * id = ggml_new_tensor_2d(cx, GGML_TYPE_I32, n_used, T);
    struct ggml_tensor * x = ggml_new_tensor_3d(cx, GGML_TYPE_F32, K, ne11, T);
    struct ggml_tensor * y = ggml_mul_mat_id(cx, as, x, id);
    ggml_backend_buffer_t bw = ggml_backend_alloc_ctx_tensors_from_buft(cw, wbuft);
    ggml_backend_buffer_t bx = ggml_backend_alloc_ctx_tensors_from_buft(cx, ggml_backend_get_default_buffer_type(be));
    ggml_backend_tensor_set(as, As, 0, ggml_nbytes(as));
    ggml_backend_tensor_set(id, ids, 0, ggml_nbytes(id));
    ggml_backend_tensor_set(x, X, 0, ggml_nbytes(x));
    struct ggml_cgraph * gf = ggml_new_graph(cx);
    ggml_build_forward_expand(gf, y);
    const int st = (int) ggml_backend_graph_compute(be, gf);
    ggml_backend_tensor_get(y, Y, 0, ggml_nbytes(y));
    ggml_backend_buffer_free(bw);
    ggml_backend_buffer_free(bx);
    ggml_free(cw);
    ggml_free(cx);
    ggml_backend_free(be);
    return st;
}

/* argsort of nrows rows of ne0 floats (order 0 asc, 1 desc) on the CPU backend */
void gg_argsort(const float * x, int64_t ne0, int64_t nrows, int order, int32_t * out) {
    struct ggml_context * ctx = mk_ctx(16 + (size_t) ((ne0 * nrows * 8) >> 20));
    struct ggml_tensor * a = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, ne0, nrows);
    memcpy(a->data, x, ggml_nbytes(a));
    struct ggml_tensor * o = ggml_argsort(ctx, a, (enum ggml_sort_order) order);
    run(ctx, o, 1);
    memcpy(out, o->data, ggml_nbytes(o));
    ggml_free(ctx);
}

void gg_sum_rows(const float * x, int64_t ne0, int64_t nrows, float * y) {
    struct ggml_context * ctx = mk_ctx(16 + (size_t) ((ne0 * nrows * 8) >> 20));
    struct ggml_tensor * a = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, ne0, nrows);
    memcpy(a->data, x, ggml_nbytes(a));
    struct ggml_tensor * o = ggml_sum_rows(ctx, a);
    run(ctx, o, 1);
    memcpy(y, o->data, ggml_nbytes(o));
    ggml_free(ctx);
}

void gg_rms_norm(const float * x, int64_t ne0, int64_t nrows, float eps, float * y) {
    struct ggml_context * ctx = mk_ctx(16 + (size_t) ((ne0 * nrows * 8) >> 20));
    struct ggml_tensor * a = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, ne0, nrows);
    memcpy(a->data, x, ggml_nbytes(a));
    struct ggml_tensor * o = ggml_rms_norm(ctx, a, eps);
    run(ctx, o, 1);
    memcpy(y, o->data, ggml_nbytes(o));
    ggml_free(ctx);
}

/* x: ggml [ne0, n_head, n_tok] f32 */
void gg_rope(const float * x, int64_t ne0, int64_t n_head, int64_t n_tok, const int32_t * pos, int n_dims, int mode,
             int n_ctx_orig, float freq_base, float freq_scale, float ext_factor, float attn_factor, float beta_fast,
             float beta_slow, const float * ff, float * y) {
    struct ggml_context * ctx = mk_ctx(32);
    struct ggml_tensor * a = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, ne0, n_head, n_tok);
    struct ggml_tensor * p = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, n_tok);
    struct ggml_tensor * f = NULL;
    memcpy(a->data, x, ggml_nbytes(a));
    memcpy(p->data, pos, ggml_nbytes(p));
    if (ff) {
        f = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, n_dims / 2);
        memcpy(f->data, ff, ggml_nbytes(f));
    }
    struct ggml_tensor * o = ggml_rope_ext(ctx, a, p, f, n_dims, mode, n_ctx_orig, freq_base, freq_scale, ext_factor,
                                           attn_factor, beta_fast, beta_slow);
    run(ctx, o, 1);
    memcpy(y, o->data, ggml_nbytes(o));
    ggml_free(ctx);
}

/* x: [nr][nc] viewed as ggml [nc, mask_rows, nr/mask_rows], mask: [mask_rows][nc] f32 or NULL
 * (the mask broadcasts over the outer dim, as for per-head KQ) */
void gg_soft_max(const float * x, int64_t nc, int64_t nr, const float * mask, int64_t mask_rows, float scale, float * y) {
    struct ggml_context * ctx = mk_ctx(32);
    struct ggml_tensor * a = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, nc, mask_rows, nr / mask_rows);
    memcpy(a->data, x, ggml_nbytes(a));
    struct ggml_tensor * m = NULL;
    if (mask) {
        m = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, nc, mask_rows);
        memcpy(m->data, mask, ggml_nbytes(m));
    }
    struct ggml_tensor * o = ggml_soft_max_ext(ctx, a, m, scale, 0.0f);
    run(ctx, o, 1);
    memcpy(y, o->data, ggml_nbytes(o));
    ggml_free(ctx);
}

/* q: [n_q][H][D] f32; k, v: [n_kv][Hkv][D] of kv_type; mask [n_q][n_kv] f16 (rows padded to
 * GGML_KQ_MASK_PAD inside); out: [n_q][H][D] */
void gg_flash_attn(const float * q, const void * k, const void * v, const uint16_t * mask, int kv_type, int64_t D,
                   int64_t n_q, int64_t H, int64_t n_kv, int64_t Hkv, float scale, float softcap, float * out, int nth) {
    struct ggml_context * ctx = mk_ctx(256);
    /* q as the graph sees it: [D, n_q, H] permuted from [D, H, n_q] */
    struct ggml_tensor * q3 = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, D, H, n_q);
    memcpy(q3->data, q, ggml_nbytes(q3));
    struct ggml_tensor * qp = ggml_permute(ctx, q3, 0, 2, 1, 3);
    struct ggml_tensor * k3 = ggml_new_tensor_3d(ctx, (enum ggml_type) kv_type, D, Hkv, n_kv);
    struct ggml_tensor * v3 = ggml_new_tensor_3d(ctx, (enum ggml_type) kv_type, D, Hkv, n_kv);
    memcpy(k3->data, k, ggml_nbytes(k3));
    memcpy(v3->data, v, ggml_nbytes(v3));
    struct ggml_tensor * kp = ggml_permute(ctx, k3, 0, 2, 1, 3);
    struct ggml_tensor * vp = ggml_permute(ctx, v3, 0, 2, 1, 3);
    struct ggml_tensor * m = NULL;
    if (mask) {
        const int64_t npad = GGML_PAD(n_q, GGML_KQ_MASK_PAD);
        m = ggml_new_tensor_2d(ctx, GGML_TYPE_F16, n_kv, npad);
        memset(m->data, 0, ggml_nbytes(m));
        memcpy(m->data, mask, sizeof(uint16_t) * n_kv * n_q);
    }
    struct ggml_tensor * o = ggml_flash_attn_ext(ctx, qp, kp, vp, m, scale, 0.0f, softcap);
    ggml_flash_attn_ext_set_prec(o, GGML_PREC_F32);
    run(ctx, o, nth);
    memcpy(out, o->data, ggml_nbytes(o));
    ggml_free(ctx);
}
