// capi.cpp — flat C ABI over the MI355X kernels for parity tests and microbenchmarks.
//
// Each entry point takes plain device pointers, sizes and a HIP stream (NULL = a private
// stream), wraps them in stack-allocated ggml_tensor descriptors with the reference's
// layout (ggml.h:576-608) and runs exactly the launcher graph_compute would run for that
// node, so tests exercise the product path without a ggml context or graph.
#include "ops.h"
#include "fattn.h"
#include "../../include/ggml-mi355x.h"

#include <cstring>
#include <functional>
#include <vector>

using namespace mi355x;

namespace mi355x {
bool mmv_q_supported_type(ggml_type t);
void mul_mat_vec(exec_ctx & ctx, ggml_tensor * dst, const q8_act * pre);
void fattn_scores_d128(hipStream_t st, const float * q, const uint16_t * k, int64_t n, float * s);
}

static void init_tensor(ggml_tensor & t, ggml_type type, const int64_t ne[4], void * data) {
    memset(&t, 0, sizeof(t));
    t.type = type;
    for (int i = 0; i < 4; ++i) t.ne[i] = ne[i];
    t.nb[0] = ggml_type_size(type);
    t.nb[1] = t.nb[0] * (t.ne[0] / ggml_blck_size(type));
    for (int i = 2; i < 4; ++i) t.nb[i] = t.nb[i - 1] * t.ne[i - 1];
    t.data = data;
}

struct scoped_ctx {
    exec_ctx ex;
    bool own = false;
    explicit scoped_ctx(void * stream) {
        if (stream) {
            ex.stream = (hipStream_t) stream;
        } else {
            MI_CHECK(hipStreamCreateWithFlags(&ex.stream, hipStreamNonBlocking));
            own = true;
        }
    }
    ~scoped_ctx() {
        MI_CHECK(hipStreamSynchronize(ex.stream));
        ex.free_scratch();
        if (own) MI_CHECK(hipStreamDestroy(ex.stream));
    }
};

extern "C" {

// ---- device memory helpers (so tests need no other HIP binding) ----------------------------
GGML_BACKEND_API void * mi355x_dev_alloc(size_t bytes) {
    void * p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    return p;
}
GGML_BACKEND_API void mi355x_dev_free(void * p) { MI_CHECK(hipFree(p)); }
GGML_BACKEND_API void mi355x_h2d(void * dst, const void * src, size_t n) { MI_CHECK(hipMemcpy(dst, src, n, hipMemcpyHostToDevice)); }
GGML_BACKEND_API void mi355x_d2h(void * dst, const void * src, size_t n) { MI_CHECK(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost)); }
GGML_BACKEND_API void mi355x_memset(void * dst, int v, size_t n) { MI_CHECK(hipMemset(dst, v, n)); }
GGML_BACKEND_API void mi355x_sync(void) { MI_CHECK(hipDeviceSynchronize()); }

// ---- activation quantization: nrows rows of k floats -> SoA (qs [nrows][k] int8,
// d [nrows][k/blk] f32, s [nrows][k/grp] i16); vdt = GGML_TYPE_Q8_K (15) or Q8_0 (8)
GGML_BACKEND_API int mi355x_quantize_rows(int vdt, const float * x, int64_t k, int64_t nrows, void * qs, void * d,
                                          void * s, void * stream) {
    const bool kq = vdt == GGML_TYPE_Q8_K;
    if (!kq && vdt != GGML_TYPE_Q8_0) return -1;
    if (k % (kq ? 256 : 32) != 0) return -2;
    scoped_ctx sc(stream);
    q8_act act;
    act.qs = (int8_t *) qs; act.d = (float *) d; act.s = (int16_t *) s; act.K = k; act.ncols = nrows; act.k_quant = kq;
    quantize_act_raw(sc.ex.stream, x, k, nrows, k, kq, act);
    return 0;
}

// ---- y[T][M] = W[M][K] (ggml_type wtype rows) x X[T][K]  — MUL_MAT node ---------------------
GGML_BACKEND_API int mi355x_mul_mat(int wtype, const void * w, int64_t K, int64_t M, const float * x, int64_t T, float * y,
                                    void * stream) {
    ggml_tensor W, X, Y;
    const int64_t new_[4] = {K, M, 1, 1}, nex[4] = {K, T, 1, 1}, ney[4] = {M, T, 1, 1};
    init_tensor(W, (ggml_type) wtype, new_, (void *) w);
    init_tensor(X, GGML_TYPE_F32, nex, (void *) x);
    init_tensor(Y, GGML_TYPE_F32, ney, y);
    Y.op = GGML_OP_MUL_MAT;
    Y.src[0] = &W;
    Y.src[1] = &X;
    if (!op_supported(&Y)) return -1;
    scoped_ctx sc(stream);
    op_mul_mat(sc.ex, &Y);
    return 0;
}

// ---- MUL_MAT_ID (ggml-cpu/ggml-cpu.c:1466): as [n_as][M][K] rows of wtype; ids [T][ids_row]
// int32 of which the first n_used per token are used (a view, as test-backend-ops builds it);
// x [T][ne11][K] f32 (ne11 = 1 broadcasts one row to every slot); y [T][n_used][M]
GGML_BACKEND_API int mi355x_mul_mat_id(int wtype, const void * as, int64_t K, int64_t M, int64_t n_as, const int32_t * ids,
                                       int64_t ids_row, int64_t n_used, const float * x, int64_t ne11, int64_t T, float * y,
                                       void * stream) {
    ggml_tensor A, I, X, Y;
    const int64_t nea[4] = {K, M, n_as, 1}, nei[4] = {n_used, T, 1, 1}, nex[4] = {K, ne11, T, 1}, ney[4] = {M, n_used, T, 1};
    init_tensor(A, (ggml_type) wtype, nea, (void *) as);
    init_tensor(I, GGML_TYPE_I32, nei, (void *) ids);
    I.nb[1] = (size_t) ids_row * sizeof(int32_t);
    I.nb[2] = I.nb[1] * T; I.nb[3] = I.nb[2];
    init_tensor(X, GGML_TYPE_F32, nex, (void *) x);
    init_tensor(Y, GGML_TYPE_F32, ney, y);
    Y.op = GGML_OP_MUL_MAT_ID;
    Y.src[0] = &A; Y.src[1] = &X; Y.src[2] = &I;
    if (!op_supported(&Y)) return -1;
    scoped_ctx sc(stream);
    op_mul_mat_id(sc.ex, &Y);
    return 0;
}

// ---- ARGSORT (ops.cpp:6956) of nrows rows of ne0 floats; order 0 = ascending, 1 = descending
GGML_BACKEND_API int mi355x_argsort(const float * x, int64_t ne0, int64_t nrows, int order, int32_t * out, void * stream) {
    ggml_tensor X, Y;
    const int64_t ne[4] = {ne0, nrows, 1, 1};
    init_tensor(X, GGML_TYPE_F32, ne, (void *) x);
    init_tensor(Y, GGML_TYPE_I32, ne, out);
    Y.op = GGML_OP_ARGSORT;
    Y.src[0] = &X;
    Y.op_params[0] = order;
    if (!op_supported(&Y)) return -1;
    scoped_ctx sc(stream);
    op_argsort(sc.ex, &Y);
    return 0;
}

// ---- SUM_ROWS (ops.cpp:1956): y[r] = sum of row r (ne0 floats)
GGML_BACKEND_API int mi355x_sum_rows(const float * x, int64_t ne0, int64_t nrows, float * y, void * stream) {
    ggml_tensor X, Y;
    const int64_t ne[4] = {ne0, nrows, 1, 1}, ney[4] = {1, nrows, 1, 1};
    init_tensor(X, GGML_TYPE_F32, ne, (void *) x);
    init_tensor(Y, GGML_TYPE_F32, ney, y);
    Y.op = GGML_OP_SUM_ROWS;
    Y.src[0] = &X;
    if (!op_supported(&Y)) return -1;
    scoped_ctx sc(stream);
    op_sum_rows(sc.ex, &Y);
    return 0;
}

// ---- rms_norm over nrows rows (optionally fused with a weight vector w[ne0]) ---------------
GGML_BACKEND_API int mi355x_rms_norm(const float * x, int64_t ne0, int64_t nrows, float eps, const float * w, float * y,
                                     float * y_mul, void * stream) {
    ggml_tensor X, Y, Wt, Ym;
    const int64_t ne[4] = {ne0, nrows, 1, 1}, new_[4] = {ne0, 1, 1, 1};
    init_tensor(X, GGML_TYPE_F32, ne, (void *) x);
    init_tensor(Y, GGML_TYPE_F32, ne, y);
    Y.op = GGML_OP_RMS_NORM;
    Y.src[0] = &X;
    memcpy(Y.op_params, &eps, sizeof(float));
    scoped_ctx sc(stream);
    if (w) {
        init_tensor(Wt, GGML_TYPE_F32, new_, (void *) w);
        init_tensor(Ym, GGML_TYPE_F32, ne, y_mul);
        op_rms_norm(sc.ex, &Y, &Wt, &Ym);
    } else {
        op_rms_norm(sc.ex, &Y, nullptr, nullptr);
    }
    return 0;
}

// ---- rope: x [n_tok][n_head][ne0] (ggml [ne0, n_head, n_tok]) -------------------------------
GGML_BACKEND_API int mi355x_rope(const float * x, int64_t ne0, int64_t n_head, int64_t n_tok, const int32_t * pos,
                                 int n_dims, int mode, int n_ctx_orig, float freq_base, float freq_scale, float ext_factor,
                                 float attn_factor, float beta_fast, float beta_slow, const float * ff, float * y,
                                 void * stream) {
    ggml_tensor X, P, F, Y;
    const int64_t ne[4] = {ne0, n_head, n_tok, 1}, nep[4] = {n_tok, 1, 1, 1}, nef[4] = {n_dims / 2, 1, 1, 1};
    init_tensor(X, GGML_TYPE_F32, ne, (void *) x);
    init_tensor(P, GGML_TYPE_I32, nep, (void *) pos);
    init_tensor(Y, GGML_TYPE_F32, ne, y);
    Y.op = GGML_OP_ROPE;
    Y.src[0] = &X;
    Y.src[1] = &P;
    if (ff) {
        init_tensor(F, GGML_TYPE_F32, nef, (void *) ff);
        Y.src[2] = &F;
    }
    int32_t * op = Y.op_params;
    op[1] = n_dims; op[2] = mode; op[4] = n_ctx_orig;
    memcpy(op + 5, &freq_base, 4); memcpy(op + 6, &freq_scale, 4); memcpy(op + 7, &ext_factor, 4);
    memcpy(op + 8, &attn_factor, 4); memcpy(op + 9, &beta_fast, 4); memcpy(op + 10, &beta_slow, 4);
    if (!op_supported(&Y)) return -1;
    scoped_ctx sc(stream);
    op_rope(sc.ex, &Y);
    return 0;
}

// ---- soft_max_ext: x viewed as ggml [nc, mask_rows, nr/mask_rows]; mask [mask_rows][nc] f32
GGML_BACKEND_API int mi355x_soft_max(const float * x, int64_t nc, int64_t nr, const float * mask, int64_t mask_rows,
                                     float scale, float * y, void * stream) {
    ggml_tensor X, Mk, Y;
    const int64_t ne[4] = {nc, mask_rows, nr / mask_rows, 1}, nem[4] = {nc, mask_rows, 1, 1};
    init_tensor(X, GGML_TYPE_F32, ne, (void *) x);
    init_tensor(Y, GGML_TYPE_F32, ne, y);
    Y.op = GGML_OP_SOFT_MAX;
    Y.src[0] = &X;
    if (mask) {
        init_tensor(Mk, GGML_TYPE_F32, nem, (void *) mask);
        Y.src[1] = &Mk;
    }
    const float mb = 0.0f;
    memcpy(Y.op_params, &scale, 4);
    memcpy(Y.op_params + 1, &mb, 4);
    scoped_ctx sc(stream);
    op_soft_max(sc.ex, &Y);
    return 0;
}

// ---- unary SiLU over n floats ------------------------------------------------------------------
GGML_BACKEND_API int mi355x_silu(const float * x, int64_t ne0, int64_t nrows, float * y, void * stream) {
    ggml_tensor X, Y;
    const int64_t ne[4] = {ne0, nrows, 1, 1};
    init_tensor(X, GGML_TYPE_F32, ne, (void *) x);
    init_tensor(Y, GGML_TYPE_F32, ne, y);
    Y.op = GGML_OP_UNARY;
    Y.src[0] = &X;
    Y.op_params[0] = GGML_UNARY_OP_SILU;
    scoped_ctx sc(stream);
    op_unary(sc.ex, &Y);
    return 0;
}

// ---- flash_attn_ext: q [n_q][H][D] f32, k/v [n_kv][Hkv][D] (f16 or q8_0 rows),
// mask [n_q][n_kv] f16 (rows padded to 64 internally by the caller or not at all),
// out [n_q][H][D] f32 — the layout llama's graph hands to FLASH_ATTN_EXT
GGML_BACKEND_API int mi355x_flash_attn(const float * q, const void * k, const void * v, const uint16_t * mask, int kv_type,
                                       int64_t D, int64_t n_q, int64_t H, int64_t n_kv, int64_t Hkv, float scale,
                                       float softcap, float * out, void * stream) {
    ggml_tensor Q, K, V, Mk, O;
    // q: [D, H, n_q] permuted to [D, n_q, H]
    const int64_t neq[4] = {D, H, n_q, 1};
    init_tensor(Q, GGML_TYPE_F32, neq, (void *) q);
    std::swap(Q.ne[1], Q.ne[2]);
    std::swap(Q.nb[1], Q.nb[2]);
    const int64_t nek[4] = {D, Hkv, n_kv, 1};
    init_tensor(K, (ggml_type) kv_type, nek, (void *) k);
    std::swap(K.ne[1], K.ne[2]);
    std::swap(K.nb[1], K.nb[2]);
    init_tensor(V, (ggml_type) kv_type, nek, (void *) v);
    std::swap(V.ne[1], V.ne[2]);
    std::swap(V.nb[1], V.nb[2]);
    const int64_t nem[4] = {n_kv, n_q, 1, 1};
    const int64_t neo[4] = {D, H, n_q, 1};
    init_tensor(O, GGML_TYPE_F32, neo, out);
    O.op = GGML_OP_FLASH_ATTN_EXT;
    O.src[0] = &Q; O.src[1] = &K; O.src[2] = &V;
    if (mask) {
        init_tensor(Mk, GGML_TYPE_F16, nem, (void *) mask);
        O.src[3] = &Mk;
    }
    const float mb = 0.0f;
    memcpy(O.op_params, &scale, 4);
    memcpy(O.op_params + 1, &mb, 4);
    memcpy(O.op_params + 2, &softcap, 4);
    O.op_params[3] = GGML_PREC_F32;
    if (!op_supported(&O)) return -1;
    scoped_ctx sc(stream);
    op_flash_attn(sc.ex, &O);
    return 0;
}

// test hook: K·Q scores of the CPU-exact flash-attention kernel (f16 K rows of 128)
GGML_BACKEND_API int mi355x_fa_scores_d128(const float * q, const uint16_t * k, int64_t n, float * s, void * stream) {
    scoped_ctx sc(stream);
    fattn_scores_d128(sc.ex.stream, q, k, n, s);
    return 0;
}

}  // extern "C"

// ---- microbenchmark hook: decode GEMV (k_gemv.hip) in isolation ---------------------------------
// nmat matrices of M x K (wtype) share one activation row; `copies` rotating weight copies
// (> MALL size in total) make every launch stream from HBM like a real layer walk.  Returns
// the average device time per grouped launch in microseconds (activation quantized once).
namespace mi355x {
}

extern "C" GGML_BACKEND_API double mi355x_bench_gemv2(int wtype, int64_t K, int64_t M, int nmat, int copies, int iters, int epi_kind);
extern "C" GGML_BACKEND_API double mi355x_bench_gemv(int wtype, int64_t K, int64_t M, int nmat, int copies, int iters) {
    return mi355x_bench_gemv2(wtype, K, M, nmat, copies, iters, 0);
}

// epi_kind: 0 plain; 1 SiLU of matrix 0; 2 f16 (KV-cache) store of every matrix through a
// dynamic-pointer slot; 3 NORM rope (Llama-3 parameters, head dim 128) of matrix 0 with its
// f16 store
extern "C" GGML_BACKEND_API double mi355x_bench_gemv2(int wtype, int64_t K, int64_t M, int nmat, int copies, int iters, int epi_kind) {
    const ggml_type t = (ggml_type) wtype;
    const size_t row = ggml_row_size(t, K);
    const size_t mat = row * (size_t) M;
    std::vector<char *> pool((size_t) copies * nmat);
    for (auto & p : pool) {
        MI_CHECK(hipMalloc(&p, mat));
        // small positive f16 scales everywhere keep values finite; content is irrelevant
        MI_CHECK(hipMemset(p, 0x11, mat));
    }
    float * x; float * y;
    MI_CHECK(hipMalloc(&x, K * 4));
    MI_CHECK(hipMalloc(&y, M * 4 * nmat));
    MI_CHECK(hipMemset(x, 0x3c, K * 4));
    scoped_ctx sc(nullptr);
    std::vector<ggml_tensor> W(nmat), Y(nmat);
    ggml_tensor X;
    const int64_t nex[4] = {K, 1, 1, 1};
    init_tensor(X, GGML_TYPE_F32, nex, x);
    std::vector<ggml_tensor *> mms(nmat);
    for (int m = 0; m < nmat; ++m) {
        const int64_t new_[4] = {K, M, 1, 1}, ney[4] = {M, 1, 1, 1};
        init_tensor(W[m], t, new_, pool[m]);
        init_tensor(Y[m], GGML_TYPE_F32, ney, y + m * M);
        Y[m].op = GGML_OP_MUL_MAT;
        Y[m].src[0] = &W[m];
        Y[m].src[1] = &X;
        mms[m] = &Y[m];
    }
    if (!gemv_supported(mms[0])) return -1.0;
    if (epi_kind == 7) {
        // the general mat-vec (k_mmv_q, one weight row per wave) on matrix 0 only
        hipEvent_t f0, f1;
        MI_CHECK(hipEventCreate(&f0));
        MI_CHECK(hipEventCreate(&f1));
        auto run7 = [&](int it) { W[0].data = pool[(size_t) (it % copies) * nmat]; mul_mat_vec(sc.ex, mms[0], nullptr); };
        for (int i = 0; i < 4; ++i) run7(i);
        MI_CHECK(hipEventRecord(f0, sc.ex.stream));
        for (int i = 0; i < iters; ++i) run7(i);
        MI_CHECK(hipEventRecord(f1, sc.ex.stream));
        MI_CHECK(hipEventSynchronize(f1));
        float ms = 0;
        MI_CHECK(hipEventElapsedTime(&ms, f0, f1));
        for (auto p : pool) MI_CHECK(hipFree(p));
        MI_CHECK(hipFree(x)); MI_CHECK(hipFree(y));
        return ms * 1000.0 / iters;
    }
    if (epi_kind == 6) {
        // MUL_MAT_ID decode: nmat = n_used experts routed out of a stack of 8 (ids 1, 5, 6),
        // one shared activation row; the stacks rotate over `copies` copies
        const int64_t n_as = 8;
        std::vector<char *> stacks((size_t) copies);
        for (auto & p : stacks) {
            MI_CHECK(hipMalloc(&p, mat * n_as));
            MI_CHECK(hipMemset(p, 0x11, mat * n_as));
        }
        int32_t * ids;
        const int32_t hid[3] = {1, 5, 6};
        MI_CHECK(hipMalloc(&ids, sizeof(hid)));
        MI_CHECK(hipMemcpy(ids, hid, sizeof(hid), hipMemcpyHostToDevice));
        float * yid;
        MI_CHECK(hipMalloc(&yid, M * 4 * nmat));
        ggml_tensor As, Id, Yid;
        const int64_t nea[4] = {K, M, n_as, 1}, nei[4] = {nmat, 1, 1, 1}, ney2[4] = {M, nmat, 1, 1};
        init_tensor(As, t, nea, stacks[0]);
        init_tensor(Id, GGML_TYPE_I32, nei, ids);
        init_tensor(Yid, GGML_TYPE_F32, ney2, yid);
        Yid.op = GGML_OP_MUL_MAT_ID;
        Yid.src[0] = &As; Yid.src[1] = &X; Yid.src[2] = &Id;
        hipEvent_t f0, f1;
        MI_CHECK(hipEventCreate(&f0));
        MI_CHECK(hipEventCreate(&f1));
        auto run_id = [&](int it) { As.data = stacks[(size_t) (it % copies)]; op_mul_mat_id(sc.ex, &Yid); };
        for (int i = 0; i < 4; ++i) run_id(i);
        MI_CHECK(hipEventRecord(f0, sc.ex.stream));
        for (int i = 0; i < iters; ++i) run_id(i);
        MI_CHECK(hipEventRecord(f1, sc.ex.stream));
        MI_CHECK(hipEventSynchronize(f1));
        float ms = 0;
        MI_CHECK(hipEventElapsedTime(&ms, f0, f1));
        for (auto p : stacks) MI_CHECK(hipFree(p));
        for (auto p : pool) MI_CHECK(hipFree(p));
        MI_CHECK(hipFree(ids)); MI_CHECK(hipFree(yid)); MI_CHECK(hipFree(x)); MI_CHECK(hipFree(y));
        return ms * 1000.0 / iters;
    }
    // epilogue operands
    gemv_epi epi;
    ggml_tensor S, Rt, P;
    float * fbuf; uint16_t * hbuf; void ** slots; int32_t * pos;
    MI_CHECK(hipMalloc(&fbuf, (M + 4 * K) * 4));
    MI_CHECK(hipMalloc(&hbuf, M * 2 * nmat));
    MI_CHECK(hipMalloc(&slots, 8 * nmat));
    MI_CHECK(hipMalloc(&pos, 4));
    MI_CHECK(hipMemset(fbuf, 0x3c, (M + 4 * K) * 4));
    MI_CHECK(hipMemset(pos, 0, 4));
    for (int m = 0; m < nmat; ++m) {
        void * h = hbuf + m * M;
        MI_CHECK(hipMemcpy(slots + m, &h, 8, hipMemcpyHostToDevice));
    }
    const int64_t nem[4] = {M, 1, 1, 1}, nek[4] = {K, 1, 1, 1};
    if (epi_kind == 1) {
        init_tensor(S, GGML_TYPE_F32, nem, fbuf);
        epi.silu[0] = &S;
    } else if (epi_kind == 2) {
        for (int m = 0; m < nmat; ++m) epi.f16out[m] = (void * const *) (slots + m);
    } else if (epi_kind == 3) {
        const int64_t ner[4] = {128, M / 128, 1, 1}, nep[4] = {1, 1, 1, 1};
        init_tensor(Rt, GGML_TYPE_F32, ner, fbuf);
        init_tensor(P, GGML_TYPE_I32, nep, pos);
        Rt.op = GGML_OP_ROPE;
        Rt.src[0] = &Y[0];
        Rt.src[1] = &P;
        int32_t * op = Rt.op_params;
        const float fb = 500000.0f, fs = 1.0f, ef = 0.0f, af = 1.0f, bf = 32.0f, bs = 1.0f;
        op[1] = 128; op[2] = 0; op[4] = 8192;
        memcpy(op + 5, &fb, 4); memcpy(op + 6, &fs, 4); memcpy(op + 7, &ef, 4);
        memcpy(op + 8, &af, 4); memcpy(op + 9, &bf, 4); memcpy(op + 10, &bs, 4);
        epi.rope[0] = &Rt;
        epi.rope_f16[0] = (void * const *) slots;
        epi.elide_rope[0] = true;
    }
    hipEvent_t e0, e1;
    MI_CHECK(hipEventCreate(&e0));
    MI_CHECK(hipEventCreate(&e1));
    auto run = [&](int it) {
        for (int m = 0; m < nmat; ++m) W[m].data = pool[(size_t) (it % copies) * nmat + m];
        gemv_group(sc.ex, mms.data(), nmat, epi_kind ? &epi : nullptr);
    };
    run(0);   // quantizes X into the cache; later launches reuse it
    for (int i = 1; i < 4; ++i) run(i);
    MI_CHECK(hipEventRecord(e0, sc.ex.stream));
    for (int i = 0; i < iters; ++i) run(i);
    MI_CHECK(hipEventRecord(e1, sc.ex.stream));
    MI_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    MI_CHECK(hipEventElapsedTime(&ms, e0, e1));
    MI_CHECK(hipEventDestroy(e0));
    MI_CHECK(hipEventDestroy(e1));
    for (auto p : pool) MI_CHECK(hipFree(p));
    MI_CHECK(hipFree(x));
    MI_CHECK(hipFree(y));
    MI_CHECK(hipFree(fbuf)); MI_CHECK(hipFree(hbuf)); MI_CHECK(hipFree(slots)); MI_CHECK(hipFree(pos));
    return ms * 1000.0 / iters;
}

// ---- microbenchmark hook: the per-layer small ops in isolation -----------------------------------
// which = 0: decode FLASH_ATTN_EXT (exact f16 path) with D = 128, H = 32, Hkv = 8, a cache
//            positions of which the first b are unmasked (Llama-3-8B layout);
//         1: fused residual ADD + RMS_NORM + MUL + Q8_K quantization of one row of a floats.
// Returns the average device time per launch in microseconds.
// streaming-read reference for the roofline: every byte of a buffer read once with 16-byte
// loads, 8 in flight per lane, grid-stride over `grid` workgroups
typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream_read(const v4u_t * __restrict__ p, int64_t n16, uint32_t * out) {
    uint32_t acc = 0;
    const int64_t stride = (int64_t) gridDim.x * 256;
    int64_t i = (int64_t) blockIdx.x * 256 + threadIdx.x;
    for (; i + 7 * stride < n16; i += 8 * stride) {
        v4u_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) { const v4u_t v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678u) out[0] = acc;
}

// the decode GEMV's q4_K access pattern without its arithmetic: a wave reads R = 4 rows of
// 16 blocks x 144 B, lane t taking block t/4's 16-byte header and quant chunks 16+32j, 32+32j
// (j = t%4) — three 16-byte loads per row; MODE 1 instead reads the same bytes as contiguous
// 16-byte chunks (2304 B = 144 chunks: lane t takes chunks t, t+64 and t+128 < 144)
template <int MODE>
__global__ __launch_bounds__(256) void k_pattern_read(const uint8_t * __restrict__ w, int64_t nrows, uint32_t * out) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t row0 = ((int64_t) blockIdx.x * 4 + wave) * 4;
    uint32_t acc = 0;
    uint4 v[12];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint8_t * rp = w + min(row0 + r, nrows - 1) * 2304;
        if (MODE == 0) {
            const uint8_t * blk = rp + (lane >> 2) * 144;
            const int j = lane & 3;
            v[3 * r + 0] = ld16(blk);
            v[3 * r + 1] = ld16(blk + 16 + 32 * j);
            v[3 * r + 2] = ld16(blk + 32 + 32 * j);
        } else {
            v[3 * r + 0] = ld16(rp + 16 * lane);
            v[3 * r + 1] = ld16(rp + 16 * (lane + 64));
            v[3 * r + 2] = lane + 128 < 144 ? ld16(rp + 16 * (lane + 128)) : make_uint4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    if (acc == 0x12345678u) out[0] = acc;
}

namespace mi355x { void mul_mat_q(exec_ctx & ctx, ggml_tensor * dst); }

// buffer_from_host_ptr check: the q4_K weights `w` [M][K/256 blocks] held in host memory are
// wrapped with the device's buffer_from_host_ptr (registered, mapped), the decode mat-vec reads
// them in place, and the result is compared bit for bit with the same weights copied to HBM.
// Returns 0 when identical, 1 on a mismatch, -1 when the device refuses the mapping.
extern "C" GGML_BACKEND_API int mi355x_check_host_ptr_matvec(const void * w, int64_t K, int64_t M, const float * x) {
    ggml_backend_reg_t reg = ggml_backend_mi355x_reg();
    ggml_backend_dev_t dev = ggml_backend_reg_dev_get(reg, 0);
    const size_t wbytes = ggml_row_size(GGML_TYPE_Q4_K, K) * (size_t) M;
    // a page-aligned host copy: hipHostRegister maps whole pages
    const size_t pg = 4096, hsz = (wbytes + 256 + pg - 1) / pg * pg;
    void * host = aligned_alloc(pg, hsz);
    memset(host, 0, hsz);
    memcpy(host, w, wbytes);
    ggml_backend_buffer_t buf = ggml_backend_dev_buffer_from_host_ptr(dev, host, hsz, wbytes);
    if (!buf) { free(host); return -1; }
    void * wdev = nullptr, * xd = nullptr, * y0 = nullptr, * y1 = nullptr;
    MI_CHECK(hipMalloc(&wdev, wbytes + 256));
    MI_CHECK(hipMemset(wdev, 0, wbytes + 256));
    MI_CHECK(hipMemcpy(wdev, w, wbytes, hipMemcpyHostToDevice));
    MI_CHECK(hipMalloc(&xd, K * 4));
    MI_CHECK(hipMemcpy(xd, x, K * 4, hipMemcpyHostToDevice));
    MI_CHECK(hipMalloc(&y0, M * 4));
    MI_CHECK(hipMalloc(&y1, M * 4));
    int rc = 0;
    {
        scoped_ctx sc(nullptr);
        ggml_tensor W0, W1, X, Y0, Y1;
        const int64_t new_[4] = {K, M, 1, 1}, nex[4] = {K, 1, 1, 1}, ney[4] = {M, 1, 1, 1};
        init_tensor(W0, GGML_TYPE_Q4_K, new_, ggml_backend_buffer_get_base(buf));
        init_tensor(W1, GGML_TYPE_Q4_K, new_, wdev);
        init_tensor(X, GGML_TYPE_F32, nex, xd);
        init_tensor(Y0, GGML_TYPE_F32, ney, y0);
        init_tensor(Y1, GGML_TYPE_F32, ney, y1);
        Y0.op = Y1.op = GGML_OP_MUL_MAT;
        Y0.src[0] = &W0; Y1.src[0] = &W1;
        Y0.src[1] = Y1.src[1] = &X;
        op_mul_mat(sc.ex, &Y0);
        sc.ex.qcache_clear();
        op_mul_mat(sc.ex, &Y1);
        MI_CHECK(hipStreamSynchronize(sc.ex.stream));
    }
    std::vector<float> a(M), b(M);
    MI_CHECK(hipMemcpy(a.data(), y0, M * 4, hipMemcpyDeviceToHost));
    MI_CHECK(hipMemcpy(b.data(), y1, M * 4, hipMemcpyDeviceToHost));
    if (memcmp(a.data(), b.data(), M * 4) != 0) rc = 1;
    ggml_backend_buffer_free(buf);
    free(host);
    MI_CHECK(hipFree(wdev)); MI_CHECK(hipFree(xd)); MI_CHECK(hipFree(y0)); MI_CHECK(hipFree(y1));
    return rc;
}

extern "C" GGML_BACKEND_API double mi355x_bench_op(int which, int64_t a, int64_t b, int iters) {
    scoped_ctx sc(nullptr);
    hipEvent_t e0, e1;
    MI_CHECK(hipEventCreate(&e0));
    MI_CHECK(hipEventCreate(&e1));
    std::vector<void *> bufs;
    auto dalloc = [&](size_t n, int pattern) {
        void * p;
        MI_CHECK(hipMalloc(&p, n));
        MI_CHECK(hipMemset(p, pattern, n));
        bufs.push_back(p);
        return p;
    };
    std::function<void()> run;
    ggml_tensor Q, K, V, Mk, O, X, R, A, N, Wt, Mu;
    unsigned long long * prof = nullptr;
    // 3: the decode flash attention of 0 over a q8_0 cache
    const ggml_type fa_kv = which == 3 ? GGML_TYPE_Q8_0 : GGML_TYPE_F16;
    if (which == 3) which = 0;
    const bool fa_probe = which == 2;
    if (which == 2) {
        MI_CHECK(hipMalloc(&prof, 8 * sizeof(unsigned long long)));
        MI_CHECK(hipMemset(prof, 0, 8 * sizeof(unsigned long long)));
        g_fa_prof = prof;
        which = 0;
    }
    if (which == 200 || which == 201) {
        // q4_K-row access pattern (k_pattern_read) over a bytes (rows of 2304 B), b copies
        const int64_t nrows = a / 2304, copies = std::max<int64_t>(1, b);
        char * buf = (char *) dalloc((size_t) (nrows * 2304 * copies), 0x11);
        uint32_t * o = (uint32_t *) dalloc(64, 0);
        int64_t c = 0;
        const int mode = which - 200;
        run = [=, &sc]() mutable {
            const uint8_t * p = (const uint8_t *) buf + (c % copies) * nrows * 2304;
            const dim3 grid((unsigned) ceil_div(nrows, 16));
            if (mode == 0) hipLaunchKernelGGL(k_pattern_read<0>, grid, dim3(256), 0, sc.ex.stream, p, nrows, o);
            else           hipLaunchKernelGGL(k_pattern_read<1>, grid, dim3(256), 0, sc.ex.stream, p, nrows, o);
            ++c;
        };
    } else if (which == 300 || which == 301) {
        // prefill MUL_MAT: Q4_K (300) / Q6_K (301) weights [K=4096][M=a] x b f32 tokens
        const ggml_type wt = which == 300 ? GGML_TYPE_Q4_K : GGML_TYPE_Q6_K;
        const int64_t Kd = 4096, M = a, T = b;
        static ggml_tensor Wm, Xm, Dm;
        const int64_t new_[4] = {Kd, M, 1, 1}, nex[4] = {Kd, T, 1, 1}, ned[4] = {M, T, 1, 1};
        init_tensor(Wm, wt, new_, dalloc(ggml_row_size(wt, Kd) * M, 0x11));
        init_tensor(Xm, GGML_TYPE_F32, nex, dalloc(Kd * T * 4, 0x3c));
        init_tensor(Dm, GGML_TYPE_F32, ned, dalloc(M * T * 4, 0));
        Dm.op = GGML_OP_MUL_MAT; Dm.src[0] = &Wm; Dm.src[1] = &Xm;
        run = [&] { mul_mat_q(sc.ex, &Dm); };
        run();
        MI_CHECK(hipStreamSynchronize(sc.ex.stream));
        float chk[4];
        MI_CHECK(hipMemcpy(chk, (const char *) Dm.data + (M * T / 2) * 4, sizeof(chk), hipMemcpyDeviceToHost));
        fprintf(stderr, "mmq probe M=%lld T=%lld: dst[mid] %g %g %g %g\n", (long long) M, (long long) T, chk[0], chk[1], chk[2], chk[3]);
    } else if (which == 302) {
        // prefill flash attention: D = 128, 32 query heads over 8 KV heads, a query rows = a cache
        // rows with the causal mask, random data (phase cycles of workgroup (0, 0) when b != 0)
        const int64_t D = 128, H = 32, Hkv = 8, nq = a, n_kv = a;
        std::vector<float> hq(D * H * nq);
        std::vector<uint16_t> hk(D * Hkv * n_kv), hv(D * Hkv * n_kv), hm(n_kv * nq);
        uint32_t st = 12345;
        auto rnd = [&]() { st = st * 1664525u + 1013904223u; return ((st >> 8) & 0xffff) / 65536.0f - 0.5f; };
        for (auto & x : hq) x = rnd();
        auto f16b = [](float f) { const _Float16 h = (_Float16) f; uint16_t u; memcpy(&u, &h, 2); return u; };
        for (auto & x : hk) x = f16b(rnd());
        for (auto & x : hv) x = f16b(rnd());
        for (int64_t i = 0; i < nq; ++i)
            for (int64_t j = 0; j < n_kv; ++j) hm[i * n_kv + j] = j <= i ? 0 : 0xFC00;
        float * q = (float *) dalloc(hq.size() * 4, 0);
        void * k = dalloc(hk.size() * 2, 0);
        void * v = dalloc(hv.size() * 2, 0);
        uint16_t * m = (uint16_t *) dalloc(hm.size() * 2, 0);
        MI_CHECK(hipMemcpy(q, hq.data(), hq.size() * 4, hipMemcpyHostToDevice));
        MI_CHECK(hipMemcpy(k, hk.data(), hk.size() * 2, hipMemcpyHostToDevice));
        MI_CHECK(hipMemcpy(v, hv.data(), hv.size() * 2, hipMemcpyHostToDevice));
        MI_CHECK(hipMemcpy(m, hm.data(), hm.size() * 2, hipMemcpyHostToDevice));
        float * out = (float *) dalloc(D * H * nq * 4, 0);
        const int64_t neq[4] = {D, nq, H, 1};
        init_tensor(Q, GGML_TYPE_F32, neq, q);
        std::swap(Q.nb[1], Q.nb[2]);   // [D, nq, H] view of rows laid out [nq][H][D]
        Q.nb[1] = D * H * 4; Q.nb[2] = D * 4; Q.nb[3] = D * H * nq * 4;
        const int64_t nek[4] = {D, n_kv, Hkv, 1};
        init_tensor(K, GGML_TYPE_F16, nek, k);
        K.nb[1] = D * Hkv * 2; K.nb[2] = D * 2; K.nb[3] = D * Hkv * n_kv * 2;
        init_tensor(V, GGML_TYPE_F16, nek, v);
        V.nb[1] = D * Hkv * 2; V.nb[2] = D * 2; V.nb[3] = D * Hkv * n_kv * 2;
        const int64_t nem[4] = {n_kv, nq, 1, 1}, neo[4] = {D, H, nq, 1};
        init_tensor(Mk, GGML_TYPE_F16, nem, m);
        init_tensor(O, GGML_TYPE_F32, neo, out);
        O.op = GGML_OP_FLASH_ATTN_EXT;
        O.src[0] = &Q; O.src[1] = &K; O.src[2] = &V; O.src[3] = &Mk;
        const float scale = 0.088f, zero = 0.0f;
        memcpy(O.op_params, &scale, 4);
        memcpy(O.op_params + 1, &zero, 4);
        memcpy(O.op_params + 2, &zero, 4);
        if (b) {
            MI_CHECK(hipMalloc(&prof, 8 * sizeof(unsigned long long)));
            MI_CHECK(hipMemset(prof, 0, 8 * sizeof(unsigned long long)));
            g_fa_prof = prof;
        }
        run = [&] { op_flash_attn(sc.ex, &O); };
    } else if (which >= 100) {
        // streaming read of a bytes per launch over b rotating copies, grid = which - 100 (x64)
        const int64_t bytes = a, copies = std::max<int64_t>(1, b);
        const int grid = (which - 100) * 64;
        char * buf = (char *) dalloc((size_t) (bytes * copies), 0x11);
        uint32_t * o = (uint32_t *) dalloc(64, 0);
        int64_t c = 0;
        run = [=, &sc]() mutable {
            hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, sc.ex.stream,
                               (const v4u_t *) (buf + (c % copies) * bytes), bytes / 16, o);
            ++c;
        };
    } else if (which == 0) {
        const int64_t D = 128, H = 32, Hkv = 8, n_kv = a;
        float * q = (float *) dalloc(D * H * 4, 0x3c);
        void * k = dalloc(ggml_row_size(fa_kv, D) * Hkv * n_kv, 0x3c);
        void * v = dalloc(ggml_row_size(fa_kv, D) * Hkv * n_kv, 0x3c);
        std::vector<uint16_t> hm(n_kv);
        for (int64_t i = 0; i < n_kv; ++i) hm[i] = i < b ? 0 : 0xFC00;
        uint16_t * m = (uint16_t *) dalloc(n_kv * 2, 0);
        MI_CHECK(hipMemcpy(m, hm.data(), n_kv * 2, hipMemcpyHostToDevice));
        float * out = (float *) dalloc(D * H * 4, 0);
        const int64_t neq[4] = {D, H, 1, 1};
        init_tensor(Q, GGML_TYPE_F32, neq, q);
        std::swap(Q.ne[1], Q.ne[2]); std::swap(Q.nb[1], Q.nb[2]);
        const int64_t nek[4] = {D, Hkv, n_kv, 1};
        init_tensor(K, fa_kv, nek, k);
        std::swap(K.ne[1], K.ne[2]); std::swap(K.nb[1], K.nb[2]);
        init_tensor(V, fa_kv, nek, v);
        std::swap(V.ne[1], V.ne[2]); std::swap(V.nb[1], V.nb[2]);
        const int64_t nem[4] = {n_kv, 1, 1, 1}, neo[4] = {D, H, 1, 1};
        init_tensor(Mk, GGML_TYPE_F16, nem, m);
        init_tensor(O, GGML_TYPE_F32, neo, out);
        O.op = GGML_OP_FLASH_ATTN_EXT;
        O.src[0] = &Q; O.src[1] = &K; O.src[2] = &V; O.src[3] = &Mk;
        const float scale = 0.088f, zero = 0.0f;
        memcpy(O.op_params, &scale, 4);
        memcpy(O.op_params + 1, &zero, 4);
        memcpy(O.op_params + 2, &zero, 4);
        run = [&] { op_flash_attn(sc.ex, &O); };
    } else {
        const int64_t n = a;
        const int64_t ne[4] = {n, 1, 1, 1};
        init_tensor(X, GGML_TYPE_F32, ne, dalloc(n * 4, 0x3c));
        init_tensor(R, GGML_TYPE_F32, ne, dalloc(n * 4, 0x3c));
        init_tensor(A, GGML_TYPE_F32, ne, dalloc(n * 4, 0));
        init_tensor(N, GGML_TYPE_F32, ne, dalloc(n * 4, 0));
        init_tensor(Wt, GGML_TYPE_F32, ne, dalloc(n * 4, 0x3c));
        init_tensor(Mu, GGML_TYPE_F32, ne, dalloc(n * 4, 0));
        A.op = GGML_OP_ADD; A.src[0] = &X; A.src[1] = &R;
        N.op = GGML_OP_RMS_NORM; N.src[0] = &A;
        const float eps = 1e-5f;
        memcpy(N.op_params, &eps, 4);
        Mu.op = GGML_OP_MUL; Mu.src[0] = &N; Mu.src[1] = &Wt;
        // a Q4_K consumer so the norm quantizes to Q8_K
        static ggml_tensor W, MM;
        const int64_t new_[4] = {n, 16, 1, 1}, nem_[4] = {16, 1, 1, 1};
        init_tensor(W, GGML_TYPE_Q4_K, new_, dalloc(ggml_row_size(GGML_TYPE_Q4_K, n) * 16, 0x11));
        init_tensor(MM, GGML_TYPE_F32, nem_, dalloc(64, 0));
        MM.op = GGML_OP_MUL_MAT; MM.src[0] = &W; MM.src[1] = &Mu;
        run = [&] { fused_norm(sc.ex, &A, &N, &Mu, &MM); };
    }
    for (int i = 0; i < 3; ++i) run();
    MI_CHECK(hipEventRecord(e0, sc.ex.stream));
    for (int i = 0; i < iters; ++i) run();
    MI_CHECK(hipEventRecord(e1, sc.ex.stream));
    MI_CHECK(hipEventSynchronize(e1));
    float ms = 0;
    MI_CHECK(hipEventElapsedTime(&ms, e0, e1));
    MI_CHECK(hipEventDestroy(e0));
    MI_CHECK(hipEventDestroy(e1));
    MI_CHECK(hipStreamSynchronize(sc.ex.stream));
    {
        const hipError_t err = hipGetLastError();
        if (err != hipSuccess) fprintf(stderr, "mi355x_bench_op %d: %s\n", which, hipGetErrorString(err));
    }
    if (prof) {
        unsigned long long h[8];
        MI_CHECK(hipMemcpy(h, prof, sizeof(h), hipMemcpyDeviceToHost));
        const char * nm[8] = {"A(mask)", "0(V issue)", "1(scores)", "2(softmax coef)", "3(wait V)", "3(recurrence)", "-", "-"};
        const char * nmp[8] = {"barrier+wait", "1(scores)", "2(coef)", "3(recurrence)", "chunks", "-", "-", "-"};
        const char * nmd[8] = {"p:mask", "p:V issue", "p:scores", "p:coef", "p:V wait", "p:barrier", "chain busy", "chain wait"};
        const char * nms[8] = {"p0:loads in", "p0:barrier", "p0:block 0 ready", "p0:done", "c0:barrier", "c0:block 0 seen", "c0:chain end", "quantized"};
        const bool dsh = fa_probe && a <= 256 && (getenv("GGML_MI355X_FA_DSH") == nullptr || atoi(getenv("GGML_MI355X_FA_DSH")) != 0);
        if (which == 302) for (int i = 0; i < 8; ++i) nm[i] = nmp[i];
        else if (dsh) for (int i = 0; i < 8; ++i) nm[i] = nms[i];
        else if (getenv("GGML_MI355X_FA_DEC2") == nullptr || atoi(getenv("GGML_MI355X_FA_DEC2")) != 0) for (int i = 0; i < 8; ++i) nm[i] = nmd[i];
        fprintf(stderr, "FA phases (s_memtime ticks per launch, wg 0):");
        for (int i = 0; i < 8; ++i) fprintf(stderr, " %s=%.0f", nm[i], (double) h[i] / (iters + 3));
        fprintf(stderr, "\n");
        g_fa_prof = nullptr;
        MI_CHECK(hipFree(prof));
    }
    for (void * p : bufs) MI_CHECK(hipFree(p));
    return ms * 1000.0 / iters;
}
