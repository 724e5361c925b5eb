// ops.h — host-side op launchers of the MI355X backend.  Each launcher takes the
// backend stream context and one ggml node (dst), reads its srcs/op_params with the
// reference's semantics, and enqueues HIP kernels on ctx.stream (never synchronises).
#pragma once

#include "common.h"

#include <vector>

namespace mi355x {

// Per-(context, device) execution state: one HIP stream plus a stream-ordered
// scratch arena for op temporaries (quantized activations, attention partials).
struct exec_ctx {
    int         device = 0;
    hipStream_t stream = nullptr;

    // scratch arena: slot i is a separate region so one op can hold several temps
    static constexpr int N_SLOTS = 4;
    void *  slot_ptr[N_SLOTS]  = {nullptr, nullptr, nullptr, nullptr};
    size_t  slot_size[N_SLOTS] = {0, 0, 0, 0};
    bool    capturing = false;   // hipGraph capture in progress: growing is forbidden

    void * scratch(int slot, size_t bytes);
    void   free_scratch();

    // kernel timing (HIP events on `stream`) for the roofline figure in bench.py
    bool   timing = false;
    struct timed { hipEvent_t beg, end; double bytes; int kind; };
    std::vector<timed> pending;
    std::vector<hipEvent_t> event_pool;
    double acc_ms[8]    = {0};
    double acc_bytes[8] = {0};
    long   acc_count[8] = {0};
    hipEvent_t get_event();
    void   time_begin(int kind, double bytes, hipEvent_t & beg);
    void   time_end(int kind, double bytes, hipEvent_t beg);
    void   collect_timing();  // after a stream synchronize
};

enum timed_kind { TK_MMV = 0, TK_MMQ = 1, TK_FATTN = 2, TK_OTHER = 3 };

// supports / dispatch
bool op_supported(const ggml_tensor * op);
// returns number of graph nodes consumed (>=1) — fused patterns consume several
int  op_compute(exec_ctx & ctx, ggml_cgraph * cgraph, int i);

// individual launchers
void op_mul_mat(exec_ctx & ctx, ggml_tensor * dst);
void op_get_rows(exec_ctx & ctx, ggml_tensor * dst);
void op_rms_norm(exec_ctx & ctx, ggml_tensor * dst, const ggml_tensor * mul_w, ggml_tensor * out);
void op_norm(exec_ctx & ctx, ggml_tensor * dst);
void op_binary(exec_ctx & ctx, ggml_tensor * dst);
void op_scale(exec_ctx & ctx, ggml_tensor * dst);
void op_unary(exec_ctx & ctx, ggml_tensor * dst);
void op_cpy(exec_ctx & ctx, const ggml_tensor * src, ggml_tensor * dst);
void op_rope(exec_ctx & ctx, ggml_tensor * dst);
void op_soft_max(exec_ctx & ctx, ggml_tensor * dst);
void op_flash_attn(exec_ctx & ctx, ggml_tensor * dst);
void op_argsort(exec_ctx & ctx, ggml_tensor * dst);
void op_sum_rows(exec_ctx & ctx, ggml_tensor * dst);
void op_mul_mat_id(exec_ctx & ctx, ggml_tensor * dst);

// activation quantization shared by mul_mat / mul_mat_id / flash-attn (q8_0 K)
struct q8_act {
    int8_t  * qs = nullptr;   // [ncols][K] int8
    float   * d  = nullptr;   // [ncols][K/blk] scale (already rounded like the CPU's)
    int16_t * s  = nullptr;   // [ncols][K/grp] partial sums (q8_K: 16-groups, q8_0: 32-blocks)
    int64_t   K  = 0;
    int64_t   ncols = 0;
    bool      k_quant = false; // Q8_K (256-blocks) vs Q8_0 (32-blocks)
    int64_t qs_stride() const { return K; }
    int64_t d_stride()  const { return k_quant ? K / 256 : K / 32; }
    int64_t s_stride()  const { return k_quant ? K / 16 : K / 32; }
    static size_t bytes(int64_t K, int64_t ncols, bool k_quant);
};

// quantizes ncols rows of an f32 tensor (row i = (i1, i2, i3) flattened) into act
void quantize_act(exec_ctx & ctx, const ggml_tensor * src, bool k_quant, q8_act & act, int slot);
void quantize_act_raw(hipStream_t stream, const float * x, int64_t K, int64_t ncols, int64_t row_stride_elems,
                      bool k_quant, q8_act & act);

}  // namespace mi355x
