// ops.h — host-side op launchers of the MI355X backend.  Each launcher takes the
// backend stream context and one ggml node (dst), reads its srcs/op_params with the
// reference's semantics, and enqueues HIP kernels on ctx.stream (never synchronises).
#pragma once

#include "common.h"

#include <vector>

namespace mi355x {

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

// Per-(context, device) execution state: one HIP stream plus a stream-ordered
// scratch arena for op temporaries (quantized activations, attention partials).
struct exec_ctx {
    int         device = 0;
    hipStream_t stream = nullptr;

    // scratch arena: slot i is a separate region so one op can hold several temps
    static constexpr int N_SLOTS = 7;   // 5: row-split mat-mul staging (op_mul_mat_split)
    static constexpr int MOE_SLOT = 6;  // the MoE routing weights between router and combine
    void *  slot_ptr[N_SLOTS]  = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t  slot_size[N_SLOTS] = {0, 0, 0, 0, 0, 0, 0};
    bool    capturing = false;   // hipGraph capture in progress: growing is forbidden
    // bumped whenever a slot is reallocated: a captured hipGraph holds slot addresses in its
    // kernel arguments, so graphs captured under an older generation are dropped (backend.cpp)
    uint64_t scratch_gen = 0;

    // arrival counters of the flash-attention output quantization (k_fattn_exact.hip)
    static constexpr int FA_CNT = 1024;
    int *   fa_cnt = nullptr;
    // arrival counters of the multi-workgroup MoE router, one per token (k_elem.hip)
    static constexpr int MOE_CNT = 4096;
    int *   moe_cnt = nullptr;
    // the pending prologue: the chain whose output `last` (and its data pointer) the next decode
    // mat-vecs read; they form it from x and w in their launch (kind 1: RMS_NORM(x) [* w])
    // instead of a launch of its own (dispatch.cpp)
    struct pro_pending { const ggml_tensor * last; const void * data; int kind; const float * x; const float * w;
                         float eps; int64_t n; };
    pro_pending pro = {};

    void * scratch(int slot, size_t bytes);
    void   free_scratch();

    // Activation-quantization cache.  Slot QSLOT holds the last quantized MUL_MAT input;
    // consecutive MUL_MATs that share src1 (Q/K/V, gate/up) reuse it, and fused producers
    // (norm / mul kernels, k_fused.hip) fill it ahead of their consumer.  Keyed on the
    // ggml node (and its data pointer) and cleared at the start of every graph_compute,
    // because libllama re-uses node objects across graphs.
    static constexpr int QSLOT = 0;
    const ggml_tensor * qc_tensor = nullptr;
    const void *        qc_data   = nullptr;
    bool                qc_kquant = false;
    q8_act              qc_act;
    void qcache_clear() { qc_tensor = nullptr; qc_data = nullptr; qc0_tensor = nullptr; qc0_data = nullptr; }

    // per-graph RoPE cos/sin table (k_elem.hip rope_table): every layer's fused Q/K rope
    // epilogue reads the same table of the token's position, built once per graph
    const float2 *  rt_table = nullptr;
    int64_t         rt_ntok = 0;
    const void *    rt_pos = nullptr;
    const void *    rt_ff = nullptr;
    int32_t         rt_params[15] = {};


    // nodes already computed ahead of their position by a grouped launch (dispatch.cpp)
    std::vector<const ggml_tensor *> done;

    // a SILU whose MUL partner's other input (the up projection) is computed after it (MoE:
    // gate, SILU, up, MUL): run as one silu*mul kernel at the MUL (dispatch.cpp)
    ggml_tensor * silu_defer = nullptr;
    ggml_tensor * silu_mul = nullptr;

    // MoE decode chain (dispatch.cpp try_moe_router): the router launch wrote the normalised
    // routing weights of `mul` (the combine's MUL) to MOE_SLOT, so the GET_ROWS / SUM_ROWS / DIV
    // nodes are skipped; `comb` (the combine's slot-sum ADD) is deferred into the residual ADD +
    // RMS_NORM launch that reads it (k_norm_fused's combine source)
    struct moe_pending { const ggml_tensor * mul; const float * wn; int n_used; const ggml_tensor * comb; const float * e; };
    moe_pending moe = {};
    // the FFN norm the router launch forms (dispatch.cpp plan_resid, its MoE branch): x the residual sum the
    // producer stored, w the norm weight; qkey the expert mat-vecs' input for the Q8_K cache
    struct moe_norm_pending { const ggml_tensor * mm; const float * x; const float * w; float eps; const ggml_tensor * qkey; };
    moe_norm_pending moe_pro = {};

    // Dynamic destinations: a KV-cache store (CPY into a view at offset n_past) changes its
    // destination every token while the rest of the graph stays identical.  Kernels read
    // such pointers from a device table refreshed before each graph launch, so a captured
    // hipGraph can be replayed (the role of ggml-cuda's cpy dest-pointer indirection).
    std::vector<const ggml_tensor *> dyn_nodes;   // CPY nodes of the current graph
    std::vector<void *>              dyn_host;    // their destination pointers
    void **                          dyn_dev = nullptr;
    size_t                           dyn_cap = 0;
    // pinned staging of the table upload, a ring: buffer k is rewritten only after the copy
    // that last read it has completed (dyn_ev[k])
    static constexpr int             DYN_RING = 8;
    void **                          dyn_pin[DYN_RING] = {};
    hipEvent_t                       dyn_ev[DYN_RING] = {};
    int                              dyn_flip = 0;
    bool prepare_dyn(ggml_cgraph * g);            // scan + upload; false = table too small (backend.cpp)
    void * const * dyn_slot(const ggml_tensor * cpy) const {
        for (size_t k = 0; k < dyn_nodes.size(); ++k) {
            if (dyn_nodes[k] == cpy) return dyn_dev + k;
        }
        return nullptr;
    }
    // a Q8_0 companion of the same activation (slot QSLOT0), written by a fused norm whose
    // output feeds both K-quant and Q8_0 mat-vecs (Mixtral's Q5_K attn_q beside Q8_0 attn_k/v)
    static constexpr int QSLOT0 = 4;
    const ggml_tensor * qc0_tensor = nullptr;
    const void *        qc0_data   = nullptr;
    q8_act              qc0_act;
    bool qcache_get(const ggml_tensor * t, bool k_quant, q8_act & act) const {
        if (!k_quant && qc0_tensor == t && qc0_data == t->data) {
            act = qc0_act;
            return true;
        }
        if (qc_tensor != t || qc_data != t->data || qc_kquant != k_quant) return false;
        act = qc_act;
        return true;
    }
    void qcache_put(const ggml_tensor * t, bool k_quant, const q8_act & act) {
        qc_tensor = t; qc_data = t->data; qc_kquant = k_quant; qc_act = act;
    }

    // in-graph kernel timeline (GGML_MI355X_KTRACE / ggml_backend_mi355x_set_ktrace): a device
    // buffer of realtime stamps (common.h kt_enter / kt_exit), one region per instrumented launch
    // of the current graph, in launch order; the list is kept with a captured graph so a replay
    // is decoded against the launches it replays
    struct kt_launch { const char * name; size_t off; unsigned nwg; unsigned stride; };
    unsigned long long * kt_buf = nullptr;
    size_t kt_cap = 0, kt_off = 0;
    std::vector<kt_launch> kt_list;
    // region for one launch of nwg workgroups of `threads` threads, or nullptr (tracing off / full)
    unsigned long long * kt_take(const char * name, unsigned nwg, unsigned threads);

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
    void   time_cancel(hipEvent_t beg);
    void   collect_timing();  // after a stream synchronize
};

enum timed_kind { TK_MMV = 0, TK_MMQ = 1, TK_FATTN = 2, TK_OTHER = 3, TK_GRAPH = 5, TK_GRAPH_HOST = 6 };

// run-time switches (backend.cpp): GGML_MI355X_NO_FUSE=1 runs every node with its own
// kernel, GGML_MI355X_NO_GRAPH=1 disables hipGraph replay; both also settable through
// ggml_backend_mi355x_set_flags (fused/unfused and graph/eager runs are compared
// bit-for-bit in tests/test_gpu_model.py)
bool fusion_enabled();
bool debug_ops();
bool graphs_enabled();
// blocks while any thread has a hipGraph capture open (backend.cpp)
void wait_no_capture();
bool ktrace_enabled();

// row-split weights (backend.cpp, the split buffer type): the row slices [lo, hi) of a matrix,
// one per device that holds rows, each in that device's memory (HIP device `hip`)
constexpr int MI_MAX_DEV = 16;
struct split_part { int hip; int64_t lo, hi; void * data; };
struct split_parts { int n = 0; split_part p[MI_MAX_DEV]; };
bool tensor_split_parts(const ggml_tensor * t, split_parts & sp);   // false: t is not in a split buffer
// MUL_MAT whose src0 is row-split: each slice on its device, the rows gathered into dst (dispatch.cpp)
void op_mul_mat_split(exec_ctx & ctx, ggml_tensor * dst);
void split_stats(long * mm, long * foreign);   // row-split mat-muls run, and slices run on another GPU

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
// node = the CPY node (its destination may live in the dynamic-pointer table) or nullptr
void op_cpy(exec_ctx & ctx, const ggml_tensor * src, ggml_tensor * dst, const ggml_tensor * node);
void op_rope(exec_ctx & ctx, ggml_tensor * dst);
void op_rope_multi(exec_ctx & ctx, ggml_tensor * const * nodes, int n, void * const * const * cache);
void op_soft_max(exec_ctx & ctx, ggml_tensor * dst);
// mm: the MUL_MAT consuming (a reshape of) dst, whose input the exact kernel may quantize
void op_flash_attn(exec_ctx & ctx, ggml_tensor * dst, const ggml_tensor * mm = nullptr);
void op_argsort(exec_ctx & ctx, ggml_tensor * dst);
void op_sum_rows(exec_ctx & ctx, ggml_tensor * dst);
void op_mul_mat_id(exec_ctx & ctx, ggml_tensor * dst);
bool op_mul_mat_id_pair(exec_ctx & ctx, ggml_tensor * dst, ggml_tensor * dst2);
// the MoE router chain (k_elem.hip): SOFT_MAX + ARGSORT in one launch, GET_ROWS + SUM_ROWS + DIV in another
bool moe_route_sort(exec_ctx & ctx, const ggml_tensor * sm, ggml_tensor * as);
// the router's input formed in the router launch: RMS_NORM(x) * w (eps), stored to the router's
// src1 and, with q, quantized to Q8_K (the expert mat-vecs' activation)
struct moe_router_pro { const float * x; const float * w; float eps; const q8_act * q; };
enum { MOE_RNONE = 0, MOE_R1, MOE_RMW, MOE_RPLAIN };
int moe_router_path(const ggml_tensor * mm, bool pro);
bool moe_router_counters(exec_ctx & ctx);
bool moe_router(exec_ctx & ctx, ggml_tensor * mm, const ggml_tensor * sm, ggml_tensor * as, int n_used, float * wscr,
                const moe_router_pro * pro = nullptr);
bool moe_route_weights(exec_ctx & ctx, ggml_tensor * gr, ggml_tensor * sr, ggml_tensor * dv);
// out = experts[:, 0] * w0 + experts[:, 1] * w1 per token: the MUL by the routing weights and the ADD
// of its two slot views in one launch (k_elem.hip)
void moe_combine(exec_ctx & ctx, const ggml_tensor * mul, ggml_tensor * add, const float * wscr = nullptr);

// quantizes ncols rows of an f32 tensor (row i = (i1, i2, i3) flattened) into act
void quantize_act(exec_ctx & ctx, const ggml_tensor * src, bool k_quant, q8_act & act, int slot);
// fused epilogues of a grouped decode GEMV (k_gemv.hip), per matrix of the group
struct gemv_epi {
    ggml_tensor *  silu[3]     = {nullptr, nullptr, nullptr};   // UNARY SILU of the output
    void * const * f16out[3]   = {nullptr, nullptr, nullptr};   // dyn slot: f16 CPY of the output
    ggml_tensor *  rope[3]     = {nullptr, nullptr, nullptr};   // ROPE (NORM mode) of the output
    void * const * rope_f16[3] = {nullptr, nullptr, nullptr};   // dyn slot: f16 CPY of the rope
    // dead intermediates (read only by nodes this launch computes in registers, then
    // overwritten): not stored
    bool elide_dst[3]  = {false, false, false};   // the projection itself
    bool elide_rope[3] = {false, false, false};   // its rope (kept only as the f16 cache row)
    // residual producer (one matrix): x = out + rres stored to rxsum
    const float * rres = nullptr; float * rxsum = nullptr;
    // norm prologue: the activation is quant(RMS_NORM(px) [* pw]) (pkind 1), formed by every
    // workgroup of the launch (k_gemv.hip)
    int pkind = 0;
    const float * px = nullptr; const float * pw = nullptr;
    float peps = 0.0f; int64_t pn = 0;
};
bool gemv_supported(const ggml_tensor * mm);
bool gemv_epilogue_ok(const ggml_tensor * mm);   // the kernel path that carries epilogues applies
void gemv_group(exec_ctx & ctx, ggml_tensor * const * mms, int nmat, const gemv_epi * epi);
bool gemv_mixed_ok(const ggml_tensor * mm0, const ggml_tensor * c);   // c may join mm0's launch as a second weight type

// lays out a q8_act (qs | d | s, 256-B aligned) in `base`
void carve_act(q8_act & act, void * base, int64_t K, int64_t ncols, bool k_quant);

// fused producers (k_fused.hip); false = pattern not applicable, nothing launched
// store_norm / store_mul = false: that output is read by no later node (dispatch.cpp dead_after;
// the consuming mat-vecs take the quantized activation from the cache), so it is not written
// qkey: the tensor the quantized activation is cached under when the consumer `mm` reads a
// reshape of the chain's output (a MoE MUL_MAT_ID behind the router); nullptr = the output itself
// a deferred MoE combine as the first operand source of fused_norm's ADD: the experts'
// outputs e ([ne0, 2, T] contiguous), the routing weights w ([T][n_used]) and the slot-sum node
struct norm_combine { const float * e; const float * w; int n_used; const ggml_tensor * sum; };
bool fused_norm(exec_ctx & ctx, const ggml_tensor * add, ggml_tensor * norm, ggml_tensor * mul, const ggml_tensor * mm,
                bool store_norm = true, bool store_mul = true, const ggml_tensor * qkey = nullptr,
                const ggml_tensor * mm0 = nullptr, const struct norm_combine * comb = nullptr);
bool fused_mul_quant(exec_ctx & ctx, ggml_tensor * mul, const ggml_tensor * mm);
bool fused_silu_mul_quant(exec_ctx & ctx, ggml_tensor * silu, ggml_tensor * mul, const ggml_tensor * mm, bool store_silu,
                          bool store_mul = true);

void quantize_act_raw(hipStream_t stream, const float * x, int64_t K, int64_t ncols, int64_t row_stride_elems,
                      bool k_quant, q8_act & act);

}  // namespace mi355x
