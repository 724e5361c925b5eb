// dispatch.cpp — supports_op gate and per-node dispatch of the MI355X backend.
//
// supports_op (device vtable, ggml-backend-impl.h:172) decides what the reference's
// scheduler places on this device (ggml-backend.cpp:697-785); everything listed here is a
// hand-written HIP kernel in this directory.  op_compute is the body of graph_compute's
// node loop (the hot loop of SURVEY.md §3.1) and applies the fusions documented in
// DESIGN.md (RMS_NORM + MUL).
#include "ops.h"
#include <atomic>
#include <mutex>

#include <algorithm>
#include <cstdio>

namespace mi355x {

bool mmv_q_supported_type(ggml_type t);
void mul_mat_vec(exec_ctx & ctx, ggml_tensor * dst, const q8_act * pre);
bool mmq_supported(const ggml_tensor * dst);
void mul_mat_q(exec_ctx & ctx, ggml_tensor * dst);

bool fattn_supported(const ggml_tensor * op);
bool mul_mat_id_supported(const ggml_tensor * op);

static bool is_f32(const ggml_tensor * t) { return t && t->type == GGML_TYPE_F32; }

static bool can_repeat(const ggml_tensor * s1, const ggml_tensor * s0) {
    for (int i = 0; i < 4; ++i) {
        if (s1->ne[i] == 0 || s0->ne[i] % s1->ne[i] != 0) return false;
    }
    return true;
}

static bool mul_mat_supported(const ggml_tensor * op) {
    const ggml_tensor * a = op->src[0];
    const ggml_tensor * b = op->src[1];
    if (!is_f32(b) || !is_f32(op)) return false;
    if (b->nb[0] != sizeof(float) || op->nb[0] != sizeof(float)) return false;
    if (a->ne[0] != b->ne[0]) return false;
    if (b->ne[2] % a->ne[2] != 0 || b->ne[3] % a->ne[3] != 0) return false;
    if (a->type == GGML_TYPE_F16 || a->type == GGML_TYPE_F32) {
        return a->nb[0] == ggml_type_size(a->type);
    }
    if (!mmv_q_supported_type(a->type)) return false;
    if (a->nb[0] != ggml_type_size(a->type)) return false;
    const bool kq = a->type == GGML_TYPE_Q4_K || a->type == GGML_TYPE_Q5_K || a->type == GGML_TYPE_Q6_K;
    if (a->ne[0] % (kq ? 256 : 32) != 0) return false;
    return true;
}

static bool cpy_supported(const ggml_tensor * src, const ggml_tensor * dst) {
    const ggml_type s = src->type, d = dst->type;
    if (ggml_nelements(src) != ggml_nelements(dst)) return false;
    if ((s == GGML_TYPE_F32 || s == GGML_TYPE_F16) && (d == GGML_TYPE_F32 || d == GGML_TYPE_F16)) return true;
    if (s == GGML_TYPE_I32 && d == GGML_TYPE_I32) return true;
    if (s == GGML_TYPE_F32 && (d == GGML_TYPE_Q8_0 || d == GGML_TYPE_Q4_0)) {
        // the KV-cache store: src Kcur [D, H, T] into a contiguous [H*D, T] view of the cache
        // (flat rows: op_cpy quantizes the element stream in 32-blocks).  With equal row lengths
        // op_cpy goes row by row, so each row must hold whole blocks (the CPU's dup-to-quant
        // asserts the same)
        if (ggml_is_contiguous(src) && ggml_is_contiguous(dst) && src->ne[0] != dst->ne[0]) return ggml_nelements(src) % 32 == 0;
        return src->ne[0] == dst->ne[0] && src->ne[0] % 32 == 0 && dst->nb[0] == ggml_type_size(d) &&
               ggml_nrows(src) == ggml_nrows(dst);
    }
    return false;
}

bool op_supported(const ggml_tensor * op) {
    switch (op->op) {
        case GGML_OP_NONE:
        case GGML_OP_RESHAPE:
        case GGML_OP_VIEW:
        case GGML_OP_PERMUTE:
        case GGML_OP_TRANSPOSE:
            return true;
        case GGML_OP_MUL_MAT:
            return mul_mat_supported(op);
        case GGML_OP_GET_ROWS: {
            const ggml_type t = op->src[0]->type;
            return (t == GGML_TYPE_F32 || t == GGML_TYPE_F16 || mmv_q_supported_type(t)) &&
                   op->src[1]->type == GGML_TYPE_I32 && is_f32(op);
        }
        case GGML_OP_RMS_NORM:
        case GGML_OP_NORM:
            return is_f32(op->src[0]) && is_f32(op) && op->src[0]->nb[0] == 4 && op->nb[0] == 4;
        case GGML_OP_ADD:
        case GGML_OP_SUB:
        case GGML_OP_MUL:
        case GGML_OP_DIV:
            return is_f32(op->src[0]) && is_f32(op->src[1]) && is_f32(op) && can_repeat(op->src[1], op->src[0]);
        case GGML_OP_SCALE:
            return is_f32(op->src[0]) && is_f32(op);
        case GGML_OP_UNARY:
            switch (ggml_get_unary_op(op)) {
                case GGML_UNARY_OP_SILU:
                case GGML_UNARY_OP_GELU:
                case GGML_UNARY_OP_GELU_ERF:
                case GGML_UNARY_OP_GELU_QUICK:
                case GGML_UNARY_OP_RELU:
                case GGML_UNARY_OP_NEG:
                case GGML_UNARY_OP_TANH:
                case GGML_UNARY_OP_SIGMOID:
                case GGML_UNARY_OP_EXP:
                case GGML_UNARY_OP_ABS:
                case GGML_UNARY_OP_SGN:
                case GGML_UNARY_OP_STEP:
                    return is_f32(op->src[0]) && is_f32(op);
                default:
                    return false;
            }
        case GGML_OP_CPY:
            return cpy_supported(op->src[0], op->src[1]);
        case GGML_OP_DUP:
        case GGML_OP_CONT:
            return cpy_supported(op->src[0], op);
        case GGML_OP_ROPE: {
            const int mode = op->op_params[2];
            if (mode != 0 && mode != 2) return false;   // NORM and NEOX
            return is_f32(op->src[0]) && is_f32(op) && op->src[1]->type == GGML_TYPE_I32 &&
                   (op->src[2] == nullptr || is_f32(op->src[2]));
        }
        case GGML_OP_SOFT_MAX: {
            const ggml_tensor * m = op->src[1];
            if (op->src[2] != nullptr) return false;
            if (m && !(m->type == GGML_TYPE_F32 || m->type == GGML_TYPE_F16)) return false;
            if (m && (m->ne[2] != 1 || m->ne[3] != 1)) return false;
            return is_f32(op->src[0]) && is_f32(op);
        }
        case GGML_OP_FLASH_ATTN_EXT:
            return fattn_supported(op);
        case GGML_OP_MUL_MAT_ID:
            return mul_mat_id_supported(op);
        case GGML_OP_ARGSORT:
            // the CPU's exchange order on one lane per row: router-sized rows (n_expert)
            return is_f32(op->src[0]) && op->type == GGML_TYPE_I32 && op->src[0]->nb[0] == 4 && op->src[0]->ne[0] <= 1024;
        case GGML_OP_SUM_ROWS:
            return is_f32(op->src[0]) && is_f32(op) && op->src[0]->nb[0] == 4;
        default:
            return false;
    }
}

void op_mul_mat(exec_ctx & ctx, ggml_tensor * dst) {
    if (gemv_supported(dst)) {
        ggml_tensor * one[1] = {dst};
        gemv_group(ctx, one, 1, nullptr);
    } else if (mmq_supported(dst)) {
        mul_mat_q(ctx, dst);
    } else {
        mul_mat_vec(ctx, dst, nullptr);
    }
}


// ---- row-split weights ------------------------------------------------------------------------
// One helper execution context per physical device for the slices that live on another GPU
// than the computing backend's (each has its own stream and scratch; enqueueing is serialised)
// ein[d]: recorded on device d's computing stream, waited on by the helper; eout: recorded on the
// helper stream, waited on by the computing stream.  Reused from slice to slice (a stream wait
// takes the event's most recent record at the time of the wait), so no event is created per
// slice and no host sync is needed: buffer reuse is ordered by the two streams' waits
struct split_helper { exec_ctx ex; std::mutex mtx; bool init = false; hipEvent_t eout = nullptr; hipEvent_t ein[MI_MAX_DEV] = {}; };
static split_helper g_split_helpers[MI_MAX_DEV];

static exec_ctx & split_helper_ctx(int hip, std::unique_lock<std::mutex> & lk) {
    GGML_ASSERT(hip >= 0 && hip < MI_MAX_DEV);
    split_helper & h = g_split_helpers[hip];
    lk = std::unique_lock<std::mutex>(h.mtx);
    if (!h.init) {
        MI_CHECK(hipSetDevice(hip));
        h.ex.device = hip;
        MI_CHECK(hipStreamCreateWithFlags(&h.ex.stream, hipStreamNonBlocking));
        MI_CHECK(hipEventCreateWithFlags(&h.eout, hipEventDisableTiming));
        h.init = true;
    }
    return h.ex;
}

// The mat-mul of one row slice [lo, hi) of a split weight against src1, into `out` (a
// contiguous [hi - lo, T] f32 block), on execution context ex (whose device holds the slice)
static void mul_mat_slice(exec_ctx & ex, const ggml_tensor * dst, const split_part & p, const ggml_tensor * src1, void * out) {
    const ggml_tensor * src0 = dst->src[0];
    ggml_tensor w = *src0;
    w.ne[1] = p.hi - p.lo;
    w.nb[2] = w.nb[3] = w.nb[1] * w.ne[1];
    w.data = p.data;
    w.buffer = nullptr;
    w.extra = nullptr;
    w.view_src = nullptr;
    ggml_tensor y = *dst;
    y.ne[0] = p.hi - p.lo;
    y.nb[1] = y.ne[0] * sizeof(float);
    y.nb[2] = y.nb[1] * y.ne[1];
    y.nb[3] = y.nb[2] * y.ne[2];
    y.data = out;
    y.buffer = nullptr;
    y.view_src = nullptr;
    y.src[0] = &w;
    y.src[1] = (ggml_tensor *) src1;
    op_mul_mat(ex, &y);
}

static std::atomic<long> g_split_mm{0}, g_split_foreign{0};
void split_stats(long * mm, long * foreign) {
    if (mm) *mm = g_split_mm.load();
    if (foreign) *foreign = g_split_foreign.load();
}

void op_mul_mat_split(exec_ctx & ctx, ggml_tensor * dst) {
    split_parts sp;
    GGML_ASSERT(tensor_split_parts(dst->src[0], sp));
    g_split_mm.fetch_add(1);
    const ggml_tensor * src1 = dst->src[1];
    GGML_ASSERT(ggml_is_contiguous(src1) && ggml_is_contiguous(dst) && dst->ne[2] == 1 && dst->ne[3] == 1);
    const int64_t T = dst->ne[1], M = dst->ne[0];
    int64_t maxr = 0;
    for (int i = 0; i < sp.n; ++i) maxr = std::max(maxr, sp.p[i].hi - sp.p[i].lo);
    char * tmp = (char *) ctx.scratch(5, (size_t) maxr * T * sizeof(float));
    for (int i = 0; i < sp.n; ++i) {
        const split_part & p = sp.p[i];
        const int64_t rows = p.hi - p.lo;
        if (p.hip == ctx.device) {
            // a slice in this device's memory (virtual devices of one GPU, or the main device's
            // own share): a one-token output is a contiguous run of dst, a batch is gathered
            if (T == 1) {
                mul_mat_slice(ctx, dst, p, src1, (float *) dst->data + p.lo);
            } else {
                mul_mat_slice(ctx, dst, p, src1, tmp);
                MI_CHECK(hipMemcpy2DAsync((char *) dst->data + p.lo * sizeof(float), M * sizeof(float), tmp, rows * sizeof(float),
                                          rows * sizeof(float), T, hipMemcpyDeviceToDevice, ctx.stream));
            }
            continue;
        }
        // a slice on another GPU: src1 over to it (peer copy), the slice computed there on its
        // helper stream, the rows back into this stream's staging, then gathered into dst
        g_split_foreign.fetch_add(1);
        std::unique_lock<std::mutex> lk;
        exec_ctx & hx = split_helper_ctx(p.hip, lk);
        split_helper & hh = g_split_helpers[p.hip];
        GGML_ASSERT(ctx.device >= 0 && ctx.device < MI_MAX_DEV);
        MI_CHECK(hipSetDevice(ctx.device));
        if (!hh.ein[ctx.device]) MI_CHECK(hipEventCreateWithFlags(&hh.ein[ctx.device], hipEventDisableTiming));
        hipEvent_t ein = hh.ein[ctx.device], eout = hh.eout;
        MI_CHECK(hipEventRecord(ein, ctx.stream));
        MI_CHECK(hipSetDevice(p.hip));
        MI_CHECK(hipStreamWaitEvent(hx.stream, ein, 0));
        const size_t b1 = ggml_nbytes(src1), bo = (size_t) rows * T * sizeof(float);
        char * hbuf = (char *) hx.scratch(5, b1 + bo + 256);
        MI_CHECK(hipMemcpyPeerAsync(hbuf, p.hip, src1->data, ctx.device, b1, hx.stream));
        ggml_tensor x = *src1;
        x.data = hbuf;
        x.buffer = nullptr;
        x.view_src = nullptr;
        hx.qcache_clear();
        mul_mat_slice(hx, dst, p, &x, hbuf + ((b1 + 255) / 256) * 256);
        MI_CHECK(hipMemcpyPeerAsync(tmp, ctx.device, hbuf + ((b1 + 255) / 256) * 256, p.hip, bo, hx.stream));
        MI_CHECK(hipEventRecord(eout, hx.stream));
        MI_CHECK(hipSetDevice(ctx.device));
        MI_CHECK(hipStreamWaitEvent(ctx.stream, eout, 0));
        // tmp is rewritten by the next foreign slice only after that slice's ein, recorded on
        // this stream behind the gather below
        MI_CHECK(hipMemcpy2DAsync((char *) dst->data + p.lo * sizeof(float), M * sizeof(float), tmp, rows * sizeof(float),
                                  rows * sizeof(float), T, hipMemcpyDeviceToDevice, ctx.stream));
    }
}

static ggml_tensor * at(ggml_cgraph * g, int i, int n) { return i < n ? ggml_graph_node(g, i) : nullptr; }

// the MUL by a norm weight row that directly follows RMS_NORM node i, or nullptr
static ggml_tensor * norm_weight_mul(ggml_cgraph * g, int i, int n) {
    ggml_tensor * node = ggml_graph_node(g, i);
    ggml_tensor * nx = at(g, i + 1, n);
    if (nx && nx->op == GGML_OP_MUL && nx->src[0] == node && is_f32(nx->src[1]) &&
        nx->src[1]->ne[0] == node->ne[0] && nx->src[1]->ne[1] == 1 && nx->src[1]->ne[2] == 1 &&
        nx->src[1]->ne[3] == 1 && ggml_are_same_shape(nx, node) && node->nb[1] == nx->nb[1]) {
        return nx;
    }
    return nullptr;
}

static bool overlaps(const ggml_tensor * a, const ggml_tensor * b) {
    if (!a || !b || !a->data || !b->data) return false;
    const char * a0 = (const char *) a->data, * a1 = a0 + ggml_nbytes(a);
    const char * b0 = (const char *) b->data, * b1 = b0 + ggml_nbytes(b);
    return a0 < b1 && b0 < a1;
}

// may node j run before the nodes i+1 .. j-1 (except those in `skip`)?  Its output must
// not touch anything those nodes read or write (ggml-alloc re-uses memory of tensors
// whose last consumer ran, so a later node's output can alias an earlier temporary).
static bool can_hoist(ggml_cgraph * g, int i, int j, const ggml_tensor * const * outs, int nout,
                      const std::vector<const ggml_tensor *> & skip) {
    for (int k = i + 1; k < j; ++k) {
        const ggml_tensor * t = ggml_graph_node(g, k);
        if (std::find(skip.begin(), skip.end(), t) != skip.end()) continue;
        // views / reshapes / permutes neither read nor write memory
        if (t->op == GGML_OP_NONE || t->op == GGML_OP_VIEW || t->op == GGML_OP_RESHAPE ||
            t->op == GGML_OP_PERMUTE || t->op == GGML_OP_TRANSPOSE) continue;
        for (int o = 0; o < nout; ++o) {
            if (overlaps(outs[o], t)) return false;
            for (int s = 0; s < GGML_MAX_SRC; ++s) {
                if (overlaps(outs[o], t->src[s])) return false;
            }
        }
    }
    return true;
}

// base node of a (chain of) view/reshape nodes
static const ggml_tensor * base_of(const ggml_tensor * t) {
    while (t && t->view_src) t = t->view_src;
    return t;
}

// index of `t` among the graph nodes, -1 for leaves (weights, inputs)
static int node_index(ggml_cgraph * g, const ggml_tensor * t) {
    const int n = ggml_graph_n_nodes(g);
    for (int k = 0; k < n; ++k) {
        if (ggml_graph_node(g, k) == t) return k;
    }
    return -1;
}

// has the data of `t` been produced when node i runs (earlier node, leaf, or hoisted)?
static bool computed_before(exec_ctx & ctx, ggml_cgraph * g, const ggml_tensor * t, int i) {
    const ggml_tensor * b = base_of(t);
    if (std::find(ctx.done.begin(), ctx.done.end(), b) != ctx.done.end()) return true;
    const int k = node_index(g, b);
    return k < i;
}

// the f32 -> f16 CPY (KV-cache store) of `out` within the next few nodes after position p:
// src is `out` itself or a contiguous reshape of it, destination contiguous f16 of the same
// size.  Returns the CPY node or nullptr.
static ggml_tensor * f16_store_of(ggml_cgraph * g, const ggml_tensor * out, int p, int n) {
    if (!ggml_is_contiguous(out) || out->type != GGML_TYPE_F32) return nullptr;
    for (int k = p + 1; k < n && k <= p + 12; ++k) {
        ggml_tensor * c = ggml_graph_node(g, k);
        if (c->op != GGML_OP_CPY) continue;
        const ggml_tensor * s = c->src[0];
        const bool same = s == out || (base_of(s) == out && s->data == out->data && ggml_is_contiguous(s));
        if (!same) continue;
        const ggml_tensor * d = c->src[1];
        if (d->type == GGML_TYPE_F16 && ggml_is_contiguous(d) && ggml_nelements(d) == ggml_nelements(out)) return c;
    }
    return nullptr;
}

// NORM-mode ROPE (one token) applied to the output of MUL_MAT `mm` within the next few
// nodes (through a contiguous reshape), or nullptr
static ggml_tensor * rope_of(ggml_cgraph * g, const ggml_tensor * mm, int p, int n) {
    for (int k = p + 1; k < n && k <= p + 4; ++k) {
        ggml_tensor * r = ggml_graph_node(g, k);
        if (r->op != GGML_OP_ROPE) continue;
        static const bool dbg = getenv("GGML_MI355X_DEBUG_FUSE") != nullptr;
        if (dbg) {
            const ggml_tensor * x = r->src[0];
            fprintf(stderr, "[mi355x] rope cand %s: base_ok=%d data_ok=%d contig=%d/%d mode=%d ne=%lld,%lld,%lld n_dims=%d\n",
                    r->name, base_of(x) == mm, x->data == mm->data, ggml_is_contiguous(x), ggml_is_contiguous(r),
                    r->op_params[2], (long long) x->ne[0], (long long) x->ne[1], (long long) x->ne[2], r->op_params[1]);
        }
        const ggml_tensor * x = r->src[0];
        if (base_of(x) != mm || x->data != mm->data || !ggml_is_contiguous(x) || !ggml_is_contiguous(r)) return nullptr;
        if (r->op_params[2] != 0 || r->type != GGML_TYPE_F32) return nullptr;   // NORM mode only
        const int n_dims = r->op_params[1];
        if (x->ne[2] != 1 || x->ne[3] != 1 || x->ne[0] % 2 != 0 || n_dims > x->ne[0] || n_dims % 2 != 0 || n_dims > 512) return nullptr;
        if (r->src[1]->type != GGML_TYPE_I32) return nullptr;
        return r;
    }
    return nullptr;
}

// does t overlap any of outs?  An exact alias of `self` (an in-place SiLU / ROPE that
// ggml-alloc placed in the projection's own buffer) is allowed: the epilogue writes the
// projection value and then the derived value to the same address from the same lane.
static bool overlaps_any(const ggml_tensor * t, const std::vector<const ggml_tensor *> & outs,
                         const ggml_tensor * self = nullptr) {
    for (const ggml_tensor * o : outs) {
        if (o == t) continue;
        if (o == self && t->data == self->data && ggml_nbytes(t) == ggml_nbytes(self)) continue;
        if (overlaps(t, o)) return true;
    }
    return false;
}

static bool f32c(const ggml_tensor * t) { return t && t->type == GGML_TYPE_F32 && ggml_is_contiguous(t); }

static bool is_view_op(const ggml_tensor * t) {
    return t->op == GGML_OP_NONE || t->op == GGML_OP_VIEW || t->op == GGML_OP_RESHAPE ||
           t->op == GGML_OP_PERMUTE || t->op == GGML_OP_TRANSPOSE;
}

// Is the memory of `t` (produced before node `from`) never read again except by `allowed`
// nodes (which this launch computes from registers), before a later node overwrites it?
// ggml-alloc re-uses a tensor's memory once its last consumer has run, so the first later
// node whose output overlaps `t` ends its life.  A graph output, or a tensor still live at
// the end of the graph (a later split may read it), is never dead.
static bool dead_after(ggml_cgraph * g, int n, int from, const ggml_tensor * t,
                       const std::vector<const ggml_tensor *> & allowed) {
    if (!t || (t->flags & GGML_TENSOR_FLAG_OUTPUT)) return false;
    for (int k = from; k < n; ++k) {
        const ggml_tensor * c = ggml_graph_node(g, k);
        if (is_view_op(c)) continue;
        const bool ok = std::find(allowed.begin(), allowed.end(), c) != allowed.end();
        if (!ok) {
            for (int s = 0; s < GGML_MAX_SRC; ++s) {
                if (c->src[s] && overlaps(c->src[s], t)) return false;
            }
        }
        if (overlaps(c, t)) return true;
    }
    return false;
}



// the next node after p that computes something (not a view), or n
static int next_compute(ggml_cgraph * g, int p, int n) {
    for (int k = p + 1; k < n; ++k) {
        if (!is_view_op(ggml_graph_node(g, k))) return k;
    }
    return n;
}

static void norm_stores(ggml_cgraph * g, int n, ggml_tensor * norm, ggml_tensor * mul, const ggml_tensor * mm,
                        bool & store_norm, bool & store_mul);

// GGML_MI355X_PROLOGUE=0: the norm chains run as their own launches (k_fused.hip)
static bool prologues_enabled() {
    static const bool on = !getenv("GGML_MI355X_PROLOGUE") || atoi(getenv("GGML_MI355X_PROLOGUE")) != 0;
    return on;
}

// Residual producer (k_gemv.hip): the single projection mm0 at node i is followed by
// ADD(mm0, res) -> RMS_NORM -> [MUL w] (the residual and the next norm, build_norm in
// src/llama-graph.cpp:464-497) whose only readers are decode mat-vecs.  The producer stores
// x = mm0 + res (mm0 itself is dead); every workgroup of the consumers' launch forms the norm
// from x in its prologue (k_gemv.hip), so neither the RMS_NORM nor the MUL runs as a node.
// Same-lane in-place aliases of mm0 / res by the ADD output are safe (each row is read before it
// is written).
static bool moe_router_nodes(ggml_cgraph * g, int i, int n, ggml_tensor ** psm, ggml_tensor ** pas);
static ggml_tensor * moe_quant_consumer(ggml_cgraph * g, int n, const ggml_tensor * out, const ggml_tensor * mm,
                                        const ggml_tensor ** qkey);

static void plan_resid(exec_ctx & ctx, ggml_cgraph * g, int i, int n, ggml_tensor * mm0, gemv_epi & epi,
                       std::vector<const ggml_tensor *> & absorbed) {
    const int pa = next_compute(g, i, n);
    ggml_tensor * ad = at(g, pa, n);
    if (!ad || ad->op != GGML_OP_ADD || !f32c(ad)) return;
    const ggml_tensor * res = ad->src[0] == mm0 ? ad->src[1] : (ad->src[1] == mm0 ? ad->src[0] : nullptr);
    if (!res || res == mm0 || !f32c(res) || !ggml_are_same_shape(res, mm0) || !ggml_are_same_shape(ad, mm0) ||
        !computed_before(ctx, g, res, i)) return;
    if (overlaps(ad, res) && ad->data != res->data) return;
    if (!dead_after(g, n, pa, mm0, {ad})) return;   // mm0 itself is not stored
    const int pn = next_compute(g, pa, n);
    ggml_tensor * nm = at(g, pn, n);
    if (!nm || nm->op != GGML_OP_RMS_NORM || nm->src[0] != ad || !f32c(nm) || nm->ne[0] % 256 != 0 || nm->ne[0] > 16384 ||
        ggml_nrows(nm) != 1) return;
    ggml_tensor * mul = norm_weight_mul(g, pn, n);
    if (mul && (!f32c(mul) || !ggml_is_contiguous(mul->src[1]))) return;
    ggml_tensor * last = mul ? mul : nm;
    ggml_tensor * mm = at(g, next_compute(g, node_index(g, last), n), n);
    if (!mm || mm->op != GGML_OP_MUL_MAT || mm->src[1] != last) return;
    if (!gemv_supported(mm)) {
        // the MoE FFN: the norm is formed by the router launch instead (try_moe_router)
        ggml_tensor * sm = nullptr, * as = nullptr;
        const ggml_tensor * qkey = nullptr;
        if (!mul || !moe_router_nodes(g, node_index(g, mm), n, &sm, &as) || nm->ne[0] % 1024 != 0 || nm->ne[0] > 4096) return;
        // the router kernel moe_router will pick must be one that forms the norm (k_elem.hip
        // moe_router_path); the counter kernel's arrival counters exist before the plan relies on them
        const int path = moe_router_path(mm, true);
        if (path == MOE_RNONE || (path == MOE_RMW && !moe_router_counters(ctx))) return;
        if (!dead_after(g, n, pn + 1, nm, {mul})) return;
        const ggml_tensor * c = moe_quant_consumer(g, n, last, mm, &qkey);
        if (c && !(c->src[0]->type == GGML_TYPE_Q4_K || c->src[0]->type == GGML_TYPE_Q5_K || c->src[0]->type == GGML_TYPE_Q6_K))
            qkey = nullptr;
        epi.rres = (const float *) res->data;
        epi.rxsum = (float *) ad->data;
        float eps;
        memcpy(&eps, nm->op_params, sizeof(float));
        ctx.moe_pro = {mm, (const float *) ad->data, (const float *) mul->src[1]->data, eps, qkey};
        absorbed.push_back(ad);
        absorbed.push_back(nm);
        absorbed.push_back(mul);
        return;
    }
    // every reader of the chain's output must be a decode mat-vec (each forms the activation in
    // its own prologue), and the norm output itself may be read only by the MUL
    std::vector<const ggml_tensor *> readers;
    const int pl = node_index(g, last);
    int64_t rows = 0;
    for (int k = pl + 1; k < n && k <= pl + 16; ++k) {
        const ggml_tensor * c = ggml_graph_node(g, k);
        if (c->op == GGML_OP_MUL_MAT && c->src[1] == last && gemv_supported(c)) {
            readers.push_back(c);
            rows += c->ne[0];
        }
    }
    // every consumer workgroup forms the norm: for wide consumers (the FFN gate/up, 28672 rows; the
    // output head) that is thousands of redundant norms, and the stand-alone norm kernel plus a
    // prologue-free launch measured faster (round 3 kernel timeline: gate/up 27.0 us with the
    // prologue vs 15 + 4 without); Q/K/V keep it
    static const long max_rows = getenv("GGML_MI355X_PRO_MAXROWS") ? atol(getenv("GGML_MI355X_PRO_MAXROWS")) : 16384;
    if (rows > max_rows) return;
    if (!dead_after(g, n, pl + 1, last, readers)) return;
    if (mul && !dead_after(g, n, pn + 1, nm, {mul})) return;
    epi.rres = (const float *) res->data;
    epi.rxsum = (float *) ad->data;
    float eps;
    memcpy(&eps, nm->op_params, sizeof(float));
    ctx.pro = {last, last->data, 1, (const float *) ad->data, mul ? (const float *) mul->src[1]->data : nullptr, eps, nm->ne[0]};
    absorbed.push_back(ad);
    absorbed.push_back(nm);
    if (mul) absorbed.push_back(mul);
}

// RMS_NORM (node i) of an x computed before -> [MUL w] whose only readers are decode mat-vecs
// and whose outputs nothing else reads (the first layer's attention norm of the embedding): the
// readers' launch forms it in its activation prologue (k_gemv.hip), no norm launch
static bool plan_norm_prologue(exec_ctx & ctx, ggml_cgraph * g, int i, int n) {
    ggml_tensor * nm = ggml_graph_node(g, i);
    const ggml_tensor * x = nm->src[0];
    if (!f32c(nm) || !f32c(x) || !ggml_are_same_shape(nm, x) || nm->ne[0] % 256 != 0 || nm->ne[0] > 16384 || ggml_nrows(nm) != 1)
        return false;
    ggml_tensor * mul = norm_weight_mul(g, i, n);
    if (mul && (!f32c(mul) || !ggml_is_contiguous(mul->src[1]))) return false;
    ggml_tensor * last = mul ? mul : nm;
    const int pl = node_index(g, last);
    ggml_tensor * mm = at(g, next_compute(g, pl, n), n);
    if (!mm || mm->op != GGML_OP_MUL_MAT || mm->src[1] != last || !gemv_supported(mm)) return false;
    std::vector<const ggml_tensor *> readers;
    for (int k = pl + 1; k < n && k <= pl + 16; ++k) {
        const ggml_tensor * c = ggml_graph_node(g, k);
        if (c->op == GGML_OP_MUL_MAT && c->src[1] == last && gemv_supported(c)) readers.push_back(c);
    }
    if (!dead_after(g, n, pl + 1, last, readers)) return false;
    if (mul && !dead_after(g, n, i + 1, nm, {mul})) return false;
    // x stays live past the readers (the residual ADD reads it), so no reader output overlaps it
    if (dead_after(g, n, pl + 1, x, {})) return false;
    float eps;
    memcpy(&eps, nm->op_params, sizeof(float));
    ctx.pro = {last, last->data, 1, (const float *) x->data, mul ? (const float *) mul->src[1]->data : nullptr, eps, nm->ne[0]};
    return true;
}

// decode mat-vec: launch node i together with up to two later MUL_MATs on the same src1
// (Q/K/V, gate/up) in one grouped kernel, with fused epilogues: the SiLU that follows a
// projection, the NORM-mode ROPE of a projection, and f16 KV-cache stores (CPY) of a
// projection or of its rope.  Every hoisted node's outputs are checked against what the
// skipped-over nodes read and write, and against the other outputs of the launch.
int op_gemv_grouped(exec_ctx & ctx, ggml_cgraph * g, int i, int n) {
    ggml_tensor * mm0 = ggml_graph_node(g, i);
    ggml_tensor * mms[3] = {mm0, nullptr, nullptr};
    gemv_epi epi;
    int nm = 1;
    // the activation of a pending prologue (planned at its producer chain)
    if (ctx.pro.last && ctx.pro.last == mm0->src[1] && ctx.pro.data == mm0->src[1]->data) {
        epi.pkind = ctx.pro.kind;
        epi.px = ctx.pro.x; epi.pw = ctx.pro.w; epi.peps = ctx.pro.eps; epi.pn = ctx.pro.n;
    }
    std::vector<const ggml_tensor *> absorbed;   // nodes this launch computes (besides node i)
    std::vector<const ggml_tensor *> outs = {mm0};

    // epilogues of matrix m (node position pm): rope (+ its cache store), or a cache store.  (The
    // SiLU of a gate projection is left to the FFN-product kernel, op_compute GGML_OP_UNARY, which
    // forms silu(gate)*up in one pass: as an epilogue it parked the row sums and cost the 66 MB
    // gate/up launch ~2 us, round 2)
    auto add_epilogues = [&](int m, int pm) {
        ggml_tensor * mm = mms[m];
        if (ggml_tensor * r = rope_of(g, mm, pm, n)) {
            const ggml_tensor * o[1] = {r};
            const int pr = node_index(g, r);
            if (!overlaps_any(r, outs, mm) && can_hoist(g, i, pr, o, 1, absorbed)) {
                epi.rope[m] = r;
                absorbed.push_back(r);
                outs.push_back(r);
                if (ggml_tensor * c = f16_store_of(g, r, pr, n)) {
                    void * const * slot = ctx.dyn_slot(c);
                    const ggml_tensor * oc[1] = {c->src[1]};
                    if (slot && !overlaps_any(c->src[1], outs) && can_hoist(g, i, node_index(g, c), oc, 1, absorbed)) {
                        epi.rope_f16[m] = slot;
                        absorbed.push_back(c);
                        outs.push_back(c->src[1]);
                    }
                }
            }
            return;
        }
        if (ggml_tensor * c = f16_store_of(g, mm, pm, n)) {
            void * const * slot = ctx.dyn_slot(c);
            const ggml_tensor * oc[1] = {c->src[1]};
            if (slot && !overlaps_any(c->src[1], outs) && can_hoist(g, i, node_index(g, c), oc, 1, absorbed)) {
                epi.f16out[m] = slot;
                absorbed.push_back(c);
                outs.push_back(c->src[1]);
            }
        }
    };
    // a projection (or its rope) read only by this launch's register epilogues is not stored,
    // and no longer constrains which other projections may join the launch
    auto settle = [&](int m, int pm) {
        if (dead_after(g, n, pm + 1, mms[m], absorbed)) {
            epi.elide_dst[m] = true;
            outs.erase(std::remove(outs.begin(), outs.end(), (const ggml_tensor *) mms[m]), outs.end());
        }
        if (epi.rope[m] && epi.rope_f16[m] && dead_after(g, n, node_index(g, epi.rope[m]) + 1, epi.rope[m], absorbed)) {
            epi.elide_rope[m] = true;
            outs.erase(std::remove(outs.begin(), outs.end(), (const ggml_tensor *) epi.rope[m]), outs.end());
        }
    };
    add_epilogues(0, i);
    settle(0, i);

    for (int j = i + 1; j < n && j <= i + 12 && nm < 3; ++j) {
        ggml_tensor * c = ggml_graph_node(g, j);
        if (c->op != GGML_OP_MUL_MAT || c->src[1] != mm0->src[1] || !gemv_supported(c)) continue;
        if (std::find(ctx.done.begin(), ctx.done.end(), c) != ctx.done.end()) continue;
        if (c->src[0]->ne[0] != mm0->src[0]->ne[0]) continue;
        if (c->src[0]->type != mm0->src[0]->type) {
            // a second K-quant type (V beside Q/K) joins as the launch's second body, one type
            // besides mm0's at most
            bool ok = gemv_mixed_ok(mm0, c);
            for (int m = 1; m < nm; ++m) {
                const ggml_type tm = mms[m]->src[0]->type;
                ok = ok && (tm == mm0->src[0]->type || tm == c->src[0]->type);
            }
            if (!ok) continue;
        }
        const ggml_tensor * o[1] = {c};
        if (overlaps_any(c, outs) || !can_hoist(g, i, j, o, 1, absorbed)) {
            static const bool dbg = getenv("GGML_MI355X_DEBUG_FUSE") != nullptr;
            if (dbg) {
                fprintf(stderr, "[mi355x] group %s + %s rejected: overlap=%d hoist=%d", mm0->name, c->name,
                        overlaps_any(c, outs), can_hoist(g, i, j, o, 1, absorbed));
                for (const ggml_tensor * t : outs) if (overlaps(c, t)) fprintf(stderr, " [overlaps %s]", t->name);
                for (int k = i + 1; k < j; ++k) {
                    const ggml_tensor * t = ggml_graph_node(g, k);
                    if (std::find(absorbed.begin(), absorbed.end(), t) != absorbed.end()) continue;
                    bool hit = overlaps(c, t);
                    for (int s2 = 0; s2 < GGML_MAX_SRC; ++s2) hit = hit || overlaps(c, t->src[s2]);
                    if (hit && t->op != GGML_OP_VIEW && t->op != GGML_OP_RESHAPE && t->op != GGML_OP_PERMUTE &&
                        t->op != GGML_OP_TRANSPOSE && t->op != GGML_OP_NONE) fprintf(stderr, " [hoist blocked by %s %s]", ggml_op_name(t->op), t->name);
                }
                fprintf(stderr, "\n");
            }
            continue;
        }
        mms[nm] = c;
        absorbed.push_back(c);
        outs.push_back(c);
        add_epilogues(nm, j);
        settle(nm, j);
        ++nm;
    }
    static const bool dbg = getenv("GGML_MI355X_DEBUG_FUSE") != nullptr;
    if (dbg) {
        fprintf(stderr, "[mi355x] gemv @%d %s: nmat=%d", i, mm0->name, nm);
        for (int m = 0; m < nm; ++m) {
            fprintf(stderr, " | %s silu=%d rope=%d rope_f16=%d f16=%d elide=%d/%d", mms[m]->name, epi.silu[m] != nullptr,
                    epi.rope[m] != nullptr, epi.rope_f16[m] != nullptr, epi.f16out[m] != nullptr, epi.elide_dst[m], epi.elide_rope[m]);
        }
        fprintf(stderr, "\n");
    }
    // the next norm chain moves into this launch (residual producer) and its consumers
    // (prologue).  GGML_MI355X_RESID=0 runs the chain as its own launch (k_fused.hip)
    static const bool resid = !getenv("GGML_MI355X_RESID") || atoi(getenv("GGML_MI355X_RESID")) != 0;
    bool plain = true;
    for (int m = 0; m < nm; ++m) {
        plain = plain && !epi.silu[m] && !epi.rope[m] && !epi.f16out[m] && !epi.rope_f16[m] && !epi.elide_dst[m];
    }
    if (resid && prologues_enabled() && plain && nm == 1) plan_resid(ctx, g, i, n, mm0, epi, absorbed);
    if (dbg && (epi.rres || epi.px)) fprintf(stderr, "[mi355x]   resid=%d prologue=%d\n", epi.rres != nullptr, epi.px != nullptr);
    gemv_group(ctx, mms, nm, &epi);
    // node i+1 when it is node i's SiLU is consumed here; everything else is skipped later
    const bool next_absorbed = epi.silu[0] && epi.silu[0] == at(g, i + 1, n);
    for (const ggml_tensor * t : absorbed) {
        if (!(next_absorbed && t == epi.silu[0])) ctx.done.push_back(t);
    }
    return next_absorbed ? 2 : 1;
}

// ROPE of Q at node i + ROPE of K (same parameters and positions, input already computed)
// in one launch, each with its f16 KV-cache store fused when present
static int op_rope_grouped(exec_ctx & ctx, ggml_cgraph * g, int i, int n) {
    ggml_tensor * r0 = ggml_graph_node(g, i);
    ggml_tensor * nodes[2] = {r0, nullptr};
    void * const * cache[2] = {nullptr, nullptr};
    std::vector<const ggml_tensor *> absorbed;
    int nr = 1;
    for (int j = i + 1; j < n && j <= i + 6; ++j) {
        ggml_tensor * c = ggml_graph_node(g, j);
        if (c->op != GGML_OP_ROPE) continue;
        if (c->src[1] != r0->src[1] || c->src[2] != r0->src[2] || memcmp(c->op_params, r0->op_params, 15 * sizeof(int32_t)) != 0) break;
        if (c->src[0]->ne[0] != r0->src[0]->ne[0] || !computed_before(ctx, g, c->src[0], i)) break;
        const ggml_tensor * outs[1] = {c};
        if (!can_hoist(g, i, j, outs, 1, absorbed)) break;
        nodes[nr++] = c;
        absorbed.push_back(c);
        break;
    }
    for (int k = 0; k < nr; ++k) {
        ggml_tensor * c = f16_store_of(g, nodes[k], node_index(g, nodes[k]), n);
        if (!c) continue;
        void * const * slot = ctx.dyn_slot(c);
        const ggml_tensor * outs[1] = {c->src[1]};
        if (!slot || !can_hoist(g, i, node_index(g, c), outs, 1, absorbed)) continue;
        cache[k] = slot;
        absorbed.push_back(c);
    }
    op_rope_multi(ctx, nodes, nr, cache);
    for (const ggml_tensor * t : absorbed) ctx.done.push_back(t);
    return 1;
}

// A MoE FFN norm feeds the f32 router first; the expert MUL_MAT_ID behind it reads a reshape of
// the same output: quantize for that consumer instead (qkey = the reshape), so it needs no
// quantize launch of its own
static ggml_tensor * moe_quant_consumer(ggml_cgraph * g, int n, const ggml_tensor * out, const ggml_tensor * mm,
                                        const ggml_tensor ** qkey) {
    // the router may follow the norm behind views (build_moe_ffn reshapes cur for the experts
    // first, src/llama-graph.cpp:682)
    if (mm && is_view_op(mm)) {
        const int lim = node_index(g, mm) + 4;
        for (int k = node_index(g, mm); mm && is_view_op(mm) && k < lim;) mm = at(g, ++k, n);
    }
    if (!mm || mm->op != GGML_OP_MUL_MAT || mm->src[1] != out || mmv_q_supported_type(mm->src[0]->type)) return nullptr;
    const int p = node_index(g, mm);
    for (int k = p + 1; k < n && k <= p + 16; ++k) {
        ggml_tensor * c = ggml_graph_node(g, k);
        if (c->op != GGML_OP_MUL_MAT_ID) continue;
        const ggml_tensor * b = c->src[1];
        if (base_of(b) == base_of(out) && b->data == out->data && ggml_is_contiguous(b) && ggml_nelements(b) == ggml_nelements(out)) {
            *qkey = b;
            return c;
        }
        return nullptr;
    }
    return nullptr;
}

// a later MUL_MAT reading the same output `out` with another weight type than the first reader
// mm (Mixtral: Q8_0 attn_k / attn_v after the Q5_K attn_q), or nullptr
static const ggml_tensor * other_type_reader(ggml_cgraph * g, int n, const ggml_tensor * out, const ggml_tensor * mm) {
    if (!mm || mm->op != GGML_OP_MUL_MAT || mm->src[1] != out) return nullptr;
    const int p = node_index(g, mm);
    for (int k = p + 1; k < n && k <= p + 12; ++k) {
        const ggml_tensor * c = ggml_graph_node(g, k);
        if (c->op == GGML_OP_MUL_MAT && c->src[1] == out && c->src[0]->type != mm->src[0]->type) return c;
    }
    return nullptr;
}

// which outputs of a fused [ADD] -> RMS_NORM -> [MUL] chain feeding mat-vec `mm` must be stored:
// the norm output when something other than the MUL reads it; the last output when something
// other than the decode mat-vecs that consume it through the quantized-activation cache reads it
static void norm_stores(ggml_cgraph * g, int n, ggml_tensor * norm, ggml_tensor * mul, const ggml_tensor * mm,
                        bool & store_norm, bool & store_mul) {
    store_norm = store_mul = true;
    const int pn = node_index(g, norm);
    const ggml_tensor * last = mul ? mul : norm;
    if (mul) store_norm = !dead_after(g, n, pn + 1, norm, {mul});
    if (!mm || mm->op != GGML_OP_MUL_MAT || mm->src[1] != last || !gemv_supported(mm)) return;
    std::vector<const ggml_tensor *> readers;
    const int pm = node_index(g, mm);
    for (int k = pm; k < n && k <= pm + 12; ++k) {
        const ggml_tensor * c = ggml_graph_node(g, k);
        if (c->op == GGML_OP_MUL_MAT && c->src[1] == last && gemv_supported(c) &&
            c->src[0]->type == mm->src[0]->type && c->src[0]->ne[0] == mm->src[0]->ne[0]) readers.push_back(c);
    }
    const bool dead = dead_after(g, n, node_index(g, last) + 1, last, readers);
    if (mul) store_mul = !dead; else store_norm = !dead;
}

// The MoE router (build_moe_ffn, src/llama-graph.cpp:661-712) in two launches instead of five.
// At the SOFT_MAX: the ARGSORT (DESC, ggml_top_k) of its output follows after views only.  At the
// GET_ROWS of the probabilities by the top-k view: SUM_ROWS and the DIV follow after views only
// (the expert mat-muls lie between the two halves in graph order).
static bool try_moe_sort(exec_ctx & ctx, ggml_cgraph * g, int i, int n) {
    ggml_tensor * sm = ggml_graph_node(g, i);
    float max_bias = 0.0f;
    memcpy(&max_bias, (const float *) sm->op_params + 1, sizeof(float));
    if (sm->src[1] || sm->src[2] || max_bias != 0.0f || !f32c(sm) || !f32c(sm->src[0])) return false;
    for (int j = i + 1; j < n && j <= i + 4; ++j) {
        ggml_tensor * c = ggml_graph_node(g, j);
        if (is_view_op(c)) continue;
        if (c->op == GGML_OP_ARGSORT && c->src[0] == sm && c->op_params[0] == GGML_SORT_ORDER_DESC &&
            c->type == GGML_TYPE_I32 && moe_route_sort(ctx, sm, c)) {
            ctx.done.push_back(c);
            return true;
        }
        return false;
    }
    return false;
}

// The expert outputs weighted and summed (build_moe_ffn :761-777, n_used = 2): MUL(experts,
// weights) followed, after views only, by the ADD of its two slot views: that ADD, or nullptr.
// The MUL output is never stored, so only that ADD may read it.
static ggml_tensor * moe_combine_sum(ggml_cgraph * g, int i, int n) {
    ggml_tensor * mul = ggml_graph_node(g, i);
    const ggml_tensor * e = mul->src[0], * w = mul->src[1];
    if (mul->op != GGML_OP_MUL || !f32c(mul) || !f32c(e) || !w || w->type != GGML_TYPE_F32 || mul->ne[1] != 2 || w->ne[0] != 1 ||
        w->ne[1] != 2 || w->ne[2] != mul->ne[2] || mul->ne[3] != 1 || !ggml_are_same_shape(mul, e)) return nullptr;
    for (int j = i + 1; j < n && j <= i + 6; ++j) {
        ggml_tensor * c = ggml_graph_node(g, j);
        if (is_view_op(c)) continue;
        if (c->op != GGML_OP_ADD || !f32c(c) || base_of(c->src[0]) != mul || base_of(c->src[1]) != mul) return nullptr;
        const ggml_tensor * v0 = c->src[0], * v1 = c->src[1];
        if (v0->data != mul->data || (const char *) v1->data != (const char *) mul->data + mul->nb[1]) return nullptr;
        if (v0->ne[0] != mul->ne[0] || v0->ne[1] != mul->ne[2] || v0->nb[1] != mul->nb[2] || v1->nb[1] != mul->nb[2] ||
            c->ne[0] != mul->ne[0] || c->ne[1] != mul->ne[2]) return nullptr;
        if (!dead_after(g, n, i + 1, mul, {c}) || overlaps(c, e) || overlaps(c, w)) return nullptr;
        return c;
    }
    return nullptr;
}

// the combine as its own launch, or — after the fused router (ctx.moe) — deferred into the
// residual ADD -> RMS_NORM launch that is the only reader of its slot sum (k_norm_fused's
// combine source: the sum is never stored)
static bool try_moe_combine(exec_ctx & ctx, ggml_cgraph * g, int i, int n) {
    ggml_tensor * mul = ggml_graph_node(g, i);
    const bool routed = ctx.moe.mul == mul;
    ggml_tensor * c = moe_combine_sum(g, i, n);
    if (!c) {
        GGML_ASSERT(!routed);   // try_moe_router checked this same pattern
        return false;
    }
    ctx.done.push_back(c);
    if (routed) {
        const ggml_tensor * e = mul->src[0];
        const int ir = next_compute(g, node_index(g, c), n);
        const ggml_tensor * r = at(g, ir, n);
        const ggml_tensor * nx = at(g, ir + 1, n);
        const bool dense = e->nb[1] == (size_t) e->ne[0] * sizeof(float) && e->nb[2] == 2 * e->nb[1];
        if (dense && r && r->op == GGML_OP_ADD && (r->src[0] == c || r->src[1] == c) && nx && nx->op == GGML_OP_RMS_NORM &&
            nx->src[0] == r && dead_after(g, n, node_index(g, c) + 1, c, {r}) &&
            std::find(ctx.done.begin(), ctx.done.end(), r) == ctx.done.end() &&
            c->ne[1] == 1) {   // one token: one workgroup reads e before any output is stored
            ctx.moe.comb = c;
            ctx.moe.e = (const float *) e->data;
            return true;
        }
    }
    moe_combine(ctx, mul, c, routed ? ctx.moe.wn : nullptr);
    if (routed) ctx.moe = {};
    return true;
}

// a deferred combine (ctx.moe.comb) whose consumer did not take it: launch it now
static void flush_moe_combine(exec_ctx & ctx) {
    if (!ctx.moe.comb) return;
    moe_combine(ctx, ctx.moe.mul, (ggml_tensor *) ctx.moe.comb, ctx.moe.wn);
    ctx.moe = {};
}

// The MoE router in one launch (k_moe_router): at the router's f32 MUL_MAT, its SOFT_MAX and the
// ARGSORT (ggml_top_k) follow after views only.  When the GET_ROWS of the probabilities by the
// top-k, its SUM_ROWS and DIV are read by nothing but the combine MUL, those three are formed in
// the same launch into a private scratch and skipped at their own nodes; the combine reads it.
// the router MUL_MAT at node i (f32 gate_inp, at most 16 experts) and its SOFT_MAX / ARGSORT
static bool moe_router_nodes(ggml_cgraph * g, int i, int n, ggml_tensor ** psm, ggml_tensor ** pas) {
    ggml_tensor * mm = ggml_graph_node(g, i);
    if (mm->op != GGML_OP_MUL_MAT || mm->src[0]->type != GGML_TYPE_F32 || mm->src[0]->ne[1] > 16) return false;
    const int is = next_compute(g, i, n);
    ggml_tensor * sm = at(g, is, n);
    if (!sm || sm->op != GGML_OP_SOFT_MAX || sm->src[0] != mm || sm->src[1] || sm->src[2]) return false;
    float max_bias = 0.0f;
    memcpy(&max_bias, (const float *) sm->op_params + 1, sizeof(float));
    if (max_bias != 0.0f || !f32c(sm)) return false;
    ggml_tensor * as = at(g, next_compute(g, is, n), n);
    if (!as || as->op != GGML_OP_ARGSORT || as->src[0] != sm || as->op_params[0] != GGML_SORT_ORDER_DESC || as->type != GGML_TYPE_I32)
        return false;
    *psm = sm;
    *pas = as;
    return true;
}

static bool try_moe_router(exec_ctx & ctx, ggml_cgraph * g, int i, int n) {
    ggml_tensor * mm = ggml_graph_node(g, i);
    ggml_tensor * sm = nullptr, * as = nullptr;
    const bool pro = ctx.moe_pro.mm == mm;
    if (!moe_router_nodes(g, i, n, &sm, &as)) {
        GGML_ASSERT(!pro);   // plan_resid's MoE branch checked this same pattern
        return false;
    }
    const int ia = node_index(g, as);
    // the weights chain and its combine
    ggml_tensor * gr = nullptr, * sr = nullptr, * dv = nullptr, * mul = nullptr;
    for (int k = ia + 1; k < n && k <= ia + 48 && !gr; ++k) {
        ggml_tensor * c = ggml_graph_node(g, k);
        if (c->op == GGML_OP_GET_ROWS && base_of(c->src[0]) == sm && base_of(c->src[1]) == as) gr = c;
    }
    if (gr) {
        const int k1 = next_compute(g, node_index(g, gr), n);
        sr = at(g, k1, n);
        if (sr && sr->op == GGML_OP_SUM_ROWS && base_of(sr->src[0]) == gr && sr->type == GGML_TYPE_F32) {
            dv = at(g, next_compute(g, k1, n), n);
            if (!dv || dv->op != GGML_OP_DIV || base_of(dv->src[0]) != gr || dv->src[1] != sr || dv->type != GGML_TYPE_F32) dv = nullptr;
        } else {
            sr = nullptr;
        }
    }
    if (dv) {
        const int id = node_index(g, dv);
        for (int k = id + 1; k < n && k <= id + 8; ++k) {
            ggml_tensor * c = ggml_graph_node(g, k);
            if (is_view_op(c)) continue;
            if (c->op == GGML_OP_MUL && base_of(c->src[1]) == dv && moe_combine_sum(g, k, n)) mul = c;
            break;
        }
    }
    const int64_t T = mm->src[1]->ne[1];
    const int n_used = gr ? (int) gr->ne[1] : 0;
    const bool chain = mul && n_used == 2 && gr->ne[0] == 1 && gr->ne[2] == T && ggml_is_contiguous(gr) &&
                       dead_after(g, n, node_index(g, gr) + 1, gr, {sr, dv}) &&
                       dead_after(g, n, node_index(g, sr) + 1, sr, {dv}) &&
                       dead_after(g, n, node_index(g, dv) + 1, dv, {mul});
    float * wscr = chain ? (float *) ctx.scratch(exec_ctx::MOE_SLOT, 3 * T * n_used * sizeof(float)) : nullptr;
    if (pro) {
        // the FFN norm formed in this launch (plan_resid's MoE branch): its output stored, its Q8_K
        // quantization cached for the expert mat-vecs
        const int64_t K = mm->src[1]->ne[0];
        q8_act act;
        carve_act(act, ctx.scratch(exec_ctx::QSLOT, q8_act::bytes(K, 1, true)), K, 1, true);
        const moe_router_pro rp = {ctx.moe_pro.x, ctx.moe_pro.w, ctx.moe_pro.eps, ctx.moe_pro.qkey ? &act : nullptr};
        GGML_ASSERT(moe_router(ctx, mm, sm, as, n_used, wscr, &rp));
        if (ctx.moe_pro.qkey) ctx.qcache_put(ctx.moe_pro.qkey, true, act);
        ctx.moe_pro = {};
    } else if (!moe_router(ctx, mm, sm, as, n_used, wscr)) {
        return false;
    }
    ctx.done.push_back(sm);
    ctx.done.push_back(as);
    if (chain) {
        ctx.done.push_back(gr);
        ctx.done.push_back(sr);
        ctx.done.push_back(dv);
        ctx.moe = {mul, wscr + 2 * T * n_used, n_used, nullptr, nullptr};
    }
    return true;
}

static bool try_moe_weights(exec_ctx & ctx, ggml_cgraph * g, int i, int n) {
    ggml_tensor * gr = ggml_graph_node(g, i);
    const ggml_tensor * pb = base_of(gr->src[0]), * ib = base_of(gr->src[1]);
    if (!pb || !ib || pb->op != GGML_OP_SOFT_MAX || ib->op != GGML_OP_ARGSORT || gr->type != GGML_TYPE_F32) return false;
    ggml_tensor * sr = nullptr, * dv = nullptr;
    for (int j = i + 1; j < n && j <= i + 6; ++j) {
        ggml_tensor * c = ggml_graph_node(g, j);
        if (is_view_op(c)) continue;
        if (!sr && c->op == GGML_OP_SUM_ROWS && base_of(c->src[0]) == gr && c->type == GGML_TYPE_F32) { sr = c; continue; }
        if (sr && c->op == GGML_OP_DIV && base_of(c->src[0]) == gr && c->src[1] == sr && c->type == GGML_TYPE_F32) dv = c;
        break;
    }
    if (!sr || !dv || !moe_route_weights(ctx, gr, sr, dv)) return false;
    ctx.done.push_back(sr);
    ctx.done.push_back(dv);
    return true;
}

int op_compute(exec_ctx & ctx, ggml_cgraph * cgraph, int i) {
    ggml_tensor * node = ggml_graph_node(cgraph, i);
    if (ctx.silu_defer && node != ctx.silu_mul && !is_view_op(node)) {
        bool reads = false;
        for (int k = 0; k < GGML_MAX_SRC; ++k) reads = reads || (node->src[k] && overlaps(node->src[k], ctx.silu_defer));
        if (reads || overlaps(node, ctx.silu_defer) || overlaps(node, ctx.silu_defer->src[0])) {
            op_unary(ctx, ctx.silu_defer);   // something else needs it now: run it stand-alone
            ctx.silu_defer = ctx.silu_mul = nullptr;
        }
    }
    if (ctx.moe.comb && !is_view_op(node) && node != ctx.moe.comb &&
        !(node->op == GGML_OP_ADD && (node->src[0] == ctx.moe.comb || node->src[1] == ctx.moe.comb))) {
        flush_moe_combine(ctx);   // something else runs before the residual ADD that takes it
    }
    if (ggml_is_empty(node)) return 1;
    if (!ctx.done.empty()) {
        auto it = std::find(ctx.done.begin(), ctx.done.end(), node);
        if (it != ctx.done.end()) {   // already computed by a grouped launch
            ctx.done.erase(it);
            return 1;
        }
    }
    const int n = ggml_graph_n_nodes(cgraph);
    if (debug_ops() && !is_view_op(node))
        fprintf(stderr, "[ops] %d %s %s (%s%s%s)\n", i, ggml_op_desc(node), node->name, node->src[0] ? ggml_type_name(node->src[0]->type) : "-",
                node->src[1] ? " " : "", node->src[1] ? node->src[1]->name : "");
    switch (node->op) {
        case GGML_OP_NONE:
        case GGML_OP_RESHAPE:
        case GGML_OP_VIEW:
        case GGML_OP_PERMUTE:
        case GGML_OP_TRANSPOSE:
            return 1;
        case GGML_OP_MUL_MAT: {
            split_parts sp;
            if (tensor_split_parts(node->src[0], sp)) {   // -sm row weights
                op_mul_mat_split(ctx, node);
                return 1;
            }
        }
            if (fusion_enabled() && gemv_supported(node)) return op_gemv_grouped(ctx, cgraph, i, n);
            if (fusion_enabled() && try_moe_router(ctx, cgraph, i, n)) return 1;
            op_mul_mat(ctx, node);
            return 1;
        case GGML_OP_GET_ROWS:
            if (fusion_enabled() && try_moe_weights(ctx, cgraph, i, n)) return 1;
            op_get_rows(ctx, node);
            return 1;
        case GGML_OP_RMS_NORM: {
            // fuse y = rms_norm(x) * w when the next node is that MUL (build_norm,
            // src/llama-graph.cpp:464-497); the norm output is still written, so other
            // readers of it stay correct.
            ggml_tensor * mul = norm_weight_mul(cgraph, i, n);
            if (fusion_enabled() && prologues_enabled() && plan_norm_prologue(ctx, cgraph, i, n)) return mul ? 2 : 1;
            if (fusion_enabled()) {
                ggml_tensor * mm = at(cgraph, i + (mul ? 2 : 1), n);
                bool sn, sm;
                norm_stores(cgraph, n, node, mul, mm, sn, sm);
                const ggml_tensor * qkey = nullptr;
                if (ggml_tensor * c = moe_quant_consumer(cgraph, n, mul ? mul : node, mm, &qkey)) mm = c;
                const ggml_tensor * mm0 = other_type_reader(cgraph, n, mul ? mul : node, mm);
                if (fused_norm(ctx, nullptr, node, mul, mm, sn, sm, qkey, mm0)) return mul ? 2 : 1;
            }
            op_rms_norm(ctx, node, mul ? mul->src[1] : nullptr, mul);
            return mul ? 2 : 1;
        }
        case GGML_OP_NORM:
            op_norm(ctx, node);
            return 1;
        case GGML_OP_ADD: {
            // a deferred MoE combine whose slot sum is an operand here
            norm_combine nc = {};
            const norm_combine * pc = nullptr;
            if (ctx.moe.comb && (node->src[0] == ctx.moe.comb || node->src[1] == ctx.moe.comb)) {
                nc = {ctx.moe.e, ctx.moe.wn, ctx.moe.n_used, ctx.moe.comb};
                pc = &nc;
            }
            // residual ADD feeding the next RMS_NORM (+ norm-weight MUL, + MUL_MAT input)
            if (fusion_enabled()) {
                ggml_tensor * nx = at(cgraph, i + 1, n);
                if (nx && nx->op == GGML_OP_RMS_NORM && nx->src[0] == node) {
                    ggml_tensor * mul = norm_weight_mul(cgraph, i + 1, n);
                    const int used = mul ? 3 : 2;
                    ggml_tensor * mm = at(cgraph, i + used, n);
                    bool sn, sm;
                    norm_stores(cgraph, n, nx, mul, mm, sn, sm);
                    const ggml_tensor * qkey = nullptr;
                    if (ggml_tensor * c = moe_quant_consumer(cgraph, n, mul ? mul : nx, mm, &qkey)) mm = c;
                    static const bool dbga = getenv("GGML_MI355X_DEBUG_ALIAS") != nullptr;
                    if (dbga) {
                        const ggml_tensor * last = mul ? mul : nx;
                        fprintf(stderr, "[alias] @%d add=%s a=%s res=%s: add==a %d add==res %d norm~a %d norm~res %d mul~norm %d |", i, node->name,
                                node->src[0]->name, node->src[1]->name, node->data == node->src[0]->data, node->data == node->src[1]->data,
                                overlaps(nx, node->src[0]), overlaps(nx, node->src[1]), mul && mul->data == nx->data);
                        for (int k = i + used; k < n && k < i + used + 14; ++k) {
                            const ggml_tensor * c = ggml_graph_node(cgraph, k);
                            if (is_view_op(c)) continue;
                            const bool r = overlaps(c, node->src[0]) || overlaps(c, node->src[1]) || overlaps(c, node) || overlaps(c, last);
                            fprintf(stderr, " %s:%s%s", ggml_op_name(c->op), c->name, r ? "[ALIAS]" : "");
                        }
                        fprintf(stderr, "\n");
                    }
                    const ggml_tensor * mm0 = other_type_reader(cgraph, n, mul ? mul : nx, mm);
                    if (fused_norm(ctx, node, nx, mul, mm, sn, sm, qkey, mm0, pc)) {
                        if (pc) ctx.moe = {};
                        return used;
                    }
                }
            }
            flush_moe_combine(ctx);
            op_binary(ctx, node);
            return 1;
        }
        case GGML_OP_MUL:
            if (ctx.silu_defer && node == ctx.silu_mul) {
                ggml_tensor * sl = ctx.silu_defer;
                ctx.silu_defer = ctx.silu_mul = nullptr;
                ggml_tensor * mm = at(cgraph, i + 1, n);
                const bool smul = !(mm && (mm->op == GGML_OP_MUL_MAT || mm->op == GGML_OP_MUL_MAT_ID) &&
                                    dead_after(cgraph, n, i + 1, node, {mm}));
                if (fused_silu_mul_quant(ctx, sl, node, mm, false, smul)) return 1;
                op_unary(ctx, sl);
                op_binary(ctx, node);
                return 1;
            }
            if (fusion_enabled() && try_moe_combine(ctx, cgraph, i, n)) return 1;
            // gated-FFN product feeding the down projection: multiply + quantize in one pass
            if (fusion_enabled()) {
                if (fused_mul_quant(ctx, node, at(cgraph, i + 1, n))) return 1;
            }
            op_binary(ctx, node);
            return 1;
        case GGML_OP_SUB:
        case GGML_OP_DIV:
            op_binary(ctx, node);
            return 1;
        case GGML_OP_SCALE:
            op_scale(ctx, node);
            return 1;
        case GGML_OP_UNARY:
            // gated FFN: SILU(gate) -> MUL(., up) -> MUL_MAT down in one pass that also quantizes
            // the down projection's input (src/llama-graph.cpp:555-616 LLM_FFN_SILU + PAR)
            // (graph order is gate, SILU, up, MUL: the up projection ran in the gate's grouped
            // launch, so the MUL is hoisted over it when nothing in between is touched)
            if (fusion_enabled() && ggml_get_unary_op(node) == GGML_UNARY_OP_SILU) {
                const ggml_tensor * between = nullptr;   // one node computing the MUL's other input
                for (int j = i + 1; j < n && j <= i + 4; ++j) {
                    ggml_tensor * c = ggml_graph_node(cgraph, j);
                    if (c->op == GGML_OP_MUL && c->src[0] == node && c->src[1] != node) {
                        if (between && base_of(c->src[1]) == between && dead_after(cgraph, n, i + 1, node, {c}) &&
                            !overlaps(between, node) && !overlaps(between, node->src[0])) {
                            // MoE order (gate, SILU, up, MUL): the SILU waits for the MUL
                            ctx.silu_defer = node;
                            ctx.silu_mul = c;
                            return 1;
                        }
                        const ggml_tensor * o[1] = {c};
                        const std::vector<const ggml_tensor *> skip(ctx.done.begin(), ctx.done.end());
                        if (!computed_before(ctx, cgraph, c->src[1], i) || !can_hoist(cgraph, i, j, o, 1, skip)) break;
                        ggml_tensor * mm = at(cgraph, j + 1, n);
                        const bool ssilu = !dead_after(cgraph, n, i + 1, node, {c});
                        const bool smul = !(mm && (mm->op == GGML_OP_MUL_MAT || mm->op == GGML_OP_MUL_MAT_ID) &&
                                            dead_after(cgraph, n, j + 1, c, {mm}));
                        if (fused_silu_mul_quant(ctx, node, c, mm, ssilu, smul)) {
                            if (j == i + 1) return 2;
                            ctx.done.push_back(c);
                            return 1;
                        }
                        break;
                    }
                    if (is_view_op(c) || std::find(ctx.done.begin(), ctx.done.end(), c) != ctx.done.end()) continue;
                    // a projection that reads neither the SILU nor writes its input may run first
                    bool reads = false;
                    for (int k = 0; k < GGML_MAX_SRC; ++k) reads = reads || (c->src[k] && base_of(c->src[k]) == node);
                    if (between || reads || (c->op != GGML_OP_MUL_MAT && c->op != GGML_OP_MUL_MAT_ID)) break;
                    between = c;
                }
            }
            op_unary(ctx, node);
            return 1;
        case GGML_OP_CPY:
            op_cpy(ctx, node->src[0], node->src[1], node);
            return 1;
        case GGML_OP_DUP:
        case GGML_OP_CONT:
            op_cpy(ctx, node->src[0], node, nullptr);
            return 1;
        case GGML_OP_ROPE:
            if (fusion_enabled()) return op_rope_grouped(ctx, cgraph, i, n);
            op_rope(ctx, node);
            return 1;
        case GGML_OP_SOFT_MAX:
            if (fusion_enabled() && try_moe_sort(ctx, cgraph, i, n)) return 1;
            op_soft_max(ctx, node);
            return 1;
        case GGML_OP_MUL_MAT_ID:
            // MoE gate and up of the same routed slots (graph order gate, SILU, up,
            // build_moe_ffn :727-741) in one launch
            if (fusion_enabled()) {
                ggml_tensor * up = nullptr;
                int j = i + 1;
                for (; j < n && j <= i + 4; ++j) {
                    ggml_tensor * c = ggml_graph_node(cgraph, j);
                    if (is_view_op(c) || (c->op == GGML_OP_UNARY && c->src[0] == node)) continue;
                    if (c->op == GGML_OP_MUL_MAT_ID && c->src[1] == node->src[1] && c->src[2] == node->src[2]) up = c;
                    break;
                }
                const ggml_tensor * o[1] = {up};
                const std::vector<const ggml_tensor *> skip(ctx.done.begin(), ctx.done.end());
                if (up && !overlaps(up, node) && can_hoist(cgraph, i, j, o, 1, skip) && op_mul_mat_id_pair(ctx, node, up)) {
                    ctx.done.push_back(up);
                    return 1;
                }
            }
            op_mul_mat_id(ctx, node);
            return 1;
        case GGML_OP_ARGSORT:
            op_argsort(ctx, node);
            return 1;
        case GGML_OP_SUM_ROWS:
            op_sum_rows(ctx, node);
            return 1;
        case GGML_OP_FLASH_ATTN_EXT: {
            // attention output -> reshape -> output projection: quantize in the FA epilogue
            const ggml_tensor * mm = nullptr;
            if (fusion_enabled()) {
                ggml_tensor * r = at(cgraph, i + 1, n);
                ggml_tensor * c = at(cgraph, i + 2, n);
                if (r && c && (r->op == GGML_OP_RESHAPE || r->op == GGML_OP_VIEW) && r->view_src == node &&
                    r->data == node->data && ggml_is_contiguous(r) && c->op == GGML_OP_MUL_MAT && c->src[1] == r &&
                    (gemv_supported(c) || mmq_supported(c))) {   // decode mat-vec / prefill MFMA tile
                    mm = c;
                }
            }
            op_flash_attn(ctx, node, mm);
            return 1;
        }
        default:
            GGML_ABORT("mi355x: op %s reached graph_compute but is not supported", ggml_op_desc(node));
    }
}

}  // namespace mi355x
