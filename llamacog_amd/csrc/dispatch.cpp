// dispatch.cpp — supports_op gate and per-node dispatch of the MI355X backend.
//
// supports_op (device vtable, ggml-backend-impl.h:172) decides what the reference's
// scheduler places on this device (ggml-backend.cpp:697-785); everything listed here is a
// hand-written HIP kernel in this directory.  op_compute is the body of graph_compute's
// node loop (the hot loop of SURVEY.md §3.1) and applies the fusions documented in
// DESIGN.md (RMS_NORM + MUL).
#include "ops.h"

namespace mi355x {

bool mmv_q_supported_type(ggml_type t);
void mul_mat_vec(exec_ctx & ctx, ggml_tensor * dst, const q8_act * pre);
bool mmq_supported(const ggml_tensor * dst);
void mul_mat_q(exec_ctx & ctx, ggml_tensor * dst);
bool fattn_supported(const ggml_tensor * op);

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
    if (s == GGML_TYPE_F32 && d == GGML_TYPE_Q8_0) {
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
        default:
            return false;
    }
}

void op_mul_mat(exec_ctx & ctx, ggml_tensor * dst) {
    if (mmq_supported(dst)) {
        mul_mat_q(ctx, dst);
    } else {
        mul_mat_vec(ctx, dst, nullptr);
    }
}

int op_compute(exec_ctx & ctx, ggml_cgraph * cgraph, int i) {
    ggml_tensor * node = ggml_graph_node(cgraph, i);
    if (ggml_is_empty(node)) return 1;
    const int n = ggml_graph_n_nodes(cgraph);
    switch (node->op) {
        case GGML_OP_NONE:
        case GGML_OP_RESHAPE:
        case GGML_OP_VIEW:
        case GGML_OP_PERMUTE:
        case GGML_OP_TRANSPOSE:
            return 1;
        case GGML_OP_MUL_MAT:
            op_mul_mat(ctx, node);
            return 1;
        case GGML_OP_GET_ROWS:
            op_get_rows(ctx, node);
            return 1;
        case GGML_OP_RMS_NORM: {
            // fuse y = rms_norm(x) * w when the next node is that MUL (build_norm,
            // src/llama-graph.cpp:464-497); the norm output is still written, so other
            // readers of it stay correct.
            if (i + 1 < n) {
                ggml_tensor * nx = ggml_graph_node(cgraph, i + 1);
                if (nx->op == GGML_OP_MUL && nx->src[0] == node && is_f32(nx->src[1]) &&
                    nx->src[1]->ne[0] == node->ne[0] && nx->src[1]->ne[1] == 1 && nx->src[1]->ne[2] == 1 &&
                    nx->src[1]->ne[3] == 1 && ggml_are_same_shape(nx, node) && node->nb[1] == nx->nb[1]) {
                    op_rms_norm(ctx, node, nx->src[1], nx);
                    return 2;
                }
            }
            op_rms_norm(ctx, node, nullptr, nullptr);
            return 1;
        }
        case GGML_OP_NORM:
            op_norm(ctx, node);
            return 1;
        case GGML_OP_ADD:
        case GGML_OP_SUB:
        case GGML_OP_MUL:
        case GGML_OP_DIV:
            op_binary(ctx, node);
            return 1;
        case GGML_OP_SCALE:
            op_scale(ctx, node);
            return 1;
        case GGML_OP_UNARY:
            op_unary(ctx, node);
            return 1;
        case GGML_OP_CPY:
            op_cpy(ctx, node->src[0], node->src[1]);
            return 1;
        case GGML_OP_DUP:
        case GGML_OP_CONT:
            op_cpy(ctx, node->src[0], node);
            return 1;
        case GGML_OP_ROPE:
            op_rope(ctx, node);
            return 1;
        case GGML_OP_SOFT_MAX:
            op_soft_max(ctx, node);
            return 1;
        case GGML_OP_FLASH_ATTN_EXT:
            op_flash_attn(ctx, node);
            return 1;
        default:
            GGML_ABORT("mi355x: op %s reached graph_compute but is not supported", ggml_op_desc(node));
    }
}

}  // namespace mi355x
