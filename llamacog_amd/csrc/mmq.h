// mmq.h — shared argument block and types of the prefill MUL_MAT tiles (k_mmq.hip: the int8
// Q4_K tile for MUL_MAT_ID and the class-exact Q6_K / Q5_K tiles; k_mmq_f16.hip: the f16 Q4_K
// tile for MUL_MAT).
#pragma once

#include "ops.h"
#include "qtypes.h"

namespace mi355x {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void * lds_ptr_t;

struct mmq_args {
    const uint8_t * W; int64_t nb01; int64_t M; int64_t K; int64_t nblk;
    const int8_t * xq; const float * xd; const int16_t * xs;   // Q8_K SoA: [T][K], [T][K/256], [T][K/16]
    int64_t T;
    int64_t gemm_cols;          // tokens below this take the gemm (per-pair) order, the rest the gemv order
    float * dst; int64_t nb1;   // dst[t * nb1 + m*4]
    // MUL_MAT_ID (expert-sorted, k_mmv.hip k_moe_sort): blockIdx.z = expert, its cnt[z] tokens are
    // activation columns off[z] .. off[z] + cnt[z] - 1, column j is pair list[j] = e + n_used * t and
    // lands at dst + e * nb1 + t * nb2; nullptr cnt = a plain MUL_MAT
    const int32_t * cnt; const int32_t * off; const int32_t * list; int64_t n_used; int64_t nb02; int64_t nb2;
    int64_t ty0 = 0;            // k_mmq_q4Kh: first token tile of the grid
};

// the f16-operand Q4_K tile (k_mmq_f16.hip), 64-token workgroups of four waves
void launch_mmq_q4Kh(hipStream_t st, const mmq_args & p);

}  // namespace mi355x
