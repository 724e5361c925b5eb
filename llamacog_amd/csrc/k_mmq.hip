// k_mmq.hip — batched (prefill) quantized mat-mul on MFMA.  Placeholder gate: until the
// MFMA tile kernel lands every MUL_MAT goes through the column-grouped mat-vec path.
#include "ops.h"

namespace mi355x {

bool mmq_supported(const ggml_tensor * dst) {
    (void) dst;
    return false;
}

void mul_mat_q(exec_ctx & ctx, ggml_tensor * dst) {
    (void) ctx; (void) dst;
    GGML_ABORT("mi355x: mmq not built");
}

}  // namespace mi355x
