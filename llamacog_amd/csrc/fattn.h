// fattn.h — shared argument block of the flash-attention kernels (k_fattn.hip: split-K
// f32 kernel; k_fattn_exact.hip: the CPU-exact f16 kernel).
#pragma once

#include "ops.h"

namespace mi355x {

struct fa_args {
    const char * q; int64_t nbq1, nbq2, nbq3;
    const char * k; int64_t nbk1, nbk2, nbk3;
    const char * v; int64_t nbv1, nbv2, nbv3;
    const char * mask; int64_t nbm1; int64_t mask_ne1;
    int k_type, v_type;
    int64_t D, n_kv, n_q, H, Hkv, chunk;
    float scale, softcap, max_bias, m0, m1; uint32_t n_head_log2;
    float * part;      // [nchunks][n_q][H][D+2]  (M, S, O[D])
    float * dst;       // final output when nchunks == 1
    int64_t nb1_dst, nb2_dst;
    int nchunks;
    // fused quantization of the output for the following MUL_MAT (exact kernel only):
    // qmode 0 none, 1 Q8_K, 2 Q8_0 over the flat [n_q][H*D] output rows
    int qmode;
    int8_t * qs; float * qd; int16_t * qsum;
    // per-Q8_K-block arrival counters of the fused output quantization (zeroed, self-resetting)
    int * cnt;
    // microbenchmark hook: per-phase s_memtime cycles of workgroup (0,0) (nullable)
    unsigned long long * prof;
    // in-graph kernel timeline region (common.h kt_enter / kt_exit; nullable)
    unsigned long long * kt;
};

// the FLASH_ATTN_EXT node's arguments (and the quantization of its output for the output
// projection mm, act); op_flash_attn launches them
void fa_args_of(exec_ctx & ctx, ggml_tensor * dst, const ggml_tensor * mm, fa_args & a, q8_act & act, int64_t & nq3);

// set by mi355x_bench_op (capi.cpp) only; copied into fa_args.prof
extern unsigned long long * g_fa_prof;


// launch the CPU-exact f16 kernel (k_fattn_exact.hip); D in {64, 128, 256}
void launch_fattn_exact(hipStream_t stream, const fa_args & a, int64_t nq3);
// decode, D = 128, f16 cache: two heads per workgroup, scores produced under the recurrence
// (4 chain waves + 2 or 4 producer waves per head: four above FA_DEC2_NQ4_MIN cache positions)
constexpr int FA_DEC2_NQ4_MIN = 256;
int fattn_dec2_threads(const fa_args & a);   // the launch's workgroup size (timeline slots)
bool fattn_dec2_ok(const fa_args & a, int64_t nq3);
// decode, D = 128, f16 cache of at most 256 positions (tg128's depths): every load issued at the
// launch's start, two heads (one KV head) per 512-thread workgroup (GGML_MI355X_FA_DSH=0: dec2)
bool fattn_dsh_ok(const fa_args & a, int64_t nq3);
void launch_fattn_dsh(hipStream_t stream, const fa_args & a, int64_t nq3);
// the prefill batch tile (k_fattn_pf) runs this batch and can quantize its output (qmode 1):
// f16 cache, D = 128, a GQA group of 4, 8 or 16 heads
bool fattn_pf_quant_ok(const fa_args & a);
void launch_fattn_dec2(hipStream_t stream, const fa_args & a, int64_t nq3);
void fattn_scores_d128(hipStream_t st, const float * q, const uint16_t * k, int64_t n, float * s);
// long-context decode (D = 128): the scores of every position by a (position block x KV head)
// grid into sco [H][n_kv], then one chain workgroup per head (coefficients of all positions in
// LDS, V streamed by stager waves); from FA_LONG_MIN cached positions (GGML_MI355X_FA_LONG)
constexpr int FAL_THREADS = 256;   // the long-context chain kernel: wave 0 the recurrence, 1-3 stage V
constexpr int FAL_PB = 128;        // positions per scores workgroup (k_fal_scores)
constexpr int FAL_DSPLIT = 2;      // chain workgroups per head (each DH = 128 / FAL_DSPLIT of its dims)
constexpr int FA_LONG_MIN = 512;     // f16 cache
constexpr int FA_LONG_MIN_Q = 384;   // q8_0 / q4_0 cache
bool fattn_long_ok(const fa_args & a, int64_t nq3);
void launch_fattn_long(hipStream_t stream, const fa_args & a, float * sco, unsigned long long * kt_scores);

}  // namespace mi355x
