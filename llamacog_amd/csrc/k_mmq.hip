// k_mmq.hip — batched (prefill) Q4_K MUL_MAT on MFMA (v_mfma_i32_16x16x32_i8), in the CPU
// backend's exact float order.
//
// libllama keeps Q4_K weights with M % 8 == 0 in the CPU_REPACK buffer; for a batch the CPU
// runs ggml_gemm_q4_K_8x8_q8_K (arch/x86/repack.cpp:1771) on the tokens in whole groups of
// four and ggml_gemv_q4_K_8x8_q8_K (:718) on the last T % 4 (repack.cpp:1261-1274).  The gemm
// accumulates once per PAIR of sub-blocks:
//   A = fma(I_pair, d·dy, A),  B = fma(Imin_pair, dmin·dy, B)   pairs in K order, result A - B,
// the gemv once per block (I and Imin summed over the block's pairs).  The activations are the
// CPU's Q8_K (the gemm's 4x8 quantizer differs only in the sign of equal-magnitude maxima,
// which flips qs, d and bsums together and leaves every product unchanged; qtypes.h).
//
// The integer dot of a 32-element chunk of 16 weight rows x 16 tokens is one MFMA; the 6-bit
// sub-block scales multiply the int32 results in VALU (24-bit multiplies: |MFMA result| <=
// 32*15*127 < 2^23), pairs and mins are exact integers, and every float step is the CPU's.
//
// Tiling (MI355X): a 256-thread workgroup owns 64 weight rows x 64 tokens; per 256-element K
// block the 64 rows' quant blocks and the 64 tokens' Q8_K rows are staged in LDS (two stages:
// block b+1 loads while block b computes), each wave computes 16 rows x 64 tokens (four 16x16
// MFMA tiles sharing the A fragment).  MFMA layouts (verified by tools/mfma_layout.hip): lane l
// holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15]; C[row 4(l>>4)+i][col l&15].
#include "ops.h"

namespace mi355x {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void * lds_ptr_t;

constexpr int MQ_BM = 64, MQ_BN = 64;

// Q4_K weight block: per-row sub-scales and mins, and the A fragment of 32-element chunk c
// (0..7), k = 8h .. 8h+7 (h = lane>>4)
struct mq_q4_K {
    static constexpr int BLK = 144, NSC = 8;
    __device__ static void unpack(const uint8_t * b, int * sc, int * mn, float & d, float & dmin) {
        d = h2f(ld2(b)); dmin = h2f(ld2(b + 2));
        const uint8_t * q = b + 4;
        for (int j = 0; j < 8; ++j) {
            int s, m;
            scale_min_k4(j, q, s, m);
            sc[j] = s; mn[j] = m;
        }
    }
    __device__ static long afrag(const uint8_t * b, int c, int h) {
        // chunk c = 2g + hi: qs[32g + k] low (hi = 0) or high nibbles
        const uint2 v = ld8(b + 16 + 32 * (c >> 1) + 8 * h);
        const int sh = 4 * (c & 1);
        const uint32_t lo = (v.x >> sh) & 0x0f0f0f0f, hi = (v.y >> sh) & 0x0f0f0f0f;
        return (long) lo | ((long) hi << 32);
    }
};

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
};

// Staging: the loads of K block b+1 are in flight while block b computes: the Q8_K token rows,
// their scales d and bsums go HBM -> LDS by global_load_lds into the other of two stages, the
// weight blocks go to registers and are written to that stage after the MFMA work.  One
// s_waitcnt + barrier per block then finds the next stage landed.
// The token tile is XOR-swizzled in LDS: the 16-byte chunk k of token row t sits in slot
// k ^ (t & 15), so the 16 lanes of an MFMA B fragment (rows t = 16n + c16, same chunk) read 16
// different bank groups instead of one (rows are 256 B = one bank period apart).  The swizzle
// is applied on the source side of the LDS-DMA (each lane picks which chunk it fetches).
template <class W> struct mq_stage {
    static constexpr int RS = (W::BLK + 15) / 16 * 16;
    static constexpr int XQ = MQ_BM * RS;            // token rows [64][256] after the weight tile
    static constexpr int XD = XQ + MQ_BN * 256;      // token scales [64] f32
    static constexpr int XS = XD + MQ_BN * 4;        // token bsums [64][16] i16
    static constexpr int BYTES = XS + MQ_BN * 32;
    static constexpr int RC = RS / 16;               // 16-byte chunks per weight row
    static constexpr int NWR = (MQ_BM * RC + 255) / 256;   // weight chunks per thread
};

// two workgroups per CU (two stages of ~56 KB LDS each)
template <class W>
__global__ __launch_bounds__(256, 2) void k_mmq_q4K(const mmq_args p) {
    using S = mq_stage<W>;
    constexpr int RS = S::RS;
    __shared__ __attribute__((aligned(16))) uint8_t st[2][S::BYTES];
    __shared__ int wsc[MQ_BM][W::NSC];
    __shared__ __attribute__((aligned(8))) int wmn[MQ_BM][8];
    __shared__ float wd[MQ_BM], wdm[MQ_BM];
    __shared__ __attribute__((aligned(8))) int xs[MQ_BN][8];   // Q8_K sums per 32-element chunk

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t row0 = (int64_t) blockIdx.x * MQ_BM;
    const int64_t tok0 = (int64_t) blockIdx.y * MQ_BN;
    const int h = lane >> 4, c16 = lane & 15;
    const uint8_t * Wb = p.W;
    int64_t T = p.T, col0 = 0;
    if (p.cnt) {
        T = p.cnt[blockIdx.z];
        if (tok0 >= T) return;   // uniform: no barrier passed yet
        col0 = p.off[blockIdx.z];
        Wb = p.W + (int64_t) blockIdx.z * p.nb02;
    }
    const int64_t KB = p.K / 256;
    // per token tile n: does this lane's token take the gemm (per-pair) order?
    bool gemm[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) gemm[n] = tok0 + 16 * n + c16 < p.gemm_cols;

    // per-thread source pointers of block 0 (block b adds b * 256 / b / b * 16 / b * BLK)
    const int8_t * xsrc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {   // token rows: instruction i = wave + 4k of 16
        const int c = 64 * (wave + 4 * k) + lane, t = c >> 4, part = (c & 15) ^ (t & 15);   // LDS slot (t, c & 15) holds chunk (c & 15) ^ (t & 15)
        xsrc[k] = p.xq + (col0 + min(tok0 + t, T - 1)) * p.K + 16 * part;
    }
    const float * dsrc = p.xd + (col0 + min(tok0 + lane, T - 1)) * KB;
    const int16_t * ssrc;
    {
        const int c = 64 * (wave == 2 ? 1 : 0) + lane, t = c >> 1, half = c & 1;
        ssrc = p.xs + (col0 + min(tok0 + t, T - 1)) * (p.K / 16) + 8 * half;
    }
    const uint8_t * wsrc[S::NWR];
#pragma unroll
    for (int j = 0; j < S::NWR; ++j) {
        const int c = min(tid + 256 * j, MQ_BM * S::RC - 1);
        const int r = c / S::RC, k = c % S::RC;
        wsrc[j] = Wb + min(row0 + r, p.M - 1) * p.nb01 + 16 * k;
    }
    // token-side loads of block b into stage s (LDS-DMA: 1 KiB, or 256 B, per wave instruction)
    auto issue_x = [&](int64_t b, int s) {
        uint8_t * base = st[s];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            __builtin_amdgcn_global_load_lds((const void *) (xsrc[k] + b * 256), (lds_ptr_t) (base + S::XQ + 1024 * (wave + 4 * k)), 16, 0, 0);
        }
        if (wave == 0) {   // scales: one 4-byte load per token
            __builtin_amdgcn_global_load_lds((const void *) (dsrc + b), (lds_ptr_t) (base + S::XD), 4, 0, 0);
        } else if (wave <= 2) {   // bsums: 32 B per token, two instructions
            __builtin_amdgcn_global_load_lds((const void *) (ssrc + b * 16), (lds_ptr_t) (base + S::XS + 1024 * (wave - 1)), 16, 0, 0);
        }
    };
    uint4 wr[S::NWR];
    auto load_w = [&](int64_t b) {
#pragma unroll
        for (int j = 0; j < S::NWR; ++j) {
            if (tid + 256 * j < MQ_BM * S::RC) wr[j] = ld16(wsrc[j] + b * W::BLK);
        }
    };
    auto store_w = [&](int s) {
#pragma unroll
        for (int j = 0; j < S::NWR; ++j) {
            const int c = tid + 256 * j;
            if (c < MQ_BM * S::RC) *(uint4 *) (st[s] + c * 16) = wr[j];   // row r, chunk k at r * RS + 16 k = 16 c
        }
    };

    // the CPU's two fp32 chains per output (qtypes.h g_q4_K_p)
    float A[4][4], B[4][4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) A[n][i] = B[n][i] = 0.0f;

    issue_x(0, 0);
    load_w(0);
    store_w(0);
    for (int64_t b = 0; b < p.nblk; ++b) {
        const int s = (int) (b & 1);
        const uint8_t * wq = st[s];
        const int8_t * xq = (const int8_t *) (st[s] + S::XQ);
        const float * xd = (const float *) (st[s] + S::XD);
        // stage s has landed for every wave, and block b-1's reads of stage s^1 are done
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const bool more = b + 1 < p.nblk;
        if (more) {
            issue_x(b + 1, s ^ 1);
            load_w(b + 1);
        }
        // ---- per-row scales and per-token chunk sums of block b ----------------------------
        if (tid < MQ_BM) {
            int sc[16], mn[8];
            float d, dmin;
            W::unpack(wq + tid * RS, sc, mn, d, dmin);
#pragma unroll
            for (int j = 0; j < W::NSC; ++j) wsc[tid][j] = sc[j];
#pragma unroll
            for (int j = 0; j < 8; ++j) wmn[tid][j] = mn[j];
            wd[tid] = d; wdm[tid] = dmin;
        } else if (tid < MQ_BM + MQ_BN) {
            const int t = tid - MQ_BM;
            const int16_t * s16 = (const int16_t *) (st[s] + S::XS) + 16 * t;
#pragma unroll
            for (int j = 0; j < 8; ++j) xs[t][j] = s16[2 * j] + s16[2 * j + 1];
        }
        __syncthreads();
        // scale products d·dy and dmin·dy of this lane's 4 rows x 4 tokens, as the CPU forms them
        float dw[4], dmw[4], dy[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { dw[i] = wd[16 * wave + 4 * h + i]; dmw[i] = wdm[16 * wave + 4 * h + i]; }
#pragma unroll
        for (int n = 0; n < 4; ++n) dy[n] = xd[16 * n + c16];
        int ib[4][4], mb[4][4];   // block sums of the gemv (tail) tokens
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) ib[n][i] = mb[n][i] = 0;
        const int rA = 16 * wave + c16;
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {   // sub-block pairs
            int ip[4][4];
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int i = 0; i < 4; ++i) ip[n][i] = 0;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int c = 2 * k + u;
                const long a = W::afrag(wq + rA * RS, c, h);
                int scv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) scv[i] = wsc[16 * wave + 4 * h + i][c];
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const long bf = *(const long *) (xq + (16 * n + c16) * 256 + 16 * ((2 * c + (h >> 1)) ^ c16) + 8 * (h & 1));
                    v4i r = {0, 0, 0, 0};
                    r = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, bf, r, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) ip[n][i] += __mul24(r[i], scv[i]);
                }
            }
            // the pair's mins integer m_2k·bsum_2k + m_2k+1·bsum_2k+1 (exact)
            int2 mr[4], xt[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) mr[i] = *(const int2 *) &wmn[16 * wave + 4 * h + i][2 * k];
#pragma unroll
            for (int n = 0; n < 4; ++n) xt[n] = *(const int2 *) &xs[16 * n + c16][2 * k];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int mn = __mul24(mr[i].x, xt[n].x) + __mul24(mr[i].y, xt[n].y);
                    if (gemm[n]) {
                        A[n][i] = fmaf((float) ip[n][i], dw[i] * dy[n], A[n][i]);
                        B[n][i] = fmaf((float) mn, dmw[i] * dy[n], B[n][i]);
                    } else {
                        ib[n][i] += ip[n][i];
                        mb[n][i] += mn;
                    }
                }
            }
        }
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            if (gemm[n]) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                A[n][i] = fmaf((float) ib[n][i], dw[i] * dy[n], A[n][i]);
                B[n][i] = fmaf((float) mb[n][i], dmw[i] * dy[n], B[n][i]);
            }
        }
        // block b+1's weights into the other stage (its readers, block b-1, passed the barrier)
        if (more) store_w(s ^ 1);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
        const int64_t t = tok0 + 16 * n + c16;
        if (t >= T) continue;
        char * drow = (char *) p.dst + t * p.nb1;
        if (p.cnt) {
            const int pair = p.list[col0 + t];
            drow = (char *) p.dst + (pair % p.n_used) * p.nb1 + (pair / p.n_used) * p.nb2;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t m = row0 + 16 * wave + 4 * h + i;
            if (m < p.M) *(float *) (drow + m * 4) = __fsub_rn(A[n][i], B[n][i]);
        }
    }
}

// ---- host --------------------------------------------------------------------------------------
// Q4_K weights with M % 8 == 0 (the repacked order) and a batch of >= 16 tokens
bool mmq_supported(const ggml_tensor * dst) {
    static const bool off = getenv("GGML_MI355X_NO_MMQ") && atoi(getenv("GGML_MI355X_NO_MMQ")) != 0;
    if (off) return false;
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    if (w->type != GGML_TYPE_Q4_K || w->ne[1] % 8 != 0) return false;
    if (x->type != GGML_TYPE_F32 || dst->type != GGML_TYPE_F32) return false;
    if (w->ne[2] != 1 || w->ne[3] != 1 || x->ne[2] != 1 || x->ne[3] != 1) return false;
    if (x->ne[1] < 16) return false;             // small batches stay on the mat-vec path
    if (w->ne[0] % 256 != 0 || x->nb[0] != 4 || dst->nb[0] != 4) return false;
    return true;
}

void mul_mat_q(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    hipEvent_t ev = nullptr;
    const double flops = 2.0 * (double) w->ne[0] * (double) w->ne[1] * (double) x->ne[1];
    if (ctx.timing) ctx.time_begin(TK_MMQ, flops, ev);
    q8_act act;
    if (!ctx.qcache_get(x, true, act)) {
        quantize_act(ctx, x, true, act, exec_ctx::QSLOT);
        ctx.qcache_put(x, true, act);
    }
    mmq_args p;
    p.W = (const uint8_t *) w->data; p.nb01 = w->nb[1]; p.M = w->ne[1]; p.K = w->ne[0]; p.nblk = w->ne[0] / 256;
    p.xq = act.qs; p.xd = act.d; p.xs = act.s;
    p.T = x->ne[1];
    p.gemm_cols = p.T - p.T % 4;   // repack.cpp:1261-1274
    p.dst = (float *) dst->data; p.nb1 = dst->nb[1];
    p.cnt = p.off = p.list = nullptr; p.n_used = 1; p.nb02 = 0; p.nb2 = 0;
    const dim3 grid((unsigned) ceil_div(p.M, MQ_BM), (unsigned) ceil_div(p.T, MQ_BN));
    hipLaunchKernelGGL(k_mmq_q4K<mq_q4_K>, grid, dim3(256), 0, ctx.stream, p);
    if (ctx.timing) ctx.time_end(TK_MMQ, flops, ev);
}

// MUL_MAT_ID prefill on the MFMA tile: the pairs sorted by expert (cnt/off/list) and their
// activations quantized in that order (k_mmv.hip op_mul_mat_id); grid z = expert, workgroups past
// an expert's token count exit at once.  The repacked CPU path runs one gemv per routed pair
// (repack.cpp:1385-1402): every token takes the per-block order.
bool mmq_id_supported(const ggml_tensor * dst) {
    static const bool off = getenv("GGML_MI355X_NO_MMQ") && atoi(getenv("GGML_MI355X_NO_MMQ")) != 0;
    const ggml_tensor * w = dst->src[0];
    return !off && w->type == GGML_TYPE_Q4_K && w->ne[1] % 8 == 0;
}

void mul_mat_q_id(exec_ctx & ctx, ggml_tensor * dst, const q8_act & act, const int32_t * cnt, const int32_t * off,
                  const int32_t * list, int64_t n_pairs) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * ids = dst->src[2];
    mmq_args p;
    p.W = (const uint8_t *) w->data; p.nb01 = w->nb[1]; p.M = w->ne[1]; p.K = w->ne[0]; p.nblk = w->ne[0] / 256;
    p.xq = act.qs; p.xd = act.d; p.xs = act.s;
    p.T = n_pairs;
    p.gemm_cols = 0;
    p.dst = (float *) dst->data; p.nb1 = dst->nb[1];
    p.cnt = cnt; p.off = off; p.list = list; p.n_used = ids->ne[0]; p.nb02 = w->nb[2]; p.nb2 = dst->nb[2];
    const dim3 grid((unsigned) ceil_div(p.M, MQ_BM), (unsigned) ceil_div(n_pairs, MQ_BN), (unsigned) w->ne[2]);
    hipLaunchKernelGGL(k_mmq_q4K<mq_q4_K>, grid, dim3(256), 0, ctx.stream, p);
}

}  // namespace mi355x
