// k_mmq.hip — batched (prefill) quantized MUL_MAT / MUL_MAT_ID on MFMA, in the CPU backend's
// exact float order.
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
// Tiles: Q4_K MUL_MAT runs the f16-operand tile (k_mmq_f16.hip); Q4_K MUL_MAT_ID (expert-sorted
// pairs, all gemv order) runs the int8 scale-folded tile below
// (v_mfma_i32_16x16x64_i8); Q6_K / Q5_K run the class-exact tile (the vec_dot order).
// MFMA layouts (tools/mfma_layout.hip, tools/mfma_probe.hip): 16x16x32 i8 / f16 lane l holds
// A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15]; 16x16x64 i8 k 16(l>>4)+j;
// C[row 4(l>>4)+i][col l&15].
#include "mmq.h"

namespace mi355x {

constexpr int MQ_BM = 64, MQ_BN = 64;




// ==== Q4_K on v_mfma_i32_16x16x64_i8 with scale-folded weights (the repacked gemm/gemv order) ========
// The gemm's integer per sub-block pair, I_pair = sc_2k·<q_2k, y> + sc_2k+1·<q_2k+1, y>, is a
// K = 64 dot product once each weight carries its 6-bit sub-block scale.  With sc = 8a + b
// (a, b <= 7) the two planes qa = q·a and qb = q·b are int8 (<= 105), so
// I_pair = 8·MFMA(qa, y) + MFMA(qb, y) exactly, and the pair's mins integer
// m_2k·Σy_2k + m_2k+1·Σy_2k+1 is a third MFMA with the mins replicated along K — three
// 16x16x64 instructions per pair and 16x16 outputs, and per output only the CPU's own work
// remains on the VALU (one shift-add, two converts, the two fp32 chain FMAs).  The fold is one
// packed 16-bit multiply per 4 weights (q·a < 256: no carry between bytes).
// Each wave folds the 16 rows it multiplies, so the planes need no workgroup barrier: the one
// barrier per K block is for the shared token stage (LDS-DMA, double-buffered).
// Workgroups of one XCD take all token tiles of a row tile (the weights are read once per XCD
// L2, not once per token tile), when the row-tile count is a multiple of 8.
// MFMA x64 lane map (tools/mfma_probe.hip): lane l holds A[row l&15][k 16(l>>4)+j], B[k 16(l>>4)+j]
// [col l&15], j < 16; C[row 4(l>>4)+i][col l&15].
constexpr int MF_RS = 272;                       // plane row stride (256 + 16: 16 rows, 16 bank groups)
constexpr int MF_PL = MQ_BM * MF_RS;             // one plane
constexpr int MF_XD = MQ_BN * 256;               // token stage: rows [64][256] (XOR-swizzled chunks), then
constexpr int MF_XB = MF_XD + MQ_BN * 4;         //   the token scales [64] f32

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_mul16(uint32_t x, uint32_t s2) {
    const us2 r = __builtin_bit_cast(us2, x) * __builtin_bit_cast(us2, s2);
    return __builtin_bit_cast(uint32_t, r);
}

__global__ __launch_bounds__(256, 2) void k_mmq_q4Kf(const mmq_args p) {
    __shared__ __attribute__((aligned(16))) uint8_t pa[MF_PL], pb[MF_PL];
    __shared__ __attribute__((aligned(16))) uint8_t xst[2][MF_XB];
    __shared__ __attribute__((aligned(16))) uint32_t wmn4[MQ_BM][8];   // mins, byte-replicated
    __shared__ __attribute__((aligned(16))) float wd[MQ_BM], wdm[MQ_BM];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int64_t bx = blockIdx.x, by = blockIdx.y;
    if (!p.cnt && (gridDim.x & 7) == 0) {   // XCD-major: one row tile's token tiles on one XCD
        const int64_t id = bx + (int64_t) gridDim.x * by, j = id >> 3;
        by = j % gridDim.y;
        bx = (j / gridDim.y) * 8 + (id & 7);
    }
    const int64_t row0 = bx * MQ_BM;
    const int64_t tok0 = by * MQ_BN;
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
    // 0: every token of the tile takes the gemm (per-pair) order, 1: every token the gemv
    // (per-block) order, 2: mixed (the last tile of a batch with T % 4 != 0)
    const int mode = tok0 + MQ_BN <= p.gemm_cols ? 0 : (tok0 >= p.gemm_cols ? 1 : 2);
    bool gemm[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) gemm[n] = tok0 + 16 * n + c16 < p.gemm_cols;

    // token-side LDS-DMA sources (as k_mmq_q4K): 16 KiB of rows + 256 B of scales per block
    const int8_t * xsrc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = 64 * (wave + 4 * k) + lane, t = c >> 4, part = (c & 15) ^ (t & 15);
        xsrc[k] = p.xq + (col0 + min(tok0 + t, T - 1)) * p.K + 16 * part;
    }
    const float * dsrc = p.xd + (col0 + min(tok0 + lane, T - 1)) * KB;
    auto issue_x = [&](int64_t b, int s) {
        uint8_t * base = xst[s];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            __builtin_amdgcn_global_load_lds((const void *) (xsrc[k] + b * 256), (lds_ptr_t) (base + 1024 * (wave + 4 * k)), 16, 0, 0);
        }
        if (wave == 0) __builtin_amdgcn_global_load_lds((const void *) (dsrc + b), (lds_ptr_t) (base + MF_XD), 4, 0, 0);
    };
    // weight side: lane (row fr, pair fq) of wave w folds 64 weights of row 16w + lane/4
    const int fr = tid >> 2, fq = tid & 3;
    const uint8_t * wrow = Wb + min(row0 + fr, p.M - 1) * p.nb01;
    uint4 whdr, wqa, wqb;   // header (d, dmin, scales) and the pair's 32 qs bytes
    auto load_w = [&](int64_t b) {
        const uint8_t * blk = wrow + b * 144;
        whdr = ld16(blk);
        wqa = ld16(blk + 16 + 32 * fq);
        wqb = ld16(blk + 32 + 32 * fq);
    };
    auto fold_w = [&]() {
        int sc_lo, sc_hi, m_lo, m_hi;
        k4_scales_g(whdr.y, whdr.z, whdr.w, fq, sc_lo, sc_hi, m_lo, m_hi);
        const uint32_t q[8] = {wqa.x, wqa.y, wqa.z, wqa.w, wqb.x, wqb.y, wqb.z, wqb.w};
        uint32_t qa[16], qb[16];
        // elements 0..31 of the pair: low nibbles (sub-block 2fq); 32..63: high nibbles (2fq+1)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const uint32_t sc = (uint32_t) (half ? sc_hi : sc_lo);
            const uint32_t a2 = (sc >> 3) * 0x10001u, b2 = (sc & 7) * 0x10001u;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t nb = half ? (q[i] >> 4) & 0x0f0f0f0fu : q[i] & 0x0f0f0f0fu;
                qa[8 * half + i] = pk_mul16(nb, a2);
                qb[8 * half + i] = pk_mul16(nb, b2);
            }
        }
        uint8_t * ap = pa + fr * MF_RS + 64 * fq;
        uint8_t * bp = pb + fr * MF_RS + 64 * fq;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            *(uint4 *) (ap + 16 * k) = make_uint4(qa[4 * k], qa[4 * k + 1], qa[4 * k + 2], qa[4 * k + 3]);
            *(uint4 *) (bp + 16 * k) = make_uint4(qb[4 * k], qb[4 * k + 1], qb[4 * k + 2], qb[4 * k + 3]);
        }
        *(uint2 *) &wmn4[fr][2 * fq] = make_uint2((uint32_t) m_lo * 0x01010101u, (uint32_t) m_hi * 0x01010101u);
        if (fq == 0) { wd[fr] = h2f(whdr.x & 0xffff); wdm[fr] = h2f(whdr.x >> 16); }
    };

    float A[4][4], B[4][4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) A[n][i] = B[n][i] = 0.0f;

    const int rA = 16 * wave + c16;
    load_w(0);
    issue_x(0, 0);
    fold_w();
    for (int64_t b = 0; b < p.nblk; ++b) {
        const int s = (int) (b & 1);
        const int8_t * xq = (const int8_t *) xst[s];
        const float * xd = (const float *) (xst[s] + MF_XD);
        // stage s landed for every wave; every wave is done with stage s^1 (block b-1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const bool more = b + 1 < p.nblk;
        if (more) {
            load_w(b + 1);
            issue_x(b + 1, s ^ 1);
        }
        // the CPU's scale products d·dy and dmin·dy of this lane's 4 rows x 4 tokens
        const float4 dw4 = *(const float4 *) &wd[16 * wave + 4 * h], dm4 = *(const float4 *) &wdm[16 * wave + 4 * h];
        const float dw[4] = {dw4.x, dw4.y, dw4.z, dw4.w}, dmw[4] = {dm4.x, dm4.y, dm4.z, dm4.w};
        float sA[4][4], sB[4][4];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const float dy = xd[16 * n + c16];
#pragma unroll
            for (int i = 0; i < 4; ++i) { sA[n][i] = dw[i] * dy; sB[n][i] = dmw[i] * dy; }
        }
        if (mode == 0) {
#pragma unroll 1
            for (int k = 0; k < 4; ++k) {
                const uint4 a1 = *(const uint4 *) (pa + rA * MF_RS + 64 * k + 16 * h);
                const uint4 a2 = *(const uint4 *) (pb + rA * MF_RS + 64 * k + 16 * h);
                const uint32_t mm = wmn4[rA][2 * k + (h >> 1)];
                const v4i va = {(int) a1.x, (int) a1.y, (int) a1.z, (int) a1.w};
                const v4i vb = {(int) a2.x, (int) a2.y, (int) a2.z, (int) a2.w};
                const v4i vm = {(int) mm, (int) mm, (int) mm, (int) mm};
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const uint4 x = *(const uint4 *) (xq + (16 * n + c16) * 256 + 16 * ((4 * k + h) ^ c16));
                    const v4i y = {(int) x.x, (int) x.y, (int) x.z, (int) x.w};
                    const v4i z = {0, 0, 0, 0};
                    const v4i ra = __builtin_amdgcn_mfma_i32_16x16x64_i8(va, y, z, 0, 0, 0);
                    const v4i rb = __builtin_amdgcn_mfma_i32_16x16x64_i8(vb, y, z, 0, 0, 0);
                    const v4i rm = __builtin_amdgcn_mfma_i32_16x16x64_i8(vm, y, z, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        A[n][i] = fmaf((float) (ra[i] * 8 + rb[i]), sA[n][i], A[n][i]);
                        B[n][i] = fmaf((float) rm[i], sB[n][i], B[n][i]);
                    }
                }
            }
        } else if (mode == 1) {
            // per-block integer sums (gemv order), accumulated in the MFMA
            v4i ca[4], cb[4], cm[4];
#pragma unroll
            for (int n = 0; n < 4; ++n) ca[n] = cb[n] = cm[n] = (v4i){0, 0, 0, 0};
#pragma unroll 1
            for (int k = 0; k < 4; ++k) {
                const uint4 a1 = *(const uint4 *) (pa + rA * MF_RS + 64 * k + 16 * h);
                const uint4 a2 = *(const uint4 *) (pb + rA * MF_RS + 64 * k + 16 * h);
                const uint32_t mm = wmn4[rA][2 * k + (h >> 1)];
                const v4i va = {(int) a1.x, (int) a1.y, (int) a1.z, (int) a1.w};
                const v4i vb = {(int) a2.x, (int) a2.y, (int) a2.z, (int) a2.w};
                const v4i vm = {(int) mm, (int) mm, (int) mm, (int) mm};
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const uint4 x = *(const uint4 *) (xq + (16 * n + c16) * 256 + 16 * ((4 * k + h) ^ c16));
                    const v4i y = {(int) x.x, (int) x.y, (int) x.z, (int) x.w};
                    ca[n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(va, y, ca[n], 0, 0, 0);
                    cb[n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(vb, y, cb[n], 0, 0, 0);
                    cm[n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(vm, y, cm[n], 0, 0, 0);
                }
            }
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    A[n][i] = fmaf((float) (ca[n][i] * 8 + cb[n][i]), sA[n][i], A[n][i]);
                    B[n][i] = fmaf((float) cm[n][i], sB[n][i], B[n][i]);
                }
        } else {
            // mixed tile: per-pair chains for the gemm tokens, block integer sums for the rest
            int ib[4][4], mb[4][4];
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int i = 0; i < 4; ++i) ib[n][i] = mb[n][i] = 0;
#pragma unroll 1
            for (int k = 0; k < 4; ++k) {
                const uint4 a1 = *(const uint4 *) (pa + rA * MF_RS + 64 * k + 16 * h);
                const uint4 a2 = *(const uint4 *) (pb + rA * MF_RS + 64 * k + 16 * h);
                const uint32_t mm = wmn4[rA][2 * k + (h >> 1)];
                const v4i va = {(int) a1.x, (int) a1.y, (int) a1.z, (int) a1.w};
                const v4i vb = {(int) a2.x, (int) a2.y, (int) a2.z, (int) a2.w};
                const v4i vm = {(int) mm, (int) mm, (int) mm, (int) mm};
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const uint4 x = *(const uint4 *) (xq + (16 * n + c16) * 256 + 16 * ((4 * k + h) ^ c16));
                    const v4i y = {(int) x.x, (int) x.y, (int) x.z, (int) x.w};
                    const v4i z = {0, 0, 0, 0};
                    const v4i ra = __builtin_amdgcn_mfma_i32_16x16x64_i8(va, y, z, 0, 0, 0);
                    const v4i rb = __builtin_amdgcn_mfma_i32_16x16x64_i8(vb, y, z, 0, 0, 0);
                    const v4i rm = __builtin_amdgcn_mfma_i32_16x16x64_i8(vm, y, z, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int ip = ra[i] * 8 + rb[i];
                        if (gemm[n]) {
                            A[n][i] = fmaf((float) ip, sA[n][i], A[n][i]);
                            B[n][i] = fmaf((float) rm[i], sB[n][i], B[n][i]);
                        } else {
                            ib[n][i] += ip;
                            mb[n][i] += rm[i];
                        }
                    }
                }
            }
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                if (gemm[n]) continue;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    A[n][i] = fmaf((float) ib[n][i], sA[n][i], A[n][i]);
                    B[n][i] = fmaf((float) mb[n][i], sB[n][i], B[n][i]);
                }
            }
        }
        if (more) {
            // this wave's plane rows for block b+1 (only this wave reads them; a wave's LDS
            // accesses complete in order, so the reads above finish first)
            asm volatile("" ::: "memory");
            fold_w();
        }
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
        const int64_t m0 = row0 + 16 * wave + 4 * h;
        if (m0 + 3 < p.M) {
            *(float4 *) (drow + m0 * 4) = make_float4(__fsub_rn(A[n][0], B[n][0]), __fsub_rn(A[n][1], B[n][1]),
                                                      __fsub_rn(A[n][2], B[n][2]), __fsub_rn(A[n][3], B[n][3]));
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (m0 + i < p.M) *(float *) (drow + (m0 + i) * 4) = __fsub_rn(A[n][i], B[n][i]);
        }
    }
}

// ==== class-exact prefill tile for Q6_K / Q5_K (the vec_dot order, qtypes.h) ====================
// The CPU's vec_dot keeps, per 256-block, eight integer "class" sums (class c = bytes 4c..4c+3
// of every 32-element chunk) and runs eight fp32 chains acc[c] = fma(dy·d, cls_b[c], acc[c])
// over the blocks, then hsum_float_8 (Q5_K adds the chain summs = fma(Imin, -dy·dmin, summs)).
// On MFMA: per K block the 64 rows' weights are folded into class-major int8 planes in LDS —
// the 32 weights of class c in K order 4·chunk + j, each pre-multiplied by its sub-block scale
// and split as w' = 64·hi + lo (Q6_K: sc·(q-32) in [-4096, 4064] -> hi in [-64, 64], lo in
// [0, 63]; Q5_K: sc·q <= 1953) — so a class integer is two v_mfma_i32_16x16x32_i8 (the lo
// product accumulates onto the hi product shifted by 6), exact.  The token tile is the Q8_K rows
// as staged by LDS-DMA (XOR-swizzled 16-byte chunks); a lane's B fragment of class c is the 4
// bytes of each of its two chunks.  8 fp32 chains per output live in registers through the K
// loop.
template <class W> struct mc_stage {
    static constexpr int XD = MQ_BN * 256;           // token scales [64] f32 after the rows
    static constexpr int XS = XD + MQ_BN * 4;        // token bsums [64][16] i16
    static constexpr int BYTES = XS + MQ_BN * 32;
};

// LDS slot of 8-byte piece s (0..31) of a folded plane row: s ^ 2(row & 15) spreads the MFMA
// A-fragment reads (rows c16, pieces 4c + h) over all banks; the extra (s >> 4) separates the fold's
// ds_write_b64 lane groups (two rows x eight classes: pieces 4fc + q), which otherwise met 2-way
__device__ __forceinline__ int mc_slot(int row, int s) { return s ^ (2 * (row & 15)) ^ (s >> 4); }

__device__ __forceinline__ uint32_t pk_bytes(uint32_t e, uint32_t o) {   // bytes 0,2 from e, 1,3 from o
    return (e & 0x00ff00ffu) | ((o & 0x00ff00ffu) << 8);
}
typedef short sh2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ sh2 as_sh2(uint32_t u) { sh2 v; __builtin_memcpy(&v, &u, 4); return v; }
__device__ __forceinline__ uint32_t as_u32(sh2 v) { uint32_t u; __builtin_memcpy(&u, &v, 4); return u; }

// four weights (bytes of q, unsigned) -> hi / lo bytes of sc·(q - bias) (16-bit lanes: exact)
__device__ __forceinline__ void fold4(uint32_t q, int sc, int bias, uint32_t & hi, uint32_t & lo) {
    const sh2 b2 = {(short) bias, (short) bias}, s2 = {(short) sc, (short) sc};
    const sh2 we = (as_sh2(q & 0x00ff00ffu) - b2) * s2;
    const sh2 wo = (as_sh2((q >> 8) & 0x00ff00ffu) - b2) * s2;
    const sh2 sh = {6, 6}, m63 = {63, 63};
    hi = pk_bytes(as_u32(we >> sh), as_u32(wo >> sh));
    lo = pk_bytes(as_u32(we & m63), as_u32(wo & m63));
}

// Q6_K: a thread folds class c of one row.  Element e = 128n + 32g + l sits in chunk 4n + g;
// its 6 bits are ql[64n + 32(g&1) + l] nibble g>>1 and qh[32n + l] bits 2g; its scale
// scales[2·chunk + (l >= 16)] (dequantize_row_q6_K, ggml-quants.c:1684); class c is l = 4c..4c+3
struct mc_q6_K {
    static constexpr int BLK = 210;
    static constexpr bool MINS = false;
    struct raw { uint32_t ql[2][2]; uint32_t qh[2]; uint4 sc; uint32_t d; };
    __device__ static void load(const uint8_t * blk, int c, raw & r) {
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            r.ql[n][0] = ld4(blk + 64 * n + 4 * c);
            r.ql[n][1] = ld4(blk + 64 * n + 32 + 4 * c);
            r.qh[n] = ld4(blk + 128 + 32 * n + 4 * c);
        }
        r.sc = ld16(blk + 192);
        r.d = ld2(blk + 208);
    }
    // hi/lo[chunk]: the 4 bytes of class c in chunk `chunk`
    __device__ static void fold(const raw & r, int c, uint32_t (&hi)[8], uint32_t (&lo)[8]) {
        const uint32_t scw[4] = {r.sc.x, r.sc.y, r.sc.z, r.sc.w};
#pragma unroll
        for (int ch = 0; ch < 8; ++ch) {
            const int n = ch >> 2, g = ch & 3;
            const uint32_t q = ((r.ql[n][g & 1] >> (4 * (g >> 1))) & 0x0f0f0f0fu) | (((r.qh[n] >> (2 * g)) & 0x03030303u) << 4);
            const int si = 2 * ch + (c >= 4 ? 1 : 0);
            const int sc = (int8_t) ((scw[si >> 2] >> (8 * (si & 3))) & 0xff);
            fold4(q, sc, 32, hi[ch], lo[ch]);
        }
    }
    __device__ static float d_of(const raw & r) { return h2f((uint16_t) r.d); }
    __device__ static float dmin_of(const raw &) { return 0.0f; }
    __device__ static void mins_of(const raw &, int (&)[8]) {}
};

// Q5_K: chunk (sub-block) s = 2j + nib: element l of it is qs[32j + l] nibble nib with bit
// (qh[l] >> s) & 1 on top (dequantize_row_q5_K, ggml-quants.c:1476); scale / min get_scale_min_k4(s)
struct mc_q5_K {
    static constexpr int BLK = 176;
    static constexpr bool MINS = true;
    struct raw { uint32_t qs[4]; uint32_t qh; uint4 hdr; };
    __device__ static void load(const uint8_t * blk, int c, raw & r) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r.qs[j] = ld4(blk + 48 + 32 * j + 4 * c);
        r.qh = ld4(blk + 16 + 4 * c);
        r.hdr = ld16(blk);
    }
    __device__ static void scmin(const raw & r, int s, int & sc, int & m) {
        const uint8_t * q = (const uint8_t *) &r.hdr + 4;
        scale_min_k4(s, q, sc, m);
    }
    __device__ static void fold(const raw & r, int, uint32_t (&hi)[8], uint32_t (&lo)[8]) {
#pragma unroll
        for (int ch = 0; ch < 8; ++ch) {
            int sc, m;
            scmin(r, ch, sc, m);
            const uint32_t q = ((r.qs[ch >> 1] >> (4 * (ch & 1))) & 0x0f0f0f0fu) | (((r.qh >> ch) & 0x01010101u) << 4);
            fold4(q, sc, 0, hi[ch], lo[ch]);
        }
    }
    __device__ static float d_of(const raw & r) { return h2f((uint16_t) (r.hdr.x & 0xffff)); }
    __device__ static float dmin_of(const raw & r) { return h2f((uint16_t) (r.hdr.x >> 16)); }
    __device__ static void mins_of(const raw & r, int (&mn)[8]) {
#pragma unroll
        for (int s = 0; s < 8; ++s) { int sc; scmin(r, s, sc, mn[s]); }
    }
};

// 512 threads: wave w computes rows 16 (w & 3) .. +15 of the 64-row tile for tokens 32 (w >> 2) ..
// +31 (two 16-token MFMA tiles): 8 x 2 x 4 = 64 chain registers per lane
template <class W>
__global__ __launch_bounds__(512, 2) void k_mmq_cls(const mmq_args p) {
    using S = mc_stage<W>;
    __shared__ __attribute__((aligned(16))) uint8_t st[2][S::BYTES];      // token stages
    __shared__ __attribute__((aligned(16))) uint8_t ph[MQ_BM * 256];       // folded planes, swizzled
    __shared__ __attribute__((aligned(16))) uint8_t pl[MQ_BM * 256];
    __shared__ float wd[MQ_BM], wdm[MQ_BM];
    __shared__ float wmn[W::MINS ? MQ_BM : 1][8];   // Q5_K mins (exact in f32)
    __shared__ float xsb[W::MINS ? MQ_BN : 1][8];   // Q5_K per-token sub-block sums

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rg = wave & 3, tg = wave >> 2;
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
    // token-side LDS-DMA sources: instruction i = wave + 8k of 16 (1 KiB each)
    const int8_t * xsrc[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int c = 64 * (wave + 8 * k) + lane, t = c >> 4, part = (c & 15) ^ (t & 15);
        xsrc[k] = p.xq + (col0 + min(tok0 + t, T - 1)) * p.K + 16 * part;
    }
    const float * dsrc = p.xd + (col0 + min(tok0 + lane, T - 1)) * KB;
    const int16_t * ssrc;
    {
        const int c = 64 * (wave == 2 ? 1 : 0) + lane, t = c >> 1, half = c & 1;
        ssrc = p.xs + (col0 + min(tok0 + t, T - 1)) * (p.K / 16) + 8 * half;
    }
    auto issue_x = [&](int64_t b, int s) {
        uint8_t * base = st[s];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            __builtin_amdgcn_global_load_lds((const void *) (xsrc[k] + b * 256), (lds_ptr_t) (base + 1024 * (wave + 8 * k)), 16, 0, 0);
        }
        if (wave == 0) {
            __builtin_amdgcn_global_load_lds((const void *) (dsrc + b), (lds_ptr_t) (base + S::XD), 4, 0, 0);
        } else if (W::MINS && wave <= 2) {
            __builtin_amdgcn_global_load_lds((const void *) (ssrc + b * 16), (lds_ptr_t) (base + S::XS + 1024 * (wave - 1)), 16, 0, 0);
        }
    };
    // the fold: thread = (row fr, class fc); its raw bytes come straight from global memory
    const int fr = tid >> 3, fc = tid & 7;
    const uint8_t * wsrc = Wb + min(row0 + fr, p.M - 1) * p.nb01;
    typename W::raw wr;

    float acc[8][2][4];
    float summs[W::MINS ? 2 : 1][4];
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[c][n][i] = 0.0f;
#pragma unroll
    for (int n = 0; n < (W::MINS ? 2 : 1); ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) summs[n][i] = 0.0f;

    issue_x(0, 0);
    typename W::raw wr1;
    W::load(wsrc, fc, wr);
    const int ra = 16 * rg + c16;   // A row of this lane
    // block b: its token stage and raw weights were issued at the start of block b-1 (before that
    // block's fold and MFMAs), so the wait at the top of b covers loads a whole block old
    auto block = [&](int64_t b, typename W::raw & cur, typename W::raw & nxt) __attribute__((always_inline)) {
        const int s = (int) (b & 1);
        const int8_t * xq = (const int8_t *) st[s];
        const float * xd = (const float *) (st[s] + S::XD);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();   // token stage s and this thread's raw weights landed; block b-1 is done with the planes and stage s^1
        if (b + 1 < p.nblk) {
            issue_x(b + 1, s ^ 1);
            W::load(wsrc + (b + 1) * W::BLK, fc, nxt);
        }
        {
            uint32_t hi[8], lo[8];
            W::fold(cur, fc, hi, lo);
#pragma unroll
            for (int q = 0; q < 4; ++q) {   // 8-byte slot 4c + q of the row, XOR-swizzled
                const int slot = mc_slot(fr, 4 * fc + q);
                *(uint2 *) (ph + fr * 256 + 8 * slot) = make_uint2(hi[2 * q], hi[2 * q + 1]);
                *(uint2 *) (pl + fr * 256 + 8 * slot) = make_uint2(lo[2 * q], lo[2 * q + 1]);
            }
            if (fc == 0) {
                wd[fr] = W::d_of(cur);
                wdm[fr] = W::dmin_of(cur);
                if constexpr (W::MINS) {
                    int mn[8];
                    W::mins_of(cur, mn);
#pragma unroll
                    for (int j = 0; j < 8; ++j) wmn[fr][j] = (float) mn[j];
                }
            }
            if constexpr (W::MINS) {
                if (tid < MQ_BN) {
                    const int16_t * s16 = (const int16_t *) (st[s] + S::XS) + 16 * tid;
#pragma unroll
                    for (int j = 0; j < 8; ++j) xsb[tid][j] = (float) (s16[2 * j] + s16[2 * j + 1]);
                }
            }
        }
        __syncthreads();
        float f[2][4];   // dy·d, as the CPU forms it
#pragma unroll
        for (int n = 0; n < 2; ++n) {
            const float dy = xd[32 * tg + 16 * n + c16];
#pragma unroll
            for (int i = 0; i < 4; ++i) f[n][i] = dy * wd[16 * rg + 4 * h + i];
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int slot = mc_slot(c16, 4 * c + h);
            const long ahi = *(const long *) (ph + ra * 256 + 8 * slot);
            const long alo = *(const long *) (pl + ra * 256 + 8 * slot);
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const int8_t * xr = xq + (32 * tg + 16 * n + c16) * 256 + 4 * (c & 3);
                const uint32_t b0 = *(const uint32_t *) (xr + 16 * ((4 * h + (c >> 2)) ^ c16));
                const uint32_t b1 = *(const uint32_t *) (xr + 16 * ((4 * h + 2 + (c >> 2)) ^ c16));
                const long bf = (long) b0 | ((long) b1 << 32);
                v4i r = {0, 0, 0, 0};
                r = __builtin_amdgcn_mfma_i32_16x16x32_i8(ahi, bf, r, 0, 0, 0);
                r[0] <<= 6; r[1] <<= 6; r[2] <<= 6; r[3] <<= 6;
                r = __builtin_amdgcn_mfma_i32_16x16x32_i8(alo, bf, r, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[c][n][i] = fmaf(f[n][i], (float) r[i], acc[c][n][i]);
            }
        }
        if constexpr (W::MINS) {
            // Imin[r][t] = sum_s mins[r][s] * bsum[t][s]: a K = 8 product, exact in fp32 (every
            // partial sum is an integer below 2^24): two f32 MFMAs per 16 x 16 tile
            const float a0 = wmn[ra][h], a1 = wmn[ra][h + 4];
#pragma unroll
            for (int n = 0; n < 2; ++n) {
                const int t = 32 * tg + 16 * n + c16;
                v4f z = {0.f, 0.f, 0.f, 0.f};
                z = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, xsb[t][h], z, 0, 0, 0);
                z = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, xsb[t][h + 4], z, 0, 0, 0);
                const float dy = xd[t];
#pragma unroll
                for (int i = 0; i < 4; ++i) summs[n][i] = fmaf(z[i], -dy * wdm[16 * rg + 4 * h + i], summs[n][i]);
            }
        }
    };
    for (int64_t b = 0; b < p.nblk; b += 2) {
        block(b, wr, wr1);
        if (b + 1 < p.nblk) block(b + 1, wr1, wr);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int64_t t = tok0 + 32 * tg + 16 * n + c16;
        if (t >= T) continue;
        char * drow = (char *) p.dst + t * p.nb1;
        if (p.cnt) {
            const int pair = p.list[col0 + t];
            drow = (char *) p.dst + (pair % p.n_used) * p.nb1 + (pair / p.n_used) * p.nb2;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t m = row0 + 16 * rg + 4 * h + i;
            // hsum_float_8: ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7))
            float v = __fadd_rn(__fadd_rn(__fadd_rn(acc[0][n][i], acc[4][n][i]), __fadd_rn(acc[2][n][i], acc[6][n][i])),
                                __fadd_rn(__fadd_rn(acc[1][n][i], acc[5][n][i]), __fadd_rn(acc[3][n][i], acc[7][n][i])));
            if constexpr (W::MINS) v = __fadd_rn(v, summs[n][i]);
            if (m < p.M) *(float *) (drow + m * 4) = v;
        }
    }
}

// ---- host --------------------------------------------------------------------------------------
// Q4_K weights with M % 8 == 0 (the repacked order), Q5_K / Q6_K (the vec_dot order), and a
// batch of >= 16 tokens
static bool mmq_type_ok(const ggml_tensor * w) {
    return (w->type == GGML_TYPE_Q4_K && w->ne[1] % 8 == 0) || w->type == GGML_TYPE_Q5_K || w->type == GGML_TYPE_Q6_K;
}

template <class W>
static void launch_cls(hipStream_t st, const dim3 & grid, const mmq_args & p) {
    hipLaunchKernelGGL(k_mmq_cls<W>, grid, dim3(512), 0, st, p);
}

static void launch_mmq(hipStream_t st, ggml_type t, const dim3 & grid, const mmq_args & p) {
    switch (t) {
        case GGML_TYPE_Q4_K: hipLaunchKernelGGL(k_mmq_q4Kf, grid, dim3(256), 0, st, p); break;
        case GGML_TYPE_Q5_K: launch_cls<mc_q5_K>(st, grid, p); break;
        case GGML_TYPE_Q6_K: launch_cls<mc_q6_K>(st, grid, p); break;
        default: GGML_ABORT("mi355x: mmq type");
    }
}

bool mmq_supported(const ggml_tensor * dst) {
    static const bool off = getenv("GGML_MI355X_NO_MMQ") && atoi(getenv("GGML_MI355X_NO_MMQ")) != 0;
    if (off) return false;
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    if (!mmq_type_ok(w)) return false;
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
    // Q4_K: the f16-operand tile, 64-token workgroups of four waves
    if (w->type == GGML_TYPE_Q4_K) {
        launch_mmq_q4Kh(ctx.stream, p);
    } else {
        const dim3 grid((unsigned) ceil_div(p.M, MQ_BM), (unsigned) ceil_div(p.T, MQ_BN));
        launch_mmq(ctx.stream, w->type, grid, p);
    }
    if (ctx.timing) ctx.time_end(TK_MMQ, flops, ev);
}

// MUL_MAT_ID prefill on the MFMA tile: the pairs sorted by expert (cnt/off/list) and their
// activations quantized in that order (k_mmv.hip op_mul_mat_id); grid z = expert, workgroups past
// an expert's token count exit at once.  The repacked CPU path runs one gemv per routed pair
// (repack.cpp:1385-1402): every token takes the per-block order.
bool mmq_id_supported(const ggml_tensor * dst) {
    static const bool off = getenv("GGML_MI355X_NO_MMQ") && atoi(getenv("GGML_MI355X_NO_MMQ")) != 0;
    return !off && mmq_type_ok(dst->src[0]);
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
    launch_mmq(ctx.stream, w->type, grid, p);
}

}  // namespace mi355x
