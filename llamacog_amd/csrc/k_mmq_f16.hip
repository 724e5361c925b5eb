// k_mmq_f16.hip — batched (prefill) Q4_K MUL_MAT on f16 MFMA in the CPU backend's exact float
// order (the repacked gemm / gemv of arch/x86/repack.cpp; the order is described in k_mmq.hip).
// Built with -fno-slp-vectorize (Makefile): the two fp32 chains stay scalar FMAs.
#include "mmq.h"

#include <type_traits>

namespace mi355x {

// ==== Q4_K on f16 MFMA: exact integers in f32 accumulators (the repacked gemm/gemv order) ======
// The scale-folded weight w' = sc·q <= 945 and the Q8_K value y in [-128, 127] are exact f16, every
// product (<= 120960) and every partial sum of a sub-block pair (<= 64·120960 < 2^23) is an exact
// f32 integer, so v_mfma_f32_16x16x32_f16 returns the pair's integer I_pair as a float with no
// rounding in any summation order — the CPU's (float) I_pair — and the VALU is left with the two
// chain FMAs per output.  The mins integer of a pair is one v_mfma_f32_16x16x16_f16 over the 16
// sums of 16 Q8_K values (|sum| <= 2048: exact f16) with the sums outside the pair zeroed.
// 64 rows x 64 tokens per workgroup of 4 waves (two workgroups per CU); wave w multiplies the 64
// rows with tokens 16w .. +15.  The folded weight planes are the only LDS data (double-buffered: the fold of
// block b+1 overlaps block b, one barrier per block; 16-byte chunks swizzled by mh_slot so the
// reads and the fold's stores are conflict-free); each wave streams its 16 tokens' Q8_K
// bytes straight into registers one block ahead and widens them to f16 there
// ((0x6400 | (y ^ 0x80)) - 1152 = y, exact).
constexpr int MH_BM = 64;

typedef _Float16 mh8 __attribute__((ext_vector_type(8)));
typedef _Float16 mh4 __attribute__((ext_vector_type(4)));
typedef _Float16 mh2 __attribute__((ext_vector_type(2)));

struct mh_tok {   // one K block of a lane's token: bytes 64pp + 16h .. +15 per pair, the 16-sums of
    uint4 x[4];   // slots 4h .. 4h+3, d
    uint2 s;
    float d;
};

// LDS slot of 16-byte chunk ch (0..31) of plane row `row`: ch ^ (row & 15) makes the 16 lanes of an
// MFMA A-fragment read (rows c16 = 0..15) hit distinct bank groups; the extra 2·(ch >> 3) makes the
// fold's ds_write_b128 (8-lane groups = two rows x four pairs, chunks 8fq + k) distinct too (without
// it four lanes of a group shared a bank group: 4-way conflicts on every fold store)
__device__ __forceinline__ int mh_slot(int row, int ch) { return ch ^ (row & 15) ^ (2 * (ch >> 3)); }

// 8 int8 (two words) -> 8 f16, exact
__device__ __forceinline__ mh8 i8x8_f16(uint32_t w0, uint32_t w1) {
    const mh2 off = {(_Float16) -1152.0f, (_Float16) -1152.0f};
    const uint32_t u[2] = {w0 ^ 0x80808080u, w1 ^ 0x80808080u};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        o[2 * k] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(mh2, __builtin_amdgcn_perm(0x64646464u, u[k], 0x04010400u)) + off);
        o[2 * k + 1] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(mh2, __builtin_amdgcn_perm(0x64646464u, u[k], 0x04030402u)) + off);
    }
    const uint4 r = make_uint4(o[0], o[1], o[2], o[3]);
    return __builtin_bit_cast(mh8, r);
}

// ALLG: every token of the grid takes the gemm order.  (Loading the tokens two or three blocks
// ahead instead of one measured 4-7 % slower: 52.9 / 54.4 vs 50.8 us at M = 4096, T = 512.)
// (Eight waves of 16 tokens sharing one fold of the 64 rows, one workgroup per CU, measured
// slower: 176 vs 152 us at M = 14336, T = 512.)
template <bool ALLG>
__global__ __launch_bounds__(256, 2) void k_mmq_q4Kh(const mmq_args p) {
    constexpr int NW = 4, BN = 16 * NW;
    __shared__ __attribute__((aligned(16))) uint8_t wpl[2][MH_BM * 512];
    __shared__ __attribute__((aligned(16))) uint32_t wmn[2][MH_BM][4];   // f16 (m_2p, m_2p+1) per pair
    __shared__ __attribute__((aligned(16))) float wd[2][MH_BM], wdm[2][MH_BM];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int64_t bx = blockIdx.x, by = blockIdx.y;
    if (ALLG && (gridDim.x & 7) == 0) {   // XCD-major: one row tile's token tiles on one XCD
        const int64_t id = bx + (int64_t) gridDim.x * by, j = id >> 3;
        by = j % gridDim.y;
        bx = (j / gridDim.y) * 8 + (id & 7);
    }
    // ALLG: every token of the grid takes the gemm order (the tiles below gemm_cols); otherwise
    // the grid is the ragged tail from token tile p.ty0 on, the order chosen per token
    const int64_t row0 = bx * MH_BM, tok0 = (ALLG ? by : by + p.ty0) * BN, T = p.T;
    const int h = lane >> 4, c16 = lane & 15;
    const int tg = wave;   // wave w: the 64 rows x tokens 16w .. +15
    const int64_t KB = p.K / 256;
    const int64_t tok = tok0 + 16 * tg + c16;                // this lane's token
    const bool gemm = tok < p.gemm_cols;

    // token side: straight to registers
    const int64_t tl = min(tok, T - 1);
    const int8_t * xrow = p.xq + tl * p.K + 16 * h;
    const int16_t * srow = p.xs + tl * (p.K / 16) + 4 * h;
    const float * drow_ = p.xd + tl * KB;
    auto load_x = [&](int64_t b, mh_tok & o) __attribute__((always_inline)) {
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) o.x[pp] = *(const uint4 *) (xrow + b * 256 + 64 * pp);
        o.s = *(const uint2 *) (srow + b * 16);
        o.d = drow_[b];
    };
    // weight side: thread (row fr, pair fq) folds 64 weights into f16
    const int fr = tid / 4, fq = tid % 4;
    const uint8_t * wrow = p.W + min(row0 + fr, p.M - 1) * p.nb01;
    uint4 whdr, wqa, wqb;
    auto load_w = [&](int64_t b) __attribute__((always_inline)) {
        const uint8_t * blk = wrow + b * 144;
        whdr = ld16(blk);
        wqa = ld16(blk + 16 + 32 * fq);
        wqb = ld16(blk + 32 + 32 * fq);
    };
    auto fold_w = [&](int buf) __attribute__((always_inline)) {
        int sc_lo, sc_hi, m_lo, m_hi;
        k4_scales_g(whdr.y, whdr.z, whdr.w, fq, sc_lo, sc_hi, m_lo, m_hi);
        uint8_t * dp = wpl[buf] + fr * 512;
        // (1024 + q)·sc - 1024·sc = q·sc, one rounding of an exact f16 value.  Chunk 8fq + k of the
        // row: k < 4 low nibbles of qs bytes 8k .. 8k+7 of the pair (sub-block 2fq), k >= 4 high
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int half = k >> 2, kq = k & 3;
            const _Float16 sc = (_Float16) (half ? sc_hi : sc_lo);
            const mh2 s2 = {sc, sc}, n2 = {(_Float16) -1024.0f * sc, (_Float16) -1024.0f * sc};
            uint32_t o[4];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int wi = 2 * kq + u;
                const uint32_t w = wi < 4 ? (&wqa.x)[wi] : (&wqb.x)[wi - 4];
                const uint32_t nb = half ? (w >> 4) & 0x0f0f0f0fu : w & 0x0f0f0f0fu;
                const mh2 lo = __builtin_bit_cast(mh2, __builtin_amdgcn_perm(0x64646464u, nb, 0x04010400u));
                const mh2 hi = __builtin_bit_cast(mh2, __builtin_amdgcn_perm(0x64646464u, nb, 0x04030402u));
                o[2 * u] = __builtin_bit_cast(uint32_t, __builtin_elementwise_fma(lo, s2, n2));
                o[2 * u + 1] = __builtin_bit_cast(uint32_t, __builtin_elementwise_fma(hi, s2, n2));
            }
            *(uint4 *) (dp + 16 * mh_slot(fr, 8 * fq + k)) = make_uint4(o[0], o[1], o[2], o[3]);
        }
        const mh2 mm = {(_Float16) m_lo, (_Float16) m_hi};
        wmn[buf][fr][fq] = __builtin_bit_cast(uint32_t, mm);
        if (fq == 0) { wd[buf][fr] = h2f(whdr.x & 0xffff); wdm[buf][fr] = h2f(whdr.x >> 16); }
    };

    float A[4][4], B[4][4];   // [row tile][row 4h + i]
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) A[r][i] = B[r][i] = 0.0f;

    // pair-outer order: for each pair pp, the token's pair bytes become two f16 B fragments and
    // the four row tiles multiply them; every chain A[r][i] / B[r][i] still takes the pairs in
    // order 0..3, so the bits are those of the row-tile-outer order
    auto compute = [&](int buf, const mh_tok & x) __attribute__((always_inline)) {
        const uint8_t * pl = wpl[buf];
        // the CPU's scale products d·dy, dmin·dy of rows 16r + 4h + i, and the mins operand of row
        // 16r + c16 (slots 4h .. 4h+3 are sub-blocks 2h, 2h, 2h+1, 2h+1)
        float sA[4][4], sB[4][4];
        mh4 mA[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float4 dw = *(const float4 *) &wd[buf][16 * r + 4 * h];
            const float4 dm = *(const float4 *) &wdm[buf][16 * r + 4 * h];
            sA[r][0] = dw.x * x.d; sA[r][1] = dw.y * x.d; sA[r][2] = dw.z * x.d; sA[r][3] = dw.w * x.d;
            sB[r][0] = dm.x * x.d; sB[r][1] = dm.y * x.d; sB[r][2] = dm.z * x.d; sB[r][3] = dm.w * x.d;
            const uint32_t w = wmn[buf][16 * r + c16][h];
            mA[r] = __builtin_bit_cast(mh4, make_uint2(__builtin_amdgcn_perm(w, w, 0x01000100u), __builtin_amdgcn_perm(w, w, 0x03020302u)));
        }
        const mh4 sf = {(_Float16) (int16_t) (x.s.x & 0xffff), (_Float16) (int16_t) (x.s.x >> 16),
                        (_Float16) (int16_t) (x.s.y & 0xffff), (_Float16) (int16_t) (x.s.y >> 16)};
        int ib[ALLG ? 1 : 4][4], mb[ALLG ? 1 : 4][4];   // gemv-order sums (exact ints: a block's I can pass 2^24)
        if constexpr (!ALLG) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i) ib[r][i] = mb[r][i] = 0;
        }
        // the token's pairs as f16 B fragments, and the pair's 16-sums (lanes h == pp)
        mh8 bf[4][2];
        mh4 bz[4];
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
            bf[pp][0] = i8x8_f16(x.x[pp].x, x.x[pp].y);
            bf[pp][1] = i8x8_f16(x.x[pp].z, x.x[pp].w);
            bz[pp] = h == pp ? sf : (mh4){0, 0, 0, 0};
        }
        // step j = (pair pp, row tile r): its A fragments are read two steps ahead and its MFMAs
        // issued one step ahead of the chain FMAs that consume them, so the matrix pipe works
        // while the VALU runs the previous step's FMAs (not waiting on each result in turn)
        mh8 af[3][2];
        auto lda = [&](int j) __attribute__((always_inline)) {
            const int pp = j >> 2, r = j & 3, sl = j % 3;
            const uint8_t * ar = pl + (16 * r + c16) * 512;
            af[sl][0] = *(const mh8 *) (ar + 16 * mh_slot(c16, 8 * pp + 2 * h));
            af[sl][1] = *(const mh8 *) (ar + 16 * mh_slot(c16, 8 * pp + 2 * h + 1));
        };
        auto mma = [&](int j, v4f & I, v4f & Im) __attribute__((always_inline)) {
            const int pp = j >> 2, r = j & 3, sl = j % 3;
            const v4f z = {0.f, 0.f, 0.f, 0.f};
            I = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[sl][0], bf[pp][0], z, 0, 0, 0);
            I = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[sl][1], bf[pp][1], I, 0, 0, 0);
            Im = __builtin_amdgcn_mfma_f32_16x16x16f16(mA[r], bz[pp], z, 0, 0, 0);
        };
        lda(0);
        lda(1);
        v4f Ic, Imc;
        mma(0, Ic, Imc);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int r = j & 3;
            if (j + 2 < 16) lda(j + 2);
            v4f In, Imn;
            if (j + 1 < 16) mma(j + 1, In, Imn);
            if constexpr (ALLG) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    A[r][i] = fmaf(Ic[i], sA[r][i], A[r][i]);
                    B[r][i] = fmaf(Imc[i], sB[r][i], B[r][i]);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (gemm) {
                        A[r][i] = fmaf(Ic[i], sA[r][i], A[r][i]);
                        B[r][i] = fmaf(Imc[i], sB[r][i], B[r][i]);
                    } else {
                        ib[r][i] += (int) Ic[i];
                        mb[r][i] += (int) Imc[i];
                    }
                }
            }
            if (j + 1 < 16) { Ic = In; Imc = Imn; }
            __builtin_amdgcn_sched_barrier(0);   // bounded live ranges
        }
        if constexpr (!ALLG) {
            if (!gemm) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        A[r][i] = fmaf((float) ib[r][i], sA[r][i], A[r][i]);
                        B[r][i] = fmaf((float) mb[r][i], sB[r][i], B[r][i]);
                    }
            }
        }
    };

    const int64_t last = p.nblk - 1;
    load_w(0);
    mh_tok xa, xb;
    load_x(0, xa);
    fold_w(0);
    load_w(min((int64_t) 1, last));
    // block b: planes[b & 1] were folded during block b-1; the fold of b+1 (planes[(b+1) & 1],
    // last read in block b-1) and the token loads of b+1 overlap block b's MFMAs
    // (no branches around the loads: the last blocks re-load the final block, so the memory
    // counter waits stay exact instead of draining every load at each block)
    for (int64_t b = 0; b < p.nblk; ++b) {
        __syncthreads();
        load_x(min(b + 1, last), xb);
        fold_w((int) ((b + 1) & 1));
        load_w(min(b + 2, last));
        compute((int) (b & 1), xa);
        xa = xb;
    }
    if (tok < T) {
        char * drow = (char *) p.dst + tok * p.nb1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t m0 = row0 + 16 * r + 4 * h;
            if (m0 + 3 < p.M) {
                *(float4 *) (drow + m0 * 4) = make_float4(__fsub_rn(A[r][0], B[r][0]), __fsub_rn(A[r][1], B[r][1]),
                                                          __fsub_rn(A[r][2], B[r][2]), __fsub_rn(A[r][3], B[r][3]));
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (m0 + i < p.M) *(float *) (drow + (m0 + i) * 4) = __fsub_rn(A[r][i], B[r][i]);
            }
        }
    }
}


void launch_mmq_q4Kh(hipStream_t st, const mmq_args & p0) {
    mmq_args p = p0;
    const int64_t gx = ceil_div(p.M, (int64_t) MH_BM);
    const int64_t full = p.gemm_cols / 64, tiles = ceil_div(p.T, (int64_t) 64);   // token tiles all in gemm order
    if (full > 0) {
        p.ty0 = 0;
        hipLaunchKernelGGL((k_mmq_q4Kh<true>), dim3((unsigned) gx, (unsigned) full), dim3(256), 0, st, p);
    }
    if (tiles > full) {
        p.ty0 = full;
        hipLaunchKernelGGL((k_mmq_q4Kh<false>), dim3((unsigned) gx, (unsigned) (tiles - full)), dim3(256), 0, st, p);
    }
}

}  // namespace mi355x
