// k_mmq.hip — batched (prefill) quantized MUL_MAT on MFMA (v_mfma_i32_16x16x32_i8).
//
// Same arithmetic contract as the mat-vec path (k_mmv.hip / k_gemv.hip): the activations are
// quantized to Q8_K with the CPU's quantizer, every integer sub-block dot product is exact,
// and the per-block combination is (dw*dy)*sumi - (dmin*dy)*summ in fp32 — the formula of
// ggml_vec_dot_q4_K_q8_K / _q6_K_q8_K (ggml-cpu/quants.c:514-722).  The integer dot of a
// 32-element chunk of 16 weight rows x 16 tokens is one MFMA; the sub-block scales (6-bit
// for Q4_K/Q5_K per 32, int8 for Q6_K per 16) are applied to the int32 MFMA results in VALU
// (Q6_K: one MFMA per 16-element half, the other half's A lanes zeroed).
//
// Tiling (MI355X): a 256-thread workgroup owns 64 weight rows x 64 tokens; per 256-element
// K block the 64 rows' quant blocks and the 64 tokens' Q8_K rows are streamed HBM -> LDS with
// global_load_lds (16 B per lane, 1 KiB per wave instruction), the rows' scales are unpacked
// once into LDS, then each wave computes 16 rows x 64 tokens (four 16x16 MFMA tiles sharing
// the A fragment).  MFMA layouts (verified by tools/mfma_layout.hip): lane l holds
// A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15]; C[row 4(l>>4)+i][col l&15].
#include "ops.h"

namespace mi355x {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void * lds_ptr_t;

constexpr int MQ_BM = 64, MQ_BN = 64;

// ---- weight traits: raw block bytes, per-row scale unpack, A fragments -------------------
// unpack(): per-row sub-scales sc[16] (int), mins mn[8] (int), d, dmin of one block.
// afrag(blk, c, h): 8 int8 of 32-element chunk c (0..7), k = 8h .. 8h+7 (h = lane>>4).
struct mq_q4_K {
    static constexpr int BLK = 144, NSC = 8;   // NSC sub-blocks of 256/NSC elements
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

struct mq_q5_K {
    static constexpr int BLK = 176, NSC = 8;
    __device__ static void unpack(const uint8_t * b, int * sc, int * mn, float & d, float & dmin) {
        mq_q4_K::unpack(b, sc, mn, d, dmin);
    }
    __device__ static long afrag(const uint8_t * b, int c, int h) {
        const uint2 v = ld8(b + 48 + 32 * (c >> 1) + 8 * h);
        const uint2 qh = ld8(b + 16 + 8 * h);   // qh[l] bit c is element 32c + l's 5th bit
        const int sh = 4 * (c & 1);
        const uint32_t lo = ((v.x >> sh) & 0x0f0f0f0f) | (((qh.x >> c) & 0x01010101) << 4);
        const uint32_t hi = ((v.y >> sh) & 0x0f0f0f0f) | (((qh.y >> c) & 0x01010101) << 4);
        return (long) lo | ((long) hi << 32);
    }
};

struct mq_q6_K {
    static constexpr int BLK = 210, NSC = 16;
    __device__ static void unpack(const uint8_t * b, int * sc, int * mn, float & d, float & dmin) {
        d = h2f(ld2(b + 208)); dmin = 0.0f;
        for (int j = 0; j < 16; ++j) sc[j] = (int8_t) b[192 + j];
        for (int j = 0; j < 8; ++j) mn[j] = 0;
    }
    __device__ static long afrag(const uint8_t * b, int c, int h) {
        // element e = 32c + 8h + i: n = e/128, grp = (e%128)/32, l = e%32
        const int n = c >> 2, grp = c & 3, l0 = 8 * h;
        const uint2 ql = ld8(b + 64 * n + 32 * (grp & 1) + l0);
        const uint2 qh = ld8(b + 128 + 32 * n + l0);
        const int shl = 4 * (grp >> 1), shh = 2 * grp;
        const uint32_t lo = ((ql.x >> shl) & 0x0f0f0f0f) | (((qh.x >> shh) & 0x03030303) << 4);
        const uint32_t hi = ((ql.y >> shl) & 0x0f0f0f0f) | (((qh.y >> shh) & 0x03030303) << 4);
        // q - 32 per byte (q in 0..63): q ^ 0x20 for q >= 32, and additionally | 0xc0 for q < 32
        const uint32_t r0 = (lo ^ 0x20202020u) | (((~lo & 0x20202020u) >> 5) * 0xc0u);
        const uint32_t r1 = (hi ^ 0x20202020u) | (((~hi & 0x20202020u) >> 5) * 0xc0u);
        return (long) r0 | ((long) r1 << 32);
    }
};

struct mmq_args {
    const uint8_t * W; int64_t nb01; int64_t M; int64_t K; int64_t nblk;
    const int8_t * xq; const float * xd; const int16_t * xs;   // Q8_K SoA: [T][K], [T][K/256], [T][K/16]
    int64_t T;
    float * dst; int64_t nb1;   // dst[t * nb1 + m*4]
    // MUL_MAT_ID (expert-sorted, k_mmv.hip k_moe_sort): blockIdx.z = expert, its cnt[z] tokens are
    // activation columns off[z] .. off[z] + cnt[z] - 1, column j is pair list[j] = e + n_used * t and
    // lands at dst + e * nb1 + t * nb2; nullptr cnt = a plain MUL_MAT
    const int32_t * cnt; const int32_t * off; const int32_t * list; int64_t n_used; int64_t nb02; int64_t nb2;
    int xcd;   // k_mmq_db: XCD-aware tile order (plain MUL_MAT, gridDim.x % 8 == 0)
};

template <class W>
__global__ __launch_bounds__(256) void k_mmq(const mmq_args p) {
    constexpr int RS = (W::BLK + 15) / 16 * 16;   // LDS row stride of the weight tile
    __shared__ __attribute__((aligned(16))) uint8_t wq[MQ_BM * RS];
    __shared__ __attribute__((aligned(16))) int8_t xq[MQ_BN * 256];
    __shared__ int wsc[MQ_BM][W::NSC];
    __shared__ int wmn[MQ_BM][8];
    __shared__ float wd[MQ_BM], wdm[MQ_BM];
    __shared__ float xd[MQ_BN];
    __shared__ int xs[MQ_BN][8];   // Q8_K sums per 32-element chunk

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t row0 = (int64_t) blockIdx.x * MQ_BM;
    const int64_t tok0 = (int64_t) blockIdx.y * MQ_BN;
    const int h = lane >> 4, c16 = lane & 15;
    // MUL_MAT_ID: this workgroup's expert, its token count and first activation column
    const uint8_t * Wb = p.W;
    int64_t T = p.T, col0 = 0;
    if (p.cnt) {
        T = p.cnt[blockIdx.z];
        if (tok0 >= T) return;   // uniform: no barrier passed yet
        col0 = p.off[blockIdx.z];
        Wb = p.W + (int64_t) blockIdx.z * p.nb02;
    }

    float acc[4][4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[n][i] = 0.0f;

    for (int64_t b = 0; b < p.nblk; ++b) {
        // ---- stage: weight blocks of the 64 rows (LDS row stride RS = BLK rounded up to 16 B;
        // the last 16-byte read of a block runs into the next block or the buffer padding),
        // Q8_K rows of the 64 tokens (LDS-DMA) ----------------------------------------------
        constexpr int RC = (W::BLK + 15) / 16;     // 16-byte chunks per row
        for (int c = tid; c < MQ_BM * RC; c += 256) {
            const int r = c / RC, k = c % RC;
            const int64_t row = min(row0 + r, p.M - 1);
            const uint4 v = ld16(Wb + row * p.nb01 + b * W::BLK + 16 * k);
            *(uint4 *) (wq + r * RS + 16 * k) = v;
        }
        for (int c0 = wave * 64; c0 < MQ_BN * 16; c0 += 256) {
            const int c = c0 + lane;
            const int t = c >> 4, part = c & 15;
            const int64_t tok = col0 + min(tok0 + t, T - 1);
            const int8_t * src = p.xq + tok * p.K + b * 256 + 16 * part;
            __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) (xq + 16 * c0), 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // ---- per-row scales, per-token scale and chunk sums --------------------------------
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
            const int64_t tok = col0 + min(tok0 + t, T - 1);
            xd[t] = p.xd[tok * (p.K / 256) + b];
            const int16_t * s16 = p.xs + tok * (p.K / 16) + b * 16;
#pragma unroll
            for (int j = 0; j < 8; ++j) xs[t][j] = s16[2 * j] + s16[2 * j + 1];
        }
        __syncthreads();
        // ---- MFMA over the 8 chunks of 32 --------------------------------------------------
        const int rA = 16 * wave + c16;            // A row of this lane
        int sumi[4][4];
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) sumi[n][i] = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const long a = W::afrag(wq + rA * RS, c, h);
            if constexpr (W::NSC == 8) {
                int scv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) scv[i] = wsc[16 * wave + 4 * h + i][c];
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const long bf = *(const long *) (xq + (16 * n + c16) * 256 + 32 * c + 8 * h);
                    v4i r = {0, 0, 0, 0};
                    r = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, bf, r, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) sumi[n][i] += r[i] * scv[i];
                }
            } else {
                // two 16-element sub-blocks per chunk: lanes h < 2 hold the first, h >= 2 the second
                const long a0 = h < 2 ? a : 0, a1 = h < 2 ? 0 : a;
                int sc0[4], sc1[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    sc0[i] = wsc[16 * wave + 4 * h + i][2 * c];
                    sc1[i] = wsc[16 * wave + 4 * h + i][2 * c + 1];
                }
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const long bf = *(const long *) (xq + (16 * n + c16) * 256 + 32 * c + 8 * h);
                    v4i r0 = {0, 0, 0, 0}, r1 = {0, 0, 0, 0};
                    r0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a0, bf, r0, 0, 0, 0);
                    r1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a1, bf, r1, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) sumi[n][i] += r0[i] * sc0[i] + r1[i] * sc1[i];
                }
            }
        }
        // ---- block combination (fp32) --------------------------------------------------------
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 16 * wave + 4 * h + i;
            const float dw = wd[r], dmw = wdm[r];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int t = 16 * n + c16;
                const float dy = xd[t];
                if constexpr (W::NSC == 8) {
                    int summ = 0;
#pragma unroll
                    for (int j = 0; j < 8; ++j) summ += wmn[r][j] * xs[t][j];
                    acc[n][i] += (dw * dy) * (float) sumi[n][i] - (dmw * dy) * (float) summ;
                } else {
                    acc[n][i] += (dw * dy) * (float) sumi[n][i];
                }
            }
        }
        __syncthreads();   // the LDS tiles are refilled next block
    }
    // ---- store ----------------------------------------------------------------------------
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
            if (m < p.M) *(float *) (drow + m * 4) = acc[n][i];
        }
    }
}

// ---- double-buffered variant ------------------------------------------------------------------
// (24-bit multiplies, full rate, for the sub-block scaling: |MFMA result| <= 32*15*127 (Q4_K),
// 32*31*127 (Q5_K), 16*32*128 (Q6_K) < 2^23, scales and mins < 2^7, Q8_K chunk sums < 2^13,
// so every product is exact)
// The same tile, arithmetic and stores as k_mmq; the loads of K block b+1 are in flight while
// block b computes: the Q8_K token rows, their scales d and bsums go HBM -> LDS by
// global_load_lds into the other of two stages, the weight blocks go to registers and are
// written to that stage after the MFMA work.  One s_waitcnt + barrier per block then finds
// the next stage landed instead of waiting a full memory latency for it.
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

// two workgroups per CU (two stages of 56-66 KB LDS each): at most 256 VGPRs + AGPRs per lane
#ifndef MQ_DB_OCC
#define MQ_DB_OCC 2
#endif
#ifndef MQ_DB_UNROLL
#define MQ_DB_UNROLL 2
#endif
template <class W>
__global__ __launch_bounds__(256, MQ_DB_OCC) void k_mmq_db(const mmq_args p) {
    using S = mq_stage<W>;
    constexpr int RS = S::RS;
    __shared__ __attribute__((aligned(16))) uint8_t st[2][S::BYTES];
    __shared__ int wsc[MQ_BM][W::NSC];
    __shared__ int wmn[MQ_BM][8];
    __shared__ float wd[MQ_BM], wdm[MQ_BM];
    __shared__ int xs[MQ_BN][8];   // Q8_K sums per 32-element chunk

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs in dispatch order, so
    // dispatch slot L runs on XCD L % 8.  With p.xcd, XCD x takes row groups x, x + 8, ... and
    // walks each one's token tiles back to back: the tiles sharing a 64-row weight slice run
    // together on one XCD and read it from that XCD's L2 (a bijection for gridDim.x % 8 == 0)
    unsigned bx = blockIdx.x, by = blockIdx.y;
    if (p.xcd) {
        const unsigned L = blockIdx.x + gridDim.x * blockIdx.y, slot = L >> 3;
        bx = (L & 7) + 8 * (slot / gridDim.y);
        by = slot % gridDim.y;
    }
    const int64_t row0 = (int64_t) bx * MQ_BM;
    const int64_t tok0 = (int64_t) by * MQ_BN;
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

    float acc[4][4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[n][i] = 0.0f;

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
        // ---- MFMA over the 8 chunks of 32 (k_mmq's arithmetic) -----------------------------
        const int rA = 16 * wave + c16;
        int sumi[4][4];
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) sumi[n][i] = 0;
#pragma unroll MQ_DB_UNROLL
        for (int c = 0; c < 8; ++c) {
            const long a = W::afrag(wq + rA * RS, c, h);
            if constexpr (W::NSC == 8) {
                int scv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) scv[i] = wsc[16 * wave + 4 * h + i][c];
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const long bf = *(const long *) (xq + (16 * n + c16) * 256 + 16 * ((2 * c + (h >> 1)) ^ c16) + 8 * (h & 1));
                    v4i r = {0, 0, 0, 0};
                    r = __builtin_amdgcn_mfma_i32_16x16x32_i8(a, bf, r, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) sumi[n][i] += __mul24(r[i], scv[i]);
                }
            } else {
                const long a0 = h < 2 ? a : 0, a1 = h < 2 ? 0 : a;
                int sc0[4], sc1[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    sc0[i] = wsc[16 * wave + 4 * h + i][2 * c];
                    sc1[i] = wsc[16 * wave + 4 * h + i][2 * c + 1];
                }
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const long bf = *(const long *) (xq + (16 * n + c16) * 256 + 16 * ((2 * c + (h >> 1)) ^ c16) + 8 * (h & 1));
                    v4i r0 = {0, 0, 0, 0}, r1 = {0, 0, 0, 0};
                    r0 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a0, bf, r0, 0, 0, 0);
                    r1 = __builtin_amdgcn_mfma_i32_16x16x32_i8(a1, bf, r1, 0, 0, 0);
#pragma unroll
                    for (int i = 0; i < 4; ++i) sumi[n][i] += __mul24(r0[i], sc0[i]) + __mul24(r1[i], sc1[i]);
                }
            }
        }
        // the mins term summ[r][t] = sum_j mn[r][j] * bsum[t][j] of the 64 x 64 tile is a K = 8
        // product: two fp32 MFMAs per 16 x 16 tile.  Every product (< 2^18) and partial sum
        // (< 2^21) is an integer below 2^24, so the result is exact in any order — the same
        // value as the integer loop of k_mmq
        v4f smm[4];
        if constexpr (W::NSC == 8) {
            const float a0 = (float) wmn[16 * wave + c16][h], a1 = (float) wmn[16 * wave + c16][h + 4];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int t = 16 * n + c16;
                v4f z = {0.f, 0.f, 0.f, 0.f};
                z = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, (float) xs[t][h], z, 0, 0, 0);
                z = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, (float) xs[t][h + 4], z, 0, 0, 0);
                smm[n] = z;
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 16 * wave + 4 * h + i;
            const float dw = wd[r], dmw = wdm[r];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int t = 16 * n + c16;
                const float dy = xd[t];
                if constexpr (W::NSC == 8) {
                    acc[n][i] += (dw * dy) * (float) sumi[n][i] - (dmw * dy) * smm[n][i];
                } else {
                    acc[n][i] += (dw * dy) * (float) sumi[n][i];
                }
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
            if (m < p.M) *(float *) (drow + m * 4) = acc[n][i];
        }
    }
}

// ---- prefetch distance 2 (16-byte-aligned weight blocks: Q4_K) ----------------------------------
// k_mmq_db waits about one memory latency per K block whenever a block's MFMA work is shorter
// than that latency, and the compiler, which cannot tell LDS stages apart, also waits for every
// LDS-DMA in flight before each LDS read.  Here every load is an LDS-DMA issued from inline asm
// (invisible to the compiler's waitcnt pass), the token side of block b+2 and the weights of
// block b+1 leave while block b computes (three token stages, two weight stages), and every wave
// issues the same number of DMA instructions per block (clamped duplicates at the edges), so
// "blocks b's stages landed" is one fixed s_waitcnt vmcnt.
__device__ __forceinline__ void dma_lds16(const void * g, const void * lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (lds_ptr_t) lds);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" :: "v"(g), "s"(m) : "memory", "m0");
}
__device__ __forceinline__ void dma_lds4(const void * g, const void * lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (lds_ptr_t) lds);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" :: "v"(g), "s"(m) : "memory", "m0");
}

template <class W> struct mq_pipe {
    static_assert(W::BLK % 16 == 0, "weight blocks must be whole 16-byte chunks");
    static constexpr int RC = W::BLK / 16;                      // 16-byte chunks per weight row
    static constexpr int WQ = MQ_BM * W::BLK;                   // a weight stage
    static constexpr int NWI = (MQ_BM * RC / 64 + 3) / 4;       // weight DMA instructions per wave
    static constexpr int XD = MQ_BN * 256, XS = XD + MQ_BN * 4;
    static constexpr int XB = XS + MQ_BN * 32;                  // a token stage: rows, d, bsums
    static constexpr int NXI = 5;                               // token DMA instructions per wave
};

template <class W>
__global__ __launch_bounds__(256, 2) void k_mmq_p2(const mmq_args p) {
    using S = mq_pipe<W>;
    constexpr int RS = W::BLK;
    __shared__ __attribute__((aligned(16))) uint8_t xst[3][S::XB];
    __shared__ __attribute__((aligned(16))) uint8_t wst[2][S::WQ];
    __shared__ uint8_t wsc[MQ_BM][W::NSC];
    __shared__ uint8_t wmn[MQ_BM][8];
    __shared__ float wd[MQ_BM], wdm[MQ_BM];
    __shared__ int xs[MQ_BN][8];

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
    const int64_t nblk = p.nblk;

    const int8_t * xsrc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = 64 * (wave + 4 * k) + lane, t = c >> 4, part = (c & 15) ^ (t & 15);   // LDS slot (t, c & 15) holds chunk (c & 15) ^ (t & 15)
        xsrc[k] = p.xq + (col0 + min(tok0 + t, T - 1)) * p.K + 16 * part;
    }
    // the fifth token instruction: the scales (wave 0, and the same bytes again by wave 3) or
    // half of the bsums (waves 1, 2)
    const uint8_t * esrc;
    int eoff;
    const bool e4 = wave == 0 || wave == 3;
    if (e4) {
        esrc = (const uint8_t *) (p.xd + (col0 + min(tok0 + lane, T - 1)) * KB);
        eoff = S::XD;
    } else {
        const int c = 64 * (wave - 1) + lane, t = c >> 1, half = c & 1;
        esrc = (const uint8_t *) (p.xs + (col0 + min(tok0 + t, T - 1)) * (p.K / 16) + 8 * half);
        eoff = S::XS + 1024 * (wave - 1);
    }
    // weight instruction i = wave + 4j covers chunks 64i .. 64i+63 (row c / RC, chunk c % RC);
    // indices past the tile repeat the last instruction (same bytes, same LDS)
    const uint8_t * wsrc[S::NWI];
    int woff[S::NWI];
#pragma unroll
    for (int j = 0; j < S::NWI; ++j) {
        const int i = min(wave + 4 * j, MQ_BM * S::RC / 64 - 1);
        const int c = 64 * i + lane, r = c / S::RC, k = c % S::RC;
        wsrc[j] = Wb + min(row0 + r, p.M - 1) * p.nb01 + 16 * k;
        woff[j] = 1024 * i;
    }
    auto issue_w = [&](int64_t b, int ws_i) {
        b = min(b, nblk - 1);
#pragma unroll
        for (int j = 0; j < S::NWI; ++j) dma_lds16(wsrc[j] + b * W::BLK, wst[ws_i] + woff[j]);
    };
    auto issue_x = [&](int64_t b, int xs_i) {
        b = min(b, nblk - 1);
        uint8_t * base = xst[xs_i];
#pragma unroll
        for (int k = 0; k < 4; ++k) dma_lds16(xsrc[k] + b * 256, base + 1024 * (wave + 4 * k));
        if (e4) dma_lds4(esrc + 4 * b, base + eoff);
        else dma_lds16(esrc + 32 * b, base + eoff);
    };

    float acc[4][4];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[n][i] = 0.0f;

    // queue per wave, oldest first: X(0) | W(0) X(1) | W(1) X(2) | ... — at block b's top the
    // newest group (W(b) X(b+1)) is in flight and only X(b+1) may stay so
    issue_x(0, 0);
    issue_w(0, 0);
    issue_x(1, 1);
    int xi = 0;
    for (int64_t b = 0; b < nblk; ++b) {
        const int wi = (int) (b & 1);
        const uint8_t * wq = wst[wi];
        const uint8_t * xb = xst[xi];
        const int8_t * xq = (const int8_t *) xb;
        const float * xd = (const float *) (xb + S::XD);
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(S::NXI) : "memory");
        __syncthreads();   // block b's stages landed for every wave; block b-1's reads are done
        issue_w(b + 1, wi ^ 1);
        issue_x(b + 2, xi == 0 ? 2 : xi - 1);
        if (tid < MQ_BM) {
            int sc[16], mn[8];
            float d, dmin;
            W::unpack(wq + tid * RS, sc, mn, d, dmin);
#pragma unroll
            for (int j = 0; j < W::NSC; ++j) wsc[tid][j] = (uint8_t) sc[j];
#pragma unroll
            for (int j = 0; j < 8; ++j) wmn[tid][j] = (uint8_t) mn[j];
            wd[tid] = d; wdm[tid] = dmin;
        } else if (tid < MQ_BM + MQ_BN) {
            const int t = tid - MQ_BM;
            const int16_t * s16 = (const int16_t *) (xb + S::XS) + 16 * t;
#pragma unroll
            for (int j = 0; j < 8; ++j) xs[t][j] = s16[2 * j] + s16[2 * j + 1];
        }
        __syncthreads();
        const int rA = 16 * wave + c16;
        int sumi[4][4];
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) sumi[n][i] = 0;
#pragma unroll 2
        for (int c = 0; c < 8; ++c) {
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
                for (int i = 0; i < 4; ++i) sumi[n][i] += __mul24(r[i], scv[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 16 * wave + 4 * h + i;
            const float dw = wd[r], dmw = wdm[r];
#pragma unroll
            for (int n = 0; n < 4; ++n) {
                const int t = 16 * n + c16;
                const float dy = xd[t];
                int summ = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) summ += __mul24((int) wmn[r][j], xs[t][j]);
                acc[n][i] += (dw * dy) * (float) sumi[n][i] - (dmw * dy) * (float) summ;
            }
        }
        xi = xi == 2 ? 0 : xi + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped tail loads land before exit
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
            if (m < p.M) *(float *) (drow + m * 4) = acc[n][i];
        }
    }
}

// GGML_MI355X_MMQ_DB: 0 = single-buffered k_mmq, 1 = k_mmq_db, 2 = k_mmq_p2
static int mmq_db_mode() {
    static const int m = getenv("GGML_MI355X_MMQ_DB") ? atoi(getenv("GGML_MI355X_MMQ_DB")) : 1;
    return m;
}

template <class W>
static void launch_mmq(hipStream_t st, const dim3 & grid, const mmq_args & p) {
    const int m = mmq_db_mode();
    if constexpr (std::is_same<W, mq_q4_K>::value) {
        if (m == 2) { hipLaunchKernelGGL(k_mmq_p2<W>, grid, dim3(256), 0, st, p); return; }
    }
    if (m == 1) hipLaunchKernelGGL(k_mmq_db<W>, grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL(k_mmq<W>, grid, dim3(256), 0, st, p);
}

// ---- host --------------------------------------------------------------------------------------
bool mmq_supported(const ggml_tensor * dst) {
    static const bool off = getenv("GGML_MI355X_NO_MMQ") && atoi(getenv("GGML_MI355X_NO_MMQ")) != 0;
    if (off) return false;
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * x = dst->src[1];
    if (w->type != GGML_TYPE_Q4_K && w->type != GGML_TYPE_Q5_K && w->type != GGML_TYPE_Q6_K) return false;
    if (x->type != GGML_TYPE_F32 || dst->type != GGML_TYPE_F32) return false;
    if (w->ne[2] != 1 || w->ne[3] != 1 || x->ne[2] != 1 || x->ne[3] != 1) return false;
    if (x->ne[1] < 16) return false;             // decode stays on the mat-vec path
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
    p.dst = (float *) dst->data; p.nb1 = dst->nb[1];
    p.cnt = p.off = p.list = nullptr; p.n_used = 1; p.nb02 = 0; p.nb2 = 0;
    const dim3 grid((unsigned) ceil_div(p.M, MQ_BM), (unsigned) ceil_div(p.T, MQ_BN));
    // measured neutral on pp512 (10.3k-10.5k tok/s either way): the tiles are not L2-bound, so off
    static const int xcd = getenv("GGML_MI355X_MMQ_XCD") ? atoi(getenv("GGML_MI355X_MMQ_XCD")) : 0;
    p.xcd = xcd && grid.x % 8 == 0;
    switch (w->type) {
        case GGML_TYPE_Q4_K: launch_mmq<mq_q4_K>(ctx.stream, grid, p); break;
        case GGML_TYPE_Q5_K: launch_mmq<mq_q5_K>(ctx.stream, grid, p); break;
        case GGML_TYPE_Q6_K: launch_mmq<mq_q6_K>(ctx.stream, grid, p); break;
        default: GGML_ABORT("mi355x: mmq type");
    }
    if (ctx.timing) ctx.time_end(TK_MMQ, flops, ev);
}

// MUL_MAT_ID prefill on the MFMA tile: the pairs sorted by expert (cnt/off/list) and their
// activations quantized in that order (k_mmv.hip op_mul_mat_id); grid z = expert, workgroups past
// an expert's token count exit at once
bool mmq_id_supported(const ggml_tensor * dst) {
    static const bool off = getenv("GGML_MI355X_NO_MMQ") && atoi(getenv("GGML_MI355X_NO_MMQ")) != 0;
    const ggml_type t = dst->src[0]->type;
    return !off && (t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K);
}

void mul_mat_q_id(exec_ctx & ctx, ggml_tensor * dst, const q8_act & act, const int32_t * cnt, const int32_t * off,
                  const int32_t * list, int64_t n_pairs) {
    const ggml_tensor * w = dst->src[0];
    const ggml_tensor * ids = dst->src[2];
    mmq_args p;
    p.W = (const uint8_t *) w->data; p.nb01 = w->nb[1]; p.M = w->ne[1]; p.K = w->ne[0]; p.nblk = w->ne[0] / 256;
    p.xq = act.qs; p.xd = act.d; p.xs = act.s;
    p.T = n_pairs;
    p.dst = (float *) dst->data; p.nb1 = dst->nb[1];
    p.cnt = cnt; p.off = off; p.list = list; p.n_used = ids->ne[0]; p.nb02 = w->nb[2]; p.nb2 = dst->nb[2];
    p.xcd = 0;
    const dim3 grid((unsigned) ceil_div(p.M, MQ_BM), (unsigned) ceil_div(n_pairs, MQ_BN), (unsigned) w->ne[2]);
    switch (w->type) {
        case GGML_TYPE_Q4_K: launch_mmq<mq_q4_K>(ctx.stream, grid, p); break;
        case GGML_TYPE_Q5_K: launch_mmq<mq_q5_K>(ctx.stream, grid, p); break;
        case GGML_TYPE_Q6_K: launch_mmq<mq_q6_K>(ctx.stream, grid, p); break;
        default: GGML_ABORT("mi355x: mmq id type");
    }
}

}  // namespace mi355x
