// k_fattn_exact.hip — CPU-exact flash attention over an f16, q8_0 or q4_0 KV cache (every
// FLASH_ATTN_EXT the backend takes runs here).
//
// Reproduces ggml_compute_forward_flash_attn_ext_f16 (ggml-cpu/ops.cpp:7015-7232) as the
// x86-64-v4 (AVX-512) CPU backend computes it — the variant the reference selects on the
// MI355X host:
//   * Q rounded to f16; K·Q with ggml_vec_dot_f16's AVX-512 order (vec.cpp:191-231): 16
//     lanes x 4 accumulators of f32 FMAs, REDUCE (x0+=x2, x1+=x3, x0+=x1) then the
//     _mm512_reduce_add_ps tree (8/4/2/1);
//   * s = s*scale (softcap: softcap*tanh(s)), + slope*mask (ops.cpp:7100-7115);
//   * the online softmax walks the cache in order and accumulates VKQ in f16 with the
//     vec_mad_f16 / vec_scale_f16 roundings (vec.h:262-290, 410-440): y = f16(fma(v,vs,y)),
//     y = f16(y*ms); S = S*ms + vs (not contracted); glibc expf (libm_exact.h).
// q8_0 cache (Q8 = true): Q is quantized to q8_0 (the x86 quantize_row_q8_0), K·Q is
// ggml_vec_dot_q8_0_q8_0's class chains (arch/x86/quants.c:965: acc[c] = fma(dk·dq, cls[c],
// acc[c]) over the blocks, hsum_float_8), V is dequantized (d·q) and VKQ accumulates in f32:
// y = fma(v, vs, y), y = y*ms (ggml_vec_mad_f32 / ggml_vec_scale_f32).
//
// MI355X structure: one workgroup of 256 threads per (query row, query head) — 32 CUs busy
// for a Llama-3-8B decode step rather than one per KV head.  The cache is walked in chunks
// of CH positions:
//   A. the chunk's mask; the last unmasked position (wave ballots) bounds all later work;
//   0. V rows up to it are streamed HBM -> LDS with global_load_lds (async, overlapping 1-2);
//   1. scores: 4 lanes per position (lane q holds the AVX-512 lane partials 4q..4q+3), K
//      read straight from HBM with every load of the chunk in flight at once, q in VGPRs,
//      the reduction tree across the quad by DPP quad_perm;
//   2. prefix max over positions (wave scans) and the (ms, vs) coefficient of every
//      position, plus a per-batch flag marking batches with a masked position or a max
//      update;
//   3. the f16 recurrence — sequential over positions, one chain per output dimension, V
//      from LDS; a flagged-free batch is two dependent instructions per position
//      (v_fma_mix_f32, v_cvt_f16_f32).
// Output: O = y / S; optional Q8_0 / Q8_K quantization of the [H*D] row for the following
// MUL_MAT: Q8_0 blocks lie inside one head; a Q8_K block spanning 256/D heads is quantized
// by the last of its workgroups to finish (device-scope counter, self-resetting).
#include "fattn.h"
#include "quant_act.h"
#include "qtypes.h"
#include "fa_chain.h"
#include "fa_util.h"

#include <cmath>

namespace mi355x {

// ggml_vec_dot_f16 (AVX-512) of a K row with q, computed by the 4 lanes of a quad.  Lane q
// holds, for m < D/16, kh[m] = the 4 halves K[16m + 4q .. 16m + 4q + 3] and qf[m][c] =
// q[16m + 4q + c] (f16-rounded): the AVX-512 lane partials l = 4q + c (accumulator j = m % 4
// FMA'd over i = m / 4), REDUCE (x0+x2)+(x1+x3), then _mm512_reduce_add_ps's tree: t3[i] =
// w[i] + w[8+i] (quad lanes 0,1 with 2,3), t6[i] = t3[i] + t3[4+i] (lane 0 with 1),
// (t6[0]+t6[2]) + (t6[1]+t6[3]).  fp add is commutative, so only the association matters.
// The result is valid in quad lane 0.
template <int D>
__device__ __forceinline__ float dot_f16_avx512_q4(const uint2 (&kh)[D / 16], const float (&qf)[D / 16][4]) {
    float w[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float acc[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const uint2 k0 = kh[jj];
            const uint32_t h0 = (c < 2 ? k0.x : k0.y) >> (16 * (c & 1));
            float a = __fmul_rn(h2f((uint16_t) h0), qf[jj][c]);
#pragma unroll
            for (int i = 1; i < D / 64; ++i) {
                const uint2 ki = kh[4 * i + jj];
                const uint32_t hi = (c < 2 ? ki.x : ki.y) >> (16 * (c & 1));
                a = fmaf(h2f((uint16_t) hi), qf[4 * i + jj][c], a);
            }
            acc[jj] = a;
        }
        w[c] = __fadd_rn(__fadd_rn(acc[0], acc[2]), __fadd_rn(acc[1], acc[3]));
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = __fadd_rn(w[c], quad_from_plus2(w[c]));   // t3 (lanes 0, 1)
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = __fadd_rn(w[c], quad_from_plus1(w[c]));   // t6 (lane 0)
    return __fadd_rn(__fadd_rn(w[0], w[2]), __fadd_rn(w[1], w[3]));
}

template <int D, int CHO = 0> struct fax_cfg {
    // positions per chunk (V chunk <= 64 KiB); CHO overrides it (prefill: a 32 KiB chunk lets
    // more workgroups share a CU)
    static constexpr int CH = CHO ? CHO : (D <= 128 ? 256 : 128);
    static constexpr int NP = CH / 64;                // score passes per chunk (64 positions each)
    static constexpr int RPP = 512 / D;               // V rows per 1 KiB global_load_lds piece
    static constexpr int U = 8;                       // phase-3 positions per batch
};

// OCC = workgroups per CU the register budget allows: 1 for decode (32-64 workgroups, every
// register for ILP), 2 for prefill (thousands of workgroups; the LDS allows two)
// Q8: a quantized cache; Q4 (with Q8): q4_0 blocks instead of q8_0 (ggml_vec_dot_q4_0_q8_0,
// arch/x86/quants.c:531: the same eight class chains over (nibble - 8) · q8, d = dk·dq; V
// dequantized as (nibble - 8)·d, dequantize_row_q4_0)
template <int D, int OCC = 1, int CHO = 0, bool Q8 = false, bool Q4 = false>
__global__ __launch_bounds__(256, OCC) void k_fattn_exact(const fa_args a) {
    constexpr int KB = Q4 ? 18 : 34;   // bytes per 32-element K / V block
    using C = fax_cfg<D, CHO>;
    constexpr int CH = C::CH, U = C::U, NM = D / 16, NB = D / 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int qd = tid & 3;                 // lane in the quad of a position (phase 1)
    kt_enter(a.kt, 5);
    const int64_t iq1 = blockIdx.x;
    const int64_t h = blockIdx.y % a.H;
    const int64_t iq3 = blockIdx.y / a.H;
    const int64_t hk = h / (a.H / a.Hkv);

    // V chunk: [pos][D] f16, or (Q8) [pos][D] int8 + [pos][D/32] block scales
    __shared__ __attribute__((aligned(16))) uint16_t vl[Q8 ? CH * D / 2 : CH * D];
    __shared__ float vd[Q8 ? CH * NB : 1];
    __shared__ __attribute__((aligned(16))) int8_t qq[Q8 ? D : 1];   // Q as q8_0 (Q8)
    __shared__ float qqd[Q8 ? NB : 1];
    __shared__ int16_t qqs[Q8 ? NB : 1];
    __shared__ __attribute__((aligned(16))) float sc[CH + 6 * U];    // scores -> vs coefficient (0 where masked)
    __shared__ __attribute__((aligned(16))) float cm[CH + 6 * U];    // ms coefficient (1 where masked)
    __shared__ __attribute__((aligned(16))) float mk[CH + 6 * U];    // mask values of the chunk (-inf = skipped)
    __shared__ uint32_t wflag[4];    // per wave: batches needing the general step (mask / max update)
    __shared__ int wlast[4];
    __shared__ float wmax[4];

    // q of this head, f16-rounded, in the quad layout of dot_f16_avx512_q4
    float qf[NM][4];
    const char * mrow = a.mask ? a.mask + (iq1 % a.mask_ne1) * a.nbm1 : nullptr;
    // the first chunk's mask value of this thread is loaded together with q, so the two
    // memory latencies overlap instead of following each other
    uint16_t mk0 = 0;
    float4 q4[NM];
    {
        const float * qrow = (const float *) (a.q + iq1 * a.nbq1 + h * a.nbq2 + iq3 * a.nbq3);
#pragma unroll
        for (int m = 0; m < NM; ++m) q4[m] = *(const float4 *) (qrow + 16 * m + 4 * qd);
        if (mrow && tid < min((int64_t) CH, a.n_kv)) mk0 = *(const uint16_t *) (mrow + 2 * tid);
    }
    {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            qf[m][0] = f16r(q4[m].x); qf[m][1] = f16r(q4[m].y); qf[m][2] = f16r(q4[m].z); qf[m][3] = f16r(q4[m].w);
        }
    }
    // Q8: q as q8_0 blocks (lane qd of a quad takes classes 2qd, 2qd+1 of every block)
    uint2 qb[Q8 ? NB : 1];
    float qdb[Q8 ? NB : 1];
    if constexpr (Q8) {
        if (wave == 0) {
            const float * qrow = (const float *) (a.q + iq1 * a.nbq1 + h * a.nbq2 + iq3 * a.nbq3);
            for (int b0 = 0; b0 < D; b0 += 256) {
                const bool valid = b0 + 4 * lane < D;
                float qv[4] = {0.f, 0.f, 0.f, 0.f};
                if (valid) { const float4 t = *(const float4 *) (qrow + b0 + 4 * lane); qv[0] = t.x; qv[1] = t.y; qv[2] = t.z; qv[3] = t.w; }
                q8_0_wave(qv, lane, valid, qq + b0, qqd + b0 / 32, qqs + b0 / 32);
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            qb[b] = *(const uint2 *) (qq + 32 * b + 8 * qd);
            qdb[b] = qqd[b];
        }
    }
    const float slope = a.max_bias > 0.0f
        ? (float) ((uint32_t) h < a.n_head_log2 ? pow((double) a.m0, (double) (h + 1))
                                               : pow((double) a.m1, (double) (2 * ((uint32_t) h - a.n_head_log2) + 1)))
        : 1.0f;

    // phase-3 state: output dim d = tid (threads < D)
    const int d = tid;
    uint32_t yb = 0;   // f16 bits (low half)
    float yf = 0.0f;   // Q8: the f32 accumulator
    float S = 0.0f;
    float mcarry = -INFINITY;   // running max of the previous chunks (uniform)

    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;

    const bool prof = a.prof && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0;
    unsigned long long tp = prof ? __builtin_amdgcn_s_memtime() : 0, pc[6] = {0, 0, 0, 0, 0, 0};
    auto mark = [&](int i) {
        if (prof) { const unsigned long long t = __builtin_amdgcn_s_memtime(); pc[i] += t - tp; tp = t; }
    };

    for (int64_t c0 = 0; c0 < a.n_kv; c0 += CH) {
        const int nch = (int) min((int64_t) CH, a.n_kv - c0);
        // ---- phase A: mask of the chunk; the last unmasked position bounds all later work --
        int last = -1;
        for (int j0 = 0; j0 < CH + U; j0 += 256) {
            const int j = j0 + tid;
            float mv = -INFINITY;
            if (j < nch) mv = mrow ? h2f(c0 == 0 && j0 == 0 ? mk0 : *(const uint16_t *) (mrow + 2 * (c0 + j))) : 0.0f;
            if (j < CH + U) mk[j] = mv;
            const unsigned long long b = __ballot(mv != -INFINITY);
            if (b) last = j0 + 64 * wave + 63 - __clzll(b);
        }
        if (lane == 0) wlast[wave] = last;
        __syncthreads();
        const int nrun = max(max(wlast[0], wlast[1]), max(wlast[2], wlast[3])) + 1;
        mark(0);
        if (nrun == 0) { __syncthreads(); continue; }   // whole chunk masked
        // ---- phase 0: V rows [0, nrun) HBM -> LDS (async; waited on before phase 3) -------
        if constexpr (!Q8) {
            const int r_in = lane / (D / 8), col = lane % (D / 8);
            for (int p = wave; p * C::RPP < nrun; p += 4) {
                const int row = min(p * C::RPP + r_in, nrun - 1);
                const char * src = vbase + (c0 + row) * a.nbv1 + col * 16;
                __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) (vl + p * 512), 16, 0, 0);
            }
        } else {
            // q8_0 / q4_0 blocks (2-byte aligned): quants to vq[pos][D] (q4_0: nibble - 8),
            // scales to vd[pos][D/32]
            int8_t * vq = (int8_t *) vl;
            for (int i = tid; i < nrun * NB; i += 256) {
                const int row = i / NB, b = i % NB;
                const uint8_t * src = (const uint8_t *) vbase + (c0 + row) * a.nbv1 + KB * b;
                if constexpr (Q4) {
                    // element j < 16: low nibble of qs[j]; j >= 16: high nibble of qs[j - 16]
                    const uint4 q = ld16(src + 2);
                    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
                    uint32_t lo[4], hi[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        // (nibble - 8) per byte: n + 0x78 stays inside its byte (<= 135), and
                        // flipping bit 7 turns it into n - 8 as an int8
                        lo[k] = ((w[k] & 0x0f0f0f0fu) + 0x78787878u) ^ 0x80808080u;
                        hi[k] = (((w[k] >> 4) & 0x0f0f0f0fu) + 0x78787878u) ^ 0x80808080u;
                    }
                    *(uint4 *) (vq + row * D + 32 * b) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
                    *(uint4 *) (vq + row * D + 32 * b + 16) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
                } else {
                    const uint4 lo = ld16(src + 2), hi = ld16(src + 18);
                    *(uint4 *) (vq + row * D + 32 * b) = lo;
                    *(uint4 *) (vq + row * D + 32 * b + 16) = hi;
                }
                vd[row * NB + b] = h2f(ld2(src));
            }
        }
        mark(1);
        // ---- phase 1: scores, 4 lanes per position, every K load of the chunk in flight ----
        if constexpr (Q8) {
            // lane qd holds bytes 8qd .. 8qd+7 of every block: classes 2qd, 2qd+1
            uint2 kb[C::NP][NB];
            uint32_t kd[C::NP][NB];
#pragma unroll
            for (int p = 0; p < C::NP; ++p) {
                const int j = min(64 * p + (tid >> 2), nrun - 1);
                const uint8_t * krow = (const uint8_t *) kbase + (c0 + j) * a.nbk1;
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    if (64 * p < nrun) {
                        if constexpr (Q4) {
                            // elements 8qd .. 8qd+7: qs[8 (qd & 1) ..] nibble qd >> 1, minus 8
                            const uint2 q = ld8(krow + KB * b + 2 + 8 * (qd & 1));
                            const int sh = 4 * (qd >> 1);
                            kb[p][b] = make_uint2((((q.x >> sh) & 0x0f0f0f0fu) + 0x78787878u) ^ 0x80808080u,
                                                  (((q.y >> sh) & 0x0f0f0f0fu) + 0x78787878u) ^ 0x80808080u);
                        } else {
                            kb[p][b] = ld8(krow + KB * b + 2 + 8 * qd);
                        }
                        kd[p][b] = ld2(krow + KB * b);
                    }
                }
            }
#pragma unroll
            for (int p = 0; p < C::NP; ++p) {
                if (64 * p >= nrun) break;
                const int j = 64 * p + (tid >> 2);
                float ae = 0.0f, ao = 0.0f;
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    const float dd = __fmul_rn(h2f((uint16_t) kd[p][b]), qdb[b]);
                    ae = fmaf(dd, (float) dot4((int) kb[p][b].x, (int) qb[b].x, 0), ae);
                    ao = fmaf(dd, (float) dot4((int) kb[p][b].y, (int) qb[b].y, 0), ao);
                }
                // hsum_float_8 over the quad: lanes hold (a[2q], a[2q+1])
                ae = __fadd_rn(ae, quad_from_plus2(ae));
                ao = __fadd_rn(ao, quad_from_plus2(ao));
                ae = __fadd_rn(ae, quad_from_plus1(ae));
                ao = __fadd_rn(ao, quad_from_plus1(ao));
                const float w = __fadd_rn(ae, ao);
                if (qd == 0 && j < nrun) {
                    float s = __fmul_rn(w, a.scale);
                    if (a.softcap != 0.0f) s = __fmul_rn(a.softcap, tanhf(s));
                    sc[j] = __fadd_rn(s, __fmul_rn(slope, mk[j]));
                }
            }
        } else {
            uint2 kh[C::NP][NM];
#pragma unroll
            for (int p = 0; p < C::NP; ++p) {
                const int j = min(64 * p + (tid >> 2), nrun - 1);
                const char * krow = kbase + (c0 + j) * a.nbk1 + 8 * qd;
#pragma unroll
                for (int m = 0; m < NM; ++m) {
                    if (64 * p < nrun) kh[p][m] = ld8(krow + 32 * m);
                }
            }
#pragma unroll
            for (int p = 0; p < C::NP; ++p) {
                if (64 * p >= nrun) break;
                const int j = 64 * p + (tid >> 2);
                const float w = dot_f16_avx512_q4<D>(kh[p], qf);
                if (qd == 0 && j < nrun) {
                    float s = __fmul_rn(w, a.scale);
                    if (a.softcap != 0.0f) s = __fmul_rn(a.softcap, tanhf(s));
                    sc[j] = __fadd_rn(s, __fmul_rn(slope, mk[j]));
                }
            }
        }
        __syncthreads();
        mark(2);
        // ---- phase 2: prefix max and the (ms, vs) coefficients (one position per thread) ---
        {
            const int j = tid;
            const bool live = j < nrun && j < CH && mk[j] != -INFINITY;
            const float sj = live ? sc[j] : -INFINITY;
            float sm = sj;   // inclusive max-scan over the wave
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const float t = __shfl_up(sm, o, WAVE);
                if (lane >= o) sm = fmaxf(sm, t);
            }
            if (lane == 63) wmax[wave] = sm;
            __syncthreads();
            float M = mcarry;   // max over every position before j
            for (int w = 0; w < wave; ++w) M = fmaxf(M, wmax[w]);
            const float ex = __shfl_up(sm, 1, WAVE);
            if (lane > 0) M = fmaxf(M, ex);
            if (j < CH) {
                if (j < nrun) {
                    if (!live) {
                        cm[j] = 1.0f; sc[j] = 0.0f;
                    } else if (sj > M) {
                        cm[j] = M == -INFINITY ? 0.0f : expf_cr(M - sj);   // ms, applied before the add
                        sc[j] = 1.0f;                                       // vs
                    } else {
                        cm[j] = 1.0f;
                        sc[j] = expf_cr(sj - M);
                    }
                }
            }
            if (tid < U) { cm[nrun + tid] = 1.0f; sc[nrun + tid] = 0.0f; mk[nrun + tid] = -INFINITY; }
            // batch flags: a masked position, a max update or padding inside the batch
            const bool general = j < nrun ? (!live || sj > M) : (j < nrun + U);
            const unsigned long long bw = __ballot(j < CH && general);
            if (lane == 0) {
                uint32_t f = 0;
#pragma unroll
                for (int b = 0; b < 64 / U; ++b) f |= ((bw >> (U * b)) & ((1ull << U) - 1)) ? 1u << b : 0u;
                wflag[wave] = f;
            }
            mcarry = fmaxf(fmaxf(mcarry, fmaxf(wmax[0], wmax[1])), fmaxf(wmax[2], wmax[3]));
        }
        mark(3);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        mark(4);
        uint64_t bmask = 0;   // bit n: batch n takes the general step (uniform)
#pragma unroll
        for (int w = 0; w < 4; ++w) bmask |= (uint64_t) wflag[w] << ((64 / U) * w);
        bmask = ((uint64_t) __builtin_amdgcn_readfirstlane((uint32_t) (bmask >> 32)) << 32) |
                __builtin_amdgcn_readfirstlane((uint32_t) bmask);
        // ---- phase 3: sequential f16 recurrence (V from LDS) --------------------------------
        // y = f16(y*ms) and S*ms only where the running max moved (ms != 1: y*1 and S*1 are
        // identities); masked / padded positions keep the state (-0 must survive)
        if (Q8 && d < D) {
            // f32 recurrence: y = y*ms where the running max moved, y = fma(v, vs, y),
            // S = S*ms + vs; masked positions keep the state
            const int8_t * vq = (const int8_t *) vl;
            for (int j = 0; j < nrun; ++j) {
                const float v = __fmul_rn((float) vq[j * D + d], vd[j * NB + d / 32]);
                const float vs = sc[j], ms = cm[j];
                const bool live = __float_as_uint(mk[j]) != 0xff800000u;
                const bool upd = __float_as_uint(ms) != 0x3f800000u;
                const float ys = upd ? __fmul_rn(yf, ms) : yf;
                const float Ss = upd ? __fmul_rn(S, ms) : S;
                yf = live ? fmaf(v, vs, ys) : yf;
                S = live ? __fadd_rn(Ss, vs) : S;
            }
        }
        if (!Q8 && d < D) {
            // batches of U positions, software-pipelined: batch n+1's V values and
            // coefficients are read from LDS while batch n computes
            // (a prefetch past the chunk end reads other LDS arrays or past the allocation, which
            // reads as 0 — never used: batches at or past nrun do not run)
            // batch n+1's V values and vs coefficients come from LDS while batch n computes: U
            // u16 reads of the thread's V column plus U/4 broadcast b128 reads of vs, few enough
            // to stay under the 15-deep LDS counter, so the prefetch really overlaps (U = 16
            // with scalar coefficient reads saturated it: ~66 cycles per position)
            auto ld4 = [&](const float * p, float (&o)[U]) {
#pragma unroll
                for (int u = 0; u < U; u += 4) {
                    const float4 t = *(const float4 *) (p + u);
                    o[u] = t.x; o[u + 1] = t.y; o[u + 2] = t.z; o[u + 3] = t.w;
                }
            };
            auto ldb = [&](int j, uint32_t (&vv)[U], float (&vs)[U]) {
                const uint16_t * vp = vl + j * D + d;
#pragma unroll
                for (int u = 0; u < U; ++u) vv[u] = vp[u * D];
                ld4(sc + j, vs);
            };
            auto run = [&](int j, const uint32_t (&vv)[U], const float (&vs)[U]) {
                if (((bmask >> (j / U)) & 1u) == 0) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        yb = f16_mad(vv[u], vs[u], yb);
                        S = __fadd_rn(S, vs[u]);   // not contracted on the CPU
                    }
                    return;
                }
                // masked / padded position: the state is kept (-0 must survive); a running-max
                // update (ms != 1): y = f16(y*ms), S = S*ms before the add — the CPU's
                // vec_scale_f16 / S*ms (ops.cpp:7120-7160); otherwise y*1 and S*1 are skipped.
                // Selects, not branches on LDS values.
                float ms[U], mv[U];
                ld4(cm + j, ms);
                ld4(mk + j, mv);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const bool live = __float_as_uint(mv[u]) != 0xff800000u;
                    const bool upd = __float_as_uint(ms[u]) != 0x3f800000u;
                    float t = __fmul_rn(h2f((uint16_t) yb), ms[u]);
                    asm("" : "+v"(t));   // two roundings, as f16r
                    const uint32_t ys = upd ? (uint32_t) f2h(t) : yb;
                    const float Ss = upd ? __fmul_rn(S, ms[u]) : S;
                    const uint32_t yn = f16_mad(vv[u], vs[u], ys);
                    const float Sn = __fadd_rn(Ss, vs[u]);
                    yb = live ? yn : yb;
                    S = live ? Sn : S;
                }
            };
            uint32_t va[U], vb[U];
            float sa[U], sb[U];
            ldb(0, va, sa);
            for (int j = 0; j < nrun; j += 2 * U) {
                ldb(j + U, vb, sb);
                run(j, va, sa);
                if (j + U >= nrun) break;
                ldb(j + 2 * U, va, sa);
                run(j + U, vb, sb);
            }
        }
        __syncthreads();
        mark(5);
    }
    if (prof) {
        for (int i = 0; i < 6; ++i) a.prof[i] += pc[i];
    }

    // ---- output and its optional quantization ------------------------------------------------
    float * drow = (float *) ((char *) a.dst + iq1 * a.nb1_dst * a.H + h * a.nb1_dst + iq3 * a.nb2_dst);
    const float o = d < D ? __fmul_rn(Q8 ? yf : h2f((uint16_t) yb), 1.0f / S) : 0.0f;
    // a Q8_K block spanning several heads is handed to the last of their workgroups: the
    // outputs are stored write-through (sc1) and drained before the counter add, and read
    // back with sc1 loads, so no L2 write-back fence is needed (MI355X_MICROARCH.md,
    // inter-workgroup visibility, first hand-off row)
    constexpr bool handoff = D < 256;
    if (d < D) {
        if (handoff && a.qmode == 1) __hip_atomic_store(drow + d, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else drow[d] = o;
    }
    if (a.qmode == 2) {
        // Q8_0: the head's D outputs are D/32 whole blocks of the flat [H*D] row
        const int64_t K = a.H * D;
        float * ol = (float *) sc;
        __syncthreads();
        if (d < D) ol[d] = o;
        __syncthreads();
        for (int b0 = 256 * wave; b0 < D; b0 += 1024) {
            const bool valid = b0 + 4 * lane < D;
            float q[4] = {0.f, 0.f, 0.f, 0.f};
            if (valid) { const float4 v4 = *(const float4 *) (ol + b0 + 4 * lane); q[0] = v4.x; q[1] = v4.y; q[2] = v4.z; q[3] = v4.w; }
            const int64_t c0 = h * D + b0;
            q8_0_wave(q, lane, valid, a.qs + iq1 * K + c0, a.qd + iq1 * (K / 32) + c0 / 32, a.qsum + iq1 * (K / 32) + c0 / 32);
        }
    } else if (a.qmode == 1) {
        // Q8_K: block b = 256 elements = NH heads; the last of its NH workgroups quantizes it
        constexpr int NH = D >= 256 ? 1 : 256 / D;
        const int64_t K = a.H * D;
        const int64_t blk = (h * D) / 256;
        __shared__ int is_last;
        if (NH > 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
            __syncthreads();
            if (tid == 0) {
                const int prev = __hip_atomic_fetch_add(a.cnt + blk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                is_last = prev == NH - 1;
                if (is_last) __hip_atomic_store(a.cnt + blk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
        } else {
            if (tid == 0) is_last = 1;
            __syncthreads();
        }
        if (is_last && wave == 0) {
            const float * brow = (const float *) ((char *) a.dst + iq1 * a.nb1_dst * a.H) + 256 * blk;
            float q[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) q[c] = __hip_atomic_load(brow + 4 * lane + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int64_t c0 = 256 * blk;
            q8K_wave(q, lane, a.qs + iq1 * K + c0, a.qsum + iq1 * (K / 16) + c0 / 16, a.qd + iq1 * (K / 256) + c0 / 256);
        }
    }
    kt_exit(a.kt, 5);
}

// ==== prefill: a block of query rows x the G query heads of one KV head per workgroup ========
// Same arithmetic as k_fattn_exact (the AVX-512 f16 dot order, the prefix-max coefficients, the
// f16 VKQ recurrence with the CPU's roundings), arranged for a batch of queries: the 16 (query
// row, head) pairs of a workgroup share every K and V row it stages, so the cache is read from
// L2 once per 16 pairs instead of once per pair, and each thread carries 8 independent f16
// chains (2 dims x 4 pairs) instead of one.  Wave w owns pairs 4w..4w+3 through all three
// phases (scores, coefficients, recurrence), so the only workgroup barrier per 64-position
// chunk is the one that publishes the next K / V / mask stage (double-buffered, LDS-DMA).
// K rows are XOR-swizzled in LDS (16-byte chunk c of row r in slot c ^ 2(r & 3)) so the four
// rows a phase-1 instruction touches sit in different banks.
constexpr int PF_CH = 64, PF_P = 16, PF_U = 8;

// two f16 chains in one register (low half = dim 2l, high half = dim 2l + 1):
// y = f16(fma(v, vs, y)) per half — the f32 fma rounded, then rounded to f16 by
// v_cvt_pk_f16_f32 (round to nearest even, as v_cvt_f16_f32), three instructions for two steps
__device__ __forceinline__ uint32_t f16x2_mad(uint32_t vbits, float vs, uint32_t ybits) {
    float t0, t1;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t0) : "v"(vbits), "v"(vs), "v"(ybits));
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(t1) : "v"(vbits), "v"(vs), "v"(ybits));
    uint32_t r;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(t0), "v"(t1));
    return r;
}

// y = f16(f32(y) * ms) per half (f16_scale on both halves)
__device__ __forceinline__ uint32_t f16x2_scale(uint32_t ybits, float ms, float nz) {
    float t0, t1;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(t0) : "v"(ybits), "v"(ms), "v"(nz));
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(t1) : "v"(ybits), "v"(ms), "v"(nz));
    uint32_t r;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(t0), "v"(t1));
    return r;
}

// two fp32 sums of the CPU's sequence, one v_pk_add_f32 (each half an IEEE add)
__device__ __forceinline__ float2 f32x2_add(float2 a, float2 b) {
    float2 r;
    asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float2 f32x2_mul(float2 a, float2 b) {
    float2 r;
    asm("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int G, int CH = PF_CH, int OCC = 2>
__global__ __launch_bounds__(256, OCC) void k_fattn_pf(const fa_args a) {
    constexpr int D = 128, NM = D / 16, QB = PF_P / G;
    // the 32-position variant: 4-position batches and q held as packed f16 pairs (its VGPR budget)
    constexpr int U = CH == 32 ? 4 : PF_U;
    constexpr bool QH = CH == 32;
    __shared__ __attribute__((aligned(16))) uint16_t kl[2][CH * D];
    __shared__ __attribute__((aligned(16))) uint16_t vl[2][CH * D];
    __shared__ __attribute__((aligned(16))) uint16_t ml[2][QB * CH];   // mask values (f16)
    __shared__ __attribute__((aligned(16))) float sc[CH * PF_P];       // scores -> vs, [pos][pair]
    __shared__ __attribute__((aligned(16))) float cm[CH * PF_P];       // ms, [pos][pair]
    __shared__ int wend[4];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // longest causal prefixes first
    const int64_t q0 = (int64_t) (gridDim.x - 1 - blockIdx.x) * QB;
    const int64_t hk = blockIdx.y % a.Hkv, iq3 = blockIdx.y / a.Hkv;
    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;
    auto qrow_of = [&](int p) { return min(q0 + p / G, a.n_q - 1); };
    auto head_of = [&](int p) { return hk * G + p % G; };
    auto slope_of = [&](int p) -> float {
        if (a.max_bias <= 0.0f) return 1.0f;
        const uint32_t h = (uint32_t) head_of(p);
        return (float) (h < a.n_head_log2 ? pow((double) a.m0, (double) (h + 1))
                                          : pow((double) a.m1, (double) (2 * (h - a.n_head_log2) + 1)));
    };

    // ---- the cache positions any of the QB query rows attends: [0, nend) --------------------
    int64_t nend = a.n_kv;
    if (a.mask) {
        int last = -1;
        for (int qi = 0; qi < QB; ++qi) {
            const uint16_t * mr = (const uint16_t *) (a.mask + (min(q0 + qi, a.n_q - 1) % a.mask_ne1) * a.nbm1);
            for (int64_t j0 = 0; j0 < a.n_kv; j0 += 256) {
                const int64_t j = j0 + tid;
                const bool live = j < a.n_kv && mr[j] != 0xfc00;   // f16 -inf
                const unsigned long long b = __ballot(live);
                if (b) last = max(last, (int) (j0 + 64 * wave + 63 - __clzll(b)));
            }
        }
        if (lane == 0) wend[wave] = last;
        __syncthreads();
        nend = max(max(wend[0], wend[1]), max(wend[2], wend[3])) + 1;
    }
    const int nchunk = (int) ((nend + CH - 1) / CH);
    // microbenchmark hook: per-phase s_memtime cycles of workgroup (0, 0) wave 0 (capi.cpp op 302)
    const bool prof = a.prof && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0;
    unsigned long long tp = prof ? __builtin_amdgcn_s_memtime() : 0, pc[6] = {0, 0, 0, 0, 0, 0};
    auto mark = [&](int i) {
        if (prof) { const unsigned long long t = __builtin_amdgcn_s_memtime(); pc[i] += t - tp; tp = t; }
    };

    // ---- staging: K (swizzled) and V rows of a chunk by LDS-DMA, its mask through registers -----
    auto issue_kv = [&](int c, int s) {
        const int64_t c0 = (int64_t) c * CH;
#pragma unroll
        for (int k = 0; k < CH / 16; ++k) {
            const int i = wave + 4 * k;                       // 1 KiB piece: rows 4i .. 4i+3
            const int r = 4 * i + (lane >> 4), cs = lane & 15;
            const int64_t row = min(c0 + r, a.n_kv - 1);
            __builtin_amdgcn_global_load_lds((const void *) (kbase + row * a.nbk1 + 16 * (cs ^ (2 * (r & 3)))),
                                             (lds_ptr_t) (kl[s] + 512 * i), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void *) (vbase + row * a.nbv1 + 16 * cs),
                                             (lds_ptr_t) (vl[s] + 512 * i), 16, 0, 0);
        }
    };
    constexpr int MPT = (QB * CH + 255) / 256;   // mask values per thread
    uint16_t mreg[MPT];
    auto load_mask = [&](int c) {
        const int64_t c0 = (int64_t) c * CH;
#pragma unroll
        for (int k = 0; k < MPT; ++k) {
            const int e = tid + 256 * k, qi = e / CH, j = e % CH;
            uint16_t v = 0xfc00;
            if (e < QB * CH && c0 + j < a.n_kv) {
                v = 0;
                if (a.mask) v = *(const uint16_t *) (a.mask + (min(q0 + qi, a.n_q - 1) % a.mask_ne1) * a.nbm1 + 2 * (c0 + j));
            }
            mreg[k] = v;
        }
    };
    auto store_mask = [&](int s) {
#pragma unroll
        for (int k = 0; k < MPT; ++k) {
            const int e = tid + 256 * k;
            if (e < QB * CH) ml[s][e] = mreg[k];
        }
    };

    // ---- phase-1 role: quad qi = lane / 4 scores pair 4w + (qi & 3) at positions 4r + qi / 4 --
    const int qd = lane & 3, qi = lane >> 2;
    const int p1 = 4 * wave + (qi & 3), r1 = qi >> 2;
    // (QH: quad qi scores pairs 4w + 2 (qi & 1) and the next one at positions 8r + qi / 2 — each K
    // row read from LDS once for two pairs; q of both as packed f16 pairs)
    const int pa = 4 * wave + 2 * (qi & 1), ra = qi >> 1;
    float qf[QH ? 1 : NM][4];
    uint32_t qh[QH ? 2 : 1][QH ? NM : 1][2];
    if constexpr (QH) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const float * qr = (const float *) (a.q + qrow_of(pa + e) * a.nbq1 + head_of(pa + e) * a.nbq2 + iq3 * a.nbq3);
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                const float4 t = *(const float4 *) (qr + 16 * m + 4 * qd);
                qh[e][m][0] = (uint32_t) f2h(t.x) | ((uint32_t) f2h(t.y) << 16);
                qh[e][m][1] = (uint32_t) f2h(t.z) | ((uint32_t) f2h(t.w) << 16);
            }
        }
    } else {
        const float * qr = (const float *) (a.q + qrow_of(p1) * a.nbq1 + head_of(p1) * a.nbq2 + iq3 * a.nbq3);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            const float4 t = *(const float4 *) (qr + 16 * m + 4 * qd);
            qf[m][0] = f16r(t.x); qf[m][1] = f16r(t.y); qf[m][2] = f16r(t.z); qf[m][3] = f16r(t.w);
        }
    }
    const float slope_a = slope_of(pa), slope_b = slope_of(pa + 1);
    const float slope1 = slope_of(p1);
    float nz = -0.0f;
    asm volatile("" : "+v"(nz));
    // ---- phase-2/3 state of the wave's 4 pairs --------------------------------------------------
    float mc[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};   // running max (uniform)
    uint32_t y[4] = {0, 0, 0, 0};                                  // f16 x 2: dims 2 lane, 2 lane + 1
    float2 S[2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};                      // pairs (0, 1), (2, 3)
    float slope2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) slope2[i] = slope_of(4 * wave + i);

    if (nchunk > 0) {
        issue_kv(0, 0);
        load_mask(0);
        store_mask(0);
    }
    for (int c = 0; c < nchunk; ++c) {
        const int s = c & 1;
        const int64_t c0 = (int64_t) c * CH;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();   // stage s (K, V, mask) is in; every wave is done with stage s^1
        const bool more = c + 1 < nchunk;
        if (more) {
            issue_kv(c + 1, s ^ 1);
            load_mask(c + 1);
        }
        mark(0);
        const uint16_t * ks = kl[s];
        const uint16_t * ms = ml[s];
        // ---- phase 1: scores of the wave's 4 pairs x 64 positions --------------------------
        auto score_of = [&](float w, float slope, int p, int j) {
            float sv = __fmul_rn(w, a.scale);
            if (a.softcap != 0.0f) sv = __fmul_rn(a.softcap, tanhf(sv));
            sc[j * PF_P + p] = __fadd_rn(sv, __fmul_rn(slope, h2f(ms[(p / G) * CH + j])));
        };
        if constexpr (QH) {
#pragma unroll 2
            for (int r = 0; r < CH / 8; ++r) {
                const int j = 8 * r + ra;
                uint2 kh[NM];
#pragma unroll
                for (int m = 0; m < NM; ++m)
                    kh[m] = *(const uint2 *) ((const char *) ks + j * 256 + 16 * ((2 * m + (qd >> 1)) ^ (2 * (j & 3))) + 8 * (qd & 1));
                const float wa = dot_f16_mix_d128_h(kh, qh[0], nz);
                const float wb = dot_f16_mix_d128_h(kh, qh[1], nz);
                if (qd == 0) {
                    score_of(wa, slope_a, pa, j);
                    score_of(wb, slope_b, pa + 1, j);
                }
            }
        } else {
#pragma unroll 4
            for (int r = 0; r < CH / 4; ++r) {
                const int j = 4 * r + r1;
                uint2 kh[NM];
#pragma unroll
                for (int m = 0; m < NM; ++m)
                    kh[m] = *(const uint2 *) ((const char *) ks + j * 256 + 16 * ((2 * m + (qd >> 1)) ^ (2 * (j & 3))) + 8 * (qd & 1));
                const float w = dot_f16_mix_d128(kh, qf, nz);
                if (qd == 0) score_of(w, slope1, p1, j);
            }
        }
        asm volatile("" ::: "memory");
        mark(1);
        // ---- phase 2: per pair, the prefix max and the (ms, vs) coefficient of every position -
        // per pair: positions that update the running max / that are masked (uniform)
        uint64_t upd[4], dead[4];
        if constexpr (CH == 32) {
            // two pairs per pass: lanes 0-31 pair 2 ii, lanes 32-63 pair 2 ii + 1 (a scan segmented
            // at 32 lanes: the row_bcast:31 step left out, the exclusive shift cut at lane 32)
            const int hf = lane >> 5, j = lane & 31;
#pragma unroll
            for (int ii = 0; ii < 2; ++ii) {
                const int i = 2 * ii + hf, p = 4 * wave + i;
                const bool live = c0 + j < nend && ms[(p / G) * CH + j] != 0xfc00;
                const float sj = live ? sc[j * PF_P + p] : -INFINITY;
                float sm = sj;
                sm = fmaxf(sm, dpp_ninf<0x111>(sm));
                sm = fmaxf(sm, dpp_ninf<0x112>(sm));
                sm = fmaxf(sm, dpp_ninf<0x114>(sm));
                sm = fmaxf(sm, dpp_ninf<0x118>(sm));
                sm = fmaxf(sm, dpp_ninf<0x142, 0xa>(sm));
                const float ex = dpp_ninf<0x138>(sm);
                float m_lo = mc[2 * ii], m_hi = mc[2 * ii + 1];
                asm volatile("" : "+v"(m_lo), "+v"(m_hi));   // (a select of two array loads would become an indexed, scratch, access)
                const float mci = hf ? m_hi : m_lo;
                const float M = fmaxf(mci, j == 0 ? -INFINITY : ex);   // max over every position before j
                float vs, mv;
                if (!live) { mv = 1.0f; vs = 0.0f; }
                else if (sj > M) { mv = M == -INFINITY ? 0.0f : expf_cr(M - sj); vs = 1.0f; }
                else { mv = 1.0f; vs = expf_cr(sj - M); }
                cm[j * PF_P + p] = mv;
                sc[j * PF_P + p] = vs;
                const uint64_t bu = __ballot(live && sj > M), bd = __ballot(!live);
                upd[2 * ii] = bu & 0xffffffffull;
                upd[2 * ii + 1] = bu >> 32;
                dead[2 * ii] = bd & 0xffffffffull;
                dead[2 * ii + 1] = bd >> 32;
                mc[2 * ii] = fmaxf(mc[2 * ii], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm), 31)));
                mc[2 * ii + 1] = fmaxf(mc[2 * ii + 1], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm), 63)));
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int p = 4 * wave + i, j = lane;
                const bool live = j < CH && c0 + j < nend && ms[(p / G) * CH + j] != 0xfc00;
                const float sj = live ? sc[j * PF_P + p] : -INFINITY;
                const float sm = wave_scan_max(sj);
                const float M = fmaxf(mc[i], dpp_ninf<0x138>(sm));   // max over every position before j
                float vs, mv;
                if (!live) { mv = 1.0f; vs = 0.0f; }
                else if (sj > M) { mv = M == -INFINITY ? 0.0f : expf_cr(M - sj); vs = 1.0f; }
                else { mv = 1.0f; vs = expf_cr(sj - M); }
                if (j < CH) {
                    cm[j * PF_P + p] = mv;
                    sc[j * PF_P + p] = vs;
                }
                upd[i] = __ballot(live && sj > M);
                dead[i] = __ballot(!live);
                mc[i] = fmaxf(mc[i], __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sm), 63)));
            }
        }
        asm volatile("" ::: "memory");
        mark(2);
        // ---- phase 3: the f16 recurrence, 2 dims x 4 pairs per lane (V from LDS) ------------
        {
            const int nrun = (int) min((int64_t) CH, nend - c0);
            const uint32_t * vrow = (const uint32_t *) vl[s] + lane;   // dims 2 lane, 2 lane + 1
            const float * scw = sc + 4 * wave;
            const float * cmw = cm + 4 * wave;
            // batch j0's V values and coefficients are read while batch j0 - U computes (a read
            // past the chunk end lands in other LDS data and is never used)
            auto ldb = [&](int j0, uint32_t (&vv)[U], float4 (&vs)[U]) __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    vv[u] = vrow[(j0 + u) * (D / 2)];
                    vs[u] = *(const float4 *) (scw + (j0 + u) * PF_P);
                }
            };
            auto run = [&](int j0, const uint32_t (&vv)[U], const float4 (&vs)[U]) __attribute__((always_inline)) {
                const uint64_t ev = (upd[0] | upd[1] | upd[2] | upd[3] | dead[0] | dead[1] | dead[2] | dead[3]) >> j0;
                if ((ev & ((1ull << U) - 1)) == 0) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const float v4[4] = {vs[u].x, vs[u].y, vs[u].z, vs[u].w};
#pragma unroll
                        for (int i = 0; i < 4; ++i) y[i] = f16x2_mad(vv[u], v4[i], y[i]);
                        S[0] = f32x2_add(S[0], make_float2(vs[u].x, vs[u].y));   // not contracted on the CPU
                        S[1] = f32x2_add(S[1], make_float2(vs[u].z, vs[u].w));
                    }
                } else {
                    // the same steps, except: a masked position keeps the state (-0 must
                    // survive); a running-max update first rescales, y = f16(y*ms), S = S*ms —
                    // the CPU's vec_scale_f16 (ops.cpp:7120-7160).  Branch-free: every live step
                    // rescales by its ms, which is exactly 1 where the max does not move (an f16
                    // value times 1 rounds back to itself, S*1 = S), and a masked step selects
                    // the old state
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int j = j0 + u;
                        const float v4[4] = {vs[u].x, vs[u].y, vs[u].z, vs[u].w};
                        const float4 m4 = *(const float4 *) (cmw + j * PF_P);
                        const float w4[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const uint32_t yn = f16x2_mad(vv[u], v4[i], f16x2_scale(y[i], w4[i], nz));
                            y[i] = (dead[i] >> j) & 1 ? y[i] : yn;
                        }
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const float2 Sn = f32x2_add(f32x2_mul(S[h], make_float2(w4[2 * h], w4[2 * h + 1])),
                                                        make_float2(v4[2 * h], v4[2 * h + 1]));
                            S[h].x = (dead[2 * h] >> j) & 1 ? S[h].x : Sn.x;
                            S[h].y = (dead[2 * h + 1] >> j) & 1 ? S[h].y : Sn.y;
                        }
                    }
                }
            };
            uint32_t va[U], vb[U];
            float4 sa[U], sb[U];
            ldb(0, va, sa);
            for (int j0 = 0; j0 < nrun; j0 += 2 * U) {
                ldb(j0 + U, vb, sb);
                run(j0, va, sa);
                if (j0 + U >= nrun) break;
                ldb(j0 + 2 * U, va, sa);
                run(j0 + U, vb, sb);
            }
        }
        if (more) store_mask(s ^ 1);   // published by the next chunk's barrier
        mark(3);
    }
    if (prof) {
        for (int i = 0; i < 4; ++i) a.prof[i] += pc[i];
        a.prof[4] += (unsigned long long) nchunk;
    }
    // ---- output O = y / S --------------------------------------------------------------------
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int p = 4 * wave + i;
        const int64_t iq = q0 + p / G;
        if (iq >= a.n_q) continue;
        float * drow = (float *) ((char *) a.dst + iq * a.nb1_dst * a.H + head_of(p) * a.nb1_dst + iq3 * a.nb2_dst);
        const float rs = 1.0f / (i & 1 ? S[i >> 1].y : S[i >> 1].x);
        *(float2 *) (drow + 2 * lane) = make_float2(__fmul_rn(h2f((uint16_t) y[i]), rs), __fmul_rn(h2f((uint16_t) (y[i] >> 16)), rs));
    }
    // the output's Q8_K quantization for the next MUL_MAT (qmode 1): the wave's four heads are
    // 512 consecutive values of one token's row = two Q8_K blocks; lane l gathers elements
    // 4l .. 4l + 3 of each block (dims 2 lane, 2 lane + 1 of the lanes 2l, 2l + 1) for q8K_wave
    if (a.qmode == 1) {
        const int64_t iq = q0 + (4 * wave) / G;   // uniform over the wave (G >= 4)
        if (iq < a.n_q) {
            float o[4][2];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float rs = 1.0f / (i & 1 ? S[i >> 1].y : S[i >> 1].x);
                o[i][0] = __fmul_rn(h2f((uint16_t) y[i]), rs);
                o[i][1] = __fmul_rn(h2f((uint16_t) (y[i] >> 16)), rs);
            }
            const int KR = a.H * D;
            const int s0 = (2 * lane) & 63, s1 = (2 * lane + 1) & 63;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                float q[4];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float lo0 = __shfl(o[2 * b][0], c ? s1 : s0, WAVE), hi0 = __shfl(o[2 * b][1], c ? s1 : s0, WAVE);
                    const float lo1 = __shfl(o[2 * b + 1][0], c ? s1 : s0, WAVE), hi1 = __shfl(o[2 * b + 1][1], c ? s1 : s0, WAVE);
                    q[2 * c] = lane < 32 ? lo0 : lo1;
                    q[2 * c + 1] = lane < 32 ? hi0 : hi1;
                }
                const int64_t c0 = iq * KR + (int64_t) head_of(4 * wave + 2 * b) * D;
                q8K_wave(q, lane, a.qs + c0, a.qsum + c0 / 16, a.qd + c0 / 256);
            }
        }
    }
}

// ==== decode, D = 128, f16 cache: two heads per workgroup, scores produced under the recurrence ====
// The same arithmetic as k_fattn_exact (scores in the AVX-512 ggml_vec_dot_f16 order, the
// prefix-max (ms, vs) coefficients, the f16 VKQ recurrence with the CPU's two roundings), laid
// out so the serial part never waits on the rest:
//   * waves 0-3 are the chains: wave w runs the recurrence of head 2j + (w >> 1), dims
//     64 (w & 1) .. + 63, one dim per lane (one chain per SIMD);
//   * waves 4-5 are the producers, one per head: for chunk c + 1 they load the mask, stream V
//     into LDS (LDS-DMA), score the K rows (every K load of the chunk in flight at once), and
//     form the coefficients and the per-batch flags, while the chains run chunk c; one
//     workgroup barrier per chunk hands a double-buffered stage over;
//   * both heads of a Q8_K block (256 = 2 x 128 outputs) finish in this workgroup, so the
//     output quantization for the following projection needs no cross-workgroup hand-off.
// Chunks of DC_CH positions; the running max carries across chunks in the producer, the f16
// state in the chains, both in cache order, so the chunking changes no result.
constexpr int DC_CH = 128, DC_U = 8;

// LDS of k_fattn_dec2, laid out by hand: the small arrays the chains read every batch first,
// the V stages last (reads at high LDS addresses measured ~5 ticks per position slower,
// tools/ubench_dc.hip); with GQA sharing only head 0's stages [0, 64 KiB) above them are used
struct dc_smem {
    float sc[2][2][DC_CH + 2 * DC_U];   // [head][stage] vs (0 where dead); read ahead by one batch
    float cm[2][2][DC_CH + 2 * DC_U];   // ms (1 where dead)
    float mk[2][2][DC_CH + 2 * DC_U];   // mask value (-inf = dead)
    uint32_t bfl[2][2][2];              // [head][stage][half]: batches taking the general step
    int nrs[2];                         // positions to run, per stage
    float mpub[2];                      // [head]: running max through the first half of the chunk
    int mseq[2];                        // [head]: chunk number + 1 that mpub belongs to
    int qseq[2][2];                     // [head][half]: chunk number + 1 whose odd-quarter scores are in
    float mcar[2];                      // [head]: running max through the whole chunk
    uint64_t etab[8][32];               // expf's table (lx_exp2f_tab), a copy per producer wave
    float ol[2 * 128];
    uint16_t vl[2][2][DC_CH * 128];     // [head][stage][position][dim]
};

// NQ producer waves per head: 4 (768 threads) for long caches, 2 (512) where one or two chunks
// leave the producers little to overlap (four cost ~0.6 us per layer more at 136 positions and
// save ~9 us at 4096)
template <int NQ>
__global__ __launch_bounds__(64 * (4 + 2 * NQ), 1) void k_fattn_dec2(const fa_args a) {
    constexpr int D = 128, NM = D / 16, CH = DC_CH, U = DC_U;
    constexpr int PQ = CH / NQ, NPQ = PQ / 16;   // positions per producer wave, score passes over them
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    kt_enter(a.kt, 1 + 4 + 2 * NQ);
    const int64_t hp = blockIdx.x;          // head pair: heads 2 hp, 2 hp + 1
    const int64_t iq3 = blockIdx.y;
    const int64_t G = a.H / a.Hkv;
    const bool vsh = (2 * hp) / G == (2 * hp + 1) / G;   // both heads read one KV head: one V stage
    __shared__ __attribute__((aligned(16))) dc_smem sm;
    const int64_t nchunk = (a.n_kv + CH - 1) / CH;
    const char * mrow = a.mask ? a.mask + (0 % a.mask_ne1) * a.nbm1 : nullptr;
    if (tid < 2) { sm.mseq[tid] = 0; sm.mcar[tid] = -INFINITY; }
    if (tid < 4) sm.qseq[tid >> 1][tid & 1] = 0;
    __syncthreads();

    if (wave >= 4) {
        // ===== producers: head ph, quarter qt (positions 32 qt .. 32 qt + 31) of each chunk; the
        // even quarters also form the prefix max and coefficients of their half (64 hf .. +63) =====
        const int pw = wave - 4, ph = pw / NQ, qt = pw % NQ, hf = qt / (NQ / 2);
        const bool cw = NQ == 2 || (qt & 1) == 0;   // the coefficient wave of half hf
        // expf's table: this wave's own copy, its load issued before the mask / K / q loads and
        // stored once they are all out (one wave filling a shared copy before the launch's first
        // barrier held every wave behind a memory round trip)
        const uint64_t etv = lx_exp2f_tab[lane & 31];
        const uint64_t * etab = sm.etab[pw];
        const int64_t h = 2 * hp + ph, hk = h / G;
        const int qd = lane & 3;
        const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
        const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;
        auto mask_at = [&](int64_t j) -> uint16_t {   // f16 bits; 0xfc00 (-inf) past the cache
            if (j >= a.n_kv) return 0xfc00;
            return mrow ? *(const uint16_t *) (mrow + 2 * j) : (uint16_t) 0;
        };
        auto load_k = [&](int64_t c0, int jmax, uint2 (&kh)[NPQ][NM]) {   // this quarter's K rows (<= jmax)
#pragma unroll
            for (int p = 0; p < NPQ; ++p) {
                const int j = min(PQ * qt + 16 * p + (lane >> 2), jmax);
                const char * krow = kbase + (c0 + j) * a.nbk1 + 8 * qd;
#pragma unroll
                for (int m = 0; m < NM; ++m) kh[p][m] = ld8(krow + 32 * m);
            }
        };
        auto nrun_of = [](uint16_t m0b, uint16_t m1b) {   // positions up to the last live one
            const unsigned long long b0 = __ballot(m0b != 0xfc00), b1 = __ballot(m1b != 0xfc00);
            return b1 ? 128 - __clzll(b1) : (b0 ? 64 - __clzll(b0) : 0);
        };
        // chunk 0's K rows go out with q and the mask (bounded by the cache, not yet by the mask);
        // later chunks' go out right after the previous chunk's scores
        uint2 kh[NPQ][NM];
        if (nchunk > 0) load_k(0, (int) min<int64_t>(CH, a.n_kv) - 1, kh);
        uint16_t mc0 = mask_at(lane), mc1 = mask_at(64 + lane);
        float qf[NM][4];
        {
            const float * qrow = (const float *) (a.q + h * a.nbq2 + iq3 * a.nbq3);
            float4 q4[NM];
#pragma unroll
            for (int m = 0; m < NM; ++m) q4[m] = *(const float4 *) (qrow + 16 * m + 4 * qd);
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                qf[m][0] = f16r(q4[m].x); qf[m][1] = f16r(q4[m].y); qf[m][2] = f16r(q4[m].z); qf[m][3] = f16r(q4[m].w);
            }
        }
        if (lane < 32) sm.etab[pw][lane] = etv;   // read back only by this wave (in order)
        float nz = -0.0f;
        asm volatile("" : "+v"(nz));
        const float slope = a.max_bias > 0.0f
            ? (float) ((uint32_t) h < a.n_head_log2 ? pow((double) a.m0, (double) (h + 1))
                                                   : pow((double) a.m1, (double) (2 * ((uint32_t) h - a.n_head_log2) + 1)))
            : 1.0f;
        const bool prof = a.prof && blockIdx.x == 0 && blockIdx.y == 0 && pw == 0 && lane == 0;
        unsigned long long tp = prof ? __builtin_amdgcn_s_memtime() : 0, pc[6] = {0, 0, 0, 0, 0, 0};
        auto mark = [&](int i) {
            if (prof) { const unsigned long long t = __builtin_amdgcn_s_memtime(); pc[i] += t - tp; tp = t; }
        };
        for (int64_t c = 0; c <= nchunk; ++c) {
            if (c < nchunk) {
                const int st = (int) (c & 1);
                const int64_t c0 = c * CH;
                const uint16_t m0b = mc0, m1b = mc1;
                bool kout = false;   // the next chunk's K loads were issued
                const int nrun = nrun_of(m0b, m1b);
                // the next chunk's mask, in flight under this one
                mc0 = mask_at(c0 + CH + lane);
                mc1 = mask_at(c0 + CH + 64 + lane);
                const float mv = h2f(hf ? m1b : m0b);   // lane's position 64 hf + lane (the coefficient wave's)
                const int jl = 64 * hf + lane;
                float * mkp = sm.mk[ph][st];
                float * scp = sm.sc[ph][st];
                float * cmp = sm.cm[ph][st];
                // this quarter's mask values: position 32 qt + i is lane (32 (qt & 1) + i)'s value of half hf
                if (NQ == 2 || (lane >> 5) == (qt & 1)) mkp[jl] = mv;
                if (qt == NQ - 1 && lane < 2 * U) { mkp[CH + lane] = -INFINITY; cmp[CH + lane] = 1.0f; scp[CH + lane] = 0.0f; }
                const float mcarry = sm.mcar[ph];   // through the previous chunk (published before the last barrier)
                float tot = mcarry;
                if (nrun > 0) {
                    const int lo = PQ * qt;   // this wave's rows to score: [lo, min(nrun, lo + PQ))
                    mark(0);
                    // V rows this wave stages: with one KV head for both heads 16 rows per producer
                    // wave, else its quarter of its head's stage (LDS-DMA issue runs at ~25 GB/s per wave)
                    const int vlo = vsh ? (PQ / 2) * pw : lo, vhi = min(nrun, vsh ? vlo + PQ / 2 : lo + PQ);
                    if (vhi > vlo) {
                        // 4 rows per instruction; the row address advances by addition (a 64-bit
                        // multiply per instruction made the issue loop ~100 cycles per KiB)
                        const int r_in = lane >> 4, col = lane & 15;
                        const int64_t step = 4 * a.nbv1;
                        const char * vp = vbase + (c0 + vlo + r_in) * a.nbv1 + 16 * col;
                        const char * vlast = vbase + (c0 + vhi - 1) * a.nbv1 + 16 * col;
                        uint16_t * dst = sm.vl[vsh ? 0 : ph][st] + 512 * (vlo / 4);
                        const int np = (vhi - vlo + 3) / 4;
                        for (int p = 0; p < np; ++p) {
                            const char * src = (4 * p + r_in < vhi - vlo) ? vp : vlast;
                            lds_dma16(src, dst);
                            vp += step;
                            dst += 512;
                        }
                    }
                    dc_wave_lds_order();                        // mask values, read back by other lanes
                    mark(1);
                    float mj[NPQ];
#pragma unroll
                    for (int p = 0; p < NPQ; ++p) mj[p] = mkp[lo + 16 * p + (lane >> 2)];
#pragma unroll
                    for (int p = 0; p < NPQ; ++p) {
                        if (lo + 16 * p >= nrun) break;
                        const int j = lo + 16 * p + (lane >> 2);
                        const float w = dot_f16_mix_d128(kh[p], qf, nz);
                        if (qd == 0 && j < nrun) {
                            float sv = __fmul_rn(w, a.scale);
                            if (a.softcap != 0.0f) sv = __fmul_rn(a.softcap, tanhf(sv));
                            scp[j] = __fadd_rn(sv, __fmul_rn(slope, mj[p]));
                        }
                    }
                    // the next chunk's K rows, in flight under the coefficients and the chains'
                    // recurrence (bounded by the cache only: waiting for the next chunk's mask here
                    // would also wait for this chunk's V DMA, issued after it)
                    if (c + 1 < nchunk) {
                        load_k(c0 + CH, (int) min<int64_t>(CH, a.n_kv - c0 - CH) - 1, kh);
                        kout = true;
                    }
                    dc_wave_lds_order();
                    if (NQ == 4 && !cw) {
                        // the odd quarter hands its scores and mask values to its half's coefficient wave
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        if (lane == 0) lds_st(&sm.qseq[ph][hf], (int) c + 1);
                    }
                    mark(2);
                    if (cw) {
                        int qguard = 0;
                        if (NQ == 4) {
                            // bounded: a hand-off that never completes traps rather than reading stale scores
                            while (lds_ld(&sm.qseq[ph][hf]) != (int) c + 1) {
                                __builtin_amdgcn_s_sleep(1);
                                if (++qguard > (1 << 24)) __builtin_trap();
                            }
                            asm volatile("" ::: "memory");   // the score reads stay after the wait
                        }
                        // prefix max over the chunk: this half's scan, the first half's total from LDS
                        const bool live = mv != -INFINITY && jl < nrun;
                        const float sj = live ? scp[jl] : -INFINITY;
                        const float smx = wave_scan_max(sj);
                        const float th = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(smx), 63));
                        float base = mcarry;   // running max before this half
                        if (hf == 0) {
                            if (lane == 0) {
                                // LDS only, in order: the value, its write done, then the sequence word
                                // (a workgroup-scope fence would also wait for this wave's V DMA and K loads)
                                lds_st(&sm.mpub[ph], fmaxf(mcarry, th));
                                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                                lds_st(&sm.mseq[ph], (int) c + 1);
                            }
                        } else {
                            // the first half of the same head publishes its max within its own chunk work
                            int guard = 0;
                            while (lds_ld(&sm.mseq[ph]) != (int) c + 1) {
                                __builtin_amdgcn_s_sleep(1);
                                if (++guard > (1 << 24)) __builtin_trap();
                            }
                            asm volatile("" ::: "memory");
                            base = lds_ld(&sm.mpub[ph]);
                        }
                        const float M = fmaxf(base, dpp_ninf<0x138>(smx));   // max over every position before jl
                        float msv, vsv;
                        if (!live) { msv = 1.0f; vsv = 0.0f; }
                        else if (sj > M) { msv = M == -INFINITY ? 0.0f : lx_expf_t(M - sj, etab); vsv = 1.0f; }
                        else { msv = 1.0f; vsv = lx_expf_t(sj - M, etab); }
                        cmp[jl] = msv;
                        scp[jl] = vsv;
                        // batch flags: a dead position, a max update or padding past nrun
                        const bool gen = jl < nrun ? (!live || sj > M) : (jl < nrun + U);
                        const unsigned long long wb = __ballot(gen);
                        uint32_t f = 0;
    #pragma unroll
                        for (int bb = 0; bb < 64 / U; ++bb) f |= ((wb >> (U * bb)) & ((1ull << U) - 1)) ? 1u << bb : 0u;
                        if (lane == 0) sm.bfl[ph][st][hf] = f;
                        tot = fmaxf(base, th);
                    }
                    mark(3);
                } else {
                    if (cw && hf == 0 && lane == 0) lds_st(&sm.mseq[ph], (int) c + 1);
                    if (c + 1 < nchunk) {
                        load_k(c0 + CH, (int) min<int64_t>(CH, a.n_kv - c0 - CH) - 1, kh);
                        kout = true;
                    }
                }
                if (cw && hf == 1 && lane == 0) sm.mcar[ph] = nrun > 0 ? tot : mcarry;   // read after the barrier
                if (pw == 0 && lane == 0) sm.nrs[st] = nrun;
                // this wave's V rows are in LDS: everything but the next chunk's K loads (the
                // NPQ x NM loads of load_k, the only vector-memory instructions after the V DMA)
                if (kout) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPQ * NM) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                mark(4);
            }
            __syncthreads();
            mark(5);
        }
        if (prof) for (int i = 0; i < 6; ++i) a.prof[i] += pc[i];
    } else {
        // ===== chains: head 2 hp + (wave >> 1), dim d =====
        const int ch = wave >> 1;
        const int d = (wave & 1) * 64 + lane;
        uint32_t yb = 0;
        float S = 0.0f;
        const bool prof = a.prof && blockIdx.x == 0 && blockIdx.y == 0 && wave == 0 && lane == 0;
        unsigned long long tp = prof ? __builtin_amdgcn_s_memtime() : 0, cbusy = 0, cwait = 0;
        for (int64_t c = 0; c <= nchunk; ++c) {
            if (c >= 1) {
                const int st = (int) ((c - 1) & 1);
                const int nrun = __builtin_amdgcn_readfirstlane(sm.nrs[st]);
                const uint32_t flags = __builtin_amdgcn_readfirstlane(sm.bfl[ch][st][0] | (sm.bfl[ch][st][1] << 8));
                const uint16_t * vrow = sm.vl[vsh ? 0 : ch][st] + d;
                const float * scp = sm.sc[ch][st];
                const float * cmp = sm.cm[ch][st];
                const float * mkp = sm.mk[ch][st];
                auto ld4 = [&](const float * p, float (&o)[U]) {
#pragma unroll
                    for (int u = 0; u < U; u += 4) {
                        const float4 t = *(const float4 *) (p + u);
                        o[u] = t.x; o[u + 1] = t.y; o[u + 2] = t.z; o[u + 3] = t.w;
                    }
                };
                auto ldb = [&](int j, uint32_t (&vv)[U], float (&vs)[U]) {
#pragma unroll
                    for (int u = 0; u < U; ++u) vv[u] = vrow[(j + u) * D];
                    ld4(scp + j, vs);
                };
                auto run = [&](const uint32_t (&vv)[U], const float (&vs)[U]) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        yb = f16_mad(vv[u], vs[u], yb);
                        S = __fadd_rn(S, vs[u]);   // not contracted on the CPU
                    }
                };
                // nf consecutive batches without a dead position or a max update, from position
                // j0: a loop with nothing else in it (a flag test and the general step inside the
                // loop cost ~15 ticks per position, tools/ubench_dc.hip)
                auto fast_run = [&](int j0, int nf) {
                    uint32_t va[U], vb[U];
                    float sa[U], sb[U];
                    ldb(j0, va, sa);
                    for (int k = 0; k < nf; k += 2) {
                        ldb(j0 + (k + 1) * U, vb, sb);
                        run(va, sa);
                        if (k + 1 >= nf) break;
                        ldb(j0 + (k + 2) * U, va, sa);
                        run(vb, sb);
                    }
                };
                // a batch with a dead position or a running-max update: a dead position keeps the
                // state (-0 must survive); an update (ms != 1) first rescales, y = f16(y*ms),
                // S = S*ms (ops.cpp:7171-7190)
                auto general = [&](int j) {
                    uint32_t vv[U];
                    float vs[U], ms[U], mv[U];
                    ldb(j, vv, vs);
                    ld4(cmp + j, ms);
                    ld4(mkp + j, mv);
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const bool live = __float_as_uint(mv[u]) != 0xff800000u;
                        const bool upd = __float_as_uint(ms[u]) != 0x3f800000u;
                        float t = __fmul_rn(h2f((uint16_t) yb), ms[u]);
                        asm("" : "+v"(t));   // two roundings, as f16r
                        const uint32_t ys = upd ? (uint32_t) f2h(t) : yb;
                        const float Ss = upd ? __fmul_rn(S, ms[u]) : S;
                        const uint32_t yn = f16_mad(vv[u], vs[u], ys);
                        const float Sn = __fadd_rn(Ss, vs[u]);
                        yb = live ? yn : yb;
                        S = live ? Sn : S;
                    }
                };
                const int nb = (nrun + U - 1) / U;
                int b = 0;
                while (b < nb) {
                    const uint32_t rest = flags >> b;
                    const int nf = min(rest ? __builtin_ctz(rest) : 32, nb - b);   // fast batches before the next general one
                    if (nf > 0) {
                        fast_run(b * U, nf);
                        b += nf;
                    }
                    if (b < nb) {
                        general(b * U);
                        ++b;
                    }
                }
            }
            if (prof) { const unsigned long long t = __builtin_amdgcn_s_memtime(); cbusy += t - tp; tp = t; }
            __syncthreads();
            if (prof) { const unsigned long long t = __builtin_amdgcn_s_memtime(); cwait += t - tp; tp = t; }
        }
        if (prof) { a.prof[6] += cbusy; a.prof[7] += cwait; }
        const int64_t h = 2 * hp + ch;
        const float o = __fmul_rn(h2f((uint16_t) yb), 1.0f / S);
        float * drow = (float *) ((char *) a.dst + h * a.nb1_dst + iq3 * a.nb2_dst);
        drow[d] = o;
        sm.ol[ch * D + d] = o;
    }
    // ---- the two heads' 256 outputs: quantized here for the following projection ----
    if (a.qmode) {
        __syncthreads();
        if (wave == 0) {
            float q[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = sm.ol[4 * lane + k];
            const int64_t c0 = 256 * hp;
            if (a.qmode == 1) q8K_wave(q, lane, a.qs + c0, a.qsum + c0 / 16, a.qd + c0 / 256);
            else q8_0_wave(q, lane, true, a.qs + c0, a.qd + c0 / 32, a.qsum + c0 / 32);
        }
    }
    kt_exit(a.kt, 1 + 4 + 2 * NQ);
}

bool fattn_dec2_ok(const fa_args & a, int64_t nq3) {
    static const bool on = !getenv("GGML_MI355X_FA_DEC2") || atoi(getenv("GGML_MI355X_FA_DEC2")) != 0;
    return on && a.n_q == 1 && a.D == 128 && a.k_type == GGML_TYPE_F16 && a.v_type == GGML_TYPE_F16 && a.H % 2 == 0 &&
           (a.qmode == 0 || nq3 == 1);
}

int fattn_dec2_threads(const fa_args & a) { return a.n_kv > FA_DEC2_NQ4_MIN ? 64 * (4 + 2 * 4) : 64 * (4 + 2 * 2); }

void launch_fattn_dec2(hipStream_t st, const fa_args & a, int64_t nq3) {
    const dim3 grid((unsigned) (a.H / 2), (unsigned) nq3);
    if (a.n_kv > FA_DEC2_NQ4_MIN) hipLaunchKernelGGL(k_fattn_dec2<4>, grid, dim3(64 * (4 + 2 * 4)), 0, st, a);
    else hipLaunchKernelGGL(k_fattn_dec2<2>, grid, dim3(64 * (4 + 2 * 2)), 0, st, a);
}

// ==== decode, D = 128, f16 cache, at most DS_MAXKV cached positions (tg128's depths) ====
// The arithmetic of k_fattn_dec2 (the AVX-512 ggml_vec_dot_f16 scores, the prefix-max (ms, vs)
// coefficients, the f16 VKQ recurrence with the CPU's two roundings; ops.cpp:7015-7232), pipelined
// in 16-position blocks so the serial recurrence starts after the first block's coefficients
// instead of after every score of the cache (dec2 hands over 128-position chunks; at tg128's
// depths that is one chunk, and its chains waited for all of it):
//   * waves 0-3 are the chains: wave c runs the recurrence of head c / 2, dims 64 (c % 2) + lane.
//     Each stages the V bytes it reads itself (its half of every row, LDS-DMA, its own copy), so
//     its own vmcnt says which rows are in and no other wave waits on V;
//   * waves 4-7 are producers: producer p owns blocks p, p + 4, p + 8, p + 12.  It loads the whole
//     mask (the last live position bounds every later load), its first block's K rows and both
//     heads' q at once, then the K of its later blocks; per block it forms both heads' scores
//     from one K load, their running max (a 16-lane DPP scan inside the block; the maximum before
//     the block handed over by the previous block's producer through LDS), the (ms, vs)
//     coefficients with libm expf and a "general" flag per 8-position batch, and marks the block
//     ready;
//   * the two heads' 256 outputs (one Q8_K block) are quantized here for the following projection.
// Both heads of a workgroup read one KV head (GQA group even), so K is fetched once.  The mask and V
// loads are inline asm with explicit waits (the compiler puts no vmcnt wait of its own behind them).
constexpr int DS_MAXKV = 256, DS_U = 8, DS_B = 16, DS_NB = DS_MAXKV / DS_B, DS_PAD = 2 * DS_U;
constexpr int DS_NP = 4, DS_OWN = DS_NB / DS_NP;   // producers, blocks per producer
constexpr int DS_VROWS = DS_MAXKV + DS_U;          // V rows staged (the chain reads one batch ahead)

struct ds_smem {
    float sc[2][DS_MAXKV + DS_PAD];        // [head] vs (0 where dead)
    float cm[2][DS_MAXKV + DS_PAD];        // ms (1 where dead)
    float mk[2][DS_MAXKV + DS_PAD];        // 0 live, -inf dead
    float sr[DS_NP][DS_OWN][2][DS_B];      // [producer][its block][head] raw scores (-inf dead)
    float carry[2][DS_NB];                 // [head] running max through block b
    int cflag[DS_NB];                      // block b's carry is in
    int ready[DS_NB];                      // block b's coefficients and flags are in
    uint8_t bfl[2][2 * DS_NB + 8];         // [head][batch] general step
    uint64_t etab[DS_NP][32];              // expf's table (lx_exp2f_tab), a copy per producer
    float ol[2 * 128];
    uint16_t vc[4][DS_VROWS * 64];         // [chain wave][position][its 64 dims]
};

__global__ __launch_bounds__(512, 1) void k_fattn_dsh(const fa_args a) {
    constexpr int D = 128, NM = D / 16, U = DS_U, B = DS_B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    kt_enter(a.kt, 9);
    // mi355x_bench_op's phase split (workgroup (0, 0), waves 0 and 4): cycles from the start to
    // each mark, kept in registers and added to a.prof at the end
    const bool prof = a.prof && blockIdx.x == 0 && blockIdx.y == 0 && lane == 0 && (wave == 0 || wave == 4);
    const unsigned long long t0 = prof ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto mark = [&](int i) { if (prof) pt[i] = __builtin_amdgcn_s_memtime() - t0; };
    const int64_t hp = blockIdx.x;          // head pair: heads 2 hp, 2 hp + 1 (one KV head)
    const int64_t iq3 = blockIdx.y;
    const int64_t hk = (2 * hp) / (a.H / a.Hkv);
    const int n_kv = (int) a.n_kv;
    __shared__ __attribute__((aligned(16))) ds_smem sm;
    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;
    // every wave reads the whole mask (4 positions a lane): nrun = the last live position + 1
    uint32_t mk4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) mk4[k] = ds_mask_ld(a.mask, 64 * k + lane, n_kv);
    if (tid < DS_NB) { sm.cflag[tid] = 0; sm.ready[tid] = 0; }
    auto nrun_of = [&]() {
        int last = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned long long bl = __ballot((mk4[k] & 0xffff) != 0xfc00);
            if (bl) last = 64 * k + 63 - __clzll(bl);
        }
        return last + 1;
    };

    if (wave >= 4) {
        // ================= producers =================
        const int pw = wave - 4, qd = lane & 3;
        const uint64_t etv = lx_exp2f_tab[lane & 31];
        uint2 kh[DS_OWN][NM];
        auto load_k = [&](int i) {   // block pw + DS_NP i: its K rows, 4 lanes a position
            const int j = min(B * (pw + DS_NP * i) + (lane >> 2), n_kv - 1);
            const char * krow = kbase + (int64_t) j * a.nbk1 + 8 * qd;
#pragma unroll
            for (int m = 0; m < NM; ++m) kh[i][m] = ld8(krow + 32 * m);
        };
        // the mask value of each owned block's position B b + lane / 4
        uint32_t mkb[DS_OWN];
#pragma unroll
        for (int i = 0; i < DS_OWN; ++i) mkb[i] = ds_mask_ld(a.mask, B * (pw + DS_NP * i) + (lane >> 2), n_kv);
        if (B * pw < n_kv) load_k(0);
        float4 q4[2][NM];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float * qrow = (const float *) (a.q + (2 * hp + h) * a.nbq2 + iq3 * a.nbq3);
#pragma unroll
            for (int m = 0; m < NM; ++m) q4[h][m] = *(const float4 *) (qrow + 16 * m + 4 * qd);
        }
        __syncthreads();   // the flags' zeros (all waves), while the loads are in flight
        // (the builtin, not asm: the compiler then knows these loads are in and puts no wait for
        // them after the later blocks' loads below; the asm mask loads are older, so in too)
        __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
        asm volatile("" : "+v"(mk4[0]), "+v"(mk4[1]), "+v"(mk4[2]), "+v"(mk4[3]), "+v"(mkb[0]), "+v"(mkb[1]), "+v"(mkb[2]),
                     "+v"(mkb[3]));
        mark(0);
        if (lane < 32) sm.etab[pw][lane] = etv;
        const int nrun = nrun_of(), nblk = (nrun + B - 1) / B;
        const int nown = nblk > pw ? (nblk - pw + DS_NP - 1) / DS_NP : 0;
#pragma unroll
        for (int i = 1; i < DS_OWN; ++i)
            if (i < nown) load_k(i);
        float qf[2][NM][4];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                qf[h][m][0] = f16r(q4[h][m].x); qf[h][m][1] = f16r(q4[h][m].y);
                qf[h][m][2] = f16r(q4[h][m].z); qf[h][m][3] = f16r(q4[h][m].w);
            }
        float nz = -0.0f;
        asm volatile("" : "+v"(nz));
        float slope[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t hh = 2 * hp + h;
            slope[h] = a.max_bias > 0.0f
                ? (float) ((uint32_t) hh < a.n_head_log2 ? pow((double) a.m0, (double) (hh + 1))
                                                        : pow((double) a.m1, (double) (2 * ((uint32_t) hh - a.n_head_log2) + 1)))
                : 1.0f;
        }
        mark(1);
        const uint64_t * etab = sm.etab[pw];
        // the scores of block i into sr (quad lane 0 of each position)
        auto scores = [&](int i) {
            const int b = pw + DS_NP * i;
            const int j = B * b + (lane >> 2);
            const float mv = h2f((uint16_t) mkb[i]);
            const bool live = mv != -INFINITY && j < nrun;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float w = dot_f16_mix_d128(kh[i], qf[h], nz);
                if (qd == 0) {
                    float sv = __fmul_rn(w, a.scale);
                    if (a.softcap != 0.0f) sv = __fmul_rn(a.softcap, tanhf(sv));
                    sm.sr[pw][i][h][lane >> 2] = live ? __fadd_rn(sv, __fmul_rn(slope[h], mv)) : -INFINITY;
                }
            }
        };
        // block i's coefficients from its scores and the running max before it
        auto coef = [&](int i) {
            const int b = pw + DS_NP * i;
            dc_wave_lds_order();
            // lanes 0-31: head lane / 16, position B b + lane % 16
            const int hc = (lane >> 4) & 1, pj = B * b + (lane & 15);
            const float sj = sm.sr[pw][i][hc][lane & 15];
            const bool lj = sj != -INFINITY;
            const float inc = fmaxf(sj, dpp_ninf<0x111>(sj));
            const float inc2 = fmaxf(inc, dpp_ninf<0x112>(inc));
            const float inc3 = fmaxf(inc2, dpp_ninf<0x114>(inc2));
            const float incl = fmaxf(inc3, dpp_ninf<0x118>(inc3));   // max over the row's lanes <= this one
            const float excl = dpp_ninf<0x111>(incl);                 // ... < this one
            const float bmax0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 15));
            const float bmax1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(incl), 31));
            float cin0 = -INFINITY, cin1 = -INFINITY;
            if (b > 0) {
                ds_wait_flag(&sm.cflag[b - 1]);
                cin0 = sm.carry[0][b - 1];
                cin1 = sm.carry[1][b - 1];
            }
            if (lane == 0) {
                sm.carry[0][b] = fmaxf(cin0, bmax0);
                sm.carry[1][b] = fmaxf(cin1, bmax1);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                lds_st(&sm.cflag[b], 1);
            }
            const float M = fmaxf(hc ? cin1 : cin0, excl);   // max over every live position before pj
            float msv, vsv;
            if (!lj) { msv = 1.0f; vsv = 0.0f; }
            else if (sj > M) { msv = M == -INFINITY ? 0.0f : lx_expf_t(M - sj, etab); vsv = 1.0f; }
            else { msv = 1.0f; vsv = lx_expf_t(sj - M, etab); }
            const bool gen = pj < nrun ? (!lj || sj > M) : true;
            const unsigned long long gb = __ballot(gen && lane < 32);
            if (lane < 32) {
                sm.sc[hc][pj] = vsv;
                sm.cm[hc][pj] = msv;
                sm.mk[hc][pj] = lj ? 0.0f : -INFINITY;
            }
            if (lane < 4) sm.bfl[lane >> 1][2 * b + (lane & 1)] = ((gb >> (8 * lane)) & 0xff) ? 1 : 0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (lane == 0) lds_st(&sm.ready[b], 1);
        };
        if (nown > 0) {
            scores(0);
            coef(0);
            mark(2);
#pragma unroll
            for (int i = 1; i < DS_OWN; ++i)
                if (i < nown) scores(i);
#pragma unroll
            for (int i = 1; i < DS_OWN; ++i)
                if (i < nown) coef(i);
        }
        mark(3);
    } else {
        // ================= chains: head ch, dim d =================
        const int ch = wave >> 1, half = wave & 1;
        uint16_t * vme = sm.vc[wave];
        // this wave's half of V rows [8 i, 8 i + 8): one 1-KiB LDS-DMA instruction
        auto stage_v = [&](int i) {
            const int jv = min(8 * i + (lane >> 3), n_kv - 1);
            lds_dma16(vbase + (int64_t) jv * a.nbv1 + 128 * half + 16 * (lane & 7), vme + 512 * i);
        };
        // rows [0, 64) go out with the mask, the rest once the mask bounds them
        const int n0 = min(8, (n_kv + 7) / 8);
        for (int i = 0; i < n0; ++i) stage_v(i);
        __syncthreads();   // the flags' zeros
        eng_vm_wait_fa(n0);   // the mask (issued first)
        asm volatile("" : "+v"(mk4[0]), "+v"(mk4[1]), "+v"(mk4[2]), "+v"(mk4[3]));
        const int nrun = nrun_of(), nb = (nrun + U - 1) / U;
        const int nvi = max(n0, min((nrun + U + 7) / 8, (DS_VROWS + 7) / 8));   // rows through the last batch read
        for (int i = n0; i < nvi; ++i) stage_v(i);
        mark(4);
        const int d = half * 64 + lane;
        uint32_t yb = 0;
        float S = 0.0f;
        const uint16_t * vrow = vme + lane;
        const float * scp = sm.sc[ch];
        const float * cmp = sm.cm[ch];
        const float * mkp = sm.mk[ch];
        auto ld4 = [&](const float * p, float (&o)[U]) {
#pragma unroll
            for (int u = 0; u < U; u += 4) {
                const float4 t = *(const float4 *) (p + u);
                o[u] = t.x; o[u + 1] = t.y; o[u + 2] = t.z; o[u + 3] = t.w;
            }
        };
        auto ldb = [&](int j, uint32_t (&vv)[U], float (&vs)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) vv[u] = vrow[(j + u) * 64];
            ld4(scp + j, vs);
        };
        auto run = [&](const uint32_t (&vv)[U], const float (&vs)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                yb = f16_mad(vv[u], vs[u], yb);
                S = __fadd_rn(S, vs[u]);   // not contracted on the CPU
            }
        };
        // a dead position keeps the state (-0 must survive); an update (ms != 1) first rescales,
        // y = f16(y*ms), S = S*ms (ops.cpp:7171-7190)
        auto general = [&](int j) {
            uint32_t vv[U];
            float vs[U], ms[U], mv[U];
            ldb(j, vv, vs);
            ld4(cmp + j, ms);
            ld4(mkp + j, mv);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool live = __float_as_uint(mv[u]) != 0xff800000u;
                const bool upd = __float_as_uint(ms[u]) != 0x3f800000u;
                float t = __fmul_rn(h2f((uint16_t) yb), ms[u]);
                asm("" : "+v"(t));   // two roundings, as f16r
                const uint32_t ys = upd ? (uint32_t) f2h(t) : yb;
                const float Ss = upd ? __fmul_rn(S, ms[u]) : S;
                const uint32_t yn = f16_mad(vv[u], vs[u], ys);
                const float Sn = __fadd_rn(Ss, vs[u]);
                yb = live ? yn : yb;
                S = live ? Sn : S;
            }
        };
        // V: rows [0, 64) before the first block, the rest (issued once the mask bounded them)
        // before block 4; a block's ready flag and batch flags are read one block ahead, so their
        // LDS latency hides under the previous block's steps
        int rdy = 0, f0 = 0, f1 = 0;
        if (nb > 0) {
            eng_vm_wait_fa(nvi - n0);
            ds_wait_flag(&sm.ready[0]);
            mark(5);
            f0 = sm.bfl[ch][0];
            f1 = sm.bfl[ch][1];
        }
        for (int b = 0; 2 * b < nb; ++b) {
            if (b == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int g0 = f0, g1 = f1;
            const bool two = 2 * b + 1 < nb, more = 2 * b + 2 < nb;
            if (more) {
                rdy = lds_ld(&sm.ready[b + 1]);
                asm volatile("" ::: "memory");
                f0 = sm.bfl[ch][2 * b + 2];
                f1 = sm.bfl[ch][2 * b + 3];
            }
            if (!g0 && !(two && g1)) {   // both batches fast (or one fast batch)
                uint32_t va[U], vb[U];
                float sa[U], sb[U];
                ldb(B * b, va, sa);
                if (two) ldb(B * b + U, vb, sb);
                run(va, sa);
                if (two) run(vb, sb);
            } else {
                if (g0) general(B * b);
                else { uint32_t va[U]; float sa[U]; ldb(B * b, va, sa); run(va, sa); }
                if (two) {
                    if (g1) general(B * b + U);
                    else { uint32_t vb[U]; float sb[U]; ldb(B * b + U, vb, sb); run(vb, sb); }
                }
            }
            if (more && !rdy) {   // the producer was behind: wait, then re-read its flags
                ds_wait_flag(&sm.ready[b + 1]);
                f0 = sm.bfl[ch][2 * b + 2];
                f1 = sm.bfl[ch][2 * b + 3];
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA of this wave outlives it
        mark(6);
        const int64_t h = 2 * hp + ch;
        const float o = __fmul_rn(h2f((uint16_t) yb), 1.0f / S);
        float * drow = (float *) ((char *) a.dst + h * a.nb1_dst + iq3 * a.nb2_dst);
        drow[d] = o;
        sm.ol[ch * D + d] = o;
    }
    // ---- the two heads' 256 outputs: quantized here for the following projection ----
    if (a.qmode) {
        __syncthreads();
        if (wave == 0) {
            float q[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = sm.ol[4 * lane + k];
            const int64_t c0 = 256 * hp;
            if (a.qmode == 1) q8K_wave(q, lane, a.qs + c0, a.qsum + c0 / 16, a.qd + c0 / 256);
            else q8_0_wave(q, lane, true, a.qs + c0, a.qd + c0 / 32, a.qsum + c0 / 32);
            mark(7);
        }
    }
    if (prof) {
        for (int i = 0; i < 8; ++i) if (pt[i]) a.prof[i] += pt[i];
    }
    kt_exit(a.kt, 9);
}

// the short-context kernel applies: one query row, D = 128, f16 K and V, at most DS_MAXKV
// positions, an even GQA group (both heads of a workgroup read one KV head), 16-B aligned V rows
bool fattn_dsh_ok(const fa_args & a, int64_t nq3) {
    static const bool on = !getenv("GGML_MI355X_FA_DSH") || atoi(getenv("GGML_MI355X_FA_DSH")) != 0;
    const int64_t G = a.Hkv > 0 ? a.H / a.Hkv : 0;
    return on && a.n_q == 1 && a.D == 128 && a.k_type == GGML_TYPE_F16 && a.v_type == GGML_TYPE_F16 && a.H % 2 == 0 &&
           a.H % a.Hkv == 0 && G % 2 == 0 && a.n_kv >= 1 && a.n_kv <= DS_MAXKV && (a.qmode == 0 || nq3 == 1) &&
           ((uintptr_t) a.v % 16) == 0 && a.nbv1 % 16 == 0 && a.nbv2 % 16 == 0 && a.nbv3 % 16 == 0 && a.nbk1 % 8 == 0 &&
           ((uintptr_t) a.k % 8) == 0 && ((uintptr_t) a.q % 16) == 0 && a.nbq2 % 16 == 0 && a.nbq3 % 16 == 0;
}

void launch_fattn_dsh(hipStream_t st, const fa_args & a, int64_t nq3) {
    hipLaunchKernelGGL(k_fattn_dsh, dim3((unsigned) (a.H / 2), (unsigned) nq3), dim3(512), 0, st, a);
}

bool fattn_pf_quant_ok(const fa_args & a) {
    const int64_t G = a.H / a.Hkv;
    return a.k_type == GGML_TYPE_F16 && a.v_type == GGML_TYPE_F16 && a.D == 128 && a.n_q >= 16 && a.H % a.Hkv == 0 &&
           (G == 4 || G == 8 || G == 16);
}

void launch_fattn_exact(hipStream_t st, const fa_args & a0, int64_t nq3) {
    GGML_ASSERT(a0.H % a0.Hkv == 0);
    fa_args a = a0;
    const dim3 grid((unsigned) a.n_q, (unsigned) (a.H * nq3));
    // prefill (more workgroups than CUs): two workgroups per CU and a 128-position chunk (32 KiB
    // of V in LDS; half the phase-1 K registers of a 256 chunk, so occupancy 2 fits 256 VGPRs
    // without its 40 spills — pp512 9.6k -> 10.6k tok/s, round 2; occupancy 3 / 4 spilled and ran
    // slower, 8.5k / 8.2k)
    const bool wide = a.n_q * a.H * nq3 > 256;
    if (a.k_type == GGML_TYPE_Q4_0) {
        switch (a.D) {
            case 64:  hipLaunchKernelGGL((k_fattn_exact<64, 1, 0, true, true>), grid, dim3(256), 0, st, a); break;
            case 128:
                if (wide) hipLaunchKernelGGL((k_fattn_exact<128, 2, 128, true, true>), grid, dim3(256), 0, st, a);
                else hipLaunchKernelGGL((k_fattn_exact<128, 1, 0, true, true>), grid, dim3(256), 0, st, a);
                break;
            case 256: hipLaunchKernelGGL((k_fattn_exact<256, 1, 0, true, true>), grid, dim3(256), 0, st, a); break;
            default: GGML_ABORT("mi355x: FA head size %d", (int) a.D);
        }
        return;
    }
    if (a.k_type == GGML_TYPE_Q8_0) {
        switch (a.D) {
            case 64:  hipLaunchKernelGGL((k_fattn_exact<64, 1, 0, true>), grid, dim3(256), 0, st, a); break;
            case 128:
                if (wide) hipLaunchKernelGGL((k_fattn_exact<128, 2, 128, true>), grid, dim3(256), 0, st, a);
                else hipLaunchKernelGGL((k_fattn_exact<128, 1, 0, true>), grid, dim3(256), 0, st, a);
                break;
            case 256: hipLaunchKernelGGL((k_fattn_exact<256, 1, 0, true>), grid, dim3(256), 0, st, a); break;
            default: GGML_ABORT("mi355x: FA head size %d", (int) a.D);
        }
        return;
    }
    // prefill, f16 cache, D = 128: query blocks x the GQA group
    const int64_t G = a.H / a.Hkv;
    if (a.D == 128 && a.n_q >= 16 && (a.qmode == 0 || (a.qmode == 1 && fattn_pf_quant_ok(a))) &&
        (G == 1 || G == 2 || G == 4 || G == 8 || G == 16)) {
        const dim3 g((unsigned) ceil_div(a.n_q, (int64_t) PF_P / G), (unsigned) (a.Hkv * nq3));
        // 32-position chunks at three workgroups per CU (half the LDS stage, a 168-VGPR budget: q
        // as packed f16, two pairs per scoring quad, two pairs per coefficient pass; n = 512:
        // 213 -> 171 us, probe_fa_pf.py); GGML_MI355X_PF_CH=64: 64-position chunks at two
        static const int pfch = getenv("GGML_MI355X_PF_CH") ? atoi(getenv("GGML_MI355X_PF_CH")) : 32;
        if (pfch == 32) {
            switch (G) {
                case 1:  hipLaunchKernelGGL((k_fattn_pf<1, 32, 3>), g, dim3(256), 0, st, a); break;
                case 2:  hipLaunchKernelGGL((k_fattn_pf<2, 32, 3>), g, dim3(256), 0, st, a); break;
                case 4:  hipLaunchKernelGGL((k_fattn_pf<4, 32, 3>), g, dim3(256), 0, st, a); break;
                case 8:  hipLaunchKernelGGL((k_fattn_pf<8, 32, 3>), g, dim3(256), 0, st, a); break;
                default: hipLaunchKernelGGL((k_fattn_pf<16, 32, 3>), g, dim3(256), 0, st, a); break;
            }
            return;
        }
        switch (G) {
            case 1:  hipLaunchKernelGGL(k_fattn_pf<1>, g, dim3(256), 0, st, a); break;
            case 2:  hipLaunchKernelGGL(k_fattn_pf<2>, g, dim3(256), 0, st, a); break;
            case 4:  hipLaunchKernelGGL(k_fattn_pf<4>, g, dim3(256), 0, st, a); break;
            case 8:  hipLaunchKernelGGL(k_fattn_pf<8>, g, dim3(256), 0, st, a); break;
            default: hipLaunchKernelGGL(k_fattn_pf<16>, g, dim3(256), 0, st, a); break;
        }
        return;
    }
    switch (a.D) {
        case 64:  hipLaunchKernelGGL(k_fattn_exact<64>, grid, dim3(256), 0, st, a); break;
        case 128:
            if (!wide) hipLaunchKernelGGL(k_fattn_exact<128>, grid, dim3(256), 0, st, a);
            else hipLaunchKernelGGL((k_fattn_exact<128, 2, 128>), grid, dim3(256), 0, st, a);
            break;
        case 256: hipLaunchKernelGGL(k_fattn_exact<256>, grid, dim3(256), 0, st, a); break;
        default: GGML_ABORT("mi355x: FA head size %d", (int) a.D);
    }
}

// ---- long-context decode: the scores in one launch, the exact recurrence in another --------------
// At thousands of cached positions the per-head workgroups above are bound by one CU's intake: a
// head's K and V (1-2 MB at 4096 positions) pass through the one CU that also runs the serial
// chain.  Here the scores — independent per position — are computed first by a grid over
// (256-position block, KV head), every K row read once for the G query heads that share it
// (k_fal_scores); then one workgroup per query head (k_fal_chain) forms the prefix max and the
// (ms, vs) coefficients of ALL positions in LDS (a scan, then expf per position: parallel), and
// its chain waves run the recurrence while its stager waves stream the next V chunk into LDS.
// The arithmetic of every step is k_fattn_exact's (the CPU's ops.cpp:7015-7232), so the bits are.
constexpr int FAL_NMAX = 8192;    // positions the chain's coefficient arrays hold
constexpr int FAL_GMAX = 8;       // query heads per KV head (GQA) the scores kernel takes
constexpr int FAL_U = 8;          // chain batch

template <int KT>   // K type: 0 f16, 1 q8_0, 2 q4_0
__global__ __launch_bounds__(256) void k_fal_scores(const fa_args a, float * __restrict__ sco) {
    constexpr int D = 128, NM = D / 16, NB = D / 32, NP = FAL_PB / 64;
    constexpr int KB = KT == 2 ? 18 : 34;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, qd = tid & 3;
    kt_enter(a.kt, 5);
    const int64_t j0 = (int64_t) blockIdx.x * FAL_PB;
    const int64_t hk = blockIdx.y % a.Hkv, iq3 = blockIdx.y / a.Hkv;
    const int G = (int) (a.H / a.Hkv);
    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * mrow = a.mask;   // decode: mask row 0
    // Q of the group as q8_0 (quantized K: Q is converted to K's vec_dot_type, ops.cpp:7147)
    __shared__ __attribute__((aligned(16))) int8_t qq[KT ? FAL_GMAX * D : 1];
    __shared__ float qqd[KT ? FAL_GMAX * NB : 1];
    __shared__ int16_t qqs[KT ? FAL_GMAX * NB : 1];
    if constexpr (KT != 0) {
        for (int g = wave; g < G; g += 4) {
            const float * qrow = (const float *) (a.q + (hk * G + g) * a.nbq2 + iq3 * a.nbq3);
            const bool valid = 4 * lane < D;
            float qv[4] = {0.f, 0.f, 0.f, 0.f};
            if (valid) { const float4 t = *(const float4 *) (qrow + 4 * lane); qv[0] = t.x; qv[1] = t.y; qv[2] = t.z; qv[3] = t.w; }
            q8_0_wave(qv, lane, valid, qq + g * D, qqd + g * NB, qqs + g * NB);
        }
        __syncthreads();
    }
    // this block's K rows, 4 lanes per position (the layout of k_fattn_exact's phase 1)
    uint2 kh[KT ? 1 : NP][KT ? 1 : NM];
    uint2 kb[KT ? NP : 1][KT ? NB : 1];
    uint32_t kd[KT ? NP : 1][KT ? NB : 1];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int64_t j = min(j0 + 64 * p + (tid >> 2), a.n_kv - 1);
        if constexpr (KT == 0) {
            const char * krow = kbase + j * a.nbk1 + 8 * qd;
#pragma unroll
            for (int m = 0; m < NM; ++m) kh[p][m] = ld8(krow + 32 * m);
        } else {
            const uint8_t * krow = (const uint8_t *) kbase + j * a.nbk1;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if constexpr (KT == 2) {
                    const uint2 q = ld8(krow + KB * b + 2 + 8 * (qd & 1));
                    const int sh = 4 * (qd >> 1);
                    kb[p][b] = make_uint2((((q.x >> sh) & 0x0f0f0f0fu) + 0x78787878u) ^ 0x80808080u,
                                          (((q.y >> sh) & 0x0f0f0f0fu) + 0x78787878u) ^ 0x80808080u);
                } else {
                    kb[p][b] = ld8(krow + KB * b + 2 + 8 * qd);
                }
                kd[p][b] = ld2(krow + KB * b);
            }
        }
    }
    float mv[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const int64_t j = j0 + 64 * p + (tid >> 2);
        mv[p] = j < a.n_kv && mrow ? h2f(*(const uint16_t *) (mrow + 2 * j)) : 0.0f;
    }
    for (int g = 0; g < G; ++g) {
        const int64_t h = hk * G + g;
        const float slope = a.max_bias > 0.0f
            ? (float) ((uint32_t) h < a.n_head_log2 ? pow((double) a.m0, (double) (h + 1))
                                                   : pow((double) a.m1, (double) (2 * ((uint32_t) h - a.n_head_log2) + 1)))
            : 1.0f;
        float * out = sco + (iq3 * a.H + h) * a.n_kv;
        float w[NP];
        if constexpr (KT == 0) {
            float qf[NM][4];
            const float * qrow = (const float *) (a.q + h * a.nbq2 + iq3 * a.nbq3);
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                const float4 q4 = *(const float4 *) (qrow + 16 * m + 4 * qd);
                qf[m][0] = f16r(q4.x); qf[m][1] = f16r(q4.y); qf[m][2] = f16r(q4.z); qf[m][3] = f16r(q4.w);
            }
#pragma unroll
            for (int p = 0; p < NP; ++p) w[p] = dot_f16_avx512_q4<D>(kh[p], qf);
        } else {
            uint2 qb[NB];
            float qdb[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                qb[b] = *(const uint2 *) (qq + g * D + 32 * b + 8 * qd);
                qdb[b] = qqd[g * NB + b];
            }
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                float ae = 0.0f, ao = 0.0f;
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    const float dd = __fmul_rn(h2f((uint16_t) kd[p][b]), qdb[b]);
                    ae = fmaf(dd, (float) dot4((int) kb[p][b].x, (int) qb[b].x, 0), ae);
                    ao = fmaf(dd, (float) dot4((int) kb[p][b].y, (int) qb[b].y, 0), ao);
                }
                ae = __fadd_rn(ae, quad_from_plus2(ae));
                ao = __fadd_rn(ao, quad_from_plus2(ao));
                ae = __fadd_rn(ae, quad_from_plus1(ae));
                ao = __fadd_rn(ao, quad_from_plus1(ao));
                w[p] = __fadd_rn(ae, ao);
            }
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const int64_t j = j0 + 64 * p + (tid >> 2);
            if (qd == 0 && j < a.n_kv) {
                float sv = __fmul_rn(w[p], a.scale);
                if (a.softcap != 0.0f) sv = __fmul_rn(a.softcap, tanhf(sv));
                out[j] = __fadd_rn(sv, __fmul_rn(slope, mv[p]));
            }
        }
    }
    kt_exit(a.kt, 5);
}

// LDS of the chain kernel
// NM: positions the coefficient arrays hold (6144 or FAL_NMAX: the smaller instance keeps the
// per-thread score registers and the unrolled passes of shorter caches small)
template <int VT, int NM = FAL_NMAX> struct fal_smem {
    static constexpr int D = 128, DH = D / FAL_DSPLIT, NBH = DH / 32;   // a workgroup's dims
    static constexpr int CV = 128;                        // V positions per stage
    static constexpr int RB = VT == 0 ? 2 * DH : (VT == 1 ? 34 * NBH : 18 * NBH);   // bytes of a row's half (raw)
    static constexpr int NSTG = 3;                        // stages: chunks c + 1 and c + 2 in flight
    float cm[NM + 2 * FAL_U];                   // ms coefficient (1 where dead)
    float sc[NM + 2 * FAL_U];                   // vs coefficient (0 where dead)
    uint32_t dead[NM / 32 + 2];                 // bit per position: masked (the state is kept)
    uint8_t gb[NM / 64 + 4];                    // per 64 positions: its 8 batches taking the general step
    float wmax[4];
    int wlast[4];
    float ol[64];
    // the workgroup's half of each V row exactly as in the cache (f16, or q8_0 / q4_0 blocks),
    // packed, by LDS-DMA
    __attribute__((aligned(16))) uint8_t vr[NSTG][CV * RB + 64];
};

// one step of a wave's inclusive max-scan: lanes without a DPP source keep -inf as the operand
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float fal_dmax(float v) {
    const int t = __builtin_amdgcn_update_dpp(__float_as_int(-INFINITY), __float_as_int(v), CTRL, ROW_MASK, 0xf, false);
    return fmaxf(v, __int_as_float(t));
}

// the chain holds the f16 V values as 32-bit words (as halves it measured 7 % slower at 4096; as a
// 16-bit asm operand the compiler packed pairs with v_perm and unpacked them again)
typedef uint32_t fal_v16;
#define FAL_MAD f16_mad
template <int VT, int NM>   // V type: 0 f16, 1 q8_0, 2 q4_0; NM: positions held (n_kv <= NM)
__global__ __launch_bounds__(FAL_THREADS, 1) void k_fal_chain(const fa_args a, const float * __restrict__ sco) {
    using SM = fal_smem<VT, NM>;
    constexpr int D = 128, NB = D / 32, CV = SM::CV, U = FAL_U;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    kt_enter(a.kt, 1 + FAL_THREADS / 64);
    // FAL_DSPLIT workgroups per head, each the recurrence of DH of its dims: V is staged through
    // the CU's LDS-DMA at ~25 GB/s per CU (MI355X_MICROARCH.md ldsdma-fill), so one CU per head
    // spent most of the chain waiting for its V stages; the split halves every CU's bytes while
    // each keeps a whole chain of its own (the dims' recurrences are independent; the
    // coefficients are formed by every workgroup of the head alike)
    const int64_t h = blockIdx.x / FAL_DSPLIT, dh = blockIdx.x % FAL_DSPLIT, iq3 = blockIdx.y;
    const int64_t hk = h / (a.H / a.Hkv);
    __shared__ __attribute__((aligned(16))) SM sm;
    constexpr int RB = SM::RB, NSTG = SM::NSTG, DH = SM::DH;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3 + dh * RB;
    const char * mrow = a.mask;
    const float * srow = sco + (iq3 * a.H + h) * a.n_kv;

    // ---- stage this half of V rows [c0, c0 + n) into buffer st by LDS-DMA: waves 1-3.  f16
    // halves (128 B) go 8 to an instruction; q8_0 / q4_0 halves (68 / 36 B, not 16-B granular) a
    // dword a lane: per wave and chunk of 128 at most 12 instructions, so two chunks in flight
    // stay within vmcnt's 63.  Returns this wave's instruction count (its vmcnt share).
    auto stage = [&](int st, int64_t c0, int n) -> int {
        const int t = tid - 64, sw = t >> 6;   // stager wave 0..2
        uint8_t * dst = sm.vr[st];
        int cnt = 0;
        if constexpr (VT == 0) {
            const int r_in = (t & 63) >> 3, col = t & 7;
            for (int q = sw; 8 * q < n; q += 3, ++cnt) {
                const int row = min(8 * q + r_in, n - 1);
                lds_dma16(vbase + (c0 + row) * a.nbv1 + 16 * col, dst + 1024 * q);
            }
        } else {
            // each stager wave moves a contiguous third of the rows
            constexpr int DW = RB / 4;   // dword i of the wave's rows = row r0 + i / DW, dword i % DW
            const int per = (n + 2) / 3, r0 = min(n, sw * per), r1 = min(n, r0 + per);
            const int ndw = (r1 - r0) * DW;
            for (int q = 0; 64 * q < ndw; ++q, ++cnt) {
                // lanes past the wave's rows stay off: their LDS slots are the next wave's rows
                const int i = 64 * q + (t & 63), row = r0 + i / DW, w = i % DW;
                if (i < ndw) lds_dma4(vbase + (c0 + row) * a.nbv1 + 4 * w, dst + r0 * RB + 256 * q);
            }
        }
        return cnt;
    };
    // chunks 0 and 1 go out first (bounded by the cache; the mask bounds them later)
    const int64_t n_kv = a.n_kv;
    int pend = 0;   // this stager wave's instructions of the chunk after the current one
    if (wave >= 1) {
        stage(0, 0, (int) min<int64_t>(CV, n_kv));
        if (n_kv > CV) pend = stage(1, CV, (int) min<int64_t>(CV, n_kv - CV));
    }

    // ---- coefficients of every position (all waves) ----
    // Wave w owns a contiguous segment of positions (64·nq of them, lane l at 64 i + l of group i),
    // so the running maximum is a scan inside the wave (DPP row shifts and row broadcasts, no LDS
    // round trips) plus ONE exchange of the four segment maxima: the CPU's M before position j is
    // the maximum over every earlier live position, which is the same set either way (max is
    // order-free).  Every score and mask value is loaded first (one memory round trip).
    constexpr int NT = NM / 256;
    const int nq = (int) ((n_kv + 255) / 256);   // 64-position groups per wave (uniform)
    // expf's 32-entry 2^(i/32) table in LDS: a global-table gather per position put one memory
    // round trip into every group of the coefficient pass
    // (its global load is issued with the score loads and stored to LDS after them: a store right
    // behind the load waited a memory round trip before any score load was issued)
    __shared__ uint64_t exptab[32];
    const uint64_t etv = lx_exp2f_tab[tid & 31];
    const int seg0 = wave * 64 * nq;   // (positions < NM: 32-bit arithmetic)
    const int nkv = (int) n_kv;
    float sv[NT];
    // mask values held as 32-bit words: as 16-bit halves each pair was packed right behind its
    // load, a wait per 64-position group (16 serial memory round trips at 4096 positions)
    uint32_t mvb[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        if (i < nq) {
            const int jc = min(seg0 + 64 * i + lane, nkv - 1);
            mvb[i] = mrow ? (uint32_t) *(const uint16_t *) (mrow + 2 * jc) : 0u;
            sv[i] = srow[jc];
        }
    }
    if (tid < 32) exptab[tid] = etv;

    // phase A: each group's own inclusive max-scan and total (the groups are independent, so their
    // latency chains interleave: one wave per SIMD has nothing else to hide them behind), then the
    // carry into every group from the totals before it; the live extent
    float pm[NT], tot[NT];
    int wlast = -1;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        if (i < nq) {   // (a guard, not a break: the loop stays unrolled and the arrays in registers)
            const int j = seg0 + 64 * i + lane;
            const bool live = j < nkv && h2f((uint16_t) mvb[i]) != -INFINITY;
            const float sj = live ? sv[i] : -INFINITY;
            sv[i] = sj;
            float v = sj;
            v = fal_dmax<0x111, 0xf>(v);   // row_shr:1
            v = fal_dmax<0x112, 0xf>(v);   // row_shr:2
            v = fal_dmax<0x114, 0xf>(v);   // row_shr:4
            v = fal_dmax<0x118, 0xf>(v);   // row_shr:8
            v = fal_dmax<0x142, 0xa>(v);   // row_bcast:15
            v = fal_dmax<0x143, 0xc>(v);   // row_bcast:31
            pm[i] = v;
            tot[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
            const unsigned long long lb = __ballot(live);
            if (lb) wlast = (int) (seg0 + 64 * i + 63 - __clzll(lb));
        }
    }
    float carry[NT];   // the maximum of the segment's groups before group i
    float run = -INFINITY;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        if (i < nq) {   // (a guard, not a break: the loop stays unrolled and the arrays in registers)
            carry[i] = run;
            pm[i] = fmaxf(pm[i], run);
            run = fmaxf(run, tot[i]);
        }
    }
    if (lane == 0) { sm.wmax[wave] = run; sm.wlast[wave] = wlast; }
    // phase stamps (GGML_MI355X_KTRACE_RAW=fa_chain): slots 2.. written by thread 0 in place of
    // waves 1-3's exit stamps
    auto stamp = [&](int i) { if (a.kt && tid == 0) a.kt[(1 + FAL_THREADS / 64) * blockIdx.x + 2 + i] = __builtin_amdgcn_s_memrealtime(); };
    stamp(0);
    __syncthreads();   // (also publishes exptab)
    float Mprev = -INFINITY;
    for (int w2 = 0; w2 < wave; ++w2) Mprev = fmaxf(Mprev, sm.wmax[w2]);
    int nrun = max(max(sm.wlast[0], sm.wlast[1]), max(sm.wlast[2], sm.wlast[3])) + 1;
    // phase B: per position the exclusive maximum M and the score go to cm / sc (the expf pass
    // below turns them into (ms, vs) chunk by chunk, ahead of the chain), dead bits, batch flags
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        if (i < nq) {   // (a guard, not a break: the loop stays unrolled and the arrays in registers)
            const int j = seg0 + 64 * i + lane;
            const float sj = sv[i];
            const bool live = j < nkv && h2f((uint16_t) mvb[i]) != -INFINITY;
            const float ex = __shfl_up(pm[i], 1, WAVE);
            const float M = fmaxf(Mprev, lane > 0 ? ex : carry[i]);
            const bool upd = live && sj > M;
            if (j < NM) { sm.cm[j] = M; sm.sc[j] = sj; }
            const unsigned long long gw = __ballot(!live || upd);
            const unsigned long long dw = __ballot(!live);
            if (lane == 0) {
                const int p0 = seg0 + 64 * i;
                sm.dead[p0 / 32] = (uint32_t) dw;
                sm.dead[p0 / 32 + 1] = (uint32_t) (dw >> 32);
                // bit b: any of batch b's U = 8 positions flagged (each byte's OR, then gathered)
                static_assert(U == 8, "byte-wise batch flags");
                uint64_t x = gw;
                x |= x >> 4; x |= x >> 2; x |= x >> 1;
                sm.gb[p0 / 64] = (uint8_t) (((x & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
            }
        }
    }
    // the expf pass of 64 positions from p0 (one per lane), in place: the CPU's ms = expf(Mold - M)
    // and vs = 1 on a max update, ms = 1 and vs = expf(s - M) otherwise, (1, 0) where dead
    auto coef64 = [&](int p0) {
        const int j = p0 + lane;
        const float M = sm.cm[j], sj = sm.sc[j];
        const bool live = ((sm.dead[j / 32] >> (j % 32)) & 1u) == 0;
        const bool upd = live && sj > M;
        float cmv = 1.0f, scv = 0.0f;
        if (live) {
            const float e = lx_expf_t(upd ? M - sj : sj - M, exptab);
            if (upd) { cmv = M == -INFINITY ? 0.0f : e; scv = 1.0f; }
            else scv = e;
        }
        sm.cm[j] = cmv;
        sm.sc[j] = scv;
    };
    __syncthreads();   // M / s and the dead bits of every position are in
    nrun = __builtin_amdgcn_readfirstlane(nrun);   // uniform (from LDS): scalar loop control below
    const int nchunk = (nrun + CV - 1) / CV;
    if (nchunk > 0 && wave < CV / 64) coef64(64 * wave);   // chunk 0's coefficients before the loop
    if (tid == 0 && nrun > 0) {
        // the positions past the last live one are dead (the last batch reads up to U - 1 of them)
        for (int j = nrun; j < ((nrun + U - 1) / U) * U + U; ++j) sm.dead[j / 32] |= 1u << (j % 32);
        sm.gb[nrun / 64] |= (uint8_t) (1u << ((nrun % 64) / U));   // the partial batch (if any)
    }
    __syncthreads();
    stamp(1);

    // ---- the recurrence: wave 0, one of the workgroup's dims per lane; waves 1-3 keep two chunks
    // in flight; wave 1 also runs the S chain (the CPU's running sum, independent of the dims),
    // so the dims' chain wave issues nothing but its own steps ----
    const int d = lane;
    uint32_t yb = 0;     // f16 bits (f16 V)
    float yf = 0.0f;     // f32 accumulator (quantized V)
    float S = 0.0f;
    // S over chunk c (wave 1; every lane alike): the same steps as the dims' chain takes — a
    // fast batch adds vs, a batch with a max update or a masked position scales first (ms != 1)
    // and keeps the state where masked; the chunk's coefficients are in (published by the
    // barrier that starts the iteration)
    auto s_chunk = [&](int c) {
        const int jc = c * CV, nr = min(CV, nrun - jc), nb = (nr + U - 1) / U;
        uint32_t flags = 0;
#pragma unroll
        for (int k = 0; k < CV / 64; ++k) flags |= (uint32_t) sm.gb[jc / 64 + k] << (8 * k);
        for (int h0 = 0; h0 < nb; h0 += 64 / U) {   // 64 positions: their vs read at once
            float4 v4[64 / 4];
#pragma unroll
            for (int k = 0; k < 64 / 4; ++k) v4[k] = *(const float4 *) (sm.sc + jc + U * h0 + 4 * k);
#pragma unroll
            for (int bb = 0; bb < 64 / U; ++bb) {
                const int b = h0 + bb;
                if (b >= nb) break;
                const float vs[U] = {v4[2 * bb].x, v4[2 * bb].y, v4[2 * bb].z, v4[2 * bb].w,
                                     v4[2 * bb + 1].x, v4[2 * bb + 1].y, v4[2 * bb + 1].z, v4[2 * bb + 1].w};
                static_assert(U == 8, "two float4 per batch");
                if (!((flags >> b) & 1u)) {
#pragma unroll
                    for (int u = 0; u < U; ++u) S = __fadd_rn(S, vs[u]);   // not contracted on the CPU
                } else {
                    const int j = jc + U * b;
                    const uint32_t db = (sm.dead[j / 32] >> (j % 32)) & ((1u << U) - 1);
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const float ms = sm.cm[j + u];
                        const bool live = ((db >> u) & 1u) == 0;
                        const bool upd = __float_as_uint(ms) != 0x3f800000u;
                        const float Ss = upd ? __fmul_rn(S, ms) : S;
                        S = live ? __fadd_rn(Ss, vs[u]) : S;
                    }
                }
            }
        }
    };
    for (int c = 0; c < nchunk; ++c) {
        const int st = c % NSTG;
        // this wave's stage-c instructions have landed (those of c + 1 may still be in flight)
        if (wave >= 1) eng_vm_wait_fa(pend);
        __syncthreads();   // stage c is in; every chain lane is done with chunk c - 1's stage
        if (wave >= 1) {
            pend = c + 2 < nchunk ? stage((c + 2) % NSTG, (int64_t) (c + 2) * CV, min(CV, nrun - (c + 2) * CV)) : 0;
            // the next chunk's coefficients, by waves 2 and 3 in turn, while the chain runs this one
            if (c + 1 < nchunk && wave >= 2 && (c + 1) % 2 == wave - 2) {
#pragma unroll
                for (int g2 = 0; g2 < CV / 64; ++g2) coef64((c + 1) * CV + 64 * g2);
            }
            if (wave == 1) s_chunk(c);
            continue;
        }
        const int jc = c * CV;                  // first position of the chunk
        const int nr = min(CV, nrun - jc);      // positions to run
        const int nb = (nr + U - 1) / U;
        // batch flags of the chunk: CV / U batches from the per-64 bytes
        uint32_t flags = 0;
#pragma unroll
        for (int k = 0; k < CV / 64; ++k) flags |= (uint32_t) sm.gb[jc / 64 + k] << (8 * k);
        flags = __builtin_amdgcn_readfirstlane(flags);
        const float * scp = sm.sc + jc;
        const float * cmp = sm.cm + jc;
        // the U dead bits of the batch at chunk position j (j a multiple of U)
        auto deadb = [&](int j) { return (sm.dead[(jc + j) / 32] >> ((jc + j) % 32)) & ((1u << U) - 1); };
        auto ld4 = [&](const float * p, float (&o)[U]) {
#pragma unroll
            for (int u = 0; u < U; u += 4) {
                const float4 t = *(const float4 *) (p + u);
                o[u] = t.x; o[u + 1] = t.y; o[u + 2] = t.z; o[u + 3] = t.w;
            }
        };
        if constexpr (VT == 0) {
            const auto * vrow = (const uint16_t *) sm.vr[st] + d;
            auto ldb = [&](int j, fal_v16 (&vv)[U], float (&vs)[U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) vv[u] = vrow[(j + u) * DH];
                ld4(scp + j, vs);
            };
            auto run = [&](const fal_v16 (&vv)[U], const float (&vs)[U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) yb = FAL_MAD(vv[u], vs[u], yb);
            };
            // the next batch's LDS reads are issued before this batch's steps (a scheduling
            // barrier: the compiler otherwise sank the vs reads to the top of their own batch and
            // waited on them there)
            auto fast_run = [&](int j0, int nf) {
                fal_v16 va[U], vb[U];
                float sa[U], sb[U];
                ldb(j0, va, sa);
                for (int k = 0; k < nf; k += 2) {
                    ldb(j0 + (k + 1) * U, vb, sb);
                    __builtin_amdgcn_sched_barrier(0);
                    run(va, sa);
                    if (k + 1 >= nf) break;
                    ldb(j0 + (k + 2) * U, va, sa);
                    __builtin_amdgcn_sched_barrier(0);
                    run(vb, sb);
                }
            };
            auto general = [&](int j) {
                fal_v16 vv[U];
                float vs[U], ms[U];
                ldb(j, vv, vs);
                ld4(cmp + j, ms);
                const uint32_t db = deadb(j);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const bool live = ((db >> u) & 1u) == 0;
                    const bool upd = __float_as_uint(ms[u]) != 0x3f800000u;
                    float t = __fmul_rn(h2f((uint16_t) yb), ms[u]);
                    asm("" : "+v"(t));   // two roundings, as f16r
                    const uint32_t ys = upd ? (uint32_t) f2h(t) : yb;
                    const uint32_t yn = FAL_MAD(vv[u], vs[u], ys);
                    yb = live ? yn : yb;
                }
            };
            int b = 0;
            while (b < nb) {
                const uint32_t rest = flags >> b;
                const int nf = min(rest ? __builtin_ctz(rest) : 32, nb - b);
                if (nf > 0) { fast_run(b * U, nf); b += nf; }
                if (b < nb) { general(b * U); ++b; }
            }
        } else {
            // f32 recurrence on dequantized V: v = (float) q * d (dequantize_row_q8_0 / _q4_0)
            // the lane's byte and its block's f16 scale in a raw half row: q8_0 block b = d / 32 at
            // 34 b (d at +2, qs at +2 + d % 32); q4_0 at 18 b (qs at +2 + d % 16, low nibble for
            // d % 32 < 16)
            constexpr int KBV = VT == 2 ? 18 : 34;
            const int bo = KBV * (d / 32);
            const int qo = bo + 2 + (VT == 2 ? (d % 16) : (d % 32));
            const int nsh = VT == 2 && (d % 32) >= 16 ? 4 : 0;
            const uint8_t * vrw = sm.vr[st];
            // a batch's raw bytes and block scales are read one batch ahead; the dequant (off the
            // chain) happens in run, so a read's wait never precedes the previous batch
            // (dequantizing whole chunks into an f32 buffer in the stager waves measured slower:
            // the stagers, not the chain, became the bound)
            struct vraw { uint32_t q[U]; uint32_t dv[U]; };
            auto ldb = [&](int j, vraw & vv, float (&vs)[U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    vv.q[u] = vrw[(j + u) * RB + qo];
                    vv.dv[u] = *(const uint16_t *) (vrw + (j + u) * RB + bo);
                }
                ld4(scp + j, vs);
            };
            // dequantize_row_q8_0 / _q4_0: (float) q * d, q4_0's q = nibble - 8
            auto deq = [&](const vraw & vv, int u) {
                const int q = VT == 2 ? (int) ((vv.q[u] >> nsh) & 15u) - 8 : (int) (int8_t) vv.q[u];
                return __fmul_rn((float) q, h2f((uint16_t) vv.dv[u]));
            };
            auto run = [&](const vraw & vv, const float (&vs)[U]) {
#pragma unroll
                for (int u = 0; u < U; ++u) yf = fmaf(deq(vv, u), vs[u], yf);   // ggml_vec_mad_f32
            };
            auto fast_run = [&](int j0, int nf) {
                vraw va, vb;
                float sa[U], sb[U];
                ldb(j0, va, sa);
                for (int k = 0; k < nf; k += 2) {
                    ldb(j0 + (k + 1) * U, vb, sb);
                    run(va, sa);
                    if (k + 1 >= nf) break;
                    ldb(j0 + (k + 2) * U, va, sa);
                    run(vb, sb);
                }
            };
            auto general = [&](int j) {
                vraw vv;
                float vs[U], ms[U];
                ldb(j, vv, vs);
                ld4(cmp + j, ms);
                const uint32_t db = deadb(j);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const bool live = ((db >> u) & 1u) == 0;
                    const bool upd = __float_as_uint(ms[u]) != 0x3f800000u;
                    const float ys = upd ? __fmul_rn(yf, ms[u]) : yf;   // ggml_vec_scale_f32
                    yf = live ? fmaf(deq(vv, u), vs[u], ys) : yf;
                }
            };
            int b = 0;
            while (b < nb) {
                const uint32_t rest = flags >> b;
                const int nf = min(rest ? __builtin_ctz(rest) : 32, nb - b);
                if (nf > 0) { fast_run(b * U, nf); b += nf; }
                if (b < nb) { general(b * U); ++b; }
            }
        }
    }

    // ---- output and its optional quantization (k_fattn_exact's epilogue) ----
    // (wave 0 holds the workgroup's DH outputs, dims DH·dh ..; wave 1 the sum S)
    if (wave == 1 && lane == 0) sm.wmax[0] = S;
    stamp(2);
    __syncthreads();
    S = sm.wmax[0];
    float * drow = (float *) ((char *) a.dst + h * a.nb1_dst + iq3 * a.nb2_dst) + DH * dh;
    const float o = wave == 0 ? __fmul_rn(VT ? yf : h2f((uint16_t) yb), 1.0f / S) : 0.0f;
    if (wave == 0) {
        if (a.qmode == 1) __hip_atomic_store(drow + d, o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else drow[d] = o;
    }
    if (a.qmode == 2) {
        // Q8_0 blocks of 32: the workgroup's DH outputs are whole blocks
        if (wave == 0) sm.ol[d] = o;
        __syncthreads();
        if (wave == 0) {
            const bool valid = 4 * lane < DH;
            float q[4] = {0.f, 0.f, 0.f, 0.f};
            if (valid) { const float4 v4 = *(const float4 *) (sm.ol + 4 * lane); q[0] = v4.x; q[1] = v4.y; q[2] = v4.z; q[3] = v4.w; }
            const int64_t c0 = h * D + DH * dh;
            q8_0_wave(q, lane, valid, a.qs + c0, a.qd + c0 / 32, a.qsum + c0 / 32);
        }
    } else if (a.qmode == 1) {
        // Q8_K: a block of 256 = two heads = 2·FAL_DSPLIT workgroups; the last of them to finish
        // quantizes it (write-through outputs drained before the counter add, read back with sc1 loads)
        const int64_t blk = (h * D) / 256;
        __shared__ int is_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const int prev = __hip_atomic_fetch_add(a.cnt + blk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            is_last = prev == 2 * FAL_DSPLIT - 1;
            if (is_last) __hip_atomic_store(a.cnt + blk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (is_last && wave == 0) {
            const float * brow = (const float *) a.dst + 256 * blk;
            float q[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) q[c] = __hip_atomic_load(brow + 4 * lane + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int64_t c0 = 256 * blk;
            q8K_wave(q, lane, a.qs + c0, a.qsum + c0 / 16, a.qd + c0 / 256);
        }
    }
    if (wave == 0) kt_exit(a.kt, 1 + FAL_THREADS / 64);
}

// the long-context pair applies: one query row, D = 128, a cache longer than FA_LONG_MIN (and
// within the chain's coefficient arrays), a GQA group the scores kernel takes, one batch
bool fattn_long_ok(const fa_args & a, int64_t nq3) {
    // from where the pair beats the per-head kernels (scripts/probe_fal.py, round 4): f16 ≈ 700
    // positions, q8_0 below 512 (its per-head kernel is slower); GGML_MI355X_FA_LONG sets both
    static const int lenv = getenv("GGML_MI355X_FA_LONG") ? atoi(getenv("GGML_MI355X_FA_LONG")) : -1;
    const int lmin = lenv >= 0 ? lenv : (a.k_type == GGML_TYPE_F16 ? FA_LONG_MIN : FA_LONG_MIN_Q);
    return lmin > 0 && a.n_q == 1 && a.D == 128 && nq3 == 1 && a.n_kv >= lmin && a.n_kv <= FAL_NMAX &&
           a.H % a.Hkv == 0 && a.H / a.Hkv <= FAL_GMAX && (a.qmode != 1 || a.H % 2 == 0) &&
           (a.k_type == GGML_TYPE_F16 || a.k_type == GGML_TYPE_Q8_0 || a.k_type == GGML_TYPE_Q4_0);
}

static size_t fal_pad(size_t static_lds) {
    const size_t half = 80 * 1024 + 1024;
    return static_lds >= half ? 0 : half - static_lds;
}

void launch_fattn_long(hipStream_t st, const fa_args & a0, float * sco, unsigned long long * kt_scores) {
    fa_args a = a0;
    a.kt = kt_scores;
    const dim3 gs((unsigned) ceil_div(a.n_kv, (int64_t) FAL_PB), (unsigned) a.Hkv);
    switch (a.k_type) {
        case GGML_TYPE_F16:  hipLaunchKernelGGL(k_fal_scores<0>, gs, dim3(256), 0, st, a, sco); break;
        case GGML_TYPE_Q8_0: hipLaunchKernelGGL(k_fal_scores<1>, gs, dim3(256), 0, st, a, sco); break;
        default:             hipLaunchKernelGGL(k_fal_scores<2>, gs, dim3(256), 0, st, a, sco); break;
    }
    a.kt = a0.kt;
    const dim3 gc((unsigned) (a.H * FAL_DSPLIT), 1);
    const bool small = a.n_kv <= 6144;
    switch (a.v_type) {
        // (dynamic LDS pads a workgroup past half the CU's 160 KiB: one per CU, so no two chains
        // share a CU's LDS-DMA stream)
#define FAL_CHAIN(VT, NM) hipLaunchKernelGGL((k_fal_chain<VT, NM>), gc, dim3(FAL_THREADS), fal_pad(sizeof(fal_smem<VT, NM>)), st, a, (const float *) sco)
        case GGML_TYPE_F16:  if (small) FAL_CHAIN(0, 6144); else FAL_CHAIN(0, FAL_NMAX); break;
        case GGML_TYPE_Q8_0: if (small) FAL_CHAIN(1, 6144); else FAL_CHAIN(1, FAL_NMAX); break;
        default:             if (small) FAL_CHAIN(2, 6144); else FAL_CHAIN(2, FAL_NMAX); break;
#undef FAL_CHAIN
    }
}

// test hook: the K·Q scores exactly as phase 1 of k_fattn_exact computes them
// (q [D] f32 is f16-rounded first), 4 lanes per cache row; D = 128
__global__ void k_fattn_scores_d128(const float * q, const uint16_t * k, int64_t n, float * s) {
    const int qd = threadIdx.x & 3;
    const int64_t j = ((int64_t) blockIdx.x * blockDim.x + threadIdx.x) >> 2;
    uint2 kh[8];
    float qf[8][4];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        kh[m] = j < n ? ld8(k + j * 128 + 16 * m + 4 * qd) : make_uint2(0, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c) qf[m][c] = f16r(q[16 * m + 4 * qd + c]);
    }
    const float w = dot_f16_avx512_q4<128>(kh, qf);
    if (qd == 0 && j < n) s[j] = w;
}

void fattn_scores_d128(hipStream_t st, const float * q, const uint16_t * k, int64_t n, float * s) {
    hipLaunchKernelGGL(k_fattn_scores_d128, dim3((unsigned) ceil_div(n * 4, 256)), dim3(256), 0, st, q, k, n, s);
}

}  // namespace mi355x
