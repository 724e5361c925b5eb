// k_fattn.hip — FLASH_ATTN_EXT over an f16 or q8_0 KV cache.
//
// Semantics follow ggml_compute_forward_flash_attn_ext_f16 (ggml-cpu/ops.cpp:7015-7232):
//   * Q is first converted to K's vec_dot_type: rounded to f16 for an f16 cache, quantized to
//     Q8_0 (x86 rounding) for a q8_0 cache, and K·Q is taken in that representation;
//   * s = (K·Q)*scale (softcap optional) + slope*mask, masked (-inf) positions are skipped;
//   * online softmax, V accumulated with weights exp(s - M), output VKQ * (1/S).
// The CPU accumulates VKQ for an f16 V in f16; we keep it in f32 (documented tolerance,
// test-backend-ops bounds FA at NMSE 5e-4, tests/test-backend-ops.cpp:3334-3336).
//
// MI355X layout: one workgroup (4 waves) per (q row, q head, KV chunk).  A wave scores 64
// KV positions at once with one position per lane (K rows read as 16-byte vectors, Q
// broadcast from LDS), does the online-softmax update with wave reductions, then streams
// the 64 V rows with lanes owning D/64 output dims each.  Long caches are split over
// chunks (split-K) so decode fills the chip; a combine kernel merges the chunk partials.
#include "ops.h"

#include <cmath>

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
};

template <int EPL>  // elements of D per lane (D = 64*EPL)
__global__ __launch_bounds__(256) void k_fattn_vec(const fa_args a) {
    constexpr int D = 64 * EPL;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t chunk = blockIdx.x;
    const int64_t iq1 = blockIdx.y;
    const int64_t h = blockIdx.z % a.H;
    const int64_t iq3 = blockIdx.z / a.H;
    const int64_t hk = h / (a.H / a.Hkv);

    __shared__ float qf[D];          // Q as f32 (f16-rounded for an f16 K)
    __shared__ int8_t qq[D];         // Q quantized to q8_0 (q8_0 K)
    __shared__ float qd[D / 32];
    __shared__ float red_m[4], red_s[4];
    __shared__ float red_o[4][D];

    const float * qrow = (const float *) (a.q + iq1 * a.nbq1 + h * a.nbq2 + iq3 * a.nbq3);
    if (a.k_type == GGML_TYPE_Q8_0) {
        if (wave == 0) {
            // x86 quantize_row_q8_0 on the Q row (see k_mmv.hip); lane handles D/64 values
            for (int b = 0; b < D / 32; ++b) {
                const float x = lane < 32 ? qrow[b * 32 + lane] : 0.0f;
                float amax = fabsf(x);
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o, WAVE));
                const float dd = amax / 127.0f;
                const float id = amax != 0.0f ? 127.0f / amax : 0.0f;
                if (lane < 32) {
                    int iv = (int) rintf(__fmul_rn(x, id));
                    iv = iv > 127 ? 127 : (iv < -128 ? -128 : iv);
                    qq[b * 32 + lane] = (int8_t) iv;
                }
                if (lane == 0) qd[b] = h2f(f2h(dd));
            }
        }
    } else {
        for (int i = threadIdx.x; i < D; i += 256) {
            const float x = qrow[i];
            qf[i] = a.k_type == GGML_TYPE_F16 ? h2f(f2h(x)) : x;
        }
    }
    __syncthreads();

    const int64_t kv0 = chunk * a.chunk;
    const int64_t kv1 = min(a.n_kv, kv0 + a.chunk);
    const uint32_t hh = (uint32_t) h;
    const float slope = a.max_bias > 0.0f ? (hh < a.n_head_log2 ? powf(a.m0, hh + 1) : powf(a.m1, 2 * (hh - a.n_head_log2) + 1)) : 1.0f;
    const char * mrow = a.mask ? a.mask + (iq1 % a.mask_ne1) * a.nbm1 : nullptr;

    float M = -INFINITY, S = 0.0f;
    float o[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) o[e] = 0.0f;

    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;

    for (int64_t t0 = kv0 + 64 * wave; t0 < kv1; t0 += 256) {
        const int64_t pos = t0 + lane;
        float s = -INFINITY;
        if (pos < kv1) {
            const float mv = mrow ? slope * h2f(*(const uint16_t *) (mrow + 2 * pos)) : 0.0f;
            if (mv != -INFINITY) {
                const char * krow = kbase + pos * a.nbk1;
                float dot = 0.0f;
                if (a.k_type == GGML_TYPE_F16) {
#pragma unroll 4
                    for (int d8 = 0; d8 < D / 8; ++d8) {
                        const uint4 kv = ld16(krow + 16 * d8);
                        const float4 qa = *(const float4 *) &qf[8 * d8];
                        const float4 qb = *(const float4 *) &qf[8 * d8 + 4];
                        dot = fmaf(h2f(kv.x & 0xffff), qa.x, dot); dot = fmaf(h2f(kv.x >> 16), qa.y, dot);
                        dot = fmaf(h2f(kv.y & 0xffff), qa.z, dot); dot = fmaf(h2f(kv.y >> 16), qa.w, dot);
                        dot = fmaf(h2f(kv.z & 0xffff), qb.x, dot); dot = fmaf(h2f(kv.z >> 16), qb.y, dot);
                        dot = fmaf(h2f(kv.w & 0xffff), qb.z, dot); dot = fmaf(h2f(kv.w >> 16), qb.w, dot);
                    }
                } else if (a.k_type == GGML_TYPE_Q8_0) {
                    for (int b = 0; b < D / 32; ++b) {
                        const char * kb = krow + 34 * b;
                        const float dk = h2f(ld2(kb));
                        const uint4 k0 = ld16(kb + 2), k1 = ld16(kb + 18);
                        const int4 q0 = *(const int4 *) &qq[32 * b];
                        const int4 q1 = *(const int4 *) &qq[32 * b + 16];
                        int is = 0;
                        is = dot4(k0.x, q0.x, is); is = dot4(k0.y, q0.y, is); is = dot4(k0.z, q0.z, is); is = dot4(k0.w, q0.w, is);
                        is = dot4(k1.x, q1.x, is); is = dot4(k1.y, q1.y, is); is = dot4(k1.z, q1.z, is); is = dot4(k1.w, q1.w, is);
                        dot += (float) is * (dk * qd[b]);
                    }
                } else {  // f32 K
                    for (int d = 0; d < D; ++d) dot = fmaf(*(const float *) (krow + 4 * d), qf[d], dot);
                }
                s = dot * a.scale;
                if (a.softcap != 0.0f) s = a.softcap * tanhf(s);
                s += mv;
            }
        }
        const float tmax = wave_max(s);
        if (tmax == -INFINITY) continue;  // whole tile masked
        const float Mnew = fmaxf(M, tmax);
        const float ms = M == -INFINITY ? 0.0f : expf(M - Mnew);
        const float p = s == -INFINITY ? 0.0f : expf(s - Mnew);
        S = S * ms + wave_sum(p);
#pragma unroll
        for (int e = 0; e < EPL; ++e) o[e] *= ms;
        M = Mnew;
        const int nvalid = (int) min((int64_t) 64, kv1 - t0);
        for (int j = 0; j < nvalid; ++j) {
            const float pj = __shfl(p, j, WAVE);
            if (pj == 0.0f) continue;  // wave-uniform
            const char * vrow = vbase + (t0 + j) * a.nbv1;
            if (a.v_type == GGML_TYPE_F16) {
                if constexpr (EPL == 2) {
                    const uint32_t vv = ld4(vrow + 4 * lane);
                    o[0] = fmaf(pj, h2f(vv & 0xffff), o[0]);
                    o[1] = fmaf(pj, h2f(vv >> 16), o[1]);
                } else {
#pragma unroll
                    for (int e = 0; e < EPL; ++e) o[e] = fmaf(pj, h2f(ld2(vrow + 2 * (lane * EPL + e))), o[e]);
                }
            } else if (a.v_type == GGML_TYPE_Q8_0) {
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int d = lane * EPL + e;
                    const char * vb = vrow + 34 * (d / 32);
                    o[e] = fmaf(pj, h2f(ld2(vb)) * (float) (int8_t) vb[2 + d % 32], o[e]);
                }
            } else {
#pragma unroll
                for (int e = 0; e < EPL; ++e) o[e] = fmaf(pj, *(const float *) (vrow + 4 * (lane * EPL + e)), o[e]);
            }
        }
    }

    // combine the 4 waves of the workgroup
    if (lane == 0) { red_m[wave] = M; red_s[wave] = S; }
#pragma unroll
    for (int e = 0; e < EPL; ++e) red_o[wave][lane * EPL + e] = o[e];
    __syncthreads();
    if (wave == 0) {
        float Mt = fmaxf(fmaxf(red_m[0], red_m[1]), fmaxf(red_m[2], red_m[3]));
        float St = 0.0f;
        float ot[EPL];
#pragma unroll
        for (int e = 0; e < EPL; ++e) ot[e] = 0.0f;
        for (int w = 0; w < 4; ++w) {
            const float f = (red_m[w] == -INFINITY) ? 0.0f : expf(red_m[w] - Mt);
            St += red_s[w] * f;
#pragma unroll
            for (int e = 0; e < EPL; ++e) ot[e] += red_o[w][lane * EPL + e] * f;
        }
        if (a.nchunks == 1) {
            const float inv = 1.0f / St;
            float * drow = (float *) ((char *) a.dst + iq1 * a.nb1_dst * a.H + h * a.nb1_dst + iq3 * a.nb2_dst);
#pragma unroll
            for (int e = 0; e < EPL; ++e) drow[lane * EPL + e] = ot[e] * inv;
        } else {
            float * pr = a.part + (((chunk * a.n_q + iq1) * a.H + h) + iq3 * a.n_q * a.H * a.nchunks) * (D + 2);
            if (lane == 0) { pr[0] = Mt; pr[1] = St; }
#pragma unroll
            for (int e = 0; e < EPL; ++e) pr[2 + lane * EPL + e] = ot[e];
        }
    }
}

template <int EPL>
__global__ __launch_bounds__(64) void k_fattn_combine(const fa_args a) {
    constexpr int D = 64 * EPL;
    const int lane = threadIdx.x;
    const int64_t iq1 = blockIdx.x, h = blockIdx.y % a.H, iq3 = blockIdx.y / a.H;
    float Mt = -INFINITY;
    for (int c = 0; c < a.nchunks; ++c) {
        const float * pr = a.part + (((c * a.n_q + iq1) * a.H + h) + iq3 * a.n_q * a.H * a.nchunks) * (D + 2);
        Mt = fmaxf(Mt, pr[0]);
    }
    float St = 0.0f, ot[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) ot[e] = 0.0f;
    for (int c = 0; c < a.nchunks; ++c) {
        const float * pr = a.part + (((c * a.n_q + iq1) * a.H + h) + iq3 * a.n_q * a.H * a.nchunks) * (D + 2);
        const float f = pr[0] == -INFINITY ? 0.0f : expf(pr[0] - Mt);
        St += pr[1] * f;
#pragma unroll
        for (int e = 0; e < EPL; ++e) ot[e] += pr[2 + lane * EPL + e] * f;
    }
    const float inv = 1.0f / St;
    float * drow = (float *) ((char *) a.dst + iq1 * a.nb1_dst * a.H + h * a.nb1_dst + iq3 * a.nb2_dst);
#pragma unroll
    for (int e = 0; e < EPL; ++e) drow[lane * EPL + e] = ot[e] * inv;
}

// ------------------------------------------------------------------------------------------
// CPU-exact flash attention for an f16 KV cache (the default; GGML_MI355X_FA_FAST=1 selects
// the split-K f32 kernel above).  Reproduces ops.cpp:7015-7232 on x86-64-v4 (the AVX-512
// CPU backend the reference selects on the MI355X host):
//   * Q rounded to f16; K·Q with ggml_vec_dot_f16's AVX-512 order (vec.cpp:191-231): 16
//     lanes x 4 accumulators of f32 FMAs, REDUCE (x0+=x2, x1+=x3, x0+=x1) then the
//     _mm512_reduce_add_ps tree (8/4/2/1);
//   * the online softmax walks the cache in order and accumulates VKQ in f16 with the
//     vec_mad_f16 / vec_scale_f16 roundings (vec.h:262-290, 410-440): y = f16(fma(v,vs,y)),
//     y = f16(y*ms); S = S*ms + vs; expf taken in double and rounded (glibc's expf is
//     correctly rounded in practice).
// MI355X structure: one workgroup per (q row, KV head) covers the G = H/Hkv query heads of
// that KV head (GQA) so each K/V row is read once for all of them.  Chunks of CH cache
// positions run three phases: (1) all scores in parallel (one position per thread, the K
// row held in VGPRs), (2) per-head prefix max + the (ms, vs) coefficients in parallel,
// (3) the f16 recurrence, sequential over positions, parallel over G*D elements.
// ------------------------------------------------------------------------------------------
constexpr int FAX_CH = 512;     // cache positions per chunk
constexpr int FAX_GMAX = 8;     // max query heads per KV head

// round through f16 AFTER the f32 result exists: the empty asm keeps hipcc from fusing the
// preceding fma/mul into v_fma_mixlo_f16, which rounds the exact product straight to f16
// (one rounding) where the CPU rounds to f32 and then to f16 (two roundings)
__device__ __forceinline__ float f16r(float x) {
    asm volatile("" : "+v"(x));
    return __half2float(__float2half_rn(x));
}

// ggml_vec_dot_f16 (AVX-512) of a K row (f16) with q (f16-rounded floats in LDS)
template <int D>
__device__ __forceinline__ float dot_f16_avx512(const uint32_t (&k)[D / 2], const float * q) {
    float w[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) {
        float a[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int s = 16 * j + l;
            float acc = 0.0f;
#pragma unroll
            for (int i = 0; i < D / 64; ++i) {
                const int e = 64 * i + s;
                const float kv = h2f((k[e >> 1] >> (16 * (e & 1))) & 0xffff);
                acc = i == 0 ? __fmul_rn(kv, q[e]) : fmaf(kv, q[e], acc);
            }
            a[j] = acc;
        }
        w[l] = __fadd_rn(__fadd_rn(a[0], a[2]), __fadd_rn(a[1], a[3]));
    }
    return reduce16_avx512(w);
}

template <int D>
__global__ __launch_bounds__(256) void k_fattn_exact(const fa_args a) {
    const int tid = threadIdx.x;
    const int64_t iq1 = blockIdx.x;
    const int64_t hk = blockIdx.y % a.Hkv;
    const int64_t iq3 = blockIdx.y / a.Hkv;
    const int G = (int) (a.H / a.Hkv);

    __shared__ float qf[FAX_GMAX][D];
    __shared__ float sc[FAX_GMAX][FAX_CH];   // scores -> vs coefficient
    __shared__ float cm[FAX_GMAX][FAX_CH];   // ms coefficient (0 marks "skip", <0 unused)
    __shared__ float red[FAX_GMAX][4];
    __shared__ float mcarry[FAX_GMAX];

    for (int i = tid; i < G * D; i += 256) {
        const int g = i / D, d = i % D;
        const float * qrow = (const float *) (a.q + iq1 * a.nbq1 + (hk * G + g) * a.nbq2 + iq3 * a.nbq3);
        qf[g][d] = f16r(qrow[d]);
    }
    if (tid < FAX_GMAX) mcarry[tid] = -INFINITY;

    // phase-3 state: each thread owns up to 4 (g, d) elements
    constexpr int EMAX = FAX_GMAX * D / 256 > 0 ? FAX_GMAX * D / 256 : 1;
    float y[EMAX], S[EMAX];
#pragma unroll
    for (int e = 0; e < EMAX; ++e) { y[e] = 0.0f; S[e] = 0.0f; }
    const int nel = G * D;

    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;
    const char * mrow = a.mask ? a.mask + (iq1 % a.mask_ne1) * a.nbm1 : nullptr;
    __syncthreads();

    for (int64_t c0 = 0; c0 < a.n_kv; c0 += FAX_CH) {
        const int nch = (int) min((int64_t) FAX_CH, a.n_kv - c0);
        // ---- phase 1: scores ---------------------------------------------------------------
        for (int j = tid; j < nch; j += 256) {
            const int64_t pos = c0 + j;
            const float mv = mrow ? h2f(*(const uint16_t *) (mrow + 2 * pos)) : 0.0f;
            if (mv == -INFINITY) {
                for (int g = 0; g < G; ++g) sc[g][j] = -INFINITY;
                continue;
            }
            uint32_t kr[D / 2];
            const char * krow = kbase + pos * a.nbk1;
#pragma unroll
            for (int i = 0; i < D / 8; ++i) {
                const uint4 v = ld16(krow + 16 * i);
                kr[4 * i] = v.x; kr[4 * i + 1] = v.y; kr[4 * i + 2] = v.z; kr[4 * i + 3] = v.w;
            }
            for (int g = 0; g < G; ++g) {
                float s = dot_f16_avx512<D>(kr, qf[g]);
                s = __fmul_rn(s, a.scale);
                if (a.softcap != 0.0f) s = __fmul_rn(a.softcap, tanhf(s));
                // ALiBi slope of head h = hk*G + g (ops.cpp:7109)
                const uint32_t hh = (uint32_t) (hk * G + g);
                const float slope = a.max_bias > 0.0f
                    ? (float) (hh < a.n_head_log2 ? pow((double) a.m0, (double) (hh + 1))
                                                  : pow((double) a.m1, (double) (2 * (hh - a.n_head_log2) + 1))) : 1.0f;
                s = __fadd_rn(s, __fmul_rn(slope, mv));
                sc[g][j] = s;
            }
        }
        __syncthreads();
        // ---- phase 2: prefix max per head and the (ms, vs) coefficients --------------------
        constexpr int PER = FAX_CH / 256;
        for (int g = 0; g < G; ++g) {
            float lm = -INFINITY;
#pragma unroll
            for (int p = 0; p < PER; ++p) {
                const int j = tid * PER + p;
                if (j < nch) lm = fmaxf(lm, sc[g][j]);
            }
            // inclusive scan of max across the 256 threads
            const int lane = tid & 63, wave = tid >> 6;
            float sm = lm;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const float t = __shfl_up(sm, o, WAVE);
                if (lane >= o) sm = fmaxf(sm, t);
            }
            if (lane == 63) red[g][wave] = sm;
            __syncthreads();
            float prev = mcarry[g];
            for (int w = 0; w < wave; ++w) prev = fmaxf(prev, red[g][w]);
            const float ex = __shfl_up(sm, 1, WAVE);
            if (lane > 0) prev = fmaxf(prev, ex);
            // sequential within the thread's positions
            float M = prev;
#pragma unroll
            for (int p = 0; p < PER; ++p) {
                const int j = tid * PER + p;
                if (j >= nch) break;
                const float s = sc[g][j];
                if (s == -INFINITY) { cm[g][j] = -1.0f; sc[g][j] = 0.0f; continue; }
                if (s > M) {
                    cm[g][j] = M == -INFINITY ? 0.0f : expf_cr(M - s);   // ms, applied before the add
                    sc[g][j] = 1.0f;                                       // vs
                    M = s;
                } else {
                    cm[g][j] = 1.0f;
                    sc[g][j] = expf_cr(s - M);
                }
            }
            __syncthreads();
            if (tid == 255) mcarry[g] = fmaxf(mcarry[g], fmaxf(red[g][0], fmaxf(red[g][1], fmaxf(red[g][2], red[g][3]))));
            __syncthreads();
        }
        // ---- phase 3: sequential f16 recurrence --------------------------------------------
        // the element loop is innermost so a thread's EMAX independent chains interleave
        if (tid < nel) {
            int ge[EMAX];
            const char * vp[EMAX];
#pragma unroll
            for (int e = 0; e < EMAX; ++e) {
                const int idx = min(tid + 256 * e, nel - 1);
                ge[e] = idx / D;
                vp[e] = vbase + c0 * a.nbv1 + 2 * (idx % D);
            }
            constexpr int U = 8;
            for (int j = 0; j < nch; j += U) {
                uint16_t vv[U][EMAX];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int e = 0; e < EMAX; ++e)
                        vv[u][e] = (j + u < nch) ? *(const uint16_t *) (vp[e] + (j + u) * a.nbv1) : 0;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (j + u >= nch) break;
#pragma unroll
                    for (int e = 0; e < EMAX; ++e) {
                        const float ms = cm[ge[e]][j + u];
                        if (ms < 0.0f) continue;
                        const float vs = sc[ge[e]][j + u];
                        float yy = y[e];
                        if (ms != 1.0f) yy = f16r(__fmul_rn(yy, ms));
                        y[e] = f16r(fmaf(h2f(vv[u][e]), vs, yy));
                        S[e] = __fadd_rn(__fmul_rn(S[e], ms), vs);   // not contracted on the CPU
                    }
                }
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
        const int idx = tid + 256 * e;
        if (idx >= nel) break;
        const int g = idx / D, d = idx % D;
        const int64_t h = hk * G + g;
        float * drow = (float *) ((char *) a.dst + iq1 * a.nb1_dst * a.H + h * a.nb1_dst + iq3 * a.nb2_dst);
        drow[d] = __fmul_rn(y[e], 1.0f / S[e]);
    }
}

// test hook: the K·Q scores exactly as phase 1 of k_fattn_exact computes them
// (q [D] f32 is f16-rounded first), one thread per cache row; D = 128
__global__ void k_fattn_scores_d128(const float * q, const uint16_t * k, int64_t n, float * s) {
    __shared__ float qf[128];
    for (int i = threadIdx.x; i < 128; i += blockDim.x) qf[i] = f16r(q[i]);
    __syncthreads();
    const int64_t j = (int64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    uint32_t kr[64];
    for (int i = 0; i < 16; ++i) {
        const uint4 v = ld16(k + j * 128 + 8 * i);
        kr[4 * i] = v.x; kr[4 * i + 1] = v.y; kr[4 * i + 2] = v.z; kr[4 * i + 3] = v.w;
    }
    s[j] = dot_f16_avx512<128>(kr, qf);
}

void fattn_scores_d128(hipStream_t st, const float * q, const uint16_t * k, int64_t n, float * s) {
    hipLaunchKernelGGL(k_fattn_scores_d128, dim3((unsigned) ceil_div(n, 64)), dim3(64), 0, st, q, k, n, s);
}

bool fattn_supported(const ggml_tensor * op) {
    const ggml_tensor * q = op->src[0];
    const ggml_tensor * k = op->src[1];
    const ggml_tensor * v = op->src[2];
    const ggml_tensor * mask = op->src[3];
    if (op->src[4] != nullptr) return false;  // attention sinks not supported
    if (q->type != GGML_TYPE_F32) return false;
    if (k->ne[0] != v->ne[0]) return false;
    const int64_t D = k->ne[0];
    if (D != 64 && D != 128 && D != 256) return false;
    if (k->type != v->type) return false;
    if (k->type != GGML_TYPE_F16 && k->type != GGML_TYPE_Q8_0) return false;
    if (mask && mask->type != GGML_TYPE_F16) return false;
    if (mask && (mask->ne[2] != 1 || mask->ne[3] != 1)) return false;
    if (q->ne[2] % k->ne[2] != 0) return false;
    if (k->ne[3] != q->ne[3] || v->ne[3] != q->ne[3]) return false;
    float max_bias;
    memcpy(&max_bias, (const float *) op->op_params + 1, 4);
    return true;
}

void op_flash_attn(exec_ctx & ctx, ggml_tensor * dst) {
    const ggml_tensor * q = dst->src[0];
    const ggml_tensor * k = dst->src[1];
    const ggml_tensor * v = dst->src[2];
    const ggml_tensor * mask = dst->src[3];
    fa_args a;
    a.q = (const char *) q->data; a.nbq1 = q->nb[1]; a.nbq2 = q->nb[2]; a.nbq3 = q->nb[3];
    a.k = (const char *) k->data; a.nbk1 = k->nb[1]; a.nbk2 = k->nb[2]; a.nbk3 = k->nb[3];
    a.v = (const char *) v->data; a.nbv1 = v->nb[1]; a.nbv2 = v->nb[2]; a.nbv3 = v->nb[3];
    a.mask = mask ? (const char *) mask->data : nullptr;
    a.nbm1 = mask ? mask->nb[1] : 0;
    a.mask_ne1 = mask ? mask->ne[1] : 1;
    a.k_type = k->type; a.v_type = v->type;
    a.D = k->ne[0]; a.n_kv = k->ne[1]; a.n_q = q->ne[1]; a.H = q->ne[2]; a.Hkv = k->ne[2];
    memcpy(&a.scale, (const float *) dst->op_params + 0, 4);
    memcpy(&a.max_bias, (const float *) dst->op_params + 1, 4);
    memcpy(&a.softcap, (const float *) dst->op_params + 2, 4);
    if (a.softcap != 0.0f) a.scale /= a.softcap;
    const uint32_t n_head = (uint32_t) a.H;
    a.n_head_log2 = 1u << (uint32_t) floor(log2((double) n_head));
    a.m0 = powf(2.0f, -(a.max_bias) / a.n_head_log2);
    a.m1 = powf(2.0f, -(a.max_bias / 2.0f) / a.n_head_log2);
    a.dst = (float *) dst->data;
    a.nb1_dst = dst->nb[1];
    a.nb2_dst = dst->nb[3];  // batch stride (dst ne = [D, H, n_q, ne3])
    const int64_t nq3 = q->ne[3];

    // split-K over the cache so that decode fills the 256 CUs
    const int64_t rows = a.n_q * a.H * nq3;
    int64_t nchunks = 1;
    if (rows < 1024) nchunks = std::max<int64_t>(1, std::min<int64_t>(ceil_div(a.n_kv, 256), ceil_div(1024, rows)));
    a.chunk = ceil_div(ceil_div(a.n_kv, nchunks), 64) * 64;
    nchunks = ceil_div(a.n_kv, a.chunk);
    a.nchunks = (int) nchunks;
    a.part = nullptr;
    if (nchunks > 1) a.part = (float *) ctx.scratch(1, sizeof(float) * nchunks * rows * (a.D + 2));

    hipEvent_t ev = nullptr;
    const double bytes = (double) (ggml_nbytes(k) + ggml_nbytes(v)) + (double) ggml_nbytes(q) + (double) ggml_nbytes(dst);
    if (ctx.timing) ctx.time_begin(TK_FATTN, bytes, ev);
    static const bool fast = getenv("GGML_MI355X_FA_FAST") != nullptr && atoi(getenv("GGML_MI355X_FA_FAST")) != 0;
    if (!fast && a.k_type == GGML_TYPE_F16 && a.H / a.Hkv <= FAX_GMAX) {
        dim3 gx((unsigned) a.n_q, (unsigned) (a.Hkv * nq3));
        switch (a.D) {
            case 64:  hipLaunchKernelGGL(k_fattn_exact<64>,  gx, dim3(256), 0, ctx.stream, a); break;
            case 128: hipLaunchKernelGGL(k_fattn_exact<128>, gx, dim3(256), 0, ctx.stream, a); break;
            case 256: hipLaunchKernelGGL(k_fattn_exact<256>, gx, dim3(256), 0, ctx.stream, a); break;
            default: GGML_ABORT("mi355x: FA head size");
        }
        if (ctx.timing) ctx.time_end(TK_FATTN, bytes, ev);
        return;
    }
    dim3 grid((unsigned) nchunks, (unsigned) a.n_q, (unsigned) (a.H * nq3));
    switch (a.D) {
        case 64:  hipLaunchKernelGGL(k_fattn_vec<1>, grid, dim3(256), 0, ctx.stream, a); break;
        case 128: hipLaunchKernelGGL(k_fattn_vec<2>, grid, dim3(256), 0, ctx.stream, a); break;
        case 256: hipLaunchKernelGGL(k_fattn_vec<4>, grid, dim3(256), 0, ctx.stream, a); break;
        default: GGML_ABORT("mi355x: FA head size");
    }
    if (nchunks > 1) {
        dim3 g2((unsigned) a.n_q, (unsigned) (a.H * nq3));
        switch (a.D) {
            case 64:  hipLaunchKernelGGL(k_fattn_combine<1>, g2, dim3(64), 0, ctx.stream, a); break;
            case 128: hipLaunchKernelGGL(k_fattn_combine<2>, g2, dim3(64), 0, ctx.stream, a); break;
            case 256: hipLaunchKernelGGL(k_fattn_combine<4>, g2, dim3(64), 0, ctx.stream, a); break;
        }
    }
    if (ctx.timing) ctx.time_end(TK_FATTN, bytes, ev);
}

}  // namespace mi355x
