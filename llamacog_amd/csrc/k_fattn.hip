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
#include "fattn.h"

#include <cmath>

namespace mi355x {

unsigned long long * g_fa_prof = nullptr;

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

// ---- long-context decode: GQA-packed split-K over 64-position chunks (f16 K/V, D <= 128) -------
// One wave per (64-position chunk, KV head, query row): the G query heads that share the KV head
// are scored together, so K and V stream from HBM once per KV head (not once per query head).
// Lane l scores position l against all G heads (its K row in registers, Q from LDS); the
// online-softmax terms are wave reductions (DPP rows + readlane); V goes to LDS with
// coalesced 16-B loads issued before the scores, and lane l accumulates dims EPL*l.. for the G
// heads, with each position's weight read from its lane as a scalar.  Partials (M, S, O) per
// (chunk, head) merge in k_fattn_combine.  f32 throughout: the CPU's f16 VKQ rounding is not
// reproduced (tests/test_gpu_model.py bounds the logit error at depth).
__device__ __forceinline__ float wave_maxf(float v) {
    v = fmaxf(v, __int_as_float(dpp<DPP_XOR1>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp<DPP_XOR2>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp<DPP_HMIRROR>(__float_as_int(v))));
    v = fmaxf(v, __int_as_float(dpp<DPP_MIRROR>(__float_as_int(v))));
    const float a0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float a1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float a2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float a3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
}
__device__ __forceinline__ float wave_sumf(float v) {
    v += __int_as_float(dpp<DPP_XOR1>(__float_as_int(v)));
    v += __int_as_float(dpp<DPP_XOR2>(__float_as_int(v)));
    v += __int_as_float(dpp<DPP_HMIRROR>(__float_as_int(v)));
    v += __int_as_float(dpp<DPP_MIRROR>(__float_as_int(v)));
    const float a0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float a1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float a2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float a3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (a0 + a1) + (a2 + a3);
}

typedef __attribute__((address_space(3))) void * fa_lds_ptr_t;

typedef _Float16 fa_h2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float fa_dot2(uint32_t a, uint32_t b, float c) {
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(fa_h2_t, a), __builtin_bit_cast(fa_h2_t, b), c, false);
}

// lanes: quad q4 = lane & 3 holds dims [D/4 q4, D/4 (q4+1)) of position 16 pass + (lane >> 2),
// four passes cover the chunk's 64 positions; Q of the G heads lives in VGPRs as f16 pairs
template <int EPL, int G>
__global__ __launch_bounds__(64) void k_fattn_dec(const fa_args a) {
    constexpr int D = 64 * EPL;
    constexpr int QW = D / 8;               // dwords (f16 pairs) of a lane's quarter row
    constexpr int PR = D * 2 / 16;          // 16-B pieces per V row
    constexpr int RPP = 64 / PR;            // V rows per 1-KiB global_load_lds piece
    const int lane = threadIdx.x, q4 = lane & 3, pl = lane >> 2;
    const int64_t chunk = blockIdx.x;
    const int64_t iq1 = blockIdx.y;
    const int64_t hk = blockIdx.z % a.Hkv, iq3 = blockIdx.z / a.Hkv;
    const int64_t pos0 = chunk * 64;
    const int nvalid = (int) min((int64_t) 64, a.n_kv - pos0);
    __shared__ __attribute__((aligned(16))) uint32_t vt[64 * D / 2];   // V tile: row-major f16 pairs

    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;
    // V rows HBM -> LDS, asynchronous (1 KiB per wave instruction), consumed after the scores
    {
        const int r_in = lane / PR, col = lane % PR;
#pragma unroll
        for (int pc = 0; pc < 64 / RPP; ++pc) {
            const int row = min(pc * RPP + r_in, nvalid - 1);
            __builtin_amdgcn_global_load_lds((const void *) (vbase + (pos0 + row) * a.nbv1 + 16 * col),
                                             (fa_lds_ptr_t) (vt + pc * 256), 16, 0, 0);
        }
    }
    // K quarter rows of the four passes (QW / 4 16-B loads each)
    uint4 kq[4][QW / 4];
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
        const int r = min(16 * ps + pl, nvalid - 1);
        const char * krow = kbase + (pos0 + r) * a.nbk1 + (D / 2) * q4;
#pragma unroll
        for (int k = 0; k < QW / 4; ++k) kq[ps][k] = ld16(krow + 16 * k);
    }
    float mraw[4];
    const char * mrow = a.mask ? a.mask + (iq1 % a.mask_ne1) * a.nbm1 : nullptr;
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
        const int r = 16 * ps + pl;
        mraw[ps] = r >= nvalid ? -INFINITY : (mrow ? h2f(*(const uint16_t *) (mrow + 2 * (pos0 + r))) : 0.0f);
    }
    // Q of the G heads, f16-rounded like the CPU's vec_dot_type, as pairs
    uint32_t qh[G][QW];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const float * qrow = (const float *) (a.q + iq1 * a.nbq1 + (hk * G + g) * a.nbq2 + iq3 * a.nbq3) + (D / 4) * q4;
#pragma unroll
        for (int i = 0; i < QW / 2; ++i) {
            const float4 f = *(const float4 *) (qrow + 4 * i);
            qh[g][2 * i] = (uint32_t) f2h(f.x) | ((uint32_t) f2h(f.y) << 16);
            qh[g][2 * i + 1] = (uint32_t) f2h(f.z) | ((uint32_t) f2h(f.w) << 16);
        }
    }
    float p[4][G];
    float M[G], S[G];
#pragma unroll
    for (int g = 0; g < G; ++g) M[g] = -INFINITY;
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float acc = 0.0f;
#pragma unroll
            for (int k = 0; k < QW / 4; ++k) {
                acc = fa_dot2(kq[ps][k].x, qh[g][4 * k], acc);
                acc = fa_dot2(kq[ps][k].y, qh[g][4 * k + 1], acc);
                acc = fa_dot2(kq[ps][k].z, qh[g][4 * k + 2], acc);
                acc = fa_dot2(kq[ps][k].w, qh[g][4 * k + 3], acc);
            }
            acc += __int_as_float(dpp<DPP_XOR1>(__float_as_int(acc)));
            acc += __int_as_float(dpp<DPP_XOR2>(__float_as_int(acc)));
            const uint32_t h = (uint32_t) (hk * G + g);
            const float slope = a.max_bias > 0.0f ? (h < a.n_head_log2 ? powf(a.m0, h + 1) : powf(a.m1, 2 * (h - a.n_head_log2) + 1)) : 1.0f;
            float sv = acc * a.scale;
            if (a.softcap != 0.0f) sv = a.softcap * tanhf(sv);
            sv = mraw[ps] == -INFINITY ? -INFINITY : sv + slope * mraw[ps];
            p[ps][g] = sv;
            M[g] = fmaxf(M[g], sv);
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        M[g] = wave_maxf(M[g]);
        float sl = 0.0f;
#pragma unroll
        for (int ps = 0; ps < 4; ++ps) {
            p[ps][g] = M[g] == -INFINITY || p[ps][g] == -INFINITY ? 0.0f : expf(p[ps][g] - M[g]);
            sl += p[ps][g];
        }
        S[g] = wave_sumf(q4 == 0 ? sl : 0.0f);   // a position's weight is in all four lanes of its quad
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the V tile has landed
    __syncthreads();
    float o[G][EPL];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < EPL; ++e) o[g][e] = 0.0f;
#pragma unroll
    for (int ps = 0; ps < 4; ++ps) {
        const int jn = min(16, nvalid - 16 * ps);
        for (int jj = 0; jj < jn; ++jj) {
            const int j = 16 * ps + jj;
            float vv[EPL];
            if constexpr (EPL == 2) {
                const uint32_t x = vt[j * (D / 2) + lane];
                vv[0] = h2f(x & 0xffff); vv[1] = h2f(x >> 16);
            } else {
                const uint32_t x = vt[j * (D / 2) + lane / 2];
                vv[0] = h2f((lane & 1) ? (x >> 16) : (x & 0xffff));
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const float pj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p[ps][g]), 4 * jj));
#pragma unroll
                for (int e = 0; e < EPL; ++e) o[g][e] = fmaf(pj, vv[e], o[g][e]);
            }
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t h = hk * G + g;
        if (a.nchunks == 1) {
            float * drow = (float *) ((char *) a.dst + iq1 * a.nb1_dst * a.H + h * a.nb1_dst + iq3 * a.nb2_dst);
            const float inv = 1.0f / S[g];
#pragma unroll
            for (int e = 0; e < EPL; ++e) drow[lane * EPL + e] = o[g][e] * inv;
        } else {
            float * pr = a.part + (((chunk * a.n_q + iq1) * a.H + h) + iq3 * a.n_q * a.H * a.nchunks) * (D + 2);
            if (lane == 0) { pr[0] = M[g]; pr[1] = S[g]; }
#pragma unroll
            for (int e = 0; e < EPL; ++e) pr[2 + lane * EPL + e] = o[g][e];
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
    if (k->type != GGML_TYPE_F16 && k->type != GGML_TYPE_Q8_0 && k->type != GGML_TYPE_Q4_0) return false;
    if (mask && mask->type != GGML_TYPE_F16) return false;
    if (mask && (mask->ne[2] != 1 || mask->ne[3] != 1)) return false;
    if (q->ne[2] % k->ne[2] != 0) return false;
    if (k->ne[3] != q->ne[3] || v->ne[3] != q->ne[3]) return false;
    float max_bias;
    memcpy(&max_bias, (const float *) op->op_params + 1, 4);
    return true;
}

bool mmv_q_supported_type(ggml_type t);

void op_flash_attn(exec_ctx & ctx, ggml_tensor * dst, const ggml_tensor * mm) {
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
    a.qmode = 0;
    a.prof = g_fa_prof;
    a.kt = nullptr;
    a.qs = nullptr; a.qd = nullptr; a.qsum = nullptr;
    if (nchunks > 1) a.part = (float *) ctx.scratch(1, sizeof(float) * nchunks * rows * (a.D + 2));

    hipEvent_t ev = nullptr;
    const double bytes = (double) (ggml_nbytes(k) + ggml_nbytes(v)) + (double) ggml_nbytes(q) + (double) ggml_nbytes(dst);
    if (ctx.timing) ctx.time_begin(TK_FATTN, bytes, ev);
    // the exact (CPU-order) kernel by default at every depth.  GGML_MI355X_FA_FAST=1 selects the
    // split-K f32 kernels; GGML_MI355X_FA_EXACT_MAX=n selects them above n cache positions only.
    // Not the default: the CPU accumulates VKQ in f16 (a rounding per position), and at depth
    // that rounding is not small — on llama3-8b-2l-q4km at 1536 positions the f32 result's
    // logits differ from the CPU's by 1.56 (max |diff| / max |logit|), far outside 1e-3
    static const int fast_env = getenv("GGML_MI355X_FA_FAST") ? atoi(getenv("GGML_MI355X_FA_FAST")) : -1;
    static const int64_t exact_max = getenv("GGML_MI355X_FA_EXACT_MAX") ? atoll(getenv("GGML_MI355X_FA_EXACT_MAX")) : INT64_MAX;
    const bool dec_ok = a.k_type == GGML_TYPE_F16 && (a.D == 64 || a.D == 128) && a.n_q <= 8 &&
                        (a.H / a.Hkv == 1 || a.H / a.Hkv == 2 || a.H / a.Hkv == 4 || a.H / a.Hkv == 8);
    // q4_0 has no split-K kernel: always the exact one
    const bool fast = a.k_type != GGML_TYPE_Q4_0 && (fast_env == 1 || (fast_env != 0 && dec_ok && a.n_kv > exact_max));
    a.cnt = nullptr;
    if (!fast && (a.k_type == GGML_TYPE_F16 || a.k_type == GGML_TYPE_Q8_0 || a.k_type == GGML_TYPE_Q4_0)) {
        // fused quantization of the output for the next MUL_MAT (decode: one row)
        q8_act act;
        if (mm && a.n_q == 1 && nq3 == 1 && mmv_q_supported_type(mm->src[0]->type) &&
            mm->src[1]->ne[0] == a.H * a.D && ggml_nrows(mm->src[1]) == 1 && ggml_is_contiguous(dst)) {
            const ggml_type wt = mm->src[0]->type;
            const bool kq = wt == GGML_TYPE_Q4_K || wt == GGML_TYPE_Q5_K || wt == GGML_TYPE_Q6_K;
            // Q8_K blocks span 256/D whole heads (D divides 256 or equals it); their
            // workgroups meet on a counter (allocated outside any capture, zeroed once)
            if (kq && !ctx.fa_cnt && !ctx.capturing) {
                MI_CHECK(hipMalloc(&ctx.fa_cnt, exec_ctx::FA_CNT * sizeof(int)));
                MI_CHECK(hipMemsetAsync(ctx.fa_cnt, 0, exec_ctx::FA_CNT * sizeof(int), ctx.stream));
            }
            if ((a.H * a.D) % (kq ? 256 : 32) == 0 && (!kq || (ctx.fa_cnt && (a.H * a.D) / 256 <= exec_ctx::FA_CNT))) {
                carve_act(act, ctx.scratch(exec_ctx::QSLOT, q8_act::bytes(a.H * a.D, 1, kq)), a.H * a.D, 1, kq);
                a.qmode = kq ? 1 : 2;
                a.qs = act.qs; a.qd = act.d; a.qsum = act.s;
                a.cnt = ctx.fa_cnt;
            }
        }
        // decode (one query row): two heads per workgroup with the scores produced under the
        // recurrence (k_fattn_dec2) where it applies, else k_fattn_exact, one workgroup per head
        if (fattn_dec2_ok(a, nq3)) {
            a.kt = ctx.kt_take("fa_dec2", (unsigned) (a.H / 2 * nq3), 512);
            launch_fattn_dec2(ctx.stream, a, nq3);
        } else {
            if (a.n_q == 1) a.kt = ctx.kt_take("fa_exact", (unsigned) (a.H * nq3), 256);
            launch_fattn_exact(ctx.stream, a, nq3);
        }
        if (a.qmode) ctx.qcache_put(mm->src[1], a.qmode == 1, act);
        if (ctx.timing) ctx.time_end(TK_FATTN, bytes, ev);
        return;
    }
    if (dec_ok) {
        // one wave per 64-position chunk and KV head
        a.chunk = 64;
        a.nchunks = (int) ceil_div(a.n_kv, 64);
        if (a.nchunks > 1) a.part = (float *) ctx.scratch(1, sizeof(float) * a.nchunks * rows * (a.D + 2));
        const int G = (int) (a.H / a.Hkv);
        dim3 gd((unsigned) a.nchunks, (unsigned) a.n_q, (unsigned) (a.Hkv * nq3));
#define DEC(E, GG) hipLaunchKernelGGL((k_fattn_dec<E, GG>), gd, dim3(64), 0, ctx.stream, a)
        if (a.D == 128) { if (G == 1) DEC(2, 1); else if (G == 2) DEC(2, 2); else if (G == 4) DEC(2, 4); else DEC(2, 8); }
        else            { if (G == 1) DEC(1, 1); else if (G == 2) DEC(1, 2); else if (G == 4) DEC(1, 4); else DEC(1, 8); }
#undef DEC
        if (a.nchunks > 1) {
            dim3 g2((unsigned) a.n_q, (unsigned) (a.H * nq3));
            if (a.D == 128) hipLaunchKernelGGL(k_fattn_combine<2>, g2, dim3(64), 0, ctx.stream, a);
            else hipLaunchKernelGGL(k_fattn_combine<1>, g2, dim3(64), 0, ctx.stream, a);
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
