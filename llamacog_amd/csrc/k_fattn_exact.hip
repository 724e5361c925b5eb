// k_fattn_exact.hip — CPU-exact flash attention over an f16 KV cache (the default; the
// split-K f32 kernel in k_fattn.hip is selected with GGML_MI355X_FA_FAST=1).
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
//     y = f16(y*ms); S = S*ms + vs (not contracted); expf taken in double and rounded.
//
// MI355X structure: one workgroup per (q row, KV head) covers the G = H/Hkv query heads of
// that head (GQA) so each K/V row is read once for all of them.  The cache is walked in
// chunks of CH positions (CH*D*2 = 64 KiB of K and of V, both staged in LDS):
//   A. the chunk's mask is read first: the last unmasked position bounds all later work;
//   0. V rows up to it are streamed HBM -> LDS with global_load_lds (dwordx4, async),
//      overlapping phases 1-2;
//   1. all scores in parallel (one position per thread, the K row held in VGPRs);
//   2. per-head prefix max (wave scans) and the (ms, vs) coefficient of every position;
//   3. the f16 recurrence — sequential over positions, parallel over the G*D elements, V
//      read from LDS.  Each thread carries E independent chains to hide the dependency.
#include "fattn.h"
#include "quant_act.h"

#include <cmath>

namespace mi355x {

// round through f16 AFTER the f32 result exists: the empty asm keeps hipcc from fusing the
// preceding fma/mul into v_fma_mixlo_f16, which rounds the exact product straight to f16
// (one rounding) where the CPU rounds to f32 and then to f16 (two roundings)
__device__ __forceinline__ float f16r(float x) {
    asm("" : "+v"(x));
    return __half2float(__float2half_rn(x));
}

// lane l of a 16-lane DPP row reads lane l + N of the same row (0 past the row end)
template <int N>
__device__ __forceinline__ float row_shl(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x100 + N, 0xf, 0xf, true));
}

// ggml_vec_dot_f16 (AVX-512) of a K row with q (f16-rounded floats), computed by the 16
// lanes of a lane group: lane l holds kv[m] = K[16m + l] and produces the lane-l partial of
// the 16 x 4 accumulator layout (elements 64i + 16j + l, accumulators j = 0..3 FMA'd over
// i), then the partials are summed in _mm512_reduce_add_ps's tree (8 / 4 / 2 / 1).  qv[m]
// is q[16m + l].  The result is valid in lane l == 0.
template <int D>
__device__ __forceinline__ float dot_f16_avx512_x16(const float (&kv)[D / 16], const float (&qv)[D / 16]) {
    float acc4[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
        float acc = __fmul_rn(kv[jj], qv[jj]);
#pragma unroll
        for (int i = 1; i < D / 64; ++i) acc = fmaf(kv[4 * i + jj], qv[4 * i + jj], acc);
        acc4[jj] = acc;
    }
    float w = __fadd_rn(__fadd_rn(acc4[0], acc4[2]), __fadd_rn(acc4[1], acc4[3]));
    w = __fadd_rn(w, row_shl<8>(w));    // t3[i] = w[8+i] + w[i]
    w = __fadd_rn(w, row_shl<4>(w));    // t6[i] = t3[4+i] + t3[i]
    w = __fadd_rn(w, row_shl<2>(w));    // (t6[0]+t6[2]), (t6[1]+t6[3])
    w = __fadd_rn(w, row_shl<1>(w));
    return w;
}

template <int D> struct fax_cfg {
    static constexpr int CH = 32768 / D < 256 ? 32768 / D : 256;   // positions per chunk (<= 64 KiB of f16 K / V)
    static constexpr int RPP = 512 / D;                  // V rows per 1 KiB global_load_lds piece
    static constexpr int PER = CH >= 256 ? CH / 256 : 1; // positions per thread in phase 2
    static constexpr int TPD = 256 / D;                  // threads sharing one output dim d
    static constexpr int U = 8;                          // phase-3 positions per register batch
};

typedef __attribute__((address_space(3))) void * lds_ptr_t;

// E = query heads per thread in phase 3 (thread owns dim d = tid % D of heads tid/D + TPD*e)
template <int D, int E>
__global__ __launch_bounds__(256) void k_fattn_exact(const fa_args a) {
    using C = fax_cfg<D>;
    constexpr int CH = C::CH, U = C::U;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t iq1 = blockIdx.x;
    const int64_t hk = blockIdx.y % a.Hkv;
    const int64_t iq3 = blockIdx.y / a.Hkv;
    const int G = (int) (a.H / a.Hkv);
    const int nel = G * D;

    __shared__ __attribute__((aligned(16))) uint16_t vl[CH * D];   // V chunk, [pos][D] f16
    __shared__ __attribute__((aligned(16))) uint16_t kl[CH * D];   // K chunk, [pos][D] f16
    __shared__ __attribute__((aligned(16))) float qt[FAX_GMAX][16][D / 16];   // q[g][16m + l] at [g][l][m]
    __shared__ float sc[FAX_GMAX][CH + U];   // scores -> vs coefficient (0 where masked)
    __shared__ float cm[FAX_GMAX][CH + U];   // ms coefficient (1 where masked)
    __shared__ float mk[CH + U];             // mask values of the chunk (-inf = skipped)
    __shared__ float red[FAX_GMAX][4];
    __shared__ float mcarry[FAX_GMAX];
    __shared__ int lastj[2];

    for (int i = tid; i < nel; i += 256) {
        const int g = i / D, d = i % D;
        const float * qrow = (const float *) (a.q + iq1 * a.nbq1 + (hk * G + g) * a.nbq2 + iq3 * a.nbq3);
        qt[g][d % 16][d / 16] = f16r(qrow[d]);
    }
    if (tid < FAX_GMAX) mcarry[tid] = -INFINITY;
    if (tid < 2) lastj[tid] = -1;

    // phase-3 state: dim d of heads gh[e]
    const int d = tid % D;
    float y[E], S[E];
    int gh[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        y[e] = 0.0f; S[e] = 0.0f;
        gh[e] = min(tid / D + C::TPD * e, G - 1);
    }

    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;
    const char * mrow = a.mask ? a.mask + (iq1 % a.mask_ne1) * a.nbm1 : nullptr;
    __syncthreads();

    int par = 0;
    for (int64_t c0 = 0; c0 < a.n_kv; c0 += CH, par ^= 1) {
        const int nch = (int) min((int64_t) CH, a.n_kv - c0);
        // ---- phase A: mask of the chunk; the last unmasked position bounds all later work --
        for (int j = tid; j < CH + U; j += 256) {
            const float mv = j < nch ? (mrow ? h2f(*(const uint16_t *) (mrow + 2 * (c0 + j))) : 0.0f) : -INFINITY;
            mk[j] = mv;
            if (mv != -INFINITY) atomicMax(&lastj[par], j);
        }
        __syncthreads();
        if (tid == 0) lastj[par ^ 1] = -1;   // the next chunk's slot (last read before this chunk)
        const int nrun = lastj[par] + 1;      // positions past the last unmasked one are skipped
        // ---- phase 0: K rows [0, nrun) HBM -> LDS (all in flight at once, then waited on),
        // then V rows [0, nrun) (async; waited on before phase 3, overlapping phases 1-2) ----
        {
            const int r_in = lane / (D / 8), col = lane % (D / 8);
            for (int p = wave; p * C::RPP < nrun; p += 4) {
                const int row = min(p * C::RPP + r_in, nrun - 1);
                const char * src = kbase + (c0 + row) * a.nbk1 + col * 16;
                __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) (kl + p * 512), 16, 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            for (int p = wave; p * C::RPP < nrun; p += 4) {
                const int row = min(p * C::RPP + r_in, nrun - 1);
                const char * src = vbase + (c0 + row) * a.nbv1 + col * 16;
                __builtin_amdgcn_global_load_lds((const void *) src, (lds_ptr_t) (vl + p * 512), 16, 0, 0);
            }
        }
        // ---- phase 1: scores, 16 lanes per position ----------------------------------------
        // lane l of the 16 computes the AVX-512 lane-l partial of ggml_vec_dot_f16
        // (accumulators j = 0..3 over i: elements 64i + 16j + l), then the 16 partials are
        // summed in _mm512_reduce_add_ps's tree (8 / 4 / 2 / 1) across the lanes
        {
            const int l = tid & 15;
            for (int j = tid >> 4; j < nrun; j += 16) {
                const float mv = mk[j];           // uniform over the 16 lanes of a position
                if (mv == -INFINITY) continue;
                const uint16_t * krow = kl + j * D;
                float kv[D / 16];
#pragma unroll
                for (int m = 0; m < D / 16; ++m) kv[m] = h2f(krow[16 * m + l]);
                for (int g = 0; g < G; ++g) {
                    float qv[D / 16];
#pragma unroll
                    for (int m = 0; m < D / 16; ++m) qv[m] = qt[g][l][m];
                    const float w = dot_f16_avx512_x16<D>(kv, qv);
                    if (l == 0) {
                        float s = __fmul_rn(w, a.scale);
                        if (a.softcap != 0.0f) s = __fmul_rn(a.softcap, tanhf(s));
                        const uint32_t hh = (uint32_t) (hk * G + g);
                        const float slope = a.max_bias > 0.0f
                            ? (float) (hh < a.n_head_log2 ? pow((double) a.m0, (double) (hh + 1))
                                                          : pow((double) a.m1, (double) (2 * (hh - a.n_head_log2) + 1))) : 1.0f;
                        sc[g][j] = __fadd_rn(s, __fmul_rn(slope, mv));
                    }
                }
            }
        }
        __syncthreads();
        // ---- phase 2: prefix max per head and the (ms, vs) coefficients --------------------
        // masked positions (and the padding up to a multiple of U) get ms = 1, vs = 0
        if (nrun > 0) {
            for (int g = 0; g < G; ++g) {
                float lm = -INFINITY;
#pragma unroll
                for (int p = 0; p < C::PER; ++p) {
                    const int j = tid * C::PER + p;
                    if (j < nrun && mk[j] != -INFINITY) lm = fmaxf(lm, sc[g][j]);
                }
                float sm = lm;   // inclusive max-scan over the 256 threads
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
                float M = prev;
#pragma unroll
                for (int p = 0; p < C::PER; ++p) {
                    const int j = tid * C::PER + p;
                    if (j >= nrun) break;
                    if (mk[j] == -INFINITY) { cm[g][j] = 1.0f; sc[g][j] = 0.0f; continue; }
                    const float s = sc[g][j];
                    if (s > M) {
                        cm[g][j] = M == -INFINITY ? 0.0f : expf_cr(M - s);   // ms, applied before the add
                        sc[g][j] = 1.0f;                                       // vs
                        M = s;
                    } else {
                        cm[g][j] = 1.0f;
                        sc[g][j] = expf_cr(s - M);
                    }
                }
                if (tid < U) { cm[g][nrun + tid] = 1.0f; sc[g][nrun + tid] = 0.0f; }
                __syncthreads();
                if (tid == 255) mcarry[g] = fmaxf(mcarry[g], fmaxf(fmaxf(red[g][0], red[g][1]), fmaxf(red[g][2], red[g][3])));
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // ---- phase 3: sequential f16 recurrence (V from LDS) --------------------------------
        // y = f16(y*ms) is the identity for ms == 1 (y is f16-exact), so it is applied at every
        // position; masked / padded positions keep the state by a select (their V rows are
        // not loaded, and -0 must survive)
        if (tid < min(G, C::TPD) * D) {
            for (int j = 0; j < nrun; j += U) {
                uint16_t vv[U];
                bool skip[U];
                float msv[U][E], vsv[U][E];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    skip[u] = mk[j + u] == -INFINITY;
                    vv[u] = vl[min(j + u, CH - 1) * D + d];
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        msv[u][e] = cm[gh[e]][j + u];
                        vsv[u][e] = sc[gh[e]][j + u];
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const float v = skip[u] ? 0.0f : h2f(vv[u]);
#pragma unroll
                    for (int e = 0; e < E; ++e) {
                        const float ms = msv[u][e];
                        const float vs = vsv[u][e];
                        const float yn = f16r(fmaf(v, vs, f16r(__fmul_rn(y[e], ms))));
                        y[e] = skip[u] ? y[e] : yn;
                        S[e] = __fadd_rn(__fmul_rn(S[e], ms), vs);   // identity where skipped; not contracted on the CPU
                    }
                }
            }
        }
        __syncthreads();
    }
    float * ol = (float *) vl;   // output staging for the fused quantization (V chunk is dead)
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int g = tid / D + C::TPD * e;
        if (g >= G) break;
        const int64_t h = hk * G + g;
        float * drow = (float *) ((char *) a.dst + iq1 * a.nb1_dst * a.H + h * a.nb1_dst + iq3 * a.nb2_dst);
        const float o = __fmul_rn(y[e], 1.0f / S[e]);
        drow[d] = o;
        if (a.qmode) ol[g * D + d] = o;
    }
    if (a.qmode) {
        // the G*D outputs of this KV head are a contiguous, 256-aligned slice of the flat
        // [H*D] row the following MUL_MAT quantizes (checked on the host)
        __syncthreads();
        const int64_t K = a.H * D;
        const int64_t c00 = hk * G * D;
        for (int b = wave; b < nel / 256; b += 4) {
            const float4 v4 = *(const float4 *) (ol + 256 * b + 4 * lane);
            const float q[4] = {v4.x, v4.y, v4.z, v4.w};
            const int64_t c0 = c00 + 256 * b;
            if (a.qmode == 1) {
                q8K_wave(q, lane, a.qs + iq1 * K + c0, a.qsum + iq1 * (K / 16) + c0 / 16, a.qd + iq1 * (K / 256) + c0 / 256);
            } else {
                q8_0_wave(q, lane, true, a.qs + iq1 * K + c0, a.qd + iq1 * (K / 32) + c0 / 32, a.qsum + iq1 * (K / 32) + c0 / 32);
            }
        }
    }
}

template <int D>
static void launch_d(hipStream_t st, const fa_args & a, dim3 grid) {
    constexpr int TPD = 256 / D;
    const int64_t per = ceil_div(a.H / a.Hkv, TPD);   // heads per thread
    if (per <= 1)      hipLaunchKernelGGL((k_fattn_exact<D, 1>), grid, dim3(256), 0, st, a);
    else if (per <= 2) hipLaunchKernelGGL((k_fattn_exact<D, 2>), grid, dim3(256), 0, st, a);
    else if (per <= 4) hipLaunchKernelGGL((k_fattn_exact<D, 4>), grid, dim3(256), 0, st, a);
    else               hipLaunchKernelGGL((k_fattn_exact<D, (D >= 256 ? 8 : 4)>), grid, dim3(256), 0, st, a);
}

void launch_fattn_exact(hipStream_t st, const fa_args & a, int64_t nq3) {
    GGML_ASSERT(a.H % a.Hkv == 0 && a.H / a.Hkv <= FAX_GMAX);
    const dim3 grid((unsigned) a.n_q, (unsigned) (a.Hkv * nq3));
    switch (a.D) {
        case 64:  launch_d<64>(st, a, grid); break;
        case 128: launch_d<128>(st, a, grid); break;
        case 256: launch_d<256>(st, a, grid); break;
        default: GGML_ABORT("mi355x: FA head size %d", (int) a.D);
    }
}

// test hook: the K·Q scores exactly as phase 1 of k_fattn_exact computes them
// (q [D] f32 is f16-rounded first), 16 lanes per cache row; D = 128
__global__ void k_fattn_scores_d128(const float * q, const uint16_t * k, int64_t n, float * s) {
    const int l = threadIdx.x & 15;
    const int64_t j = ((int64_t) blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    float kv[8], qv[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        kv[m] = j < n ? h2f(k[j * 128 + 16 * m + l]) : 0.0f;
        qv[m] = f16r(q[16 * m + l]);
    }
    const float w = dot_f16_avx512_x16<128>(kv, qv);
    if (l == 0 && j < n) s[j] = w;
}

void fattn_scores_d128(hipStream_t st, const float * q, const uint16_t * k, int64_t n, float * s) {
    hipLaunchKernelGGL(k_fattn_scores_d128, dim3((unsigned) ceil_div(n * 16, 256)), dim3(256), 0, st, q, k, n, s);
}

}  // namespace mi355x
