// fa_dsh4.h — the short-context decode attention (D = 128, f16 cache, at most 256 positions) as a
// four-wave workgroup body, so it can ride in the Q/K/V projection's own launch (k_gemv.hip
// k_gemv_os_fa): its workgroups load the mask and the cached K / V rows while the projection's
// workgroups compute the token's Q, K and V, wait on a per-head-pair counter the projection's
// workgroups add their stored rows to, and then need only q and the token's own K / V row.
//
// Arithmetic as k_fattn_dsh / k_fattn_dec2 (ops.cpp:7015-7232: ggml_vec_dot_f16's AVX-512 order,
// the prefix-max (ms, vs) coefficients, the f16 VKQ recurrence with the CPU's two roundings):
//   * waves 0 and 1 are the chains, head 2 hp + wave, dims 2 lane and 2 lane + 1 (two independent
//     f16 chains per lane, V read as one dword a position); they sit alone on SIMDs 0 and 1;
//   * waves 2 and 3 are producers: producer p owns the 16-position blocks p, p + 2, ...; it loads
//     the whole mask, then the K rows and (LDS-DMA) V rows of its blocks up to the last live
//     position, then both heads' q (packed f16); per block it forms both heads' scores from one K
//     load, the block's running max (a 16-lane DPP scan, the maximum before the block handed over
//     by the other producer through LDS), the (ms, vs) coefficients with libm expf and a
//     "general" flag per 8-position batch, and marks the block ready;
//   * the two heads' 256 outputs (one Q8_K block) are quantized for the output projection.
#pragma once

#include "fattn.h"
#include "fa_util.h"
#include "libm_exact.h"
#include "quant_act.h"

namespace mi355x {

constexpr int D4_MAXKV = 256, D4_U = 8, D4_B = 16, D4_NB = D4_MAXKV / D4_B, D4_PAD = 2 * D4_U;
constexpr int D4_OWN = D4_NB / 2;          // blocks per producer
constexpr int D4_SLOTS = 5;                // K blocks a producer holds in registers at once (the rest
                                           // reuse a slot once its block is scored)
constexpr int D4_VROWS = D4_MAXKV;         // V rows staged (the chains read no row past the last batch;
                                           // two workgroups of the two-type launch share a CU with it)

struct ds4_smem {
    float sc[2][D4_MAXKV + D4_PAD];        // [head] vs (0 where dead)
    float cm[2][D4_MAXKV + D4_PAD];        // ms (1 where dead)
    float mk[2][D4_MAXKV + D4_PAD];        // 0 live, -inf dead
    float sr[2][D4_OWN][2][D4_B];          // [producer][its block][head] raw scores (-inf dead)
    float carry[2][D4_NB];                 // [head] running max through block b
    int cflag[D4_NB];                      // block b's carry is in
    int ready[D4_NB];                      // block b's coefficients, flags and V rows are in
    uint8_t bfl[2][2 * D4_NB + 8];         // [head][batch] general step
    uint64_t etab[2][32];                  // expf's table, a copy per producer
    float ol[2 * 128];
    uint16_t vl[D4_VROWS * 128];           // [position][dim]
};

// s_waitcnt vmcnt(0) that the compiler knows about (it then puts no wait of its own behind it for
// the loads before it)
__device__ __forceinline__ void fa4_vm_drain() { __builtin_amdgcn_s_waitcnt(0x0f70); }

template <bool FUSED>
__device__ __forceinline__ void fa_dsh4_body(const fa_args & a, int64_t hp, int64_t iq3, const fa_fuse & fz, ds4_smem & sm) {
    constexpr int D = 128, NM = D / 16, U = D4_U, B = D4_B;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool pr = FUSED && fz.dbg && blockIdx.x == 0 && lane == 0;
    const unsigned long long t0 = pr ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long tm[6] = {0, 0, 0, 0, 0, 0};
    auto mark = [&](int i) { if (pr) tm[i] = __builtin_amdgcn_s_memtime() - t0; };
    const int64_t hk = (2 * hp) / (a.H / a.Hkv);
    const int n_kv = (int) a.n_kv;
    const char * kbase = a.k + hk * a.nbk2 + iq3 * a.nbk3;
    const char * vbase = a.v + hk * a.nbv2 + iq3 * a.nbv3;
    // every wave reads the whole mask (4 positions a lane): nrun = the last live position + 1
    uint32_t mk4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) mk4[k] = ds_mask_ld(a.mask, 64 * k + lane, n_kv);
    if (tid < D4_NB) { sm.cflag[tid] = 0; sm.ready[tid] = 0; }
    auto nrun_of = [&]() {
        int last = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned long long bl = __ballot((mk4[k] & 0xffff) != 0xfc00);
            if (bl) last = 64 * k + 63 - __clzll(bl);
        }
        return last + 1;
    };

    if (wave >= 2) {
        // ================= producers =================
        const int pw = wave - 2, qd = lane & 3;
        const uint64_t etv = lx_exp2f_tab[lane & 31];
        // the mask value of each owned block's position B b + lane / 4
        uint32_t mkb[D4_OWN];
#pragma unroll
        for (int i = 0; i < D4_OWN; ++i) mkb[i] = ds_mask_ld(a.mask, B * (pw + 2 * i) + (lane >> 2), n_kv);
        fa4_vm_drain();
        asm volatile("" : "+v"(mk4[0]), "+v"(mk4[1]), "+v"(mk4[2]), "+v"(mk4[3]));
#pragma unroll
        for (int i = 0; i < D4_OWN; ++i) asm volatile("" : "+v"(mkb[i]));
        if (lane < 32) sm.etab[pw][lane] = etv;
        const int nrun = nrun_of(), nblk = (nrun + B - 1) / B;
        const int nown = nblk > pw ? (nblk - pw + 1) / 2 : 0;
        // the K rows (4 lanes a position) of the first D4_SLOTS owned live blocks, the V rows (LDS-DMA)
        // of all of them
        uint2 kh[D4_SLOTS][NM];
        const int r_in = lane >> 4, col = lane & 15;
        auto krow_of = [&](int i) {
            const int j = min(B * (pw + 2 * i) + (lane >> 2), n_kv - 1);
            return kbase + (int64_t) j * a.nbk1 + 8 * qd;
        };
#pragma unroll
        for (int i = 0; i < D4_OWN; ++i) {
            if (i < nown) {
                const int b = pw + 2 * i;
                if (i < D4_SLOTS) {
                    const char * krow = krow_of(i);
#pragma unroll
                    for (int m = 0; m < NM; ++m) kh[i][m] = fa_ld8(krow + 32 * m);
                }
#pragma unroll
                for (int r = 0; r < B / 4; ++r) {
                    const int jv = min(B * b + 4 * r + r_in, n_kv - 1);
                    lds_dma16(vbase + (int64_t) jv * a.nbv1 + 16 * col, sm.vl + 128 * (B * b + 4 * r));
                }
            }
        }
        __syncthreads();   // the flags' zeros and the expf table (all waves)
        mark(0);
        int jfk = -1, jfv = -1;   // the token's own K / V row (stored by this launch), if it is in the cache view
        if constexpr (FUSED) {
            // every projection row of this head pair is stored (write-through) and counted
            if (lane == 0) {
                int guard = 0;
                // (a returning atomic reads the counter where the adds land; a load poll may be served
                // from this XCD's L2 copy for microseconds)
                while (__hip_atomic_fetch_add(fz.cnt + hp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < fz.expect) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++guard > (1 << 22)) break;   // a miscount shows as wrong output, never as a hang
                }
            }
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
            mark(1);
            const char * kd = fz.kslot ? (const char *) *fz.kslot : nullptr;
            const char * vd = fz.vslot ? (const char *) *fz.vslot : nullptr;
            if (kd) {
                const int64_t o = kd - a.k;
                if (o >= 0 && o % a.nbk1 == 0 && o / a.nbk1 < n_kv) jfk = (int) (o / a.nbk1);
            }
            if (vd) {
                const int64_t o = vd - a.v;
                if (o >= 0 && o % a.nbv1 == 0 && o / a.nbv1 < n_kv) jfv = (int) (o / a.nbv1);
            }
            jfk = __builtin_amdgcn_readfirstlane(jfk);
            jfv = __builtin_amdgcn_readfirstlane(jfv);
            // no usable destination: every K / V row is re-read write-through below
        }
        // q of both heads (f16-rounded, packed pairs); FUSED: written by this launch, read past L2
        uint32_t qh[2][NM][2];
        {
            float4 q4[2][NM];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float * qrow = (const float *) (a.q + (2 * hp + h) * a.nbq2 + iq3 * a.nbq3);
#pragma unroll
                for (int m = 0; m < NM; ++m) q4[h][m] = fa_ld16<FUSED>(qrow + 16 * m + 4 * qd);
            }
            // the token's own K row (or all K rows without a usable destination), read past L2
            if (FUSED) {
#pragma unroll
                for (int i = 0; i < D4_SLOTS; ++i) {
                    if (i < nown) {
                        const int j = min(B * (pw + 2 * i) + (lane >> 2), n_kv - 1);
                        if (jfk < 0 || j == jfk) {
                            const char * krow = krow_of(i);
#pragma unroll
                            for (int m = 0; m < NM; ++m) kh[i][m] = fa_ld8<true>(krow + 32 * m);
                        }
                    }
                }
            }
            fa4_vm_drain();   // q, the K rows and this wave's V DMAs
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int m = 0; m < NM; ++m) {
                    asm volatile("" : "+v"(q4[h][m].x), "+v"(q4[h][m].y), "+v"(q4[h][m].z), "+v"(q4[h][m].w));
                    qh[h][m][0] = (uint32_t) f2h(q4[h][m].x) | ((uint32_t) f2h(q4[h][m].y) << 16);
                    qh[h][m][1] = (uint32_t) f2h(q4[h][m].z) | ((uint32_t) f2h(q4[h][m].w) << 16);
                }
#pragma unroll
            for (int i = 0; i < D4_SLOTS; ++i)
#pragma unroll
                for (int m = 0; m < NM; ++m) asm volatile("" : "+v"(kh[i][m].x), "+v"(kh[i][m].y));
        }
        if (FUSED) {
            // the token's own V row (or every V row of the owned blocks) over the staged copy
#pragma unroll
            for (int i = 0; i < D4_OWN; ++i) {
                if (i < nown) {
                    const int b = pw + 2 * i;
                    for (int r = 0; r < B; ++r) {
                        const int j = B * b + r;
                        if (j >= n_kv || (jfv >= 0 && j != jfv)) continue;
                        *(uint32_t *) (sm.vl + 128 * j + 2 * lane) = fa_ld4<true>(vbase + (int64_t) j * a.nbv1 + 4 * lane);
                    }
                }
            }
        }
        mark(2);
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
        const uint64_t * etab = sm.etab[pw];
        // block i's scores from slot i % D4_SLOTS; a block past the slots has its K loaded into the
        // slot of the block D4_SLOTS before it right after that block is scored (write-through reads
        // in the fused launch: any of its rows may be the token's own)
        auto scores = [&](int i) {
            const int b = pw + 2 * i;
            const int j = B * b + (lane >> 2);
            const float mv = h2f((uint16_t) mkb[i]);
            const bool live = mv != -INFINITY && j < nrun;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float w = dot_f16_mix_d128_h(kh[i % D4_SLOTS], qh[h], nz);
                if (qd == 0) {
                    float sv = __fmul_rn(w, a.scale);
                    if (a.softcap != 0.0f) sv = __fmul_rn(a.softcap, tanhf(sv));
                    sm.sr[pw][i][h][lane >> 2] = live ? __fadd_rn(sv, __fmul_rn(slope[h], mv)) : -INFINITY;
                }
            }
            if (i + D4_SLOTS < nown) {
                const char * krow = krow_of(i + D4_SLOTS);
#pragma unroll
                for (int m = 0; m < NM; ++m) kh[i % D4_SLOTS][m] = fa_ld8<FUSED>(krow + 32 * m);
            }
        };
        auto coef = [&](int i) {
            const int b = pw + 2 * i;
            dc_wave_lds_order();
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
#pragma unroll
            for (int i = 1; i < D4_OWN; ++i)
                if (i < nown) scores(i);
#pragma unroll
            for (int i = 1; i < D4_OWN; ++i)
                if (i < nown) coef(i);
        }
        mark(3);
        if (pr && wave == 2) printf("[fa4] hp0 jfk %d jfv %d n_kv %d nrun %d nown %d | cycles: loads+sync %llu wait %llu q/K/V %llu coef %llu\n",
                                    jfk, jfv, n_kv, nrun, nown, tm[0], tm[1], tm[2], tm[3]);
    } else {
        // ================= chains: head 2 hp + wave, dims 2 lane, 2 lane + 1 =================
        const int ch = wave;
        fa4_vm_drain();
        asm volatile("" : "+v"(mk4[0]), "+v"(mk4[1]), "+v"(mk4[2]), "+v"(mk4[3]));
        const int nrun = nrun_of(), nb = (nrun + U - 1) / U;
        __syncthreads();   // the flags' zeros
        uint32_t y0 = 0, y1 = 0;
        float S = 0.0f;
        const uint32_t * vrow = (const uint32_t *) sm.vl + lane;
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
            for (int u = 0; u < U; ++u) vv[u] = vrow[(j + u) * (D / 2)];
            ld4(scp + j, vs);
        };
        auto run = [&](const uint32_t (&vv)[U], const float (&vs)[U]) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                y0 = f16_mad(vv[u], vs[u], y0);
                y1 = f16_mad_hi(vv[u], vs[u], y1);
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
                float t0f = __fmul_rn(h2f((uint16_t) y0), ms[u]);
                float t1f = __fmul_rn(h2f((uint16_t) y1), ms[u]);
                asm("" : "+v"(t0f), "+v"(t1f));   // two roundings, as f16r
                const uint32_t ys0 = upd ? (uint32_t) f2h(t0f) : y0;
                const uint32_t ys1 = upd ? (uint32_t) f2h(t1f) : y1;
                const float Ss = upd ? __fmul_rn(S, ms[u]) : S;
                const uint32_t yn0 = f16_mad(vv[u], vs[u], ys0);
                const uint32_t yn1 = f16_mad_hi(vv[u], vs[u], ys1);
                const float Sn = __fadd_rn(Ss, vs[u]);
                y0 = live ? yn0 : y0;
                y1 = live ? yn1 : y1;
                S = live ? Sn : S;
            }
        };
        // a block's ready flag and batch flags are read one block ahead
        int rdy = 0, f0 = 0, f1 = 0;
        if (nb > 0) {
            ds_wait_flag(&sm.ready[0]);
            f0 = sm.bfl[ch][0];
            f1 = sm.bfl[ch][1];
        }
        for (int b = 0; 2 * b < nb; ++b) {
            const int g0 = f0, g1 = f1;
            const bool two = 2 * b + 1 < nb, more = 2 * b + 2 < nb;
            if (more) {
                rdy = lds_ld(&sm.ready[b + 1]);
                asm volatile("" ::: "memory");
                f0 = sm.bfl[ch][2 * b + 2];
                f1 = sm.bfl[ch][2 * b + 3];
            }
            if (!g0 && !(two && g1)) {
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
            if (more && !rdy) {
                ds_wait_flag(&sm.ready[b + 1]);
                f0 = sm.bfl[ch][2 * b + 2];
                f1 = sm.bfl[ch][2 * b + 3];
            }
        }
        mark(4);
        if (pr && wave == 0) printf("[fa4] hp0 chain end %llu\n", tm[4]);
        const int64_t h = 2 * hp + ch;
        const float rS = 1.0f / S;
        const float o0 = __fmul_rn(h2f((uint16_t) y0), rS), o1 = __fmul_rn(h2f((uint16_t) y1), rS);
        float * drow = (float *) ((char *) a.dst + h * a.nb1_dst + iq3 * a.nb2_dst);
        *(float2 *) (drow + 2 * lane) = make_float2(o0, o1);
        *(float2 *) (sm.ol + ch * D + 2 * lane) = make_float2(o0, o1);
    }
    // ---- the two heads' 256 outputs: quantized here for the following projection ----
    __syncthreads();
    if (a.qmode && wave == 0) {
        float q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = sm.ol[4 * lane + k];
        const int64_t c0 = 256 * hp;
        if (a.qmode == 1) q8K_wave(q, lane, a.qs + c0, a.qsum + c0 / 16, a.qd + c0 / 256);
        else q8_0_wave(q, lane, true, a.qs + c0, a.qd + c0 / 32, a.qsum + c0 / 32);
    }
    // the counter is this workgroup's alone and every projection row has arrived: reset for the
    // next launch (a graph replay)
    if (FUSED && tid == 0) __hip_atomic_store(fz.cnt + hp, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace mi355x
