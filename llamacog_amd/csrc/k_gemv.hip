// k_gemv.hip — decode mat-vec (one activation column) over quantized weights, with grouped
// launches and fused epilogues, in the CPU backend's exact float order (qtypes.h).
//
// Layout, built for HBM latency on MI355X:
//   * a persistent grid of ~2 workgroups per CU walks the row groups; each wave owns R
//     consecutive weight rows, keeps the activation slice of its task in VGPRs and walks the R
//     rows, fetching the NEXT group's weight slices into registers before it works on the
//     current one, so dequantization overlaps the HBM stream;
//   * for long rows WPR waves split a row's K range; WPR depends on K only;
//   * every lane forms its task's exact integers; the block records (integers + scale
//     products, qtypes.h) go to LDS, and LPR lanes per row run the CPU's fp32 chain over them
//     (the "walker"): the result is bit-identical to the reference CPU backend;
//   * one launch covers up to three matrices that share src1 (Q/K/V, gate/up), and two weight
//     types in one launch (k_gemv_pipe2: Q4_K Q/K beside a Q6_K V);
//   * fused epilogues: the NORM-mode RoPE of Q/K (rows 2i, 2i+1 lie in one group), f16
//     KV-cache stores (destinations from the dynamic-pointer table, exec_ctx::dyn_slot), and
//     optionally the SiLU of a gate projection;
//   * tail (SwiGLU): a gate/up launch also forms silu(gate) * up and its Q8_K / Q8_0 blocks for
//     the down projection: per Q8_K block, the last of the block's row groups to finish (a
//     device-scope arrival counter; the projection rows travel write-through, sc1) runs it.
//     Bits as the stand-alone k_mul_quant (k_fused.hip), one launch fewer;
//   * residual producer / norm prologue (a mat-vec followed by ADD -> RMS_NORM -> [MUL] ->
//     mat-vec): the producer stores x = v + res instead of v and adds its rows' sum of
//     (double)(x*x) to one of 64 words; every workgroup of the consumer forms the CPU's
//     mean from them (quant_act.h rms_mean_decided), y = x * scale * w, and quantizes it into
//     LDS as its activation.  The RMS_NORM launch disappears; nothing waits on a last arriver.
#include "ops.h"
#include <hip/hip_ext.h>
#include <mutex>
#include "rope.h"
#include "qtypes.h"
#include "quant_act.h"

namespace mi355x {

constexpr int GEMV_MAXMAT = 3;
constexpr int GEMV_ROPE_MAXPAIRS = 256;   // fused rope: n_dims <= 512
constexpr int GEMV_MAXG = 16;             // row groups per workgroup when epilogues park row sums

struct gemv_args {
    const uint8_t * W[GEMV_MAXMAT]; int64_t nb01[GEMV_MAXMAT]; int64_t M[GEMV_MAXMAT];
    float * dst[GEMV_MAXMAT];
    float * silu[GEMV_MAXMAT];            // SiLU epilogue output (nullable)
    uint16_t * const * f16out[GEMV_MAXMAT];   // fused f32->f16 CPY (KV-cache store) slot (nullable)
    int64_t blk0[GEMV_MAXMAT + 1];        // first row group of each matrix
    gemv_act A;
    int ntasks;
    // fused ROPE (NORM mode, one token) of the projection output: adjacent rows (2i, 2i+1)
    // of a head are rotated in the epilogue; optional f16 copy of the result (KV-cache store)
    float * rope_out[GEMV_MAXMAT];
    uint16_t * const * rope_f16[GEMV_MAXMAT];
    rope_params rp;
    const int32_t * rope_pos; const float * rope_ff; int64_t rope_d;
    int need_pairs;
    const float2 * rtab_g;                // the graph's cos/sin table of the position (rope_table)
    // SwiGLU tail (see above); kind 0 = none, 2 = silu(dst[gate]) * dst[up]
    struct tail_t {
        int kind; int64_t n;
        int gate, up; float * silu_out; float * mul_out;
        int qmode; int8_t * qs; float * qd; int16_t * qsum;
        int * cnt;
    } tl;
    // residual producer (MODE 0, one matrix): x = v + rres[row] goes to rxsum[row] (v itself is
    // dead), sum of (double)(x*x) to rsum[RSUM_STRIDE * (workgroup % RSUM_SHARDS)]
    const float * rres; float * rxsum; double * rsum;
    // norm prologue: the activation is quant(RMS_NORM(x) [* w]) formed in LDS at byte lds_off
    struct pro_t {
        const float * x; const float * w; const double * sum; float eps; int64_t n; int qmode; uint32_t lds_off;
    } pro;
    unsigned long long * kt;              // in-graph kernel timeline region (nullable)
    uint32_t wl_off;                      // one-shot kernel: LDS byte offset of the weight slices
    unsigned long long * eprof;           // engine phase counters (microbenchmark only; nullable)
    // one-shot body in a chained launch (k_gemv_ffn): after issuing its weight DMA the workgroup
    // waits until the FFN_SHARDS counters at dep sum to dep_n (its activation is complete)
    const int * dep; int dep_n;
};
constexpr int FFN_SHARDS = 8, FFN_SHARD_STRIDE = 32;   // ints: one 128-B line per shard

// the producer's partial sums: no-return f64 atomics serialize per 128-B line at the memory
// side (MI355X_MICROARCH.md dequeue row), so 64 shards, one line each, keep each line's count
// of adds (workgroups / 64) small
constexpr int RSUM_SHARDS = 64, RSUM_STRIDE = 16;   // doubles

// ---- SwiGLU tail (the last workgroup of each Q8_K block) -------------------------------------------
__device__ __forceinline__ float ld_wt(const float * p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float4 ld_wt4(const float * p) { return make_float4(ld_wt(p), ld_wt(p + 1), ld_wt(p + 2), ld_wt(p + 3)); }

// tail 2, one wave per finished Q8_K block: m = silu(gate) * up (ggml_vec_silu_f32's AVX-512
// ggml_v_silu on the 16-element chunks, libm expf on the tail; vec.cpp:233), quantized
// (WT: the quantized block write-through, read in the same launch)
template <bool WT = false>
__device__ __forceinline__ void tail_swiglu(const gemv_args & p, int blk, int lane) {
    const auto & t = p.tl;
    const int64_t e = 256 * (int64_t) blk + 4 * lane;
    const float4 g = ld_wt4(p.dst[t.gate] + e), u = ld_wt4(p.dst[t.up] + e);
    const int64_t nvec = (t.n / 16) * 16;
    float s[4] = {g.x, g.y, g.z, g.w};
    const float uu[4] = {u.x, u.y, u.z, u.w};
    float m[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        s[c] = e + c < nvec ? s[c] / (1.0f + v_expf_avx512(-s[c])) : s[c] / (1.0f + expf_cr(-s[c]));
        m[c] = __fmul_rn(s[c], uu[c]);
    }
    if (t.silu_out) *(float4 *) (t.silu_out + e) = make_float4(s[0], s[1], s[2], s[3]);
    if (t.mul_out) *(float4 *) (t.mul_out + e) = make_float4(m[0], m[1], m[2], m[3]);
    const int64_t c0 = 256 * (int64_t) blk;
    if (t.qmode == 1) q8K_wave<WT>(m, lane, t.qs + c0, t.qsum + c0 / 16, t.qd + c0 / 256);
    else if (t.qmode == 2) q8_0_wave(m, lane, true, t.qs + c0, t.qd + c0 / 32, t.qsum + c0 / 32);
}

// arrival: every workgroup drains its write-through stores, then one lane reports each of its
// row groups on its Q8_K block's counter (MI355X_MICROARCH.md, inter-workgroup visibility, first
// hand-off row); the report that completes a block's count makes this workgroup run that block.
// Returning atomics on one word serialize at the memory side (~88 per us, MI355X_MICROARCH.md
// dequeue row) and words of one line share that limit, so each counter owns a 4-KiB line.
// Ordering: this is the first row of MI355X_MICROARCH.md's measured hand-off table (sc1 stores,
// every storing wave's vmcnt(0) wait, a workgroup barrier, then one lane's agent-scope atomic add
// per counter; the last adder — told by the returned value — and only after that return, loads
// the bytes with sc1 loads after a workgroup barrier).  An acq_rel add would instead put an L2
// write-back + invalidate (≈1.7–3.5 us per workgroup, the fence rows there) into every launch;
// the form kept here is the measured-valid one the guide prescribes for write-through payloads.
constexpr int TAIL_STRIDE = 1024;   // ints between counter words
__device__ __forceinline__ void gemv_tail(const gemv_args & p, int kg, int64_t wg0, int64_t nwg, int rpg) {
    const auto & t = p.tl;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int tlist[GEMV_MAXG];
    // lane k of wave 0 reports row group k: the workgroup's returning atomics are in flight
    // together rather than one round trip after another
    if (threadIdx.x < GEMV_MAXG) {
        int done = -1;
        if ((int) threadIdx.x < kg) {
            const int per = 2 * (256 / rpg);   // row groups of a Q8_K block: gate and up
            const int64_t g = wg0 + (int64_t) threadIdx.x * nwg;
            const int mi = g >= p.blk0[1] ? 1 : 0;
            const int blk = (int) ((g - p.blk0[mi]) * rpg / 256);
            int * c = t.cnt + blk * TAIL_STRIDE;
            if (__hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == per - 1) {
                done = blk;
                __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        tlist[threadIdx.x] = done;
    }
    __syncthreads();
    for (int i = threadIdx.x >> 6; i < kg; i += 4) {
        if (tlist[i] >= 0) tail_swiglu(p, tlist[i], threadIdx.x & 63);   // wave-uniform
    }
}

// ---- norm prologue ---------------------------------------------------------------------------------
// The consumer's activation, formed by every workgroup: mean from the producer's 64 partial
// sums (summed in a fixed order; decided, else the CPU's own loop over x), y = x * scale (* w),
// quantized (Q8_K: q8K_row16, wave w lane l owns elements 16 (l & 15) .. +15 of block
// 16 pass + 4 w + (l >> 4); Q8_0: q8_0_row16 over the same elements) into buf in the gemv_act layout.
__device__ __forceinline__ void gemv_prologue(const gemv_args & p, uint8_t * buf, gemv_act & A) {
    const auto & r = p.pro;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int NB = (int) (r.n / 256);
    static_assert(RSUM_SHARDS == WAVE, "one shard per lane");
    const double s = wave_sum(r.sum[RSUM_STRIDE * lane]);   // a fixed tree: the same s in every workgroup
    float mean;
    if (!rms_mean_decided(s, r.n, mean)) {   // uniform: every thread holds the same s
        __shared__ float pmean;
        if (tid == 0) pmean = rms_mean_sequential(r.x, nullptr, r.n);
        __syncthreads();
        mean = pmean;
    }
    const float scale = 1.0f / sqrtf(mean + r.eps);
    int8_t * qs = (int8_t *) buf;
    float * qd = (float *) (buf + r.n);
    int16_t * qsum = (int16_t *) (buf + r.n + 4 * (r.qmode == 1 ? r.n / 256 : r.n / 32));
    for (int b0 = 0; b0 < NB; b0 += 16) {
        const int b = b0 + 4 * wave + (lane >> 4);
        if (b >= NB) continue;   // whole rows of 16 lanes
        const int64_t e0 = 256 * (int64_t) b + 16 * (lane & 15);
        float4 xv[4], wv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            xv[k] = *(const float4 *) (r.x + e0 + 4 * k);
            wv[k] = r.w ? *(const float4 *) (r.w + e0 + 4 * k) : make_float4(1.f, 1.f, 1.f, 1.f);
        }
        float y[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float xx[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
            const float ww[4] = {wv[k].x, wv[k].y, wv[k].z, wv[k].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float yn = __fmul_rn(xx[c], scale);
                y[4 * k + c] = r.w ? __fmul_rn(yn, ww[c]) : yn;
            }
        }
        if (r.qmode == 1) q8K_row16(y, lane, qs + 256 * (int64_t) b, qsum + 16 * (int64_t) b, qd + b);
        else q8_0_row16(y, lane, qs + 256 * (int64_t) b, qd + 8 * (int64_t) b, qsum + 8 * (int64_t) b);
    }
    __syncthreads();
    A = {qs, qd, qsum};
}

// The same prologue in two halves for the one-shot kernel: gemv_pro_load issues the partial-sum
// load and the first 4096 elements' x / w loads into registers BEFORE the weight DMAs, so that
// the wait for them (vmcnt counts the DMAs issued after) leaves the weight stream in flight;
// gemv_pro_finish forms the activation (later passes of n > 4096 load inline).
struct pro_regs { double s; float4 xv[4], wv[4]; };
__device__ __forceinline__ void gemv_pro_load(const gemv_args & p, pro_regs & pr) {
    const auto & r = p.pro;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    pr.s = r.sum[RSUM_STRIDE * lane];
    const int b = 4 * wave + (lane >> 4);
    const int64_t e0 = 256 * (int64_t) min(b, (int) (r.n / 256) - 1) + 16 * (lane & 15);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        pr.xv[k] = *(const float4 *) (r.x + e0 + 4 * k);
        pr.wv[k] = r.w ? *(const float4 *) (r.w + e0 + 4 * k) : make_float4(1.f, 1.f, 1.f, 1.f);
    }
}
__device__ __forceinline__ void gemv_pro_finish(const gemv_args & p, const pro_regs & pr, uint8_t * buf, gemv_act & A) {
    const auto & r = p.pro;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int NB = (int) (r.n / 256);
    const double s = wave_sum(pr.s);   // a fixed tree: the same s in every workgroup
    float mean;
    if (!rms_mean_decided(s, r.n, mean)) {   // uniform: every thread holds the same s
        __shared__ float pmean;
        if (tid == 0) pmean = rms_mean_sequential(r.x, nullptr, r.n);
        __syncthreads();
        mean = pmean;
    }
    const float scale = 1.0f / sqrtf(mean + r.eps);
    int8_t * qs = (int8_t *) buf;
    float * qd = (float *) (buf + r.n);
    int16_t * qsum = (int16_t *) (buf + r.n + 4 * (r.qmode == 1 ? r.n / 256 : r.n / 32));
    for (int b0 = 0; b0 < NB; b0 += 16) {
        const int b = b0 + 4 * wave + (lane >> 4);
        if (b >= NB) continue;   // whole rows of 16 lanes
        const int64_t e0 = 256 * (int64_t) b + 16 * (lane & 15);
        float4 xv[4], wv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (b0 == 0) {
                xv[k] = pr.xv[k];
                wv[k] = pr.wv[k];
            } else {
                xv[k] = *(const float4 *) (r.x + e0 + 4 * k);
                wv[k] = r.w ? *(const float4 *) (r.w + e0 + 4 * k) : make_float4(1.f, 1.f, 1.f, 1.f);
            }
        }
        float y[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float xx[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
            const float ww[4] = {wv[k].x, wv[k].y, wv[k].z, wv[k].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float yn = __fmul_rn(xx[c], scale);
                y[4 * k + c] = r.w ? __fmul_rn(yn, ww[c]) : yn;
            }
        }
        if (r.qmode == 1) q8K_row16(y, lane, qs + 256 * (int64_t) b, qsum + 16 * (int64_t) b, qd + b);
        else q8_0_row16(y, lane, qs + 256 * (int64_t) b, qd + 8 * (int64_t) b, qsum + 8 * (int64_t) b);
    }
    __syncthreads();
    A = {qs, qd, qsum};
}

// LDS bytes of the prologue's activation (gemv_act layout, 16-B aligned pieces)
static inline uint32_t pro_lds_bytes(int64_t n, int qmode) {
    const int64_t nd = qmode == 1 ? n / 256 : n / 32, ns = qmode == 1 ? n / 16 : n / 32;
    return (uint32_t) (n + 4 * nd + ((2 * ns + 15) / 16) * 16);
}

// epilogue of one output row; v = this row's value, vp = the value of its rope partner row^1
__device__ __forceinline__ void gemv_store(const gemv_args & p, int mi, int64_t M, int64_t row, float v, float vp,
                                           const float2 * rtab, uint16_t * const * f16p) {
    if (p.dst[mi]) p.dst[mi][row] = v;
    if (p.f16out[mi]) f16p[2 * mi][row] = f2h(v);
    if (p.silu[mi]) {
        // ggml_vec_silu_f32 (vec.cpp:233): AVX-512 ggml_v_silu on 16-element chunks, libm tail
        const int64_t nvec = (M / 16) * 16;
        p.silu[mi][row] = row < nvec ? v / (1.0f + v_expf_avx512(-v)) : v / (1.0f + expf_cr(-v));
    }
    if (p.rope_out[mi] || p.rope_f16[mi]) {
        const int64_t i0 = row % p.rope_d;
        float o = v;
        if (i0 < p.rp.n_dims) {
            const float c = rtab[i0 / 2].x, sn = rtab[i0 / 2].y;
            float o0, o1;
            const bool odd = row & 1;
            rope_rotate(odd ? vp : v, odd ? v : vp, c, sn, o0, o1);
            o = odd ? o1 : o0;
        }
        if (p.rope_out[mi]) p.rope_out[mi][row] = o;
        if (p.rope_f16[mi]) f16p[2 * mi + 1][row] = f2h(o);
    }
}

// LDS dwords of the block records: two buffers (groups alternate) of RPG rows x nb blocks
template <class T>
static constexpr size_t xrec_dwords(int rpg, int64_t nb) { return (size_t) 2 * rpg * nb * T::RS; }

// The body runs as workgroup wg0 of nwg over the launch's ngroups row groups, so one launch can
// hold two bodies of different weight types (k_gemv_pipe2).  MODE 0: plain stores; 1: row
// values parked in LDS and the epilogues run after the loop on all threads.
// the matrix of row group g as a wave-uniform (SGPR) index: kernel-argument arrays indexed by a
// VGPR are read with vector loads from the kernarg segment, a memory round trip in front of the
// first weight load of every workgroup (the one-shot gate/up launch ran 20.3 instead of 14.3 us)
__device__ __forceinline__ int gemv_mat(const gemv_args & p, int64_t g) {
    const int gi = __builtin_amdgcn_readfirstlane((int) g);
    int mi = 0;
#pragma unroll
    for (int k = 1; k < GEMV_MAXMAT; ++k) mi += gi >= p.blk0[k] ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(mi);
}

template <class T, int R, int WPR, int MODE>
__device__ __forceinline__ void gemv_pipe_body(const gemv_args & p, const int64_t ngroups, const int64_t wg0, const int64_t nwg,
                                               uint32_t * xr) {
    constexpr int NWV = 4;
    constexpr int NT = 64 * NWV;
    constexpr int RPG = (NWV / WPR) * R;   // rows per group
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wsub = wave % WPR;
    const int t = wsub * WAVE + lane;
    const bool active = t < p.ntasks;
    const int tt = active ? t : 0;
    const int nb = p.ntasks / T::per_block;
    const int rowl0 = (wave / WPR) * R;    // this wave's first row within the group
    auto locate = [&](int64_t g, int & mi, int64_t & row0) {
        mi = gemv_mat(p, g);
        row0 = (g - p.blk0[mi]) * RPG + rowl0;
    };
    auto fetch = [&](int64_t g, typename T::raw (&w)[R]) {
        int mi;
        int64_t row0;
        locate(g, mi, row0);
        const int64_t M = p.M[mi];
        const uint8_t * Wm = p.W[mi];
#pragma unroll
        for (int r = 0; r < R; ++r) T::fetch(Wm + min(row0 + r, M - 1) * p.nb01[mi], tt, w[r]);
    };

    // the first group's weight loads leave before anything else, so the rope table and the
    // activation loads below overlap that HBM latency
    typename T::raw cur[R], nxt[R];
    int64_t g = wg0;
    if (g < ngroups) fetch(g, cur);
    typename T::act x;
    gemv_act A = p.A;
    if (p.pro.x) gemv_prologue(p, (uint8_t *) xr + p.pro.lds_off, A);
    T::load(A, tt, x);
    __shared__ float2 rtab[MODE ? GEMV_ROPE_MAXPAIRS : 1];
    // KV-cache destinations of the f16 epilogues, read from the dynamic-pointer table now
    // rather than as a dependent load in the epilogue
    __shared__ uint16_t * f16p[2 * GEMV_MAXMAT];
    if (MODE) {
        if (threadIdx.x < 2 * GEMV_MAXMAT) {
            const int mi = threadIdx.x >> 1;
            uint16_t * const * slot = (threadIdx.x & 1) ? p.rope_f16[mi] : p.f16out[mi];
            f16p[threadIdx.x] = slot ? *slot : nullptr;
        }
        if (p.need_pairs) {
            for (int ip = threadIdx.x; ip < p.rp.n_dims / 2; ip += NT) rtab[ip] = p.rtab_g[ip];
        }
        __syncthreads();
    }
    __shared__ float res[MODE ? GEMV_MAXG * RPG : 1];
    // walker lanes: row wr of this wave's R rows, class / sub-lane ws
    const int wr = lane / T::LPR, ws = lane % T::LPR;
    const int wrc = wr < R ? wr : 0;
    // residual producer: the residual of the walker lane's row, loaded a group ahead
    auto res_of = [&](int64_t gg) {
        int mi;
        int64_t row0;
        locate(gg, mi, row0);
        return p.rres[min(row0 + wrc, p.M[0] - 1)];
    };
    float rc = 0.0f, rn = 0.0f;
    double ss = 0.0;
    if (MODE == 0 && p.rres && g < ngroups) rc = res_of(g);
    int par = 0, kg = 0;
    for (; g < ngroups; g += nwg, par ^= 1, ++kg) {
        const int64_t gn = g + nwg;
        if (gn < ngroups) fetch(gn, nxt);
        if (MODE == 0 && p.rres && gn < ngroups) rn = res_of(gn);
        uint32_t * xb = xr + (size_t) par * RPG * nb * T::RS;
#pragma unroll
        for (int r = 0; r < R; ++r) T::rec(cur[r], tt, x, active, xb + (size_t) (rowl0 + r) * nb * T::RS);
        if constexpr (WPR > 1) __syncthreads();
        else wave_lds_sync();
        if (wsub == 0) {
            const float v = T::walk(xb + (size_t) (rowl0 + wrc) * nb * T::RS, nb, ws);
            if (wr < R && ws == 0) {
                if constexpr (MODE == 0) {
                    int mi;
                    int64_t row0;
                    locate(g, mi, row0);
                    if (row0 + wr < p.M[mi]) {
                        if (p.rres) {   // ADD(v, res): the CPU's single f32 add
                            const float xv = __fadd_rn(v, rc);
                            p.rxsum[row0 + wr] = xv;
                            ss = __dadd_rn(ss, (double) __fmul_rn(xv, xv));
                        } else if (p.tl.kind) {
                            __hip_atomic_store(p.dst[mi] + row0 + wr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        } else {
                            p.dst[mi][row0 + wr] = v;
                        }
                    }
                } else {
                    res[kg * RPG + rowl0 + wr] = v;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) cur[r] = nxt[r];
        rc = rn;
    }
    if constexpr (MODE == 0) {
        if (p.tl.kind) gemv_tail(p, kg, wg0, nwg, RPG);
        if (p.rres) {
            // this workgroup's rows' sum of squares (RPG walker lanes hold partials) to its shard
            // (no-return atomic)
            __shared__ double rpart[RPG];
            if (wsub == 0 && wr < R && ws == 0) rpart[rowl0 + wr] = ss;
            __syncthreads();
            if (threadIdx.x == 0) {
                double tot = 0.0;
#pragma unroll
                for (int k = 0; k < RPG; ++k) tot = __dadd_rn(tot, rpart[k]);
                __hip_atomic_fetch_add(p.rsum + RSUM_STRIDE * (wg0 % RSUM_SHARDS), tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if constexpr (MODE >= 1) {
        __syncthreads();
        for (int i = threadIdx.x; i < kg * RPG; i += NT) {
            const int64_t gg = wg0 + (int64_t) (i / RPG) * nwg;
            int mi = 0;
#pragma unroll
            for (int k = 1; k < GEMV_MAXMAT; ++k) mi += gg >= p.blk0[k] ? 1 : 0;
            const int64_t row = (gg - p.blk0[mi]) * RPG + i % RPG;
            // rope partner row ^ 1 lies in the same group (RPG is even whenever rope is fused)
            if (row < p.M[mi]) gemv_store(p, mi, p.M[mi], row, res[i], res[RPG > 1 ? i ^ 1 : i], rtab, f16p);
        }
    }
}

template <class T, int R, int WPR, int MODE>
__global__ __launch_bounds__(256) void k_gemv_pipe(const gemv_args p, const int64_t ngroups) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    kt_enter(p.kt);
    gemv_pipe_body<T, R, WPR, MODE>(p, ngroups, blockIdx.x, gridDim.x, xr);
    kt_exit(p.kt);
}

// Q/K of one K-quant and V of another (Llama-3 Q4_K_M: Q4_K and Q6_K on 16 of 32 layers) in
// one launch with epilogues: workgroups [0, nwg1) run p1's matrices, the rest p2's.  Each
// row's arithmetic is its type's own, so the bits are those of two separate launches.
template <class T1, class T2, int R2, int WPR>
__global__ __launch_bounds__(256) void k_gemv_pipe2(const gemv_args p1, const int64_t ng1, const int64_t nwg1,
                                                    const gemv_args p2, const int64_t ng2) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    kt_enter(p1.kt);
    if ((int64_t) blockIdx.x < nwg1) gemv_pipe_body<T1, 2, WPR, 1>(p1, ng1, blockIdx.x, nwg1, xr);
    else gemv_pipe_body<T2, R2, WPR, 1>(p2, ng2, (int64_t) blockIdx.x - nwg1, (int64_t) gridDim.x - nwg1, xr);
    kt_exit(p1.kt);
}

// ---- one-shot body: one row group per workgroup, weights staged by LDS-DMA ----------------------
// Each wave copies its R row slices (at most 64 tasks of a row: os_geo<T>::SEG bytes each) HBM ->
// LDS with global_load_lds, 1 KiB of contiguous bytes per wave instruction, so every 128-B line
// is requested once (the register fetch of a task's header + quants asks each line three
// times), and no VGPR is held for bytes in flight; the dispatcher's workgroup turnover does the
// pipelining.  The norm prologue's sources are loaded before the DMAs are issued, so waiting
// for them leaves the weight stream in flight; a Q8 activation slice is loaded after them.
// Records, walker and epilogues are the pipelined kernel's (the same bits).
// a chained launch's consumer: wave 0 spins (lanes 0-7 read one shard each, a few hundred
// cycles apart: thousands of waiting workgroups polling the same lines would crowd out the
// producers' own atomics) until the producers' shards sum to n; the other waves wait at the
// barrier.  The producers wrote their outputs write-through before adding, and nothing in this
// launch read those bytes before, so plain loads after this see them.
__device__ __forceinline__ void os_dep_wait(const int * dep, int n) {
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < WAVE) {
        for (int it = 0;; ++it) {
            int v = lane < FFN_SHARDS ? __hip_atomic_load(dep + FFN_SHARD_STRIDE * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
            v = __builtin_amdgcn_readfirstlane(wave_sum(v));
            if (v >= n) break;
            if (it > (1 << 22)) __builtin_trap();   // a producer never reported: fail loudly, not hang
            __builtin_amdgcn_s_sleep(8);
        }
    }
    __syncthreads();
}

template <class T> struct os_geo {
    static constexpr int SEG = (WAVE / T::per_block) * T::blk_bytes;   // a wave's row slice
    static constexpr int NI = (SEG + 1023) / 1024;                        // DMA instructions per slice
    static constexpr int SLICE = NI * 1024;                               // LDS bytes per slice
};
typedef __attribute__((address_space(3))) void * gemv_lds_t;

template <class T, int R, int WPR, int MODE, bool PRO>
__device__ __forceinline__ void gemv_os_body(const gemv_args & p, const int64_t g, uint8_t * wl, uint32_t * xr) {
    constexpr int NWV = 4;
    constexpr int NT = 64 * NWV;
    constexpr int RPG = (NWV / WPR) * R;
    using G = os_geo<T>;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wsub = wave % WPR;
    const int t = wsub * WAVE + lane;
    const bool active = t < p.ntasks;
    const int tt = active ? t : 0;
    const int nb = p.ntasks / T::per_block;
    const int rowl0 = (wave / WPR) * R;
    const int mi = gemv_mat(p, g);
    const int64_t row0 = (g - p.blk0[mi]) * RPG + rowl0;
    const int64_t M = p.M[mi];
    // ---- activation sources first ----
    pro_regs pr;
    if constexpr (PRO) gemv_pro_load(p, pr);
    const int wr = lane / T::LPR, ws = lane % T::LPR;
    const int wrc = wr < R ? wr : 0;
    // one walking wave (W1): after every wave's records, wave 0 walks all RPG rows of the group
    // (its lanes in parallel: one walk where four waves each ran one, the other waves retire)
    constexpr bool W1 = WPR == 1 && MODE == 0 && RPG * T::LPR <= WAVE;
    const int64_t grow0 = (g - p.blk0[mi]) * RPG;
    const int wr1 = lane / T::LPR, ws1 = lane % T::LPR, wrc1 = wr1 < RPG ? wr1 : 0;
    float rc = 0.0f;
    if (MODE == 0 && p.rres) rc = p.rres[min((W1 ? grow0 + wrc1 : row0 + wrc), p.M[0] - 1)];
    // ---- weight DMA: this wave's R row slices -> its LDS region (nt: read once per token) ----
    uint8_t * mine = wl + (size_t) wave * R * G::SLICE;
    {
        const int nt_w = min(WAVE, p.ntasks - WAVE * wsub);
        const int seg = (nt_w / T::per_block) * T::blk_bytes;
        const uint8_t * Wm = p.W[mi];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint8_t * src = Wm + min(row0 + r, M - 1) * p.nb01[mi] + (int64_t) wsub * G::SEG;
#pragma unroll
            for (int i = 0; i < G::NI; ++i) {
                const int off = min(i * 1024 + 16 * lane, seg - 16);
                __builtin_amdgcn_global_load_lds((const void *) (src + off), (gemv_lds_t) (mine + r * G::SLICE + i * 1024), 16, 0,
                                                 MI_WNT ? 2 : 0);
            }
        }
    }
    if (p.dep) os_dep_wait(p.dep, p.dep_n);
    // the activation slice after the DMAs: T::load computes on what it loads (bsum pairs, the
    // Q6_K -32 sums), and a wait for a load issued BEFORE the DMAs would hold the DMA issue back
    // by an L2 round trip (the one-shot kernel's rec stage took ~35 % longer that way)
    typename T::act x;
    if constexpr (PRO) {
        gemv_act A = p.A;
        gemv_pro_finish(p, pr, (uint8_t *) xr + p.pro.lds_off, A);
        T::load(A, tt, x);
    } else {
        T::load(p.A, tt, x);
    }
    __shared__ float2 rtab[MODE ? GEMV_ROPE_MAXPAIRS : 1];
    __shared__ uint16_t * f16p[2 * GEMV_MAXMAT];
    if (MODE) {
        if (threadIdx.x < 2 * GEMV_MAXMAT) {
            const int m2 = threadIdx.x >> 1;
            uint16_t * const * slot = (threadIdx.x & 1) ? p.rope_f16[m2] : p.f16out[m2];
            f16p[threadIdx.x] = slot ? *slot : nullptr;
        }
        if (p.need_pairs) {
            for (int ip = threadIdx.x; ip < p.rp.n_dims / 2; ip += NT) rtab[ip] = p.rtab_g[ip];
        }
    }
    // ---- this wave's weights are in LDS (the issuing wave's vmcnt covers its own DMAs) ----
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t * xb = xr;
#ifndef MI_EXP
#define MI_EXP 0
#endif
    // MI_EXP (time-split experiments only, wrong results): 1 no walk, 2 no records, 3 neither
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (MI_EXP & 2) break;
        typename T::raw w;
        T::template fetch<typename lds_loader<T>::type>(mine + r * G::SLICE - (int64_t) wsub * G::SEG, tt, w);
        T::rec(w, tt, x, active, xb + (size_t) (rowl0 + r) * nb * T::RS);
    }
    if constexpr (W1) {
        __syncthreads();   // every wave's records are in
        if (wave != 0) return;
        const float v = T::walk(xb + (size_t) wrc1 * nb * T::RS, nb, ws1);
        const int64_t row = grow0 + wr1;
        const bool mine_row = wr1 < RPG && ws1 == 0 && row < M;
        double sq = 0.0;
        if (mine_row) {
            if (p.rres) {   // ADD(v, res): the CPU's single f32 add
                const float xv = __fadd_rn(v, rc);
                p.rxsum[row] = xv;
                sq = (double) __fmul_rn(xv, xv);
            } else if (p.tl.kind) {   // the SwiGLU tail reads it back: write-through
                __hip_atomic_store(p.dst[mi] + row, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                p.dst[mi][row] = v;
            }
        }
        if (p.tl.kind) {   // only this wave stored: drain, then one lane reports the group
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                const int blk = (int) (grow0 / 256);
                __hip_atomic_fetch_add(p.tl.cnt + blk * TAIL_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (p.rres) {   // the group's rows' sum of squares, in row order, to the workgroup's shard
            __shared__ double rpart1[RPG];
            if (wr1 < RPG && ws1 == 0) rpart1[wr1] = sq;
            wave_lds_sync();
            if (lane == 0) {
                double tot = 0.0;
#pragma unroll
                for (int k = 0; k < RPG; ++k) tot = __dadd_rn(tot, rpart1[k]);
                __hip_atomic_fetch_add(p.rsum + RSUM_STRIDE * (g % RSUM_SHARDS), tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return;
    }
    if constexpr (WPR > 1 || MODE != 0) __syncthreads();
    else wave_lds_sync();
    __shared__ float res[MODE ? RPG : 1];
    // epilogue launches: wave 0 walks every row of the group into res (one walk where four waves
    // each ran one); the stores below are the whole workgroup's as before
    constexpr bool W1E = WPR == 1 && MODE != 0 && RPG * T::LPR <= WAVE;
    if constexpr (W1E) {
        if (wave == 0) {
            const float v = T::walk(xb + (size_t) wrc1 * nb * T::RS, nb, ws1);
            if (wr1 < RPG && ws1 == 0) res[wr1] = v;
        }
    } else if (wsub == 0) {
        const float v = (MI_EXP & 1) ? xb[lane] * 0.5f : T::walk(xb + (size_t) (rowl0 + wrc) * nb * T::RS, nb, ws);
        if (wr < R && ws == 0) {
            if constexpr (MODE == 0) {
                if (row0 + wr < M) {
                    if (p.rres) {   // ADD(v, res): the CPU's single f32 add
                        const float xv = __fadd_rn(v, rc);
                        p.rxsum[row0 + wr] = xv;
                        rc = xv;
                    } else if (p.tl.kind) {   // the SwiGLU tail reads it back: write-through
                        __hip_atomic_store(p.dst[mi] + row0 + wr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        p.dst[mi][row0 + wr] = v;
                    }
                }
            } else {
                res[rowl0 + wr] = v;
            }
        }
    }
    if constexpr (MODE == 0) {
        // the workgroup's row group reports on its Q8_K block's counter (stores drained first, a
        // no-return add: no round trip before the workgroup retires); the block's tail workgroup
        // (k_gemv_os past the row groups) runs SILU(gate) * up and its quantization
        if (p.tl.kind) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                const int blk = (int) ((g - p.blk0[mi]) * RPG / 256);
                __hip_atomic_fetch_add(p.tl.cnt + blk * TAIL_STRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (p.rres) {
            // this workgroup's rows' sum of squares (walker lanes hold x) to its shard (no-return atomic)
            __shared__ double rpart[RPG];
            if (wsub == 0 && wr < R && ws == 0) rpart[rowl0 + wr] = row0 + wr < M ? (double) __fmul_rn(rc, rc) : 0.0;
            __syncthreads();
            if (threadIdx.x == 0) {
                double tot = 0.0;
#pragma unroll
                for (int k = 0; k < RPG; ++k) tot = __dadd_rn(tot, rpart[k]);
                __hip_atomic_fetch_add(p.rsum + RSUM_STRIDE * (g % RSUM_SHARDS), tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if constexpr (MODE >= 1) {
        __syncthreads();
        for (int i = threadIdx.x; i < RPG; i += NT) {
            const int64_t row = (g - p.blk0[mi]) * RPG + i;
            // rope partner row ^ 1 lies in the same group (RPG is even whenever rope is fused)
            if (row < M) gemv_store(p, mi, M, row, res[i], res[RPG > 1 ? i ^ 1 : i], rtab, f16p);
        }
    }
}

// a SwiGLU tail workgroup (one per Q8_K block, after every row group in dispatch order, so every
// producer it waits for is already resident or done): wave 0 waits until the block's gate and up
// row groups have all reported, re-arms the counter and runs the block's tail
// done (k_gemv_ffn): the block is quantized write-through and reported on done's shards
__device__ __forceinline__ void os_tail_block(const gemv_args & p, int blk, int per, int * done = nullptr) {
    if (threadIdx.x >= WAVE) return;
    int * c = p.tl.cnt + blk * TAIL_STRIDE;
    for (int it = 0;; ++it) {
        const int v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (v >= per) break;
        if (it > (1 << 24)) __builtin_trap();   // a producer never reported: fail loudly, not hang
        __builtin_amdgcn_s_sleep(2);
    }
    if (threadIdx.x == 0) __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done) {
        tail_swiglu<true>(p, blk, threadIdx.x);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0)
            __hip_atomic_fetch_add(done + FFN_SHARD_STRIDE * (blk % FFN_SHARDS), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        tail_swiglu(p, blk, threadIdx.x);
    }
}

// ---- looping one-shot body: several row groups per workgroup, weights double-buffered ----------
// The one-shot body's per-group work (DMA -> records -> walk -> store; the same records, walker
// and bits), but a workgroup runs groups g, g + grid, ... and issues group g + grid's weight DMA
// into its second slice set BEFORE computing group g, so its own compute overlaps its next
// stream and the activation is loaded once per workgroup instead of once per group (the
// one-shot kernel moves ~9 KB per workgroup and then computes with no bytes of its own in
// flight).  No prologue, epilogue or tail (MODE 0); the residual producer accumulates its sum
// of squares over the workgroup's groups and adds it once.
template <class T, int R, int WPR>
__device__ __forceinline__ void os_issue(const gemv_args & p, int64_t g, uint8_t * mine, int wave, int lane) {
    using G = os_geo<T>;
    constexpr int RPG = (4 / WPR) * R;
    const int wsub = wave % WPR;
    const int rowl0 = (wave / WPR) * R;
    const int mi = gemv_mat(p, g);
    const int64_t row0 = (g - p.blk0[mi]) * RPG + rowl0;
    const int64_t M = p.M[mi];
    const int nt_w = min(WAVE, p.ntasks - WAVE * wsub);
    const int seg = (nt_w / T::per_block) * T::blk_bytes;
    const uint8_t * Wm = p.W[mi];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint8_t * src = Wm + min(row0 + r, M - 1) * p.nb01[mi] + (int64_t) wsub * G::SEG;
#pragma unroll
        for (int i = 0; i < G::NI; ++i) {
            const int off = min(i * 1024 + 16 * lane, seg - 16);
            __builtin_amdgcn_global_load_lds((const void *) (src + off), (gemv_lds_t) (mine + r * G::SLICE + i * 1024), 16, 0,
                                             MI_WNT ? 2 : 0);
        }
    }
}

template <class T, int R, int WPR>
__global__ __launch_bounds__(256) void k_gemv_osl(const gemv_args p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    kt_enter(p.kt);
    constexpr int RPG = (4 / WPR) * R;
    using G = os_geo<T>;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wsub = wave % WPR;
    const int t = wsub * WAVE + lane;
    const bool active = t < p.ntasks;
    const int tt = active ? t : 0;
    const int nb = p.ntasks / T::per_block;
    const int rowl0 = (wave / WPR) * R;
    const int wr = lane / T::LPR, ws = lane % T::LPR;
    const int wrc = wr < R ? wr : 0;
    const int64_t ng = p.blk0[GEMV_MAXMAT], grid = gridDim.x;
    uint8_t * wl = (uint8_t *) xr + p.wl_off;
    uint8_t * buf[2] = {wl + (size_t) wave * 2 * R * G::SLICE, wl + (size_t) wave * 2 * R * G::SLICE + (size_t) R * G::SLICE};
    int64_t g = blockIdx.x;
    os_issue<T, R, WPR>(p, g, buf[0], wave, lane);
    typename T::act x;
    T::load(p.A, tt, x);
    double ss = 0.0;
    int cur = 0;
    for (; g < ng; g += grid) {
        const int64_t gn = g + grid;
        const bool more = gn < ng;   // uniform
        if (more) os_issue<T, R, WPR>(p, gn, buf[cur ^ 1], wave, lane);
        const int mi = gemv_mat(p, g);
        const int64_t row0 = (g - p.blk0[mi]) * RPG + rowl0;
        const int64_t M = p.M[mi];
        float rc = 0.0f;
        if (p.rres) rc = p.rres[min(row0 + wrc, p.M[0] - 1)];
        // this group's weights have landed (the next group's DMA may still be in flight)
        if (more) {
            if constexpr (G::NI * R == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
            else if constexpr (G::NI * R == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            else if constexpr (G::NI * R == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            else if constexpr (G::NI * R == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if constexpr (G::NI * R == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else if constexpr (G::NI * R == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        uint32_t * xb = xr;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            typename T::raw w;
            T::template fetch<typename lds_loader<T>::type>(buf[cur] + r * G::SLICE - (int64_t) wsub * G::SEG, tt, w);
            T::rec(w, tt, x, active, xb + (size_t) (rowl0 + r) * nb * T::RS);
        }
        if constexpr (WPR > 1) __syncthreads();
        else wave_lds_sync();
        if (wsub == 0) {
            const float v = T::walk(xb + (size_t) (rowl0 + wrc) * nb * T::RS, nb, ws);
            if (wr < R && ws == 0 && row0 + wr < M) {
                if (p.rres) {   // ADD(v, res): the CPU's single f32 add
                    const float xv = __fadd_rn(v, rc);
                    p.rxsum[row0 + wr] = xv;
                    ss = __dadd_rn(ss, (double) __fmul_rn(xv, xv));
                } else {
                    p.dst[mi][row0 + wr] = v;
                }
            }
        }
        // the records are rewritten by the next group: every wave's walk is done with them
        if constexpr (WPR > 1) __syncthreads();
        else wave_lds_sync();
        cur ^= 1;
    }
    if (p.rres) {
        // this workgroup's rows' sum of squares (walker lanes hold partials) to its shard
        __shared__ double rpart[RPG];
        if (wsub == 0 && wr < R && ws == 0) rpart[rowl0 + wr] = ss;
        __syncthreads();
        if (threadIdx.x == 0) {
            double tot = 0.0;
#pragma unroll
            for (int k = 0; k < RPG; ++k) tot = __dadd_rn(tot, rpart[k]);
            __hip_atomic_fetch_add(p.rsum + RSUM_STRIDE * (blockIdx.x % RSUM_SHARDS), tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    kt_exit(p.kt);
}

template <class T, int R, int WPR, int MODE, bool PRO>
__global__ __launch_bounds__(256) void k_gemv_os(const gemv_args p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    if (MODE == 0 && p.tl.kind && (int64_t) blockIdx.x >= p.blk0[GEMV_MAXMAT]) {
        constexpr int RPG = (4 / WPR) * R;
        os_tail_block(p, (int) (blockIdx.x - p.blk0[GEMV_MAXMAT]), 2 * (256 / RPG));
        return;
    }
    kt_enter(p.kt);
    // dynamic LDS: [records RPG x nb x RS dwords | prologue activation | weight slices]
    gemv_os_body<T, R, WPR, MODE, PRO>(p, blockIdx.x, (uint8_t *) xr + p.wl_off, xr);
    kt_exit(p.kt);
}

// ---- chained FFN launch (k_gemv_ffn) ---------------------------------------------------------------
// The decode FFN of one layer, gate/up -> SILU * MUL -> down, as ONE grid in dispatch order:
//   [gate/up row groups | one SwiGLU tail workgroup per Q8_K block | down row groups]
// Each part is the one-shot body (the same records, walkers and bits as separate launches).  A tail
// workgroup waits for its block's gate and up row groups, quantizes the block write-through and
// reports on the done shards; a down workgroup issues its weight DMA FIRST and only then waits for
// all tails, so the down weights stream in while the gate/up stragglers and the tails finish (the
// separate launches paid the gate/up tail, a product kernel and the down ramp in series).  Every
// workgroup waits only for workgroups dispatched before it, so the grid cannot deadlock.
template <class T1, int R1, int WPR1, class T2, int R2, int WPR2>
__global__ __launch_bounds__(256) void k_gemv_ffn(const gemv_args p1, const gemv_args p2, int * done) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    kt_enter(p1.kt);
    const int64_t ng1 = p1.blk0[GEMV_MAXMAT], nt = p1.tl.n / 256, b = blockIdx.x;
    if (b < ng1) gemv_os_body<T1, R1, WPR1, 0, false>(p1, b, (uint8_t *) xr + p1.wl_off, xr);
    else if (b < ng1 + nt) os_tail_block(p1, (int) (b - ng1), 2 * (256 / ((4 / WPR1) * R1)), done);
    else gemv_os_body<T2, R2, WPR2, 0, false>(p2, b - ng1 - nt, (uint8_t *) xr + p2.wl_off, xr);
    kt_exit(p1.kt);
}

template <class T1, class T2, int R2, int WPR, bool PRO, int R1 = 2>
__global__ __launch_bounds__(256) void k_gemv_os2(const gemv_args p1, const int64_t ng1, const gemv_args p2) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    kt_enter(p1.kt);
    if ((int64_t) blockIdx.x < ng1) gemv_os_body<T1, R1, WPR, 1, PRO>(p1, blockIdx.x, (uint8_t *) xr + p1.wl_off, xr);
    else gemv_os_body<T2, R2, WPR, 1, PRO>(p2, (int64_t) blockIdx.x - ng1, (uint8_t *) xr + p2.wl_off, xr);
    kt_exit(p1.kt);
}


// ---- persistent loader / consumer engine (k_gemv_eng) --------------------------------------------
// One workgroup per CU streams a contiguous range of rows (over the launch's matrices) through an
// LDS ring, with the roles of MI355X_MICROARCH.md's ldsdma-fill / engine rows:
//   * wave 0, the loader, walks the workgroup's CHUNKS in order (a chunk = 64 tasks of one row:
//     16 K-quant super-blocks or 64 Q8_0 / Q4_0 blocks, the one-shot kernel's wave slice) and
//     copies each HBM -> ring slot k % ns with LDS-DMA (1 KiB per wave instruction, nt), keeping
//     L = 60 / P chunks in flight (P instructions per chunk; vmcnt counts at most 63); after
//     issuing chunk k it waits vmcnt(L * P), i.e. for chunk k - L, and publishes it (full[slot]);
//     before reusing a slot it waits for the consumer that read it (fre[slot]);
//   * waves 1 .. NC, the consumers, own rows c, c + NC, ... of the workgroup; per chunk they wait
//     for full[slot], read their task's bytes into registers, hand the slot back, and run the
//     unchanged records (qtypes.h) and the walker, whose fp32 chain carries from chunk to chunk in
//     block order — the row's bits are the one-shot kernel's.
// The activation lives in LDS, formed once per workgroup while the loader's first chunks are in
// flight: a copy of the quantized activation, the RMS-norm prologue from the residual producer's
// partial sums, or the SwiGLU product silu(gate) * up of the FFN (the k_mul_quant arithmetic).
// The weight stream therefore never waits for a prologue, and no launch of its own forms one.
constexpr int ENG_LDS = 160 * 1024;
constexpr int ENG_NSMAX = 64;
constexpr int ENG_CTRL = 2048;   // bytes of control words in front of the activation
constexpr int ENG_RMAX = 128;    // residual rows per workgroup staged in LDS
constexpr int ENG_GPMAX = 4;     // rows per packet

struct eng_geo {
    int ns;              // ring slots (one packet each)
    int nch;             // chunks (64 tasks) per row
    int last_bytes;      // weight bytes of a row's last chunk
    int gp;              // rows per packet
    int pk;              // DMA pieces (KiB) per packet slot
    int rowb;            // bytes per row (== nb01 of every matrix)
    int ll;              // packets in flight per loader wave (ll * pk <= 63: vmcnt's range)
    int act_mode;        // 0: copy p.A; 1: RMS-norm prologue (p.pro); 2: SwiGLU prologue
    int qmode;           // activation quantization: 1 Q8_K, 2 Q8_0
    int nmat;
    int64_t n;           // activation length (K)
    uint32_t rec_off, ring_off, slot, trash_off;
    const float * sw_gate; const float * sw_up;   // act_mode 2
};

// s_waitcnt vmcnt(n) for a runtime n <= 63 (an immediate operand: one case per count)
__device__ __forceinline__ void eng_vmwait(int n) {
#define EW(k) case k: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(k) : "memory"); break;
#define EW8(k) EW(k) EW(k + 1) EW(k + 2) EW(k + 3) EW(k + 4) EW(k + 5) EW(k + 6) EW(k + 7)
    switch (n) {
        EW8(0) EW8(8) EW8(16) EW8(24) EW8(32) EW8(40) EW8(48) EW(56) EW(57) EW(58) EW(59) EW(60) EW(61) EW(62) EW(63)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef EW8
#undef EW
}

// LDS layout of the control words
struct eng_ctrl {
    int full[ENG_NSMAX];   // packet number last landed in the slot
    int fre[ENG_NSMAX];    // packet number last consumed from the slot
    int cnt[ENG_NSMAX];    // rows of the slot's packet consumed so far
    int rdy;               // consumer waves done forming the activation
    float pmean;
    double rpart[16];      // residual producer: sum of squares per consumer wave
    float rres[ENG_RMAX];  // residual producer: the workgroup's residual rows
};
static_assert(sizeof(eng_ctrl) <= ENG_CTRL, "engine control words");

template <class V> __device__ __forceinline__ V eng_ld(V * p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
template <class V> __device__ __forceinline__ void eng_st(V * p, V v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// 16 B per lane HBM -> LDS as inline asm: the compiler sees no LDS write in flight and adds no
// vmcnt(0) before the loader's LDS flag accesses (k_fattn_exact.hip lds_dma16); nt: read once
__device__ __forceinline__ void eng_dma16(const void * src, const void * lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (gemv_lds_t) lds);
#if MI_WNT
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m), "v"(src) : "memory", "m0");
#else
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(src) : "memory", "m0");
#endif
}

// the same as a buffer load: the chunk's address in the resource's base, the lane's 16-B offset
// in a VGPR that never changes, the piece's 1 KiB step in the immediate — two instructions a piece
typedef int eng_rsrc __attribute__((ext_vector_type(4)));
__device__ __forceinline__ eng_rsrc eng_rsrc_of(const void * base) {
    const uint64_t a = (uint64_t) (uintptr_t) base;
    eng_rsrc r;
    r.x = __builtin_amdgcn_readfirstlane((int) (uint32_t) a);
    r.y = __builtin_amdgcn_readfirstlane((int) ((uint32_t) (a >> 32) & 0xffffu));   // stride 0
    r.z = -1;                                                                          // no range check
    r.w = 0x00020000;                                                                  // raw dword access (gfx9)
    return r;
}
template <int IMM>
__device__ __forceinline__ void eng_bdma(eng_rsrc r, uint32_t voff, const void * lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (gemv_lds_t) lds);
#if MI_WNT
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen offset:%3 nt lds" ::"v"(voff), "s"(r), "s"(m), "n"(IMM)
                 : "memory", "m0");
#else
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen offset:%3 lds" ::"v"(voff), "s"(r), "s"(m), "n"(IMM)
                 : "memory", "m0");
#endif
}
// one packet: `bytes` contiguous bytes from src into the slot at dst as pk KiB pieces (pieces
// wholly past a short packet land in the trash line, a piece's lanes past its end are masked),
// so every packet is exactly pk instructions and vmcnt counts packets
__device__ __forceinline__ void eng_issue(const uint8_t * src, uint8_t * dst, int bytes, int pk, int lane, uint8_t * trash) {
    const uint32_t vo = 16u * (uint32_t) lane;
    for (int q0 = 0; q0 < pk; q0 += 4) {
        const eng_rsrc r = eng_rsrc_of(src + 1024 * q0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = q0 + u;
            if (q >= pk) break;
            const int rem = bytes - 1024 * q;
            // the instruction offset moves the LDS destination as well as the source
            // (tools/lds_dma_probe.hip): M0 stays at the group's base
            uint8_t * d = dst + 1024 * q0;
            if (rem >= 1024 || 16 * lane < rem) {
                if (u == 0) eng_bdma<0>(r, vo, d);
                else if (u == 1) eng_bdma<1024>(r, vo, d);
                else if (u == 2) eng_bdma<2048>(r, vo, d);
                else eng_bdma<3072>(r, vo, d);
            } else if (rem <= 0 && lane == 0) {
                eng_bdma<0>(eng_rsrc_of(src), 0u, trash);   // keeps the instruction count
            }
        }
    }
}

// bounded LDS spin: a hand-off that never completes traps instead of hanging the device
__device__ __forceinline__ void eng_wait_eq(int * w, int v) {
    for (int it = 0; eng_ld(w) != v; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if (it > (1 << 24)) __builtin_trap();
    }
}

// the fp32 chain of one row carried over its chunks (qtypes.h walk(), split at chunk bounds).
// The records of a chunk are read 16 at a time before the chain consumes them: a loop that waits
// for each record's LDS read in turn made a consumer wave's chunk ~3.5k cycles (16 dependent LDS
// round trips), the engine's bound at 3-7 consumer waves
constexpr int ENG_WG = 8;
template <class T> struct eng_walk;
template <> struct eng_walk<g_q4_K> {
    float A = 0.0f, B = 0.0f;
    __device__ void step(const uint32_t * rr, int nb, int) {
        for (int b0 = 0; b0 < nb; b0 += ENG_WG) {
            uint4 r[ENG_WG];
#pragma unroll
            for (int b = 0; b < ENG_WG; ++b) r[b] = *(const uint4 *) (rr + (b0 + b) * g_q4_K::RS);
#pragma unroll
            for (int b = 0; b < ENG_WG; ++b) {
                if (b0 + b < nb) {
                    A = fmaf((float) (int) r[b].x, asf(r[b].z), A);
                    B = fmaf((float) (int) r[b].y, asf(r[b].w), B);
                }
            }
        }
    }
    __device__ float result() const { return __fsub_rn(A, B); }
};
template <> struct eng_walk<g_q4_0> {
    float A = 0.0f;
    __device__ void step(const uint32_t * rr, int nb, int) {
        for (int b0 = 0; b0 < nb; b0 += ENG_WG) {
            uint2 r[ENG_WG];
#pragma unroll
            for (int b = 0; b < ENG_WG; ++b) r[b] = *(const uint2 *) (rr + (b0 + b) * g_q4_0::RS);
#pragma unroll
            for (int b = 0; b < ENG_WG; ++b) {
                if (b0 + b < nb) A = fmaf((float) (int) r[b].x, asf(r[b].y), A);
            }
        }
    }
    __device__ float result() const { return A; }
};
template <class T, int FO> struct eng_walk_cls {   // class chains (LPR = 8), scale product at dword FO
    float acc = 0.0f;
    __device__ void step(const uint32_t * rr, int nb, int s) {
        for (int b0 = 0; b0 < nb; b0 += ENG_WG) {
            float f[ENG_WG];
            int c[ENG_WG];
#pragma unroll
            for (int b = 0; b < ENG_WG; ++b) {
                f[b] = asf(rr[(b0 + b) * T::RS + FO]);
                c[b] = (int) rr[(b0 + b) * T::RS + s];
            }
#pragma unroll
            for (int b = 0; b < ENG_WG; ++b) {
                if (b0 + b < nb) acc = fmaf(f[b], (float) c[b], acc);
            }
        }
    }
    __device__ float result() const { return hsum8_lanes(acc); }
};
template <> struct eng_walk<g_q6_K> : eng_walk_cls<g_q6_K, 8> {};
template <> struct eng_walk<g_q8_0> : eng_walk_cls<g_q8_0, 8> {};
template <> struct eng_walk<g_q5_K> {
    float acc = 0.0f, summs = 0.0f;
    __device__ void step(const uint32_t * rr, int nb, int s) {
        for (int b0 = 0; b0 < nb; b0 += ENG_WG) {
            float f[ENG_WG], fm[ENG_WG];
            int c[ENG_WG], im[ENG_WG];
#pragma unroll
            for (int b = 0; b < ENG_WG; ++b) {
                const uint32_t * r = rr + (b0 + b) * g_q5_K::RS;
                f[b] = asf(r[9]); c[b] = (int) r[s]; im[b] = (int) r[8]; fm[b] = asf(r[10]);
            }
#pragma unroll
            for (int b = 0; b < ENG_WG; ++b) {
                if (b0 + b < nb) {
                    acc = fmaf(f[b], (float) c[b], acc);
                    summs = fmaf((float) im[b], fm[b], summs);
                }
            }
        }
    }
    __device__ float result() const { return __fadd_rn(hsum8_lanes(acc), summs); }
};

// the activation of consumer wave cw (of NC) into LDS, in the gemv_act layout at buf
template <int NC>
__device__ __forceinline__ void eng_act(const gemv_args & p, const eng_geo & e, uint8_t * buf, int cw, int lane, eng_ctrl * cc) {
    const int64_t n = e.n;
    const bool kq = e.qmode == 1;
    const int64_t nd = kq ? n / 256 : n / 32, nsum = kq ? n / 16 : n / 32;
    int8_t * qs = (int8_t *) buf;
    float * qd = (float *) (buf + n);
    int16_t * qsum = (int16_t *) (buf + n + 4 * nd);
    const int NB = (int) (n / 256);
    if (e.act_mode == 0) {
        const int tc = cw * 64 + lane;
        for (int64_t o = 16 * (int64_t) tc; o < n; o += 16 * 64 * NC) *(uint4 *) (qs + o) = *(const uint4 *) (p.A.qs + o);
        for (int64_t o = tc; o < nd; o += 64 * NC) qd[o] = p.A.d[o];
        for (int64_t o = tc; o < nsum; o += 64 * NC) qsum[o] = p.A.s[o];
        return;
    }
    float scale = 1.0f;
    if (e.act_mode == 1) {
        const auto & r = p.pro;
        const double s = wave_sum(r.sum[RSUM_STRIDE * lane]);   // a fixed tree: the same s in every wave
        float mean;
        if (!rms_mean_decided(s, n, mean)) mean = rms_mean_sequential(r.x, nullptr, n);   // rare (~1e-5 of rows)
        scale = 1.0f / sqrtf(mean + r.eps);
    }
    // wave cw, row of 16 lanes (lane >> 4): 256-element block b, lane owns 16 elements
    for (int b0 = 0; b0 < NB; b0 += 4 * NC) {
        const int b = b0 + 4 * cw + (lane >> 4);
        if (b >= NB) continue;   // whole rows of 16 lanes
        const int64_t e0 = 256 * (int64_t) b + 16 * (lane & 15);
        float y[16];
        if (e.act_mode == 1) {
            const auto & r = p.pro;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 xv = *(const float4 *) (r.x + e0 + 4 * k);
                const float4 wv = r.w ? *(const float4 *) (r.w + e0 + 4 * k) : make_float4(1.f, 1.f, 1.f, 1.f);
                const float xx[4] = {xv.x, xv.y, xv.z, xv.w}, ww[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float yn = __fmul_rn(xx[c], scale);
                    y[4 * k + c] = r.w ? __fmul_rn(yn, ww[c]) : yn;
                }
            }
        } else {
            // silu(gate) * up: ggml_vec_silu_f32's AVX-512 ggml_v_silu on the 16-element chunks
            // (vec.cpp:233; n is a multiple of 256), then the MUL (k_mul_quant's arithmetic)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 gv = *(const float4 *) (e.sw_gate + e0 + 4 * k);
                const float4 uv = *(const float4 *) (e.sw_up + e0 + 4 * k);
                const float gg[4] = {gv.x, gv.y, gv.z, gv.w}, uu[4] = {uv.x, uv.y, uv.z, uv.w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float sv = gg[c] / (1.0f + v_expf_avx512(-gg[c]));
                    y[4 * k + c] = __fmul_rn(sv, uu[c]);
                }
            }
        }
        if (kq) q8K_row16(y, lane, qs + 256 * (int64_t) b, qsum + 16 * (int64_t) b, qd + b);
        else q8_0_row16(y, lane, qs + 256 * (int64_t) b, qd + 8 * (int64_t) b, qsum + 8 * (int64_t) b);
    }
}

// The work of workgroup w: rows [w M / nwg, (w + 1) M / nwg) of EACH matrix (the same rows of
// gate and up), cut into packets of up to gp rows that never cross a matrix; a packet is one
// contiguous byte range (rows are nb01 apart and nb01 is the row size)
struct eng_work {
    int64_t r0[GEMV_MAXMAT], nr[GEMV_MAXMAT];
    int np[GEMV_MAXMAT + 1];   // packets before matrix m
    __device__ void init(const gemv_args & p, const eng_geo & e, int64_t w, int64_t nwg) {
        np[0] = 0;
#pragma unroll
        for (int m = 0; m < GEMV_MAXMAT; ++m) {
            const int64_t M = m < e.nmat ? p.M[m] : 0;
            r0[m] = w * M / nwg;
            nr[m] = (w + 1) * M / nwg - r0[m];
            np[m + 1] = np[m] + (int) ((nr[m] + e.gp - 1) / e.gp);
        }
    }
    // element m of a three-entry array by selects: a runtime index into a private array would
    // put the array in scratch memory
    template <class V> __device__ static V sel(const V (&a)[GEMV_MAXMAT], int m) { return m == 0 ? a[0] : (m == 1 ? a[1] : a[2]); }
    // packet k: its matrix, first row (in the matrix) and row count
    __device__ void packet(const eng_geo & e, int k, int & m, int64_t & row, int & n) const {
        m = k >= np[2] ? 2 : (k >= np[1] ? 1 : 0);
        const int npm = m == 0 ? 0 : (m == 1 ? np[1] : np[2]);
        const int64_t i = (int64_t) (k - npm) * e.gp;
        row = sel(r0, m) + i;
        n = (int) min<int64_t>(e.gp, sel(nr, m) - i);
    }
};

template <class T, int NL, int NC, bool ONECH>
__global__ __launch_bounds__(64 * (NL + NC)) void k_gemv_eng(const gemv_args p, const eng_geo e) {
    using G = os_geo<T>;
    constexpr int BPC = WAVE / T::per_block; // blocks (records) per full chunk
    __shared__ __attribute__((aligned(16))) uint8_t lds[ENG_LDS];
    eng_ctrl * cc = (eng_ctrl *) lds;
    uint8_t * act = lds + ENG_CTRL;
    uint8_t * ring = lds + e.ring_off;
    kt_enter(p.kt);
    // the wave index as a wave-uniform (SGPR) value: every row / packet / slot computation of the
    // roles below is then scalar (derived from threadIdx it was VGPR math with quarter-rate
    // 32-bit multiplies, hundreds of cycles per row)
    const int wave = __builtin_amdgcn_readfirstlane((int) (threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int ns = e.ns, nch = e.nch, gp = e.gp;
    const int64_t w = blockIdx.x, nwg = gridDim.x;
    eng_work wk;
    wk.init(p, e, w, nwg);
    const int npk = wk.np[GEMV_MAXMAT];
    if (threadIdx.x < ENG_NSMAX) {
        cc->full[threadIdx.x] = -1;
        cc->fre[threadIdx.x] = (int) threadIdx.x - ns;   // "slot s held packet s - ns": the first round is free
        cc->cnt[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) cc->rdy = 0;
    __syncthreads();

    if (wave < NL) {
        // ---- loader l: packets l, l + NL, ... ----
        const int l = wave;
        const int ll = e.ll, pk = e.pk;
        int it = 0;
        const bool prof = p.eprof != nullptr && lane == 0;
        unsigned long long tw0 = prof ? __builtin_amdgcn_s_memtime() : 0, t_fre = 0, t_vm = 0;
        for (int k = l; k < npk; k += NL, ++it) {
            const int s = k % ns;
            if (prof) { const unsigned long long t = __builtin_amdgcn_s_memtime(); if (k >= ns) eng_wait_eq(&cc->fre[s], k - ns); t_fre += __builtin_amdgcn_s_memtime() - t; }
            else if (k >= ns) eng_wait_eq(&cc->fre[s], k - ns);
            int m, n;
            int64_t row;
            wk.packet(e, k, m, row, n);
            const uint8_t * src = (m == 0 ? p.W[0] : (m == 1 ? p.W[1] : p.W[2])) + row * e.rowb;
            eng_issue(src, ring + (size_t) s * e.slot, n * e.rowb, pk, lane, lds + e.trash_off);
            if (it >= ll) {
                const unsigned long long t = prof ? __builtin_amdgcn_s_memtime() : 0;
                eng_vmwait(ll * pk);
                if (prof) t_vm += __builtin_amdgcn_s_memtime() - t;
                const int kp = k - ll * NL;
                if (lane == 0) eng_st(&cc->full[kp % ns], kp);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            for (int kk = l + NL * max(0, it - ll); kk < npk; kk += NL) eng_st(&cc->full[kk % ns], kk);
        }
        if (prof) {
            unsigned long long * pe = p.eprof + 8 * w;
            atomicAdd(pe + 0, t_fre); atomicAdd(pe + 1, t_vm); atomicAdd(pe + 2, __builtin_amdgcn_s_memtime() - tw0);
            atomicAdd(pe + 3, (unsigned long long) it);
        }
    } else {
        // ---- consumers: packets c, c + NC, ... (every row of a packet by one wave) ----
        const int cw = wave - NL;
        eng_act<NC>(p, e, act, cw, lane, cc);
        // the residual rows go to LDS now: a global load in the packet loop would make the wave
        // wait vmcnt(0) there, i.e. for its previous outputs' stores as well (gfx9 counts stores
        // in vmcnt), a memory round trip per packet
        if (p.rres) {
            for (int i = cw * 64 + lane; i < wk.nr[0]; i += 64 * NC) cc->rres[i] = p.rres[wk.r0[0] + i];
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(&cc->rdy, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        eng_wait_eq(&cc->rdy, NC);
        const bool kq = e.qmode == 1;
        const int64_t nd = kq ? e.n / 256 : e.n / 32;
        const gemv_act A = {(const int8_t *) act, (const float *) (act + e.n), (const int16_t *) (act + e.n + 4 * nd)};
        // records of up to ENG_GPMAX rows of a chunk; walker lanes: row wr = lane / LPR, class ws
        uint32_t * rr = (uint32_t *) (lds + e.rec_off) + (size_t) cw * ENG_GPMAX * BPC * T::RS;
        const int nblk = p.ntasks / T::per_block;
        const int wr = lane / T::LPR, ws = lane % T::LPR;
        typename T::act x0;
        if constexpr (ONECH) T::load(A, lane < p.ntasks ? lane : 0, x0);
        double ss = 0.0;
        const bool prof = p.eprof != nullptr && lane == 0;
        unsigned long long tc0 = prof ? __builtin_amdgcn_s_memtime() : 0, t_full = 0, nrw = 0;
        int s = cw % ns;
        for (int k = cw; k < npk; k += NC) {
            int m, n;
            int64_t row0;
            wk.packet(e, k, m, row0, n);
            if (prof) { const unsigned long long t = __builtin_amdgcn_s_memtime(); eng_wait_eq(&cc->full[s], k); t_full += __builtin_amdgcn_s_memtime() - t; nrw += n; }
            else eng_wait_eq(&cc->full[s], k);
            const uint8_t * pb = ring + (size_t) s * e.slot;
            const int wrc = wr < n ? wr : n - 1;
            eng_walk<T> wkr;
            for (int j = 0; j < nch; ++j) {
                const int tg = WAVE * j + lane;            // the task in the row
                const bool active = tg < p.ntasks;
                typename T::act xj;
                if constexpr (!ONECH) T::load(A, active ? tg : 0, xj);
                const typename T::act & x = ONECH ? x0 : xj;
#pragma unroll
                for (int r = 0; r < ENG_GPMAX; ++r) {
                    if (r < n) {
                        typename T::raw wraw;
                        T::template fetch<typename lds_loader<T>::type>(pb + (size_t) r * e.rowb + (size_t) j * G::SEG, active ? lane : 0, wraw);
                        T::rec(wraw, lane, x, active, rr + (size_t) r * BPC * T::RS);
                    }
                }
                if (j == nch - 1) {
                    // every row's bytes have been read (a wave's LDS accesses complete in order)
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (lane == 0) eng_st(&cc->fre[s], k);
                }
                wave_lds_sync();
                wkr.step(rr + (size_t) wrc * BPC * T::RS, min(BPC, nblk - BPC * j), ws);
                asm volatile("" ::: "memory");
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
            }
            const float v = wkr.result();
            if (ws == 0 && wr < n) {
                const int64_t row = row0 + wr;
                if (p.rres) {   // ADD(v, res): the CPU's single f32 add (one matrix)
                    const float xv = __fadd_rn(v, cc->rres[row - wk.r0[0]]);
                    p.rxsum[row] = xv;
                    ss = __dadd_rn(ss, (double) __fmul_rn(xv, xv));
                } else {
                    (m == 0 ? p.dst[0] : (m == 1 ? p.dst[1] : p.dst[2]))[row] = v;
                }
            }
            s += NC;
            while (s >= ns) s -= ns;
        }
        ss = wave_sum(ss);   // the walker lanes' sums (the others hold 0)
        if (p.rres && lane == 0) cc->rpart[cw] = ss;
        if (prof) {
            unsigned long long * pe = p.eprof + 8 * w;
            atomicAdd(pe + 4, t_full); atomicAdd(pe + 5, __builtin_amdgcn_s_memtime() - tc0); atomicAdd(pe + 6, nrw);
        }
    }
    if (p.rres) {
        __syncthreads();
        if (threadIdx.x == 0) {
            double tot = 0.0;
#pragma unroll
            for (int c = 0; c < NC; ++c) tot = __dadd_rn(tot, cc->rpart[c]);
            __hip_atomic_fetch_add(p.rsum + RSUM_STRIDE * (w % RSUM_SHARDS), tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    kt_exit(p.kt);
}

// ---- host ----------------------------------------------------------------------------------------
// kernel-timing mode: the GEMV kernel itself is launched with start/stop events
// (hipExtLaunchKernel records them at the dispatch's start and completion, without extra
// marker packets around it), so bench.py's per-launch time is the kernel's own duration
static thread_local hipEvent_t t_ev_beg = nullptr, t_ev_end = nullptr;
// the launching context while a gemv_group runs (kernel timeline regions come from it)
static thread_local exec_ctx * g_kt_ctx = nullptr;

static int g_gemv_wgs = -1;    // the pipelined kernel's persistent grid (2048: 8 per CU)
static int g_num_cu = 0;
static std::once_flag g_gemv_once;   // several contexts may launch from several threads

static void gemv_init() {
    std::call_once(g_gemv_once, [] {
        g_gemv_wgs = 2048;
        int dev = 0;
        hipDeviceProp_t prop;
        MI_CHECK(hipGetDevice(&dev));
        MI_CHECK(hipGetDeviceProperties(&prop, dev));
        g_num_cu = prop.multiProcessorCount;
    });
}

static int64_t set_groups(gemv_args & a, int nmat, int rpg) {
    a.blk0[0] = 0;
    for (int i = 0; i < GEMV_MAXMAT; ++i) a.blk0[i + 1] = a.blk0[i] + (i < nmat ? ceil_div(a.M[i], rpg) : 0);
    for (int i = nmat; i < GEMV_MAXMAT; ++i) a.blk0[i] = a.blk0[nmat];   // never selected
    return a.blk0[nmat];
}

template <class T, int R, int WPR, int MODE>
static void launch_pipe_m(hipStream_t st, gemv_args & a, int nmat) {
    constexpr int RPG = (4 / WPR) * R;
    const int64_t ng = set_groups(a, nmat, RPG);
    int64_t grid = std::min<int64_t>(ng, g_gemv_wgs);
    if constexpr (WPR == 4 && !std::is_same<T, g_q6_K>::value) {
        // four waves per row (K = 14336, the FFN down projection): one resident round of
        // workgroups beats 2048 single-group workgroups in two rounds (Q4_K 4096 x 14336: 12.0 ->
        // 11.2 us at 5 per CU, scripts/probe_geom.py); with the residual producer's epilogue 3 per
        // CU (768) is faster again, 12.5 -> 11.2 us (scripts/gpu_trace_var.sh, round 2)
        grid = std::min<int64_t>(ng, 3 * g_num_cu);
    }
    if (a.pro.x) {
        // every workgroup forms the activation: one resident round (1024), so no
        // workgroup pays the prologue after the weight stream is under way
        grid = std::min<int64_t>(grid, 1024);
    }
    if (MODE >= 1 || a.tl.kind) grid = std::max<int64_t>(grid, ceil_div(ng, GEMV_MAXG));   // LDS-parked row sums / tail lists
    size_t lds = 4 * xrec_dwords<T>(RPG, a.ntasks / T::per_block);
    if (a.pro.x) {   // the prologue's activation follows the records
        lds = (lds + 15) / 16 * 16;
        a.pro.lds_off = (uint32_t) lds;
        lds += pro_lds_bytes(a.pro.n, a.pro.qmode);
    }
    if (g_kt_ctx) {
        // timeline label: the fused pieces of this launch
        static const char * names[16] = {"gemv", "gemv+pro", "gemv+epi", "gemv+pro+epi", "gemv+tail", "gemv+pro+tail",
                                         "gemv+epi+tail", "gemv+pro+epi+tail", "gemv+resid", "gemv+pro+resid",
                                         "gemv+epi+resid", "gemv+pro+epi+resid", "gemv+tail+resid", "gemv+pro+tail+resid",
                                         "gemv+epi+tail+resid", "gemv+all"};
        const int k = (a.pro.x ? 1 : 0) | (MODE ? 2 : 0) | (a.tl.kind ? 4 : 0) | (a.rres ? 8 : 0);
        a.kt = g_kt_ctx->kt_take(names[k], (unsigned) grid, 256);
    }
    if (t_ev_beg) {
        hipExtLaunchKernelGGL((k_gemv_pipe<T, R, WPR, MODE>), dim3((unsigned) grid), dim3(256), lds, st, t_ev_beg, t_ev_end, 0, a, ng);
    } else {
        hipLaunchKernelGGL((k_gemv_pipe<T, R, WPR, MODE>), dim3((unsigned) grid), dim3(256), lds, st, a, ng);
    }
}

static bool needs_epilogue(const gemv_args & a, int nmat) {
    bool epi = a.need_pairs;
    for (int i = 0; i < nmat; ++i) epi = epi || (!a.dst[i] && !a.rres) || a.silu[i] || a.f16out[i] || a.rope_out[i] || a.rope_f16[i];
    return epi;
}

template <class T, int R, int WPR>
static void launch_pipe(hipStream_t st, gemv_args & a, int nmat) {
    GGML_ASSERT(!((a.tl.kind || a.rres) && needs_epilogue(a, nmat)) && "mi355x: GEMV tail / residual with epilogues");
    if (needs_epilogue(a, nmat)) launch_pipe_m<T, R, WPR, 1>(st, a, nmat);
    else launch_pipe_m<T, R, WPR, 0>(st, a, nmat);
}

static int wpr_of(int ntasks) { return ntasks <= WAVE ? 1 : (ntasks <= 2 * WAVE ? 2 : 4); }

// ---- one-shot launches (k_gemv_os): one row group per workgroup ---------------------------------
// GGML_MI355X_GEMV_OS=0 keeps the persistent pipelined kernel (A/B only)
static bool os_enabled() {
    static const bool on = !getenv("GGML_MI355X_GEMV_OS") || atoi(getenv("GGML_MI355X_GEMV_OS")) != 0;
    return on;
}

static inline size_t r16(size_t x) { return (x + 15) / 16 * 16; }

// LDS-DMA moves 16-B pieces: every row slice must start 16-B aligned and end on a 16-B boundary
template <class T>
static bool os_aligned(const gemv_args & a, int nmat) {
    const int wpr = a.ntasks <= WAVE ? 1 : (a.ntasks <= 2 * WAVE ? 2 : 4);
    const int nt_last = a.ntasks - WAVE * (wpr - 1);
    if ((os_geo<T>::SEG % 16) != 0 || ((nt_last / T::per_block) * T::blk_bytes) % 16 != 0) return false;
    for (int i = 0; i < nmat; ++i) {
        if (((uintptr_t) a.W[i] % 16) != 0 || (a.nb01[i] % 16) != 0) return false;
    }
    return true;
}

template <class T, int R, int WPR>
static size_t os_lds_layout(gemv_args & a) {
    constexpr int RPG = (4 / WPR) * R;
    size_t off = r16((size_t) RPG * (a.ntasks / T::per_block) * T::RS * 4);
    if (a.pro.x) {
        a.pro.lds_off = (uint32_t) off;
        off = r16(off + pro_lds_bytes(a.pro.n, a.pro.qmode));
    }
    a.wl_off = (uint32_t) off;
    return off + (size_t) 4 * R * os_geo<T>::SLICE;
}

static const char * gemv_kt_name(const gemv_args & a, int mode) {
    static const char * names[16] = {"gemv", "gemv+pro", "gemv+epi", "gemv+pro+epi", "gemv+tail", "gemv+pro+tail",
                                     "gemv+epi+tail", "gemv+pro+epi+tail", "gemv+resid", "gemv+pro+resid",
                                     "gemv+epi+resid", "gemv+pro+epi+resid", "gemv+tail+resid", "gemv+pro+tail+resid",
                                     "gemv+epi+tail+resid", "gemv+all"};
    return names[(a.pro.x ? 1 : 0) | (mode ? 2 : 0) | (a.tl.kind ? 4 : 0) | (a.rres ? 8 : 0)];
}

template <class T, int R, int WPR, int MODE>
static void launch_os_m(hipStream_t st, gemv_args & a, int nmat) {
    constexpr int RPG = (4 / WPR) * R;
    const int64_t ng = set_groups(a, nmat, RPG);
    const size_t lds = os_lds_layout<T, R, WPR>(a);
    a.kt = g_kt_ctx ? g_kt_ctx->kt_take(gemv_kt_name(a, MODE), (unsigned) ng, 256) : nullptr;
    // SwiGLU tail: one more workgroup per Q8_K block of the product, after the row groups
    int64_t grid = ng;
    if (a.tl.kind) {
        GGML_ASSERT(MODE == 0 && nmat == 2 && a.tl.n % 256 == 0 && 256 % RPG == 0 && a.blk0[GEMV_MAXMAT] == ng);
        GGML_ASSERT(a.M[0] == a.tl.n && a.M[1] == a.tl.n);
        grid += a.tl.n / 256;
    }
#define OS_LAUNCH(P)                                                                                              \
    if (t_ev_beg) hipExtLaunchKernelGGL((k_gemv_os<T, R, WPR, MODE, P>), dim3((unsigned) grid), dim3(256), lds, st, t_ev_beg, t_ev_end, 0, a); \
    else hipLaunchKernelGGL((k_gemv_os<T, R, WPR, MODE, P>), dim3((unsigned) grid), dim3(256), lds, st, a)
    if (a.pro.x) { OS_LAUNCH(true); } else { OS_LAUNCH(false); }
#undef OS_LAUNCH
}

// GGML_MI355X_OSL = workgroups per CU of the looping one-shot kernel (0: off, the default)
static int osl_per_cu() {
    static const int v = getenv("GGML_MI355X_OSL") ? atoi(getenv("GGML_MI355X_OSL")) : 0;
    return v;
}

template <class T, int R, int WPR>
static bool launch_osl(hipStream_t st, gemv_args & a, int nmat) {
    constexpr int RPG = (4 / WPR) * R;
    const int64_t ng = set_groups(a, nmat, RPG);
    const size_t rec = r16((size_t) RPG * (a.ntasks / T::per_block) * T::RS * 4);
    a.wl_off = (uint32_t) rec;
    const size_t lds = rec + (size_t) 4 * 2 * R * os_geo<T>::SLICE;
    if (lds > 64 * 1024) return false;
    const int64_t grid = std::min<int64_t>(ng, (int64_t) osl_per_cu() * g_num_cu);
    a.kt = g_kt_ctx ? g_kt_ctx->kt_take(a.rres ? "gemvl+resid" : "gemvl", (unsigned) grid, 256) : nullptr;
    if (t_ev_beg) hipExtLaunchKernelGGL((k_gemv_osl<T, R, WPR>), dim3((unsigned) grid), dim3(256), lds, st, t_ev_beg, t_ev_end, 0, a);
    else hipLaunchKernelGGL((k_gemv_osl<T, R, WPR>), dim3((unsigned) grid), dim3(256), lds, st, a);
    return true;
}

template <class T, int R, int WPR>
static void launch_os(hipStream_t st, gemv_args & a, int nmat) {
    if (osl_per_cu() > 0 && !needs_epilogue(a, nmat) && !a.pro.x && !a.tl.kind && launch_osl<T, R, WPR>(st, a, nmat)) return;
    if (needs_epilogue(a, nmat)) launch_os_m<T, R, WPR, 1>(st, a, nmat);
    else launch_os_m<T, R, WPR, 0>(st, a, nmat);
}

// rows per wave of the one-shot kernel (tools/gemv_lab.hip, round 3; round 4 below): two for the
// 4-bit K-quants at K = 14336, two (four at K <= 4096) wherever a norm prologue is formed per
// workgroup (fewer workgroups form it), and two for the plain one-wave-per-row launches
template <class T>
static bool launch_os_t(hipStream_t st, gemv_args & a, int nmat) {
    if (!os_enabled() || !os_aligned<T>(a, nmat)) return false;
    if (a.tl.kind && needs_epilogue(a, nmat)) return false;
    const int wpr = wpr_of(a.ntasks);
    int R = 1;
    if (a.pro.x || (wpr == 4 && !std::is_same<T, g_q6_K>::value)) R = 2;
    if (a.pro.x && wpr == 1) R = 4;   // a norm prologue per workgroup: half as many of them (9.9 -> 9.3 us)
    // with one walking wave per workgroup, two rows per wave for the plain (no prologue / epilogue)
    // launches: gate/up 16.5 -> 14.9 us (scripts/probe_mall_gemv.py, round 4); the 6-bit output
    // head keeps one (71 vs 77 us). GGML_MI355X_OS_R overrides it (A/B only)
    if (!a.pro.x && wpr == 1 && !needs_epilogue(a, nmat) && !std::is_same<T, g_q6_K>::value) R = 2;
    static const int r_env = getenv("GGML_MI355X_OS_R") ? atoi(getenv("GGML_MI355X_OS_R")) : 0;
    if (r_env > 0 && !a.pro.x && wpr == 1 && !needs_epilogue(a, nmat)) R = r_env;
    if (wpr == 4 && needs_epilogue(a, nmat)) return false;   // rope pairs need an even group
    gemv_args b = a;
    const size_t lds = R == 4 ? os_lds_layout<T, 4, 1>(b)
                     : R == 2 ? (wpr == 1 ? os_lds_layout<T, 2, 1>(b) : wpr == 2 ? os_lds_layout<T, 2, 2>(b) : os_lds_layout<T, 2, 4>(b))
                              : (wpr == 1 ? os_lds_layout<T, 1, 1>(b) : wpr == 2 ? os_lds_layout<T, 1, 2>(b) : os_lds_layout<T, 1, 4>(b));
    if (lds > 64 * 1024) return false;
    switch (R * 8 + wpr) {
        case 4 * 8 + 1: launch_os<T, 4, 1>(st, a, nmat); break;
        case 2 * 8 + 1: launch_os<T, 2, 1>(st, a, nmat); break;
        case 2 * 8 + 2: launch_os<T, 2, 2>(st, a, nmat); break;
        case 2 * 8 + 4: launch_os<T, 2, 4>(st, a, nmat); break;
        case 1 * 8 + 1: launch_os<T, 1, 1>(st, a, nmat); break;
        case 1 * 8 + 2: launch_os<T, 1, 2>(st, a, nmat); break;
        default:        launch_os<T, 1, 4>(st, a, nmat); break;
    }
    return true;
}

// two weight types in one one-shot launch: p1's matrices at two rows per wave, p2's at R2
template <class T1, class T2, int R2, int WPR, int R1 = 2>
static void launch_os2_v(hipStream_t st, gemv_args & a1, int n1, gemv_args & a2, int n2) {
    constexpr int NWV = 4;
    const int64_t ng1 = set_groups(a1, n1, (NWV / WPR) * R1), ng2 = set_groups(a2, n2, (NWV / WPR) * R2);
    size_t rec = r16(std::max((size_t) (NWV / WPR) * R1 * (a1.ntasks / T1::per_block) * T1::RS * 4,
                              (size_t) (NWV / WPR) * R2 * (a2.ntasks / T2::per_block) * T2::RS * 4));
    size_t off = rec;
    if (a1.pro.x) {
        a1.pro.lds_off = a2.pro.lds_off = (uint32_t) off;
        off = r16(off + pro_lds_bytes(a1.pro.n, a1.pro.qmode));
    }
    a1.wl_off = a2.wl_off = (uint32_t) off;
    const size_t lds = off + std::max((size_t) 4 * R1 * os_geo<T1>::SLICE, (size_t) 4 * R2 * os_geo<T2>::SLICE);
    a1.kt = g_kt_ctx ? g_kt_ctx->kt_take("gemv2+pro+epi", (unsigned) (ng1 + ng2), 64 * NWV) : nullptr;
#define OS2_LAUNCH(P)                                                                                                 \
    if (t_ev_beg) hipExtLaunchKernelGGL((k_gemv_os2<T1, T2, R2, WPR, P, R1>), dim3((unsigned) (ng1 + ng2)), dim3(64 * NWV), lds, st, t_ev_beg, \
                                        t_ev_end, 0, a1, ng1, a2);                                                        \
    else hipLaunchKernelGGL((k_gemv_os2<T1, T2, R2, WPR, P, R1>), dim3((unsigned) (ng1 + ng2)), dim3(64 * NWV), lds, st, a1, ng1, a2)
    if (a1.pro.x) { OS2_LAUNCH(true); } else { OS2_LAUNCH(false); }
#undef OS2_LAUNCH
}

// ---- engine launches (k_gemv_eng) -----------------------------------------------------------------
// GGML_MI355X_GEMV_ENG=1 selects the engine (A/B while it is measured); GGML_MI355X_ENG_NC = consumer waves (3, 7, 15)
static bool eng_enabled() {
    static const bool on = getenv("GGML_MI355X_GEMV_ENG") && atoi(getenv("GGML_MI355X_GEMV_ENG")) != 0;
    return on;
}
// loader / consumer waves per workgroup: GGML_MI355X_ENG_CFG = 17 (1 + 7), 26, 214 (default), 412
static int eng_cfg() {
    static const int c = [] {
        const int v = getenv("GGML_MI355X_ENG_CFG") ? atoi(getenv("GGML_MI355X_ENG_CFG")) : 412;
        return v == 214 || v == 88 || v == 610 ? v : 412;
    }();
    return c;
}
static int eng_nc() { const int c = eng_cfg(); return c == 214 ? 14 : (c == 88 ? 8 : (c == 610 ? 10 : 12)); }
static int eng_nl() { const int c = eng_cfg(); return c == 214 ? 2 : (c == 88 ? 8 : (c == 610 ? 6 : 4)); }
// engine phase counters of the microbenchmark (capi mi355x_bench_gemv2, GGML_MI355X_ENG_PROF):
// per workgroup 8 counters, s_memtime ticks summed over waves
unsigned long long * g_eng_prof = nullptr;
// the SwiGLU prologue's sources for the next engine launch (gemv_group sets them)
static thread_local const float * g_sw_gate = nullptr;
static thread_local const float * g_sw_up = nullptr;

template <class T>
static bool eng_geometry(const gemv_args & a, int nmat, int nc, eng_geo & e) {
    constexpr int BPC = WAVE / T::per_block;
    e.nch = (int) ceil_div(a.ntasks, WAVE);
    const int last_tasks = a.ntasks - WAVE * (e.nch - 1);
    e.last_bytes = (last_tasks / T::per_block) * T::blk_bytes;
    constexpr bool kq = T::per_block == 4;
    e.qmode = kq ? 1 : 2;
    e.n = (int64_t) (a.ntasks / T::per_block) * (kq ? 256 : 32);
    e.rowb = (a.ntasks / T::per_block) * T::blk_bytes;
    if (e.n % 256 != 0 || e.n > 16384 || e.rowb % 16 != 0 || e.last_bytes % 16 != 0) return false;
    for (int i = 0; i < nmat; ++i) {
        if (a.nb01[i] != e.rowb) return false;   // packets are contiguous rows
    }
    e.nmat = nmat;
    // rows per packet: the most (up to 4) whose bytes fill whole KiB within 1/32 (12 KiB at most)
    e.gp = 1;
    for (int g = 4; g >= 1; --g) {
        const int by = g * e.rowb, kib = (by + 1023) / 1024;
        if (kib <= 12 && (kib * 1024 - by) * 32 <= kib * 1024) { e.gp = g; break; }
    }
    e.pk = (e.gp * e.rowb + 1023) / 1024;
    if (e.pk > 16) return false;
    e.rec_off = (uint32_t) (ENG_CTRL + r16(pro_lds_bytes(e.n, e.qmode)));
    e.ring_off = (uint32_t) ((e.rec_off + (size_t) nc * ENG_GPMAX * BPC * T::RS * 4 + 1023) / 1024 * 1024);
    e.slot = (uint32_t) (e.pk * 1024);
    e.trash_off = (uint32_t) (ENG_LDS - 1024);
    e.ns = (int) std::min<int64_t>(ENG_NSMAX, (ENG_LDS - 1024 - (int64_t) e.ring_off) / e.slot);
    // packets in flight per loader: what the ring holds beside the consumers' working set (a
    // packet per gp consumer rows), within vmcnt's 63 instructions per loader wave
    const int nl = eng_nl();
    // (no deadlock while ns > ll * nl: a loader publishes packet k once it has issued k + ll * nl)
    e.ll = std::min(63 / e.pk, (e.ns - 1 - nc / 4) / nl);
    return e.ll >= 1;
}

template <class T, int NL, int NC>
static void launch_eng_v(hipStream_t st, gemv_args & a, const eng_geo & e) {
    const unsigned grid = (unsigned) g_num_cu;
    a.kt = g_kt_ctx ? g_kt_ctx->kt_take(a.rres ? "eng+resid" : (e.act_mode == 1 ? "eng+pro" : (e.act_mode == 2 ? "eng+swiglu" : "eng")),
                                        grid, 64 * (NL + NC)) : nullptr;
#define ENG_LAUNCH(OC)                                                                                                  \
    if (t_ev_beg) hipExtLaunchKernelGGL((k_gemv_eng<T, NL, NC, OC>), dim3(grid), dim3(64 * (NL + NC)), 0, st, t_ev_beg, t_ev_end, 0, a, e); \
    else hipLaunchKernelGGL((k_gemv_eng<T, NL, NC, OC>), dim3(grid), dim3(64 * (NL + NC)), 0, st, a, e)
    if (e.nch == 1) { ENG_LAUNCH(true); } else { ENG_LAUNCH(false); }
#undef ENG_LAUNCH
}

template <class T>
static bool launch_eng_t(hipStream_t st, gemv_args & a, int nmat) {
    if (!eng_enabled() || a.tl.kind || needs_epilogue(a, nmat) || !os_aligned<T>(a, nmat)) return false;
    const int nc = eng_nc();
    eng_geo e = {};
    if (!eng_geometry<T>(a, nmat, nc, e)) return false;
    set_groups(a, nmat, 1);
    e.act_mode = g_sw_gate ? 2 : (a.pro.x ? 1 : 0);
    e.sw_gate = g_sw_gate;
    e.sw_up = g_sw_up;
    a.eprof = g_eng_prof;
    if (e.act_mode == 1 && a.pro.qmode != e.qmode) return false;
    if (a.rres && (nmat != 1 || ceil_div(a.M[0], g_num_cu) > ENG_RMAX)) return false;
    switch (eng_cfg()) {
        case 214: launch_eng_v<T, 2, 14>(st, a, e); break;
        case 88:  launch_eng_v<T, 8, 8>(st, a, e); break;
        case 610: launch_eng_v<T, 6, 10>(st, a, e); break;
        default:  launch_eng_v<T, 4, 12>(st, a, e); break;
    }
    return true;
}

// the engine takes this mat-vec (one activation column, no register epilogues) — the
// dispatcher's test before it plans a prologue (norm / SwiGLU) that only the engine forms
bool gemv_engine_ok(const ggml_tensor * mm) {
    if (!eng_enabled() || !gemv_supported(mm)) return false;
    const ggml_tensor * w = mm->src[0];
    gemv_args a = {};
    a.W[0] = (const uint8_t *) w->data;
    a.nb01[0] = w->nb[1];
    a.M[0] = w->ne[1];
    const int64_t nblk = w->ne[0] / ggml_blck_size(w->type);
    eng_geo e = {};
    switch (w->type) {
        case GGML_TYPE_Q4_K: a.ntasks = (int) (nblk * 4); return os_aligned<g_q4_K>(a, 1) && eng_geometry<g_q4_K>(a, 1, eng_nc(), e);
        case GGML_TYPE_Q5_K: a.ntasks = (int) (nblk * 4); return os_aligned<g_q5_K>(a, 1) && eng_geometry<g_q5_K>(a, 1, eng_nc(), e);
        case GGML_TYPE_Q6_K: a.ntasks = (int) (nblk * 4); return os_aligned<g_q6_K>(a, 1) && eng_geometry<g_q6_K>(a, 1, eng_nc(), e);
        case GGML_TYPE_Q8_0: a.ntasks = (int) nblk;       return os_aligned<g_q8_0>(a, 1) && eng_geometry<g_q8_0>(a, 1, eng_nc(), e);
        case GGML_TYPE_Q4_0: a.ntasks = (int) nblk;       return os_aligned<g_q4_0>(a, 1) && eng_geometry<g_q4_0>(a, 1, eng_nc(), e);
        default: return false;
    }
}

template <class T>
static void launch_t(hipStream_t st, gemv_args & a, int nmat) {
    if (launch_eng_t<T>(st, a, nmat)) return;
    GGML_ASSERT(!g_sw_gate && "mi355x: SwiGLU prologue without the engine");
    if (launch_os_t<T>(st, a, nmat)) return;
    int64_t Mt = 0;
    for (int i = 0; i < nmat; ++i) Mt += a.M[i];
    GGML_ASSERT(a.ntasks <= 4 * WAVE);
    const int wpr = wpr_of(a.ntasks);
    // geometry measured on MI355X (tools/gemv_lab.hip, back-to-back launches over cold
    // weights): two rows per wave and a grid of up to 2048 workgroups is the fastest or within
    // 5 % of it on every Llama-3-8B shape; the 6-bit K-quant at K = 14336 prefers four rows;
    // a matrix too short to give 256 workgroups at two rows per wave takes one (the rope
    // epilogue reads its partner row from the LDS-parked sums of the same group)
    int R = 2;
    if (std::is_same<T, g_q6_K>::value && wpr == 4) R = 4;
    if (ceil_div(Mt * wpr, 8) < 256) R = 1;
    switch (R * 8 + wpr) {
        case 4 * 8 + 1: launch_pipe<T, 4, 1>(st, a, nmat); break;
        case 4 * 8 + 2: launch_pipe<T, 4, 2>(st, a, nmat); break;
        case 4 * 8 + 4: launch_pipe<T, 4, 4>(st, a, nmat); break;
        case 2 * 8 + 1: launch_pipe<T, 2, 1>(st, a, nmat); break;
        case 2 * 8 + 2: launch_pipe<T, 2, 2>(st, a, nmat); break;
        case 2 * 8 + 4: launch_pipe<T, 2, 4>(st, a, nmat); break;
        case 1 * 8 + 1: launch_pipe<T, 1, 1>(st, a, nmat); break;
        case 1 * 8 + 2: launch_pipe<T, 1, 2>(st, a, nmat); break;
        default:        launch_pipe<T, 1, 4>(st, a, nmat); break;
    }
}

// two weight types in one launch (k_gemv_pipe2): p1's matrices at two rows per wave, p2's at
// R2 by the single-type rule
template <class T1, class T2, int R2, int WPR>
static void launch_pipe2_v(hipStream_t st, gemv_args & a1, int n1, gemv_args & a2, int n2) {
    constexpr int NWV = 4;
    const int64_t ng1 = set_groups(a1, n1, (NWV / WPR) * 2), ng2 = set_groups(a2, n2, (NWV / WPR) * R2);
    auto grid_of = [](int64_t ng) {
        return std::max<int64_t>(std::min<int64_t>(ng, g_gemv_wgs), ceil_div(ng, GEMV_MAXG));   // LDS-parked row sums
    };
    const int64_t w1 = grid_of(ng1), w2 = grid_of(ng2);
    size_t lds = 4 * std::max(xrec_dwords<T1>((NWV / WPR) * 2, a1.ntasks / T1::per_block),
                               xrec_dwords<T2>((NWV / WPR) * R2, a2.ntasks / T2::per_block));
    if (a1.pro.x) {   // the prologue's activation follows the records (both bodies)
        lds = (lds + 15) / 16 * 16;
        a1.pro.lds_off = a2.pro.lds_off = (uint32_t) lds;
        lds += pro_lds_bytes(a1.pro.n, a1.pro.qmode);
    }
    a1.kt = g_kt_ctx ? g_kt_ctx->kt_take("gemv_pipe2", (unsigned) (w1 + w2), 64 * NWV) : nullptr;
    if (t_ev_beg) {
        hipExtLaunchKernelGGL((k_gemv_pipe2<T1, T2, R2, WPR>), dim3((unsigned) (w1 + w2)), dim3(64 * NWV), lds, st, t_ev_beg, t_ev_end,
                              0, a1, ng1, w1, a2, ng2);
    } else {
        hipLaunchKernelGGL((k_gemv_pipe2<T1, T2, R2, WPR>), dim3((unsigned) (w1 + w2)), dim3(64 * NWV), lds, st, a1, ng1, w1, a2, ng2);
    }
}

template <class T1, class T2>
static bool launch_pipe2_t(hipStream_t st, gemv_args & a1, int n1, gemv_args & a2, int n2) {
    if (a1.ntasks != a2.ntasks || a1.ntasks > 2 * WAVE) return false;
    const int wpr = a1.ntasks <= WAVE ? 1 : 2;
    int64_t m1 = 0, m2 = 0;
    for (int i = 0; i < n1; ++i) m1 += a1.M[i];
    for (int i = 0; i < n2; ++i) m2 += a2.M[i];
    if (os_enabled() && os_aligned<T1>(a1, n1) && os_aligned<T2>(a2, n2)) {
        // one-shot: the second type at one row per wave (two rows for the prologue consumers)
        // with the norm prologue formed per workgroup: four rows per wave for the first type (half
        // the prologues; Q/K/V 10.1 -> 9.1 us, in-graph timeline round 3), two for the second
        if (wpr == 1 && a1.pro.x) launch_os2_v<T1, T2, 2, 1, 4>(st, a1, n1, a2, n2);
        else if (wpr == 1) launch_os2_v<T1, T2, 1, 1>(st, a1, n1, a2, n2);
        else launch_os2_v<T1, T2, 1, 2>(st, a1, n1, a2, n2);
        return true;
    }
    // the single-type launch's rows-per-wave rule (launch_t), per part
    if (ceil_div(m1 * wpr, 8) < 256) return false;
    const int r2 = ceil_div(m2 * wpr, 8) < 256 ? 1 : 2;
    switch (r2 * 8 + wpr) {
        case 1 * 8 + 1: launch_pipe2_v<T1, T2, 1, 1>(st, a1, n1, a2, n2); break;
        case 1 * 8 + 2: launch_pipe2_v<T1, T2, 1, 2>(st, a1, n1, a2, n2); break;
        case 2 * 8 + 1: launch_pipe2_v<T1, T2, 2, 1>(st, a1, n1, a2, n2); break;
        default:        launch_pipe2_v<T1, T2, 2, 2>(st, a1, n1, a2, n2); break;
    }
    return true;
}

// Q/K/V of two K-quant types (gemv_group); false: launch the parts separately
static bool launch_mixed(hipStream_t st, ggml_type t1, gemv_args & a1, int n1, ggml_type t2, gemv_args & a2, int n2) {
    if (t1 == GGML_TYPE_Q4_K && t2 == GGML_TYPE_Q6_K) return launch_pipe2_t<g_q4_K, g_q6_K>(st, a1, n1, a2, n2);
    if (t1 == GGML_TYPE_Q4_K && t2 == GGML_TYPE_Q5_K) return launch_pipe2_t<g_q4_K, g_q5_K>(st, a1, n1, a2, n2);
    if (t1 == GGML_TYPE_Q5_K && t2 == GGML_TYPE_Q6_K) return launch_pipe2_t<g_q5_K, g_q6_K>(st, a1, n1, a2, n2);
    return false;
}

bool gemv_mixed_ok(const ggml_tensor * mm0, const ggml_tensor * c) {
    const ggml_type t1 = mm0->src[0]->type, t2 = c->src[0]->type;
    return ((t1 == GGML_TYPE_Q4_K && (t2 == GGML_TYPE_Q6_K || t2 == GGML_TYPE_Q5_K)) ||
                  (t1 == GGML_TYPE_Q5_K && t2 == GGML_TYPE_Q6_K));
}

static bool is_kq(ggml_type t) { return t == GGML_TYPE_Q4_K || t == GGML_TYPE_Q5_K || t == GGML_TYPE_Q6_K; }

// one activation column, a matrix the pipelined kernel covers in one pass per wave (at most
// 256 tasks), and — for the types the CPU repacks — the repacked order's row multiple
bool gemv_supported(const ggml_tensor * mm) {
    const ggml_tensor * w = mm->src[0];
    const ggml_tensor * x = mm->src[1];
    split_parts sp;
    if (tensor_split_parts(w, sp)) return false;   // row-split weights: op_mul_mat_split, never grouped
    int per = 0;
    switch (w->type) {
        case GGML_TYPE_Q4_K: case GGML_TYPE_Q4_0:
            if (w->ne[1] % 8 != 0) return false;   // not repacked: vec_dot order (k_mmv.hip)
            per = w->type == GGML_TYPE_Q4_K ? 4 : 1;
            break;
        case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K: per = 4; break;
        case GGML_TYPE_Q8_0: per = 1; break;
        default: return false;
    }
    if (w->ne[0] % ggml_blck_size(w->type) != 0 || (w->ne[0] / ggml_blck_size(w->type)) * per > 4 * WAVE) return false;
    return x->type == GGML_TYPE_F32 && x->ne[1] == 1 && x->ne[2] == 1 && x->ne[3] == 1 && w->ne[2] == 1 && w->ne[3] == 1 &&
           mm->type == GGML_TYPE_F32 && ggml_is_contiguous(mm) && x->nb[0] == 4 && w->nb[0] == ggml_type_size(w->type);
}

bool gemv_epilogue_ok(const ggml_tensor * mm) { return gemv_supported(mm); }

// ---- chained FFN launch (host) ------------------------------------------------------------------
// GGML_MI355X_FFN=1: gate/up with a SwiGLU tail is held back until its down projection arrives,
// then both go out as one k_gemv_ffn grid (any other node in between launches it alone first)
static bool ffn_enabled() {
    static const bool on = getenv("GGML_MI355X_FFN") && atoi(getenv("GGML_MI355X_FFN")) != 0;
    return on;
}

struct ffn_state {
    gemv_args a1;
    int n1 = 0;
    ggml_type t1 = GGML_TYPE_COUNT;
};

static ffn_state & ffn_of(exec_ctx & ctx) {
    if (!ctx.ffn) ctx.ffn = new ffn_state();
    return *(ffn_state *) ctx.ffn;
}

void gemv_ffn_release(exec_ctx & ctx) {
    delete (ffn_state *) ctx.ffn;
    ctx.ffn = nullptr;
    ctx.ffn_down = nullptr;
}

static void launch_by_type(hipStream_t st, ggml_type t, gemv_args & a, int nmat) {
    switch (t) {
        case GGML_TYPE_Q4_K: launch_t<g_q4_K>(st, a, nmat); break;
        case GGML_TYPE_Q5_K: launch_t<g_q5_K>(st, a, nmat); break;
        case GGML_TYPE_Q6_K: launch_t<g_q6_K>(st, a, nmat); break;
        case GGML_TYPE_Q8_0: launch_t<g_q8_0>(st, a, nmat); break;
        case GGML_TYPE_Q4_0: launch_t<g_q4_0>(st, a, nmat); break;
        default: GGML_ABORT("mi355x: gemv type");
    }
}

// the held-back gate/up goes out alone (something other than its down projection comes next)
void gemv_ffn_flush(exec_ctx & ctx) {
    if (!ctx.ffn_down) return;
    ffn_state & f = ffn_of(ctx);
    ctx.ffn_down = nullptr;
    g_kt_ctx = ctx.kt_buf && ktrace_enabled() ? &ctx : nullptr;
    launch_by_type(ctx.stream, f.t1, f.a1, f.n1);
    g_kt_ctx = nullptr;
}

// the one-shot geometry rule of launch_os_t (no prologue): rows per wave and waves per row
template <class T>
static void os_rule(const gemv_args & a, int & R, int & wpr) {
    wpr = wpr_of(a.ntasks);
    R = (wpr == 4 && !std::is_same<T, g_q6_K>::value) ? 2 : 1;
}

template <class T1, int R1, int WPR1, class T2, int R2, int WPR2>
static bool launch_ffn_v(exec_ctx & ctx, gemv_args & a1, int n1, gemv_args & a2, int * done) {
    constexpr int RPG1 = (4 / WPR1) * R1, RPG2 = (4 / WPR2) * R2;
    const int64_t ng1 = set_groups(a1, n1, RPG1), ng2 = set_groups(a2, 1, RPG2);
    if (256 % RPG1 != 0 || a1.M[0] != a1.tl.n || a1.M[1] != a1.tl.n) return false;
    const size_t l1 = os_lds_layout<T1, R1, WPR1>(a1), l2 = os_lds_layout<T2, R2, WPR2>(a2);
    const size_t lds = std::max(l1, l2);
    if (lds > 64 * 1024) return false;
    const int64_t nt = a1.tl.n / 256;
    a2.dep = done;
    a2.dep_n = (int) nt;
    const int64_t grid = ng1 + nt + ng2;
    a1.kt = g_kt_ctx ? g_kt_ctx->kt_take("ffn", (unsigned) grid, 256) : nullptr;
    a2.kt = nullptr;
    if (a1.kt) {
        // the timeline shows the three parts as their own rows (one region, three ranges)
        const auto l = g_kt_ctx->kt_list.back();
        g_kt_ctx->kt_list.pop_back();
        g_kt_ctx->kt_list.push_back({"ffn:gate_up", l.off, (unsigned) ng1, l.stride});
        g_kt_ctx->kt_list.push_back({"ffn:tail", l.off + (size_t) ng1 * l.stride, (unsigned) nt, l.stride});
        g_kt_ctx->kt_list.push_back({"ffn:down", l.off + (size_t) (ng1 + nt) * l.stride, (unsigned) ng2, l.stride});
    }
    hipLaunchKernelGGL((k_gemv_ffn<T1, R1, WPR1, T2, R2, WPR2>), dim3((unsigned) grid), dim3(256), lds, ctx.stream, a1, a2, done);
    return true;
}

// gate/up (Q4_K, one row per wave) with a Q4_K / Q6_K down projection at K <= 256 tasks
static bool launch_ffn(exec_ctx & ctx, ffn_state & f, ggml_type t2, gemv_args & a2) {
    if (f.t1 != GGML_TYPE_Q4_K || f.n1 != 2 || !os_enabled() || a2.tl.kind || a2.pro.x || needs_epilogue(a2, 1) ||
        needs_epilogue(f.a1, 2) || f.a1.tl.qmode != 1) return false;
    if (!os_aligned<g_q4_K>(f.a1, 2)) return false;
    int R1, W1, R2, W2;
    os_rule<g_q4_K>(f.a1, R1, W1);
    if (R1 != 1 || W1 != 1) return false;
    int * done = (int *) gemv_rsum_site(ctx);   // zeroed per graph (run_nodes)
    if (!done) return false;
    gemv_args a1 = f.a1;
    if (t2 == GGML_TYPE_Q4_K) {
        // one row per workgroup here (not the stand-alone launch's two): the grid's dynamic LDS is
        // the larger part's, and two-row down groups (31 KB) would cut the gate/up part from
        // eight resident workgroups per CU to five
        os_rule<g_q4_K>(a2, R2, W2);
        if (!os_aligned<g_q4_K>(a2, 1) || W2 != 4) return false;
        return launch_ffn_v<g_q4_K, 1, 1, g_q4_K, 1, 4>(ctx, a1, 2, a2, done);
    }
    if (t2 == GGML_TYPE_Q6_K) {
        os_rule<g_q6_K>(a2, R2, W2);
        if (!os_aligned<g_q6_K>(a2, 1) || R2 != 1 || W2 != 4) return false;
        return launch_ffn_v<g_q4_K, 1, 1, g_q6_K, 1, 4>(ctx, a1, 2, a2, done);
    }
    return false;
}

// one launch for up to three MUL_MATs sharing src1 (all gemv_supported, same K; a second
// K-quant type joins as the second body of k_gemv_pipe2)
void gemv_group(exec_ctx & ctx, ggml_tensor * const * mms, int nmat, const gemv_epi * epi) {
    GGML_ASSERT(nmat >= 1 && nmat <= GEMV_MAXMAT);
    gemv_init();
    const bool ffn_down = ctx.ffn_down && nmat == 1 && mms[0] == ctx.ffn_down;
    if (ctx.ffn_down && !ffn_down) gemv_ffn_flush(ctx);
    g_kt_ctx = ctx.kt_buf && ktrace_enabled() ? &ctx : nullptr;
    const ggml_tensor * src1 = mms[0]->src[1];
    const ggml_type wt = mms[0]->src[0]->type;
    const bool kq = is_kq(wt);
    double bytes = 0;
    for (int i = 0; i < nmat; ++i) bytes += (double) ggml_nbytes(mms[i]->src[0]) + (double) ggml_nbytes(mms[i]);
    bytes += (double) src1->ne[0] * (kq ? 1.14 : 1.0);

    const bool pro = epi && epi->px;
    const bool swp = epi && epi->sw_gate;
    GGML_ASSERT(!(pro && swp));
    q8_act act = {};
    if (!pro && !swp && !ctx.qcache_get(src1, kq, act)) {
        quantize_act(ctx, src1, kq, act, exec_ctx::QSLOT);
        ctx.qcache_put(src1, kq, act);
    }
    gemv_args a = {};
    for (int i = 0; i < nmat; ++i) {
        const ggml_tensor * w = mms[i]->src[0];
        a.W[i] = (const uint8_t *) w->data;
        a.nb01[i] = w->nb[1];
        a.M[i] = w->ne[1];
        a.dst[i] = epi && epi->elide_dst[i] ? nullptr : (float *) mms[i]->data;
        a.silu[i] = epi && epi->silu[i] ? (float *) epi->silu[i]->data : nullptr;
        a.f16out[i] = epi ? (uint16_t * const *) epi->f16out[i] : nullptr;
        a.rope_out[i] = epi && epi->rope[i] && !epi->elide_rope[i] ? (float *) epi->rope[i]->data : nullptr;
        a.rope_f16[i] = epi ? (uint16_t * const *) epi->rope_f16[i] : nullptr;
        if (epi && epi->rope[i]) {
            const ggml_tensor * r = epi->rope[i];
            rope_params_of(r, a.rp);
            a.rope_pos = (const int32_t *) r->src[1]->data;
            a.rope_ff = r->src[2] ? (const float *) r->src[2]->data : nullptr;
            a.rope_d = r->src[0]->ne[0];
            a.need_pairs = 1;
        }
    }
    a.rtab_g = nullptr;
    if (a.need_pairs) {
        GGML_ASSERT(a.rp.n_dims <= 2 * GEMV_ROPE_MAXPAIRS);
        for (int i = 0; i < nmat; ++i) {
            if (epi->rope[i]) { a.rtab_g = rope_table(ctx, epi->rope[i], a.rp, a.rope_pos, a.rope_ff, 1); break; }
        }
    }
    a.A = {act.qs, act.d, act.s};
    if (pro) {
        GGML_ASSERT(epi->pn == src1->ne[0] && epi->pn % 256 == 0);
        a.pro = {epi->px, epi->pw, epi->psum, epi->peps, epi->pn, kq ? 1 : 2, 0};
    }
    if (epi && epi->rres) {
        GGML_ASSERT(nmat == 1 && epi->rsum);
        a.rres = epi->rres; a.rxsum = epi->rxsum; a.rsum = epi->rsum;
        a.dst[0] = nullptr;   // v is dead: only x = v + res is stored
    }
    // SwiGLU tail: the down projection's quantized input goes to the slot this launch does not read
    q8_act tact = {};
    const bool tkq = epi && epi->tq_for && is_kq(epi->tq_for->src[0]->type);
    if (epi && epi->tail) {
        GGML_ASSERT(ctx.tail_cnt && !needs_epilogue(a, nmat));
        auto & t = a.tl;
        t.kind = 2;
        t.n = mms[epi->t_gate]->ne[0];
        GGML_ASSERT(nmat == 2 && t.n % 256 == 0 && t.n / 256 <= exec_ctx::TAIL_CNT);
        t.gate = epi->t_gate;
        t.up = epi->t_up;
        t.silu_out = epi->t_silu && epi->t_store_silu ? (float *) epi->t_silu->data : nullptr;
        t.mul_out = epi->t_mul && epi->t_store_mul ? (float *) epi->t_mul->data : nullptr;
        t.qmode = epi->tq_for ? (tkq ? 1 : 2) : 0;
        if (t.qmode) {
            const int slot = act.qs && ctx.qslot_of(act.qs) == exec_ctx::QSLOT ? exec_ctx::QSLOT2 : exec_ctx::QSLOT;
            carve_act(tact, ctx.scratch(slot, q8_act::bytes(t.n, 1, tkq)), t.n, 1, tkq);
            t.qs = tact.qs; t.qd = tact.d; t.qsum = tact.s;
        }
        t.cnt = ctx.tail_cnt;
    }
    const int64_t nblk = src1->ne[0] / ggml_blck_size(wt);
    if (swp) {
        GGML_ASSERT(nmat == 1 && !a.tl.kind);
        g_sw_gate = epi->sw_gate;
        g_sw_up = epi->sw_up;
    }
    if (ctx.timing) {
        t_ev_beg = ctx.get_event();
        t_ev_end = ctx.get_event();
    }
    // matrices of a second K-quant type (V beside Q/K, gemv_mixed_ok): one two-body launch
    int ia[GEMV_MAXMAT], ib[GEMV_MAXMAT], n1 = 0, n2 = 0;
    ggml_type wt2 = wt;
    for (int i = 0; i < nmat; ++i) {
        const ggml_type ti = mms[i]->src[0]->type;
        if (ti == wt) ia[n1++] = i;
        else { GGML_ASSERT((wt2 == wt || wt2 == ti) && is_kq(ti) && kq); wt2 = ti; ib[n2++] = i; }
    }
    auto one = [&](ggml_type t, gemv_args & d, int cnt) {
        switch (t) {
            case GGML_TYPE_Q4_K: d.ntasks = (int) (nblk * 4); launch_t<g_q4_K>(ctx.stream, d, cnt); break;
            case GGML_TYPE_Q5_K: d.ntasks = (int) (nblk * 4); launch_t<g_q5_K>(ctx.stream, d, cnt); break;
            case GGML_TYPE_Q6_K: d.ntasks = (int) (nblk * 4); launch_t<g_q6_K>(ctx.stream, d, cnt); break;
            case GGML_TYPE_Q8_0: d.ntasks = (int) nblk;       launch_t<g_q8_0>(ctx.stream, d, cnt); break;
            case GGML_TYPE_Q4_0: d.ntasks = (int) nblk;       launch_t<g_q4_0>(ctx.stream, d, cnt); break;
            default: GGML_ABORT("mi355x: gemv type");
        }
    };
    if (n2) {
        GGML_ASSERT(!a.tl.kind);
        auto part = [&](gemv_args & d, const int * idx, int cnt) {
            d.need_pairs = 0;
            for (int k = 0; k < GEMV_MAXMAT; ++k) {
                const int s = idx[k < cnt ? k : 0];
                d.W[k] = a.W[s]; d.nb01[k] = a.nb01[s]; d.M[k] = a.M[s];
                d.dst[k] = a.dst[s]; d.silu[k] = a.silu[s]; d.f16out[k] = a.f16out[s];
                d.rope_out[k] = a.rope_out[s]; d.rope_f16[k] = a.rope_f16[s];
                if (k < cnt && epi && epi->rope[s]) d.need_pairs = 1;
            }
            d.ntasks = (int) (nblk * 4);
        };
        gemv_args a1 = a, a2 = a;
        part(a1, ia, n1);
        part(a2, ib, n2);
        if (!launch_mixed(ctx.stream, wt, a1, n1, wt2, a2, n2)) {
            one(wt, a1, n1);
            if (ctx.timing) {   // the second launch is timed as its own mat-vec
                ctx.pending.push_back({t_ev_beg, t_ev_end, bytes, TK_MMV});
                t_ev_beg = ctx.get_event();
                t_ev_end = ctx.get_event();
                bytes = 0;
            }
            one(wt2, a2, n2);
        }
    } else if (ffn_down) {
        // the held-back gate/up and this down projection as one chained grid, else one by one
        ctx.ffn_down = nullptr;
        a.ntasks = (int) (nblk * (kq ? 4 : 1));
        if (!launch_ffn(ctx, ffn_of(ctx), wt, a)) {
            ffn_state & f = ffn_of(ctx);
            launch_by_type(ctx.stream, f.t1, f.a1, f.n1);
            one(wt, a, nmat);
        }
    } else if (a.tl.kind && a.tl.qmode == 1 && ffn_enabled() && !ctx.timing && epi->tq_for && wt == GGML_TYPE_Q4_K &&
               nmat == 2) {
        // hold back: the down projection (epi->tq_for) may join this launch
        ffn_state & f = ffn_of(ctx);
        a.ntasks = (int) (nblk * 4);
        f.a1 = a;
        f.n1 = nmat;
        f.t1 = wt;
        ctx.ffn_down = epi->tq_for;
    } else {
        one(wt, a, nmat);
    }
    if (ctx.timing) {
        ctx.pending.push_back({t_ev_beg, t_ev_end, bytes, TK_MMV});
        t_ev_beg = t_ev_end = nullptr;
    }
    if (a.tl.qmode) ctx.qcache_put(epi->tq_key, tkq, tact);
    g_sw_gate = g_sw_up = nullptr;
    g_kt_ctx = nullptr;
}

// the SwiGLU tails' arrival counters exist (allocated outside any capture, zeroed once)
bool gemv_tail_ready(exec_ctx & ctx) {
    if (!ctx.tail_cnt && !ctx.capturing) {
        MI_CHECK(hipMalloc(&ctx.tail_cnt, (size_t) exec_ctx::TAIL_CNT * TAIL_STRIDE * sizeof(int)));
        MI_CHECK(hipMemsetAsync(ctx.tail_cnt, 0, (size_t) exec_ctx::TAIL_CNT * TAIL_STRIDE * sizeof(int), ctx.stream));
    }
    return ctx.tail_cnt != nullptr;
}

double * gemv_rsum_site(exec_ctx & ctx) {
    if (!ctx.rsum_buf && !ctx.capturing) {
        const size_t bytes = (size_t) exec_ctx::MAX_SITES * exec_ctx::SITE_DOUBLES * sizeof(double);
        MI_CHECK(hipMalloc(&ctx.rsum_buf, bytes));
        MI_CHECK(hipMemsetAsync(ctx.rsum_buf, 0, bytes, ctx.stream));
    }
    if (!ctx.rsum_buf || ctx.nsite >= exec_ctx::MAX_SITES) return nullptr;
    return ctx.rsum_buf + (size_t) exec_ctx::SITE_DOUBLES * ctx.nsite++;
}

}  // namespace mi355x
