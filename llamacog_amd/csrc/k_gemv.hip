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
//   * residual producer (a mat-vec followed by ADD -> RMS_NORM -> [MUL] -> mat-vec): the
//     producer stores x = v + res instead of v;
//   * norm prologue: every workgroup of a narrow consumer (Q/K/V) forms RMS_NORM(x) [* w] and its
//     quantization in LDS from x itself (loaded before its weight DMA, so the wait for it leaves
//     the weight stream in flight); the stand-alone norm launch disappears.
#include "ops.h"
#include <hip/hip_ext.h>
#include <mutex>
#include "rope.h"
#include "qtypes.h"
#include "quant_act.h"

namespace mi355x {

typedef __attribute__((address_space(3))) void * gemv_lds_t;
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
    // residual producer (MODE 0, one matrix): x = v + rres[row] goes to rxsum[row] (v itself is
    // dead: the ADD is in place over it)
    const float * rres; float * rxsum;
    // norm prologue: the launch's activation is quant(RMS_NORM(x) [* w]) (kind 1), formed by every
    // workgroup in LDS at byte lds_off
    struct pro_t {
        int kind; const float * x; const float * w; float eps; int64_t n; int qmode; uint32_t lds_off;
    } pro;
    unsigned long long * kt;              // in-graph kernel timeline region (nullable)
    uint32_t wl_off;                      // one-shot kernel: LDS byte offset of the weight slices
    // one-shot kernel: LDS bytes between a wave's row slices (os_geo SLICE, or the slice itself
    // rounded to 16 B when compact), the records' LDS byte offset and their dwords per row (in
    // place: a row's records overwrite its own slice once fetched, os_lds_layout)
    uint32_t sls, rec_off, rec_st;
    int rec_bar;                          // in place at several waves per row: all fetches, a barrier, then the records
    // MUL_MAT_ID of one token (gemv_mmid; the one-shot kernel's ID instance only): matrix i is a
    // stack (W[i], experts xnb02 bytes apart) whose routed slots are stacked as its rows: row
    // s * xme + r is row r of expert *(xids + s * xids_nb0) (read on the device), its output
    // dst[i][s * xme + r] (the slots' output rows are contiguous), its activation column
    // A + s * (xqs_st, xd_st, xs_st) (0: one column shared by the slots).  gate and up of the
    // same slots are two such matrices of one launch
    const char * xids; int64_t xids_nb0, xnb02, xme; int xn_as;
    int64_t xqs_st, xd_st, xs_st;
};

// MI_KT_PHASE=1 (a profiling build, EXTRA=-DMI_KT_PHASE=1): thread 0 of every one-shot workgroup
// stamps the chip's realtime counter at its phase boundaries into the timeline slots after the
// waves' exit stamps (GGML_MI355X_KTRACE_RAW=<label> prints workgroup 0's; scripts/ktrace.py)
#ifndef MI_KT_PHASE
#define MI_KT_PHASE 0
#endif
constexpr int KT_NPH = 8;   // phase slots per workgroup in a MI_KT_PHASE build
constexpr unsigned KT_STRIDE = 1 + 4 + (MI_KT_PHASE ? KT_NPH : 0);   // the one-shot kernels' slots per workgroup
__device__ __forceinline__ void kt_phase(unsigned long long * kt, int k) {
    if (MI_KT_PHASE && kt && threadIdx.x == 0) kt[KT_STRIDE * blockIdx.x + 5 + k] = __builtin_amdgcn_s_memrealtime();
}
static inline unsigned kt_threads() { return 256 + (MI_KT_PHASE ? 64 * KT_NPH : 0); }

// ---- norm prologue ---------------------------------------------------------------------------------
// A decode mat-vec whose input is RMS_NORM(x) [* w] (build_norm, src/llama-graph.cpp:464-497; x the
// residual sum its producer stored, or an input of the graph) forms that activation itself: every
// workgroup loads x (and w), sums (double)(x*x), decides the CPU's float mean from it
// (quant_act.h rms_mean_decided; undecided: the CPU's own loop) and quantizes y = x * scale * w
// into LDS.  Worth it where the consumer launch has few workgroups (Q/K/V: ~900); a wide one
// (gate/up, 3,600) pays more in redundant norms than the stand-alone launch costs (k_fused.hip).
// Measured and not kept (round 5): LEAD workgroups in front of the row groups forming it once and
// publishing it write-through for the others to copy after a counter -- the lead's loads queue
// behind the row groups' weight stream (6-8 us for a 4096-wide norm; gate/up 15 -> 25 us).
// this thread's 16 elements of pass ps in q8K_row16 / q8_0_row16's layout: wave w lane l owns
// elements 16 (l & 15) .. +15 of block 16 ps + 4 w + (l >> 4); false past the row's last block
// (the loads are clamped to the last block, their values unused)
__device__ __forceinline__ bool pro_load(const gemv_args::pro_t & r, int ps, float4 (&xv)[4], float4 (&wv)[4]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = (int) (r.n / 256);
    const int b = 16 * ps + 4 * wave + (lane >> 4);
    const int64_t e0 = 256 * (int64_t) min(b, nb - 1) + 16 * (lane & 15);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        xv[k] = *(const float4 *) (r.x + e0 + 4 * k);
        wv[k] = r.w ? *(const float4 *) (r.w + e0 + 4 * k) : make_float4(1.f, 1.f, 1.f, 1.f);
    }
    return b < nb;
}

// Loads and LDS-DMAs the compiler does not see (inline asm), for the norm-prologue launches: the
// compiler puts no vmcnt wait of its own behind them, so the prologue's sources are waited for
// exactly (gemv_vm_wait: everything but this wave's n youngest weight DMAs) and the prologue
// overlaps the weight stream.  With the builtins its wait for x was a vmcnt(0) behind every weight
// DMA (their per-lane guards made its count conservative), and the rope table and KV-slot loads
// issued after the prologue cost another round trip in front of the records.
__device__ __forceinline__ float4 gemv_ald16(const void * p) {
    float4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint2 gemv_ald8(const void * p) {
    uint2 v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
    return v;
}
// 16 B per lane HBM -> LDS, non-temporal (read once per token), as __builtin_amdgcn_global_load_lds
__device__ __forceinline__ void gemv_dma16(const void * src, const void * lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (gemv_lds_t) lds);
    if (MI_WNT) asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(m), "v"(src) : "memory");
    else asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(src) : "memory");
}
// s_waitcnt vmcnt(n) for a wave-uniform runtime n (<= 31)
__device__ __forceinline__ void gemv_vm_wait(int n) {
#define GW(k) case k: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(k) : "memory"); break;
    switch (n) {
        GW(0) GW(1) GW(2) GW(3) GW(4) GW(5) GW(6) GW(7) GW(8) GW(9) GW(10) GW(11) GW(12) GW(13) GW(14) GW(15)
        GW(16) GW(17) GW(18) GW(19) GW(20) GW(21) GW(22) GW(23) GW(24) GW(25) GW(26) GW(27) GW(28) GW(29) GW(30) GW(31)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef GW
}

// MI_PRO_ASM=0 builds the previous arrangement (builtin loads and DMAs, the epilogue's table loaded
// after the prologue) for A/B runs
#ifndef MI_PRO_ASM
#define MI_PRO_ASM 1
#endif

// pro_load through gemv_ald16 (the caller waits)
__device__ __forceinline__ bool pro_load_asm(const gemv_args::pro_t & r, int ps, float4 (&xv)[4], float4 (&wv)[4]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nb = (int) (r.n / 256);
    const int b = 16 * ps + 4 * wave + (lane >> 4);
    const int64_t e0 = 256 * (int64_t) min(b, nb - 1) + 16 * (lane & 15);
    // (no branch on r.w: the weight-less norm loads x twice and the caller selects 1.0 after its
    // wait, so no kernel-argument round trip sits between the loads)
    const float * wsrc = r.w ? r.w : r.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        xv[k] = gemv_ald16(r.x + e0 + 4 * k);
        wv[k] = gemv_ald16(wsrc + e0 + 4 * k);
    }
    return b < nb;
}

// kind 1's scale 1 / sqrt(mean + eps) from each thread's partial sum s of (double)(x*x): a
// fixed tree over the workgroup, then the mean decided as the CPU's sequential one (quant_act.h
// rms_mean_decided; undecided: the CPU's loop)
__device__ float pro_scale(const gemv_args::pro_t & r, double s) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    s = wave_sum_rows_f64(s);   // (DPP: any order, decided below)
    __shared__ double wp[4];
    __shared__ float pm;
    if (lane == 0) wp[wave] = s;
    __syncthreads();
    const double t = __dadd_rn(__dadd_rn(wp[0], wp[1]), __dadd_rn(wp[2], wp[3]));
    float mean;
    if (!rms_mean_decided(t, r.n, mean)) {   // uniform: every thread holds the same t
        if (tid == 0) pm = rms_mean_sequential(r.x, nullptr, r.n);
        __syncthreads();
        mean = pm;
    }
    return 1.0f / sqrtf(mean + r.eps);
}

__device__ __forceinline__ double pro_sq(const float4 (&xv)[4]) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) s = __dadd_rn(s, sq4(xv[k]));
    return s;
}

// pass ps of the activation (blocks 16 ps .. 16 ps + 15 of 256 elements) into buf, in the gemv_act
// layout, from the thread's loaded slice: y = x * scale [* w], quantized by q8K_row16 (Q8_K) or
// q8_0_row16 (Q8_0)
__device__ void pro_pass(const gemv_args::pro_t & r, float scale, int ps, const float4 (&xv)[4], const float4 (&wv)[4], uint8_t * buf) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = 16 * ps + 4 * wave + (lane >> 4);
    if (b >= (int) (r.n / 256)) return;   // whole rows of 16 lanes
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
    int8_t * qs = (int8_t *) buf;
    float * qd = (float *) (buf + r.n);
    int16_t * qsum = (int16_t *) (buf + r.n + 4 * (r.qmode == 1 ? r.n / 256 : r.n / 32));
    if (r.qmode == 1) q8K_row16(y, lane, qs + 256 * (int64_t) b, qsum + 16 * (int64_t) b, qd + b);
    else q8_0_row16(y, lane, qs + 256 * (int64_t) b, qd + 8 * (int64_t) b, qsum + 8 * (int64_t) b);
}

__device__ __forceinline__ int pro_npass(const gemv_args::pro_t & r) { return (int) ((r.n / 256 + 15) / 16); }

// the whole activation into buf from pass 0's slice of x and w already in registers (loaded
// before the weight DMA, so waiting for it leaves the DMA in flight; v0: the slice exists); the
// later passes of n > 4096 are loaded here.  The mean needs every pass's squares first
__device__ void pro_form_regs(const gemv_args::pro_t & r, uint8_t * buf, bool v0, const float4 (&xv)[4], const float4 (&wv)[4],
                              unsigned long long * kt = nullptr) {
    const int np = pro_npass(r);
    double s = v0 ? pro_sq(xv) : 0.0;
    for (int ps = 1; ps < np; ++ps) {
        float4 xo[4], wo[4];
        if (pro_load(r, ps, xo, wo)) s = __dadd_rn(s, pro_sq(xo));
    }
    if (MI_KT_PHASE) {   // the squares are formed: x has arrived
        asm volatile("" ::"v"(s));
        kt_phase(kt, 1);
    }
    const float scale = pro_scale(r, s);
    kt_phase(kt, 2);
    pro_pass(r, scale, 0, xv, wv, buf);
    for (int ps = 1; ps < np; ++ps) {
        float4 xo[4], wo[4];
        pro_load(r, ps, xo, wo);
        pro_pass(r, scale, ps, xo, wo, buf);
    }
}

// the whole activation, formed by this workgroup (the pipelined kernel's prologue)
__device__ void pro_form_all(const gemv_args::pro_t & r, uint8_t * buf) {
    float4 xv[4], wv[4];
    const bool v0 = pro_load(r, 0, xv, wv);
    pro_form_regs(r, buf, v0, xv, wv);
    __syncthreads();
}

// the activation's pieces in buf (the gemv_act layout of pro_lds_bytes)
__device__ __forceinline__ gemv_act pro_act(const gemv_args::pro_t & r, const uint8_t * buf) {
    return {(const int8_t *) buf, (const float *) (buf + r.n), (const int16_t *) (buf + r.n + 4 * (r.qmode == 1 ? r.n / 256 : r.n / 32))};
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
    if (p.pro.kind) {   // every workgroup forms the activation
        uint8_t * buf = (uint8_t *) xr + p.pro.lds_off;
        pro_form_all(p.pro, buf);
        A = pro_act(p.pro, buf);
    }
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
    kt_enter(p.kt, 5);
    gemv_pipe_body<T, R, WPR, MODE>(p, ngroups, blockIdx.x, gridDim.x, xr);
    kt_exit(p.kt, 5);
}

// Q/K of one K-quant and V of another (Llama-3 Q4_K_M: Q4_K and Q6_K on 16 of 32 layers) in
// one launch with epilogues: workgroups [0, nwg1) run p1's matrices, the rest p2's.  Each
// row's arithmetic is its type's own, so the bits are those of two separate launches.
template <class T1, class T2, int R2, int WPR>
__global__ __launch_bounds__(256) void k_gemv_pipe2(const gemv_args p1, const int64_t ng1, const int64_t nwg1,
                                                    const gemv_args p2, const int64_t ng2) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    kt_enter(p1.kt, 5);
    if ((int64_t) blockIdx.x < nwg1) gemv_pipe_body<T1, 2, WPR, 1>(p1, ng1, blockIdx.x, nwg1, xr);
    else gemv_pipe_body<T2, R2, WPR, 1>(p2, ng2, (int64_t) blockIdx.x - nwg1, (int64_t) gridDim.x - nwg1, xr);
    kt_exit(p1.kt, 5);
}

// ---- one-shot body: one row group per workgroup, weights staged by LDS-DMA ----------------------
// Each wave copies its R row slices (at most 64 tasks of a row: os_geo<T>::SEG bytes each) HBM ->
// LDS with global_load_lds, 1 KiB of contiguous bytes per wave instruction, so every 128-B line
// is requested once (the register fetch of a task's header + quants asks each line three
// times), and no VGPR is held for bytes in flight; the dispatcher's workgroup turnover does the
// pipelining.  The norm prologue's sources are loaded before the DMAs are issued, so waiting
// for them leaves the weight stream in flight; a Q8 activation slice is loaded after them.
// Records, walker and epilogues are the pipelined kernel's (the same bits).
template <class T> struct os_geo {
    static constexpr int SEG = (WAVE / T::per_block) * T::blk_bytes;   // a wave's row slice
    static constexpr int NI = (SEG + 1023) / 1024;                        // DMA instructions per slice
    static constexpr int SLICE = NI * 1024;                               // LDS bytes per slice
};

template <class T, int R, int WPR, int MODE, bool PRO, bool ID = false>
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
    // ID: the routed slot of this row group (xme % RPG == 0: uniform over the workgroup)
    const int xsl = ID ? __builtin_amdgcn_readfirstlane((int) ((uint32_t) ((g - p.blk0[mi]) * RPG) / (uint32_t) p.xme)) : 0;
    // ---- activation sources first: pass 0 of x and w for the norm prologue ----
    float4 pxv[4], pwv[4];
    bool pv0 = false;
    constexpr bool PA = PRO && MI_PRO_ASM;
    if constexpr (PA) pv0 = pro_load_asm(p.pro, 0, pxv, pwv);
    else if constexpr (PRO) pv0 = pro_load(p.pro, 0, pxv, pwv);
    // the epilogue's rope table and KV-slot pointers, loaded with the prologue's sources (PRO)
    uint2 rtv = make_uint2(0, 0), fpv = make_uint2(0, 0);
    const bool has_rt = PA && MODE && ((p.need_pairs != 0) & ((int) threadIdx.x < p.rp.n_dims / 2));
    uint16_t * const * fslot = nullptr;
    if constexpr (PA && MODE != 0) {
        // (selected from the six uniform kernel arguments: a per-lane index into them is a vector
        // load of the kernarg segment and a wait in front of the DMAs)
        const int ti = threadIdx.x;
        uint16_t * const * sl = nullptr;
#pragma unroll
        for (int k = 0; k < GEMV_MAXMAT; ++k) {
            sl = ti == 2 * k ? p.f16out[k] : sl;
            sl = ti == 2 * k + 1 ? p.rope_f16[k] : sl;
        }
        fslot = sl;
        // unconditional loads (a harmless address where there is nothing to load), no branches on
        // kernel arguments between them
        rtv = gemv_ald8(has_rt ? (const void *) (p.rtab_g + threadIdx.x) : (const void *) p.pro.x);
        fpv = gemv_ald8(fslot ? (const void *) fslot : (const void *) p.pro.x);
    }
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
    uint8_t * mine = wl + (size_t) wave * R * p.sls;
    {
        const int nt_w = min(WAVE, p.ntasks - WAVE * wsub);
        const int seg = (nt_w / T::per_block) * T::blk_bytes;
        const uint8_t * Wm = p.W[mi];
        if constexpr (ID) {   // the routed expert (uniform over the workgroup, before any barrier)
            const int ex = *(const int32_t *) (p.xids + xsl * p.xids_nb0);
            if (ex < 0 || ex >= p.xn_as) return;
            Wm += (int64_t) ex * p.xnb02 - (int64_t) xsl * p.xme * p.nb01[mi];
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint8_t * src = Wm + min(row0 + r, M - 1) * p.nb01[mi] + (int64_t) wsub * G::SEG;
#pragma unroll
            for (int i = 0; i < G::NI; ++i) {
                const int off = min(i * 1024 + 16 * lane, seg - 16);
                // lanes past the slice write nothing (a compact stride leaves no padding after it)
                if (i * 1024 + 16 * lane < seg) {
                    if constexpr (PA) gemv_dma16(src + off, mine + r * p.sls + i * 1024);
                    else __builtin_amdgcn_global_load_lds((const void *) (src + off), (gemv_lds_t) (mine + r * p.sls + i * 1024), 16, 0,
                                                          MI_WNT ? 2 : 0);
                }
            }
        }
        if constexpr (PA) {
            // the prologue's sources and the epilogue's table are in; this wave's R * ceil(seg / 1 KiB)
            // weight DMAs (lane 0 of every one of them is inside the slice) stay in flight
            gemv_vm_wait(R * ((seg + 1023) / 1024));
            // (the values are used only after the wait)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                asm volatile("" : "+v"(pxv[k].x), "+v"(pxv[k].y), "+v"(pxv[k].z), "+v"(pxv[k].w));
                asm volatile("" : "+v"(pwv[k].x), "+v"(pwv[k].y), "+v"(pwv[k].z), "+v"(pwv[k].w));
            }
            asm volatile("" : "+v"(rtv.x), "+v"(rtv.y), "+v"(fpv.x), "+v"(fpv.y));
            if (!p.pro.w) {
#pragma unroll
                for (int k = 0; k < 4; ++k) pwv[k] = make_float4(1.f, 1.f, 1.f, 1.f);
            }
        }
    }
    kt_phase(p.kt, 0);
    // the activation slice after the DMAs: T::load computes on what it loads (bsum pairs, the
    // Q6_K -32 sums), and a wait for a load issued BEFORE the DMAs would hold the DMA issue back
    // by an L2 round trip (the one-shot kernel's rec stage took ~35 % longer that way)
    typename T::act x;
    if constexpr (PRO) {
        uint8_t * buf = (uint8_t *) xr + p.pro.lds_off;
        pro_form_regs(p.pro, buf, pv0, pxv, pwv, p.kt);
        __syncthreads();
        kt_phase(p.kt, 3);
        T::load(pro_act(p.pro, buf), tt, x);
    } else if constexpr (ID) {   // this slot's column
        const gemv_act A = {p.A.qs + xsl * p.xqs_st, p.A.d + xsl * p.xd_st, p.A.s + xsl * p.xs_st};
        T::load(A, tt, x);
    } else {
        T::load(p.A, tt, x);
    }
    __shared__ float2 rtab[MODE ? GEMV_ROPE_MAXPAIRS : 1];
    __shared__ uint16_t * f16p[2 * GEMV_MAXMAT];
    if constexpr (PA && MODE != 0) {   // loaded before the weight DMAs
        if (threadIdx.x < 2 * GEMV_MAXMAT) f16p[threadIdx.x] = fslot ? (uint16_t *) (((uint64_t) fpv.y << 32) | fpv.x) : nullptr;
        if (has_rt) rtab[threadIdx.x] = make_float2(__uint_as_float(rtv.x), __uint_as_float(rtv.y));
    } else if (MODE) {
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
    kt_phase(p.kt, 4);
    uint32_t * xb = xr + p.rec_off / 4;
    const int rst = (int) p.rec_st;
    if (WPR > 1 && R > 1 && p.rec_bar) {
        // a row's records go over wave 0's slice of it, written by all of the row's waves: every
        // wave has fetched its slices before any record is stored
        typename T::raw w[R];
#pragma unroll
        for (int r = 0; r < R; ++r) T::template fetch<typename lds_loader<T>::type>(mine + r * p.sls - (int64_t) wsub * G::SEG, tt, w[r]);
        __syncthreads();
#pragma unroll
        for (int r = 0; r < R; ++r) T::rec(w[r], tt, x, active, xb + (size_t) (rowl0 + r) * rst);
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            typename T::raw w;
            T::template fetch<typename lds_loader<T>::type>(mine + r * p.sls - (int64_t) wsub * G::SEG, tt, w);
            T::rec(w, tt, x, active, xb + (size_t) (rowl0 + r) * rst);
        }
    }
    if constexpr (W1) {
        __syncthreads();   // every wave's records are in
        if (wave != 0) return;
        const float v = T::walk(xb + (size_t) wrc1 * rst, nb, ws1);
        const int64_t row = grow0 + wr1;
        if (wr1 < RPG && ws1 == 0 && row < M) {
            if (p.rres) p.rxsum[row] = __fadd_rn(v, rc);   // ADD(v, res): the CPU's single f32 add
            else p.dst[mi][row] = v;
        }
        return;
    }
    kt_phase(p.kt, 5);
    if constexpr (WPR > 1 || MODE != 0) __syncthreads();
    else wave_lds_sync();
    __shared__ float res[MODE ? RPG : 1];
    // epilogue launches: wave 0 walks every row of the group into res (one walk where four waves
    // each ran one); the stores below are the whole workgroup's as before
    constexpr bool W1E = WPR == 1 && MODE != 0 && RPG * T::LPR <= WAVE;
    if constexpr (W1E) {
        if (wave == 0) {
            const float v = T::walk(xb + (size_t) wrc1 * rst, nb, ws1);
            if (wr1 < RPG && ws1 == 0) res[wr1] = v;
        }
    } else if (wsub == 0) {
        const float v = T::walk(xb + (size_t) (rowl0 + wrc) * rst, nb, ws);
        if (wr < R && ws == 0) {
            if constexpr (MODE == 0) {
                if (row0 + wr < M) {
                    if (p.rres) {   // ADD(v, res): the CPU's single f32 add
                        p.rxsum[row0 + wr] = __fadd_rn(v, rc);
                    } else {
                        p.dst[mi][row0 + wr] = v;
                    }
                }
            } else {
                res[rowl0 + wr] = v;
            }
        }
    }
    if constexpr (MODE >= 1) {
        __syncthreads();
        kt_phase(p.kt, 6);
        for (int i = threadIdx.x; i < RPG; i += NT) {
            const int64_t row = (g - p.blk0[mi]) * RPG + i;
            // rope partner row ^ 1 lies in the same group (RPG is even whenever rope is fused)
            if (row < M) gemv_store(p, mi, M, row, res[i], res[RPG > 1 ? i ^ 1 : i], rtab, f16p);
        }
    }
}

// dynamic LDS: [records RPG x nb x RS dwords | prologue activation | weight slices]; ID: the
// routed-expert instance of MUL_MAT_ID (the dense instances carry none of its branches)
template <class T, int R, int WPR, int MODE, bool PRO, bool ID>
__global__ __launch_bounds__(256) void k_gemv_os(const gemv_args p) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    kt_enter(p.kt, KT_STRIDE);
    gemv_os_body<T, R, WPR, MODE, PRO, ID>(p, blockIdx.x, (uint8_t *) xr + p.wl_off, xr);
    kt_exit(p.kt, KT_STRIDE);
}

template <class T1, class T2, int R2, int WPR, bool PRO, int R1 = 2, int WPR2 = WPR>
__global__ __launch_bounds__(256) void k_gemv_os2(const gemv_args p1, const int64_t ng1, const gemv_args p2) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    kt_enter(p1.kt, KT_STRIDE);
    const int64_t b = blockIdx.x;
    if (b < ng1) gemv_os_body<T1, R1, WPR, 1, PRO>(p1, b, (uint8_t *) xr + p1.wl_off, xr);
    else gemv_os_body<T2, R2, WPR2, 1, PRO>(p2, b - ng1, (uint8_t *) xr + p2.wl_off, xr);
    kt_exit(p1.kt, KT_STRIDE);
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

// in-graph timeline label of a launch: its fused pieces, and "/w" for rows split over waves
// (the K = 14336 down projection)
static const char * gemv_kt_name(const gemv_args & a, int mode) {
    static const char * names[16] = {"gemv", "gemv+pro", "gemv+epi", "gemv+pro+epi", "gemv+resid", "gemv+pro+resid",
                                     "gemv+epi+resid", "gemv+pro+epi+resid",
                                     "gemv/w", "gemv+pro/w", "gemv+epi/w", "gemv+pro+epi/w", "gemv+resid/w", "gemv+pro+resid/w",
                                     "gemv+epi+resid/w", "gemv+pro+epi+resid/w"};
    return names[(a.pro.kind ? 1 : 0) | (mode ? 2 : 0) | (a.rres ? 4 : 0) | (a.ntasks > WAVE ? 8 : 0)];
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
    if (a.pro.kind) {
        // every workgroup forms the activation: one resident round (1024), so no
        // workgroup pays the prologue after the weight stream is under way
        grid = std::min<int64_t>(grid, 1024);
    }
    if (MODE >= 1) grid = std::max<int64_t>(grid, ceil_div(ng, GEMV_MAXG));   // LDS-parked row sums
    size_t lds = 4 * xrec_dwords<T>(RPG, a.ntasks / T::per_block);
    if (a.pro.kind) {   // the prologue's activation follows the records
        lds = (lds + 15) / 16 * 16;
        a.pro.lds_off = (uint32_t) lds;
        lds += pro_lds_bytes(a.pro.n, a.pro.qmode);
    }
    if (g_kt_ctx) a.kt = g_kt_ctx->kt_take(gemv_kt_name(a, MODE), (unsigned) grid, 256);
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
    GGML_ASSERT(!(a.rres && needs_epilogue(a, nmat)) && "mi355x: GEMV residual with epilogues");
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

// GGML_MI355X_OS_COMPACT=0: row slices at os_geo's 1-KiB multiple and records in a region of
// their own (A/B); default: slices at their own size rounded to 16 B, and at one wave per row
// the records in place over the slices
static bool os_compact() {
    static const bool on = !getenv("GGML_MI355X_OS_COMPACT") || atoi(getenv("GGML_MI355X_OS_COMPACT")) != 0;
    return on;
}

// the plain slice layout (the two-body launches): records first, slices at os_geo's stride
template <class T, int R, int WPR>
static void os_plain_geo(gemv_args & a) {
    a.sls = os_geo<T>::SLICE;
    a.rec_off = 0;
    a.rec_bar = 0;
    a.rec_st = (uint32_t) ((a.ntasks / T::per_block) * T::RS);
}

template <class T, int R, int WPR>
static size_t os_lds_layout(gemv_args & a) {
    constexpr int RPG = (4 / WPR) * R;
    const int64_t nb = a.ntasks / T::per_block;
    const uint32_t sls = os_compact() ? (uint32_t) r16(os_geo<T>::SEG) : (uint32_t) os_geo<T>::SLICE;
    // in place: a row's records fit a slice; at one wave per row they overwrite the row's own
    // slice once fetched, at several (GGML_MI355X_OS_IPW=0: not in place) wave 0's slice of the
    // row after a barrier behind every wave's fetches
    static const bool ipw = !getenv("GGML_MI355X_OS_IPW") || atoi(getenv("GGML_MI355X_OS_IPW")) != 0;
    // (not at one row per wave group: there the barrier's registers cost more workgroups per CU
    // than the records' LDS, Q6_K down 72 vs 57 VGPRs)
    const bool inplace = os_compact() && (WPR == 1 || (ipw && R > 1)) && (size_t) nb * T::RS * 4 <= sls;
    a.rec_bar = inplace && WPR > 1;
    size_t off = inplace ? 0 : r16((size_t) RPG * nb * T::RS * 4);
    if (a.pro.kind) {
        a.pro.lds_off = (uint32_t) off;
        off = r16(off + pro_lds_bytes(a.pro.n, a.pro.qmode));
    }
    a.wl_off = (uint32_t) off;
    a.sls = sls;
    a.rec_off = inplace ? (uint32_t) off : 0;
    a.rec_st = inplace ? sls / 4 : (uint32_t) (nb * T::RS);
    return off + (size_t) 4 * R * sls;
}

template <class T, int R, int WPR, int MODE>
static void launch_os_m(hipStream_t st, gemv_args & a, int nmat) {
    constexpr int RPG = (4 / WPR) * R;
    const int64_t ng = set_groups(a, nmat, RPG);
    const size_t lds = os_lds_layout<T, R, WPR>(a);
    const int64_t grid = ng;
    a.kt = g_kt_ctx ? g_kt_ctx->kt_take(gemv_kt_name(a, MODE), (unsigned) grid, kt_threads()) : nullptr;
#define OS_LAUNCH(P)                                                                                              \
    if (t_ev_beg) hipExtLaunchKernelGGL((k_gemv_os<T, R, WPR, MODE, P, false>), dim3((unsigned) grid), dim3(256), lds, st, t_ev_beg, t_ev_end, 0, a); \
    else hipLaunchKernelGGL((k_gemv_os<T, R, WPR, MODE, P, false>), dim3((unsigned) grid), dim3(256), lds, st, a)
    if (a.pro.kind) { OS_LAUNCH(true); } else { OS_LAUNCH(false); }
#undef OS_LAUNCH
}

template <class T, int R, int WPR>
static void launch_os(hipStream_t st, gemv_args & a, int nmat) {
    if (needs_epilogue(a, nmat)) launch_os_m<T, R, WPR, 1>(st, a, nmat);
    else launch_os_m<T, R, WPR, 0>(st, a, nmat);
}

// rows per wave of a prologue launch at one wave per row: four (every workgroup forms the norm,
// so half as many of them form it; Q/K/V 9.9 -> 9.3 us, round 3).  GGML_MI355X_PRO_R = 1 / 2
// for A/B; anything else is ignored
static int pro_rows() {
    static const int v = [] {
        const int e = getenv("GGML_MI355X_PRO_R") ? atoi(getenv("GGML_MI355X_PRO_R")) : 4;
        return e == 1 || e == 2 ? e : 4;
    }();
    return v;
}

// rows per wave of the one-shot kernel (tools/gemv_lab.hip, round 3; round 4 below): two for the
// 4-bit K-quants at K = 14336, two for the plain one-wave-per-row launches, pro_rows() for the
// norm-prologue launches
template <class T>
static bool launch_os_t(hipStream_t st, gemv_args & a, int nmat) {
    if (!os_enabled() || !os_aligned<T>(a, nmat)) return false;
    const int wpr = wpr_of(a.ntasks);
    int R = 1;
    if (a.pro.kind || (wpr == 4 && !std::is_same<T, g_q6_K>::value)) R = 2;
    if (a.pro.kind && wpr == 1) R = pro_rows();
    // with one walking wave per workgroup, two rows per wave for the plain (no prologue / epilogue)
    // launches: gate/up 16.5 -> 14.9 us (scripts/probe_mall_gemv.py, round 4); the 6-bit output
    // head keeps one (71 vs 77 us)
    if (!a.pro.kind && wpr == 1 && !needs_epilogue(a, nmat) && !std::is_same<T, g_q6_K>::value) R = 2;
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

// MUL_MAT_ID of one token: the routed experts as the matrices of one one-shot launch of the ID
// instance (no prologue or epilogue), rows per wave by launch_os_t's plain rule
template <class T, int R, int WPR>
static void launch_os_id_v(hipStream_t st, gemv_args & a, int nmat) {
    constexpr int RPG = (4 / WPR) * R;
    const int64_t ng = set_groups(a, nmat, RPG);
    const size_t lds = os_lds_layout<T, R, WPR>(a);
    a.kt = g_kt_ctx ? g_kt_ctx->kt_take("gemv_id", (unsigned) ng, kt_threads()) : nullptr;
    if (t_ev_beg) hipExtLaunchKernelGGL((k_gemv_os<T, R, WPR, 0, false, true>), dim3((unsigned) ng), dim3(256), lds, st, t_ev_beg, t_ev_end, 0, a);
    else hipLaunchKernelGGL((k_gemv_os<T, R, WPR, 0, false, true>), dim3((unsigned) ng), dim3(256), lds, st, a);
}

template <class T>
static bool launch_os_id(hipStream_t st, gemv_args & a, int nmat) {
    if (!os_enabled() || !os_aligned<T>(a, nmat)) return false;
    const int wpr = wpr_of(a.ntasks);
    int R = std::is_same<T, g_q6_K>::value || wpr == 2 ? 1 : 2;
    // GGML_MI355X_MMID_R: rows per wave of the K = 14336 (four waves per row) launches (geometry probe)
    static const int r4 = getenv("GGML_MI355X_MMID_R") ? atoi(getenv("GGML_MI355X_MMID_R")) : 0;
    if (wpr == 4 && (r4 == 1 || r4 == 2 || r4 == 4)) R = r4;
    // GGML_MI355X_MMID_R1: rows per wave of the one-wave-per-row launches (gate / up)
    static const int r1 = getenv("GGML_MI355X_MMID_R1") ? atoi(getenv("GGML_MI355X_MMID_R1")) : 0;
    if (wpr == 1 && (r1 == 1 || r1 == 2 || r1 == 4)) R = r1;
    if (a.xme % ((4 / wpr) * R) != 0) return false;   // whole row groups per routed slot
    gemv_args b = a;
    const size_t lds = R == 4 ? (wpr == 1 ? os_lds_layout<T, 4, 1>(b) : os_lds_layout<T, 4, 4>(b))
                     : R == 2 ? (wpr == 1 ? os_lds_layout<T, 2, 1>(b) : os_lds_layout<T, 2, 4>(b))
                              : (wpr == 1 ? os_lds_layout<T, 1, 1>(b) : wpr == 2 ? os_lds_layout<T, 1, 2>(b) : os_lds_layout<T, 1, 4>(b));
    if (lds > 64 * 1024) return false;
    switch (R * 8 + wpr) {
        case 4 * 8 + 4: launch_os_id_v<T, 4, 4>(st, a, nmat); break;
        case 4 * 8 + 1: launch_os_id_v<T, 4, 1>(st, a, nmat); break;
        case 2 * 8 + 1: launch_os_id_v<T, 2, 1>(st, a, nmat); break;
        case 2 * 8 + 4: launch_os_id_v<T, 2, 4>(st, a, nmat); break;
        case 1 * 8 + 1: launch_os_id_v<T, 1, 1>(st, a, nmat); break;
        case 1 * 8 + 2: launch_os_id_v<T, 1, 2>(st, a, nmat); break;
        default:        launch_os_id_v<T, 1, 4>(st, a, nmat); break;
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
    if (a1.pro.kind) {
        a1.pro.lds_off = a2.pro.lds_off = (uint32_t) off;
        off = r16(off + pro_lds_bytes(a1.pro.n, a1.pro.qmode));
    }
    a1.wl_off = a2.wl_off = (uint32_t) off;
    os_plain_geo<T1, R1, WPR>(a1);
    os_plain_geo<T2, R2, WPR>(a2);
    const size_t lds = off + std::max((size_t) 4 * R1 * os_geo<T1>::SLICE, (size_t) 4 * R2 * os_geo<T2>::SLICE);
    const unsigned grid = (unsigned) (ng1 + ng2);
    a1.kt = g_kt_ctx ? g_kt_ctx->kt_take(a1.pro.kind ? "gemv2+pro+epi" : "gemv2+epi", grid, kt_threads()) : nullptr;
#define OS2_LAUNCH(P)                                                                                                 \
    if (t_ev_beg) hipExtLaunchKernelGGL((k_gemv_os2<T1, T2, R2, WPR, P, R1>), dim3(grid), dim3(64 * NWV), lds, st, t_ev_beg, \
                                        t_ev_end, 0, a1, ng1, a2);                                                        \
    else hipLaunchKernelGGL((k_gemv_os2<T1, T2, R2, WPR, P, R1>), dim3(grid), dim3(64 * NWV), lds, st, a1, ng1, a2)
    if (a1.pro.kind) { OS2_LAUNCH(true); } else { OS2_LAUNCH(false); }
#undef OS2_LAUNCH
}

// a K-quant part beside a Q8_0 part (Mixtral: Q5_K attn_q, Q8_0 attn_k / attn_v), each with its
// own activation quantization and its own waves per row; no prologue
template <class T1, int R1, int WPR1, class T2, int R2, int WPR2>
static void launch_os2m_v(hipStream_t st, gemv_args & a1, int n1, gemv_args & a2, int n2) {
    constexpr int NWV = 4;
    const int64_t ng1 = set_groups(a1, n1, (NWV / WPR1) * R1), ng2 = set_groups(a2, n2, (NWV / WPR2) * R2);
    const size_t off = r16(std::max((size_t) (NWV / WPR1) * R1 * (a1.ntasks / T1::per_block) * T1::RS * 4,
                                    (size_t) (NWV / WPR2) * R2 * (a2.ntasks / T2::per_block) * T2::RS * 4));
    a1.wl_off = a2.wl_off = (uint32_t) off;
    os_plain_geo<T1, R1, WPR1>(a1);
    os_plain_geo<T2, R2, WPR2>(a2);
    const size_t lds = off + std::max((size_t) 4 * R1 * os_geo<T1>::SLICE, (size_t) 4 * R2 * os_geo<T2>::SLICE);
    const unsigned grid = (unsigned) (ng1 + ng2);
    a1.kt = g_kt_ctx ? g_kt_ctx->kt_take("gemv2+epi", grid, kt_threads()) : nullptr;
    if (t_ev_beg) hipExtLaunchKernelGGL((k_gemv_os2<T1, T2, R2, WPR1, false, R1, WPR2>), dim3(grid), dim3(64 * NWV), lds, st,
                                        t_ev_beg, t_ev_end, 0, a1, ng1, a2);
    else hipLaunchKernelGGL((k_gemv_os2<T1, T2, R2, WPR1, false, R1, WPR2>), dim3(grid), dim3(64 * NWV), lds, st, a1, ng1, a2);
}

template <class T1>
static bool launch_os2m_t(hipStream_t st, gemv_args & a1, int n1, gemv_args & a2, int n2) {
    if (!os_enabled() || a1.pro.kind || a1.ntasks != WAVE || a2.ntasks != 2 * WAVE ||
        !os_aligned<T1>(a1, n1) || !os_aligned<g_q8_0>(a2, n2)) return false;
    launch_os2m_v<T1, 1, 1, g_q8_0, 1, 2>(st, a1, n1, a2, n2);
    return true;
}

template <class T>
static void launch_t(hipStream_t st, gemv_args & a, int nmat) {
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
    if (a1.pro.kind) {   // the prologue's activation follows the records (both bodies), formed by each
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
        if (wpr == 1 && a1.pro.kind && pro_rows() == 4) launch_os2_v<T1, T2, 2, 1, 4>(st, a1, n1, a2, n2);
        else if (wpr == 1 && a1.pro.kind && pro_rows() == 1) launch_os2_v<T1, T2, 1, 1, 1>(st, a1, n1, a2, n2);
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
    if (t1 == GGML_TYPE_Q5_K && t2 == GGML_TYPE_Q8_0) return launch_os2m_t<g_q5_K>(st, a1, n1, a2, n2);
    if (t1 == GGML_TYPE_Q4_K && t2 == GGML_TYPE_Q8_0) return launch_os2m_t<g_q4_K>(st, a1, n1, a2, n2);
    return false;
}

bool gemv_mixed_ok(const ggml_tensor * mm0, const ggml_tensor * c) {
    const ggml_type t1 = mm0->src[0]->type, t2 = c->src[0]->type;
    return ((t1 == GGML_TYPE_Q4_K && (t2 == GGML_TYPE_Q6_K || t2 == GGML_TYPE_Q5_K)) ||
            (t1 == GGML_TYPE_Q5_K && t2 == GGML_TYPE_Q6_K) ||
            // a Q8_0 part with its own activation (Mixtral's attn_k / attn_v beside the Q5_K attn_q)
            ((t1 == GGML_TYPE_Q5_K || t1 == GGML_TYPE_Q4_K) && t2 == GGML_TYPE_Q8_0));
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

// one launch for up to three MUL_MATs sharing src1 (all gemv_supported, same K; a second
// K-quant type joins as the second body of k_gemv_pipe2)
void gemv_group(exec_ctx & ctx, ggml_tensor * const * mms, int nmat, const gemv_epi * epi) {
    GGML_ASSERT(nmat >= 1 && nmat <= GEMV_MAXMAT);
    gemv_init();
    g_kt_ctx = ctx.kt_buf && ktrace_enabled() ? &ctx : nullptr;
    const ggml_tensor * src1 = mms[0]->src[1];
    const ggml_type wt = mms[0]->src[0]->type;
    const bool kq = is_kq(wt);
    double bytes = 0;
    for (int i = 0; i < nmat; ++i) bytes += (double) ggml_nbytes(mms[i]->src[0]) + (double) ggml_nbytes(mms[i]);
    bytes += (double) src1->ne[0] * (kq ? 1.14 : 1.0);

    const bool pro = epi && epi->px;
    q8_act act = {};
    if (!pro && !ctx.qcache_get(src1, kq, act)) {
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
        GGML_ASSERT(epi->pn == src1->ne[0] && epi->pn % 256 == 0 && epi->pkind == 1);
        auto & r = a.pro;
        r.kind = epi->pkind;
        r.x = epi->px; r.w = epi->pw; r.eps = epi->peps; r.n = epi->pn;
        r.qmode = kq ? 1 : 2;
        r.lds_off = 0;
    }
    if (epi && epi->rres) {
        GGML_ASSERT(nmat == 1);
        a.rres = epi->rres; a.rxsum = epi->rxsum;
        a.dst[0] = nullptr;   // v is dead: only x = v + res is stored
    }
    const int64_t nblk = src1->ne[0] / ggml_blck_size(wt);
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
        else { GGML_ASSERT((wt2 == wt || wt2 == ti) && (is_kq(ti) || ti == GGML_TYPE_Q8_0) && kq); wt2 = ti; ib[n2++] = i; }
    }
    // a Q8_0 second part reads the Q8_0 quantization of the same input (the fused norm's
    // companion, else quantized here)
    q8_act act2 = act;
    const bool q0 = n2 && wt2 == GGML_TYPE_Q8_0;
    if (q0 && !pro && !ctx.qcache_get(src1, false, act2)) {
        quantize_act(ctx, src1, false, act2, exec_ctx::QSLOT0);
        ctx.qc0_tensor = src1; ctx.qc0_data = src1->data; ctx.qc0_act = act2;
    }
    auto one = [&](ggml_type t, gemv_args & d, int cnt) {
        const int64_t nblk = src1->ne[0] / ggml_blck_size(t);
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
        if (q0) {
            a2.ntasks = (int) (src1->ne[0] / 32);
            a2.A = {act2.qs, act2.d, act2.s};
            a2.pro.qmode = 2;
        }
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
    } else {
        one(wt, a, nmat);
    }
    if (ctx.timing) {
        ctx.pending.push_back({t_ev_beg, t_ev_end, bytes, TK_MMV});
        t_ev_beg = t_ev_end = nullptr;
    }
    g_kt_ctx = nullptr;
}

// ---- MUL_MAT_ID of one token on the one-shot kernel ----------------------------------------------
// The n_used routed experts of a decode step as the matrices of one launch of the ID instance:
// each workgroup reads its expert id from ids on the device and streams that expert's rows (k_mmx
// KIND 1 does the same one row per wave with register loads).  Same records and walk (qtypes.h),
// so the same bits as ggml_compute_forward_mul_mat_id (ggml-cpu.c:1466).  The dense launches are
// other template instances and carry none of these branches.  GGML_MI355X_MMID_OS=0 keeps k_mmx.
bool gemv_mmid(exec_ctx & ctx, ggml_tensor * dst, const q8_act & act, ggml_tensor * dst2) {
    static const bool on = !getenv("GGML_MI355X_MMID_OS") || atoi(getenv("GGML_MI355X_MMID_OS")) != 0;
    const ggml_tensor * as = dst->src[0];
    const ggml_tensor * b = dst->src[1];
    const ggml_tensor * ids = dst->src[2];
    const int64_t n_used = ids->ne[0];
    const int nmat = dst2 ? 2 : 1;
    if (!on || !os_enabled() || ids->ne[1] != 1 || n_used < 1 || n_used > 8) return false;
    // the slots' output rows contiguous, and whole row groups per slot (RPG <= 8)
    if (dst->nb[1] != (size_t) as->ne[1] * sizeof(float) || as->ne[1] % 8 != 0) return false;
    if (b->ne[1] != 1 && b->ne[1] != n_used) return false;   // slot e reads column e % ne11
    if (dst2) {   // the up projection of the same slots: same stack shape, type and input
        const ggml_tensor * as2 = dst2->src[0];
        if (as2->type != as->type || !ggml_are_same_shape(as2, as) || as2->nb[1] != as->nb[1] || as2->nb[2] != as->nb[2] ||
            dst2->src[1] != b || dst2->src[2] != ids || dst2->nb[1] != dst->nb[1]) return false;
    }
    int per = 0;
    switch (as->type) {
        case GGML_TYPE_Q4_K: case GGML_TYPE_Q4_0:
            if (as->ne[1] % 8 != 0) return false;   // k_mmx's vec_dot order (not repacked)
            per = as->type == GGML_TYPE_Q4_K ? 4 : 1;
            break;
        case GGML_TYPE_Q5_K: case GGML_TYPE_Q6_K: per = 4; break;
        case GGML_TYPE_Q8_0: per = 1; break;
        default: return false;
    }
    const int64_t nblk = as->ne[0] / ggml_blck_size(as->type);
    if (nblk * per > 4 * WAVE || as->nb[2] % 16 != 0) return false;
    gemv_init();
    g_kt_ctx = ctx.kt_buf && ktrace_enabled() ? &ctx : nullptr;
    gemv_args a = {};
    for (int i = 0; i < nmat; ++i) {
        const ggml_tensor * d = i == 0 ? dst : dst2;
        a.W[i] = (const uint8_t *) d->src[0]->data;
        a.nb01[i] = as->nb[1];
        a.M[i] = n_used * as->ne[1];
        a.dst[i] = (float *) d->data;
    }
    a.A = {act.qs, act.d, act.s};
    a.xids = (const char *) ids->data; a.xids_nb0 = ids->nb[0]; a.xnb02 = as->nb[2]; a.xn_as = (int) as->ne[2];
    a.xme = as->ne[1];
    if (b->ne[1] > 1) { a.xqs_st = act.qs_stride(); a.xd_st = act.d_stride(); a.xs_st = act.s_stride(); }
    a.ntasks = (int) (nblk * per);
    bool ok = false;
    switch (as->type) {
        case GGML_TYPE_Q4_K: ok = launch_os_id<g_q4_K>(ctx.stream, a, nmat); break;
        case GGML_TYPE_Q5_K: ok = launch_os_id<g_q5_K>(ctx.stream, a, nmat); break;
        case GGML_TYPE_Q6_K: ok = launch_os_id<g_q6_K>(ctx.stream, a, nmat); break;
        case GGML_TYPE_Q8_0: ok = launch_os_id<g_q8_0>(ctx.stream, a, nmat); break;
        case GGML_TYPE_Q4_0: ok = launch_os_id<g_q4_0>(ctx.stream, a, nmat); break;
        default: break;
    }
    g_kt_ctx = nullptr;
    return ok;
}

}  // namespace mi355x
