// gemv_lab.hip — decode mat-vec design lab: time candidate Q4_K / Q6_K GEMV loop structures
// on the Llama-3-8B decode shapes against a plain streaming read of the same bytes.
// Launches run back to back (as in a decode graph), each on a different copy of the weights
// so nothing is served from the 256 MB MALL.  Arithmetic per task is k_gemv.hip's.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#ifdef LAB_EXACT
#include "qtypes.h"   // the product's tasks, records and walkers (llamacog_amd/csrc)
#endif

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

template <bool NT> __device__ __forceinline__ uint4 L16(const uint8_t * p) {
    if constexpr (NT) { const v4u v = __builtin_nontemporal_load((const v4u *) p); return make_uint4(v.x, v.y, v.z, v.w); }
    else { uint4 v; __builtin_memcpy(&v, p, 16); return v; }
}
template <bool NT> __device__ __forceinline__ uint2 L8(const uint8_t * p) {
    if constexpr (NT) { const v2u v = __builtin_nontemporal_load((const v2u *) p); return make_uint2(v.x, v.y); }
    else { uint2 v; __builtin_memcpy(&v, p, 8); return v; }
}
template <bool NT> __device__ __forceinline__ uint32_t L2(const uint8_t * p) {
    if constexpr (NT) return __builtin_nontemporal_load((const unsigned short *) p);
    else { uint16_t v; __builtin_memcpy(&v, p, 2); return v; }
}
__device__ __forceinline__ float h2f(uint32_t h) { return __half2float(__ushort_as_half((unsigned short) h)); }
__device__ __forceinline__ int dot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

struct act_t { const int8_t * qs; const float * d; const int16_t * s; };

struct q4K {
    static constexpr int BB = 144;
    struct act { int a[16]; int bs0, bs1; float dy; };
    struct raw { uint4 hdr, qa, qb; };
    __device__ static void load(const act_t & A, int t, act & x) {
        const int b = t >> 2, j = t & 3;
        const int4 * v = (const int4 *) (A.qs + b * 256 + 64 * j);
#pragma unroll
        for (int i = 0; i < 4; ++i) { const int4 q = v[i]; x.a[4 * i] = q.x; x.a[4 * i + 1] = q.y; x.a[4 * i + 2] = q.z; x.a[4 * i + 3] = q.w; }
        const int16_t * bs = A.s + b * 16 + 4 * j;
        x.bs0 = bs[0] + bs[1]; x.bs1 = bs[2] + bs[3]; x.dy = A.d[b];
    }
    template <bool NT> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const uint8_t * blk = wrow + (t >> 2) * 144;
        const int j = t & 3;
        w.hdr = L16<NT>(blk); w.qa = L16<NT>(blk + 16 + 32 * j); w.qb = L16<NT>(blk + 32 + 32 * j);
    }
    __device__ static void fetch_lds(const uint8_t * row, int t, raw & w) {
        const uint8_t * blk = row + (t >> 2) * 144;
        const int j = t & 3;
        w.hdr = *(const uint4 *) blk; w.qa = *(const uint4 *) (blk + 16 + 32 * j); w.qb = *(const uint4 *) (blk + 32 + 32 * j);
    }
    __device__ static float dotr(const raw & w, int t, const act & x) {
        const int j = t & 3;
        const float d = h2f(w.hdr.x & 0xffff), dmin = h2f(w.hdr.x >> 16);
        const uint32_t s0 = w.hdr.y, s1 = w.hdr.z, s2 = w.hdr.w;
        const uint32_t km1 = 0x3f3f3f3f, km2 = 0x0f0f0f0f, km3 = 0x03030303;
        const uint32_t sw = j < 2 ? (s0 & km1) : ((s2 & km2) | (((s0 >> 6) & km3) << 4));
        const uint32_t mw = j < 2 ? (s1 & km1) : (((s2 >> 4) & km2) | (((s1 >> 6) & km3) << 4));
        const int sh = 16 * (j & 1);
        const int sc_lo = (sw >> sh) & 0xff, sc_hi = (sw >> (sh + 8)) & 0xff;
        const int m_lo = (mw >> sh) & 0xff, m_hi = (mw >> (sh + 8)) & 0xff;
        const uint32_t q[8] = {w.qa.x, w.qa.y, w.qa.z, w.qa.w, w.qb.x, w.qb.y, w.qb.z, w.qb.w};
        int dl = 0, dh = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            dl = dot4((int) (q[i] & 0x0f0f0f0f), x.a[i], dl);
            dh = dot4((int) ((q[i] >> 4) & 0x0f0f0f0f), x.a[8 + i], dh);
        }
        return (d * x.dy) * (float) (sc_lo * dl + sc_hi * dh) - (dmin * x.dy) * (float) (m_lo * x.bs0 + m_hi * x.bs1);
    }
};

struct q6K {
    static constexpr int BB = 210;
    struct act { int4 a0, a1, a2, a3; int b0, b1, b2, b3; float dy; };
    struct raw { uint4 la, lb, hh; uint2 sc8; uint32_t d16; };
    __device__ static void load(const act_t & A, int t, act & x) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        const int8_t * ap = A.qs + b * 256 + 128 * h + 16 * lr;
        x.a0 = *(const int4 *) ap; x.a1 = *(const int4 *) (ap + 32); x.a2 = *(const int4 *) (ap + 64); x.a3 = *(const int4 *) (ap + 96);
        const int16_t * bs = A.s + b * 16 + 8 * h + lr;
        x.b0 = 32 * bs[0]; x.b1 = 32 * bs[2]; x.b2 = 32 * bs[4]; x.b3 = 32 * bs[6]; x.dy = A.d[b];
    }
    template <bool NT> __device__ static void fetch(const uint8_t * wrow, int t, raw & w) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        const uint8_t * blk = wrow + b * 210;
        w.la = L16<false>(blk + 64 * h + 16 * lr); w.lb = L16<false>(blk + 64 * h + 32 + 16 * lr);
        w.hh = L16<false>(blk + 128 + 32 * h + 16 * lr); w.sc8 = L8<false>(blk + 192 + 8 * h); w.d16 = L2<false>(blk + 208);
    }
    __device__ static void fetch_lds(const uint8_t * row, int t, raw & w) {
        const int b = t >> 2, h = (t >> 1) & 1, lr = t & 1;
        const uint8_t * blk = row + b * 210;
        uint4 v; __builtin_memcpy(&v, blk + 64 * h + 16 * lr, 16); w.la = v;
        __builtin_memcpy(&v, blk + 64 * h + 32 + 16 * lr, 16); w.lb = v;
        __builtin_memcpy(&v, blk + 128 + 32 * h + 16 * lr, 16); w.hh = v;
        uint2 u; __builtin_memcpy(&u, blk + 192 + 8 * h, 8); w.sc8 = u;
        uint16_t dd; __builtin_memcpy(&dd, blk + 208, 2); w.d16 = dd;
    }
    __device__ static float dotr(const raw & w, int t, const act & x) {
        const int lr = t & 1;
        const float d = h2f(w.d16 & 0xffff);
        const int sc0 = (int8_t) ((w.sc8.x >> (8 * lr)) & 0xff), sc1 = (int8_t) ((w.sc8.x >> (8 * lr + 16)) & 0xff);
        const int sc2 = (int8_t) ((w.sc8.y >> (8 * lr)) & 0xff), sc3 = (int8_t) ((w.sc8.y >> (8 * lr + 16)) & 0xff);
        const uint32_t L[4] = {w.la.x, w.la.y, w.la.z, w.la.w}, M[4] = {w.lb.x, w.lb.y, w.lb.z, w.lb.w}, H[4] = {w.hh.x, w.hh.y, w.hh.z, w.hh.w};
        const int A0[4] = {x.a0.x, x.a0.y, x.a0.z, x.a0.w}, A1[4] = {x.a1.x, x.a1.y, x.a1.z, x.a1.w};
        const int A2[4] = {x.a2.x, x.a2.y, x.a2.z, x.a2.w}, A3[4] = {x.a3.x, x.a3.y, x.a3.z, x.a3.w};
        int s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            s0 = dot4((int) ((L[i] & 0x0f0f0f0f) | ((H[i] & 0x03030303) << 4)), A0[i], s0);
            s1 = dot4((int) ((M[i] & 0x0f0f0f0f) | (((H[i] >> 2) & 0x03030303) << 4)), A1[i], s1);
            s2 = dot4((int) (((L[i] >> 4) & 0x0f0f0f0f) | (((H[i] >> 4) & 0x03030303) << 4)), A2[i], s2);
            s3 = dot4((int) (((M[i] >> 4) & 0x0f0f0f0f) | (((H[i] >> 6) & 0x03030303) << 4)), A3[i], s3);
        }
        return (d * x.dy) * (float) (sc0 * (s0 - x.b0) + sc1 * (s1 - x.b1) + sc2 * (s2 - x.b2) + sc3 * (s3 - x.b3));
    }
};

struct args { const uint8_t * W; int64_t nb01; int64_t M; float * dst; act_t A; int ntasks; int64_t ngroups; };

// one-shot: one row group per workgroup, every load of the group issued at once
template <class T, int R, int WPR, bool NT>
__global__ __launch_bounds__(256) void k_oneshot(const args p) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wsub = wave % WPR;
    const int t = wsub * 64 + lane;
    const bool active = t < p.ntasks;
    const int tt = active ? t : 0;
    const int64_t row0 = (int64_t) blockIdx.x * (4 / WPR) * R + (wave / WPR) * R;
    typename T::raw w[R];
#pragma unroll
    for (int r = 0; r < R; ++r) T::template fetch<NT>(p.W + min(row0 + r, p.M - 1) * p.nb01, tt, w[r]);
    typename T::act x;
    T::load(p.A, tt, x);
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = wsum(active ? T::dotr(w[r], tt, x) : 0.0f);
    if constexpr (WPR > 1) {
        __shared__ float red[4][R];
        if (lane == 0) for (int r = 0; r < R; ++r) red[wave][r] = acc[r];
        __syncthreads();
        if (wsub == 0) for (int r = 0; r < R; ++r) { float s = red[wave][r]; for (int k = 1; k < WPR; ++k) s += red[wave + k][r]; acc[r] = s; }
    }
    if (wsub == 0 && lane < R) {
        float v = acc[0];
#pragma unroll
        for (int r = 1; r < R; ++r) v = lane == r ? acc[r] : v;
        if (row0 + lane < p.M) p.dst[row0 + lane] = v;
    }
}

// persistent, prefetch one group ahead (k_gemv_pipe's structure); weights fetched before the
// activation so the first HBM request leaves at once
template <class T, int R, int WPR, bool NT>
__global__ __launch_bounds__(256) void k_pipe(const args p) {
    constexpr int RPG = (4 / WPR) * R;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wsub = wave % WPR;
    const int t = wsub * 64 + lane;
    const bool active = t < p.ntasks;
    const int tt = active ? t : 0;
    auto fetch = [&](int64_t g, typename T::raw (&w)[R]) {
        const int64_t row0 = g * RPG + (wave / WPR) * R;
#pragma unroll
        for (int r = 0; r < R; ++r) T::template fetch<NT>(p.W + min(row0 + r, p.M - 1) * p.nb01, tt, w[r]);
    };
    typename T::raw cur[R], nxt[R];
    int64_t g = blockIdx.x;
    if (g < p.ngroups) fetch(g, cur);
    typename T::act x;
    T::load(p.A, tt, x);
    __shared__ float red[2][4][R];
    int par = 0;
    for (; g < p.ngroups; g += gridDim.x, par ^= 1) {
        const int64_t gn = g + gridDim.x;
        if (gn < p.ngroups) fetch(gn, nxt);
        float acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = wsum(active ? T::dotr(cur[r], tt, x) : 0.0f);
        if constexpr (WPR > 1) {
            if (lane == 0) for (int r = 0; r < R; ++r) red[par][wave][r] = acc[r];
            __syncthreads();
            if (wsub == 0) for (int r = 0; r < R; ++r) { float s = red[par][wave][r]; for (int k = 1; k < WPR; ++k) s += red[par][wave + k][r]; acc[r] = s; }
        }
        if (wsub == 0 && lane < R) {
            const int64_t row0 = g * RPG + (wave / WPR) * R;
            float v = acc[0];
#pragma unroll
            for (int r = 1; r < R; ++r) v = lane == r ? acc[r] : v;
            if (row0 + lane < p.M) p.dst[row0 + lane] = v;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) cur[r] = nxt[r];
    }
}


// LDS ring: each wave streams its row groups HBM -> LDS by LDS-DMA (global_load_lds, 1 KiB of
// contiguous bytes per wave instruction: every 128-B line requested once), NS - 1 groups ahead;
// its lanes then read their task slices (T::fetch_lds) from the slot.  In flight per wave:
// NS - 1 groups, without VGPRs.
typedef __attribute__((address_space(3))) void * lds_ptr_t;
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }

template <class T, int R, int WPR, int NS, bool NT>
__global__ __launch_bounds__(256) void k_ring(const args p) {
    constexpr int RPG = (4 / WPR) * R;
    constexpr int SEG = 16 * T::BB;                       // a wave's row slice: 16 blocks = 64 tasks
    constexpr int NI = (SEG + 1023) / 1024;               // DMA instructions per row slice
    constexpr int SLOT = R * NI * 1024;                   // bytes per group slot
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wsub = wave % WPR;
    const int t = wsub * 64 + lane;
    const bool active = t < p.ntasks;
    const int tt = active ? t : 0;
    const int nt_w = min(64, p.ntasks - 64 * wsub);       // this wave's tasks in a row
    const int seg = (nt_w / 4) * T::BB;
    uint8_t * ring = lds + (size_t) wave * NS * SLOT;
    auto issue = [&](int64_t g, int slot) {
        const int64_t row0 = g * RPG + (wave / WPR) * R;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint8_t * src = p.W + min(row0 + r, p.M - 1) * p.nb01 + (int64_t) wsub * SEG;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int off = min(i * 1024 + 16 * lane, seg - 16);
                __builtin_amdgcn_global_load_lds((const void *) (src + off), (lds_ptr_t) (ring + slot * SLOT + r * NI * 1024 + i * 1024),
                                                 16, 0, NT ? 2 : 0);
            }
        }
    };
    typename T::act x;
    T::load(p.A, tt, x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int64_t g0 = blockIdx.x, st = gridDim.x;
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) {
        if (g0 + s * st < p.ngroups) issue(g0 + s * st, s);
    }
    __shared__ float red[2][4][R];
    int par = 0, slot = 0;
    for (int64_t g = g0; g < p.ngroups; g += st, par ^= 1) {
        const int64_t ga = g + (NS - 1) * st;   // the group issued now
        int ahead = 0;                          // groups issued after g (still in flight)
#pragma unroll
        for (int s = 1; s < NS; ++s) ahead += g + s * st < p.ngroups ? 1 : 0;
        if (ga < p.ngroups) issue(ga, (slot + NS - 1) % NS);
        if (ahead == NS - 1) wait_vm<(NS - 1) * R * NI>();
        else if (ahead == NS - 2 && NS >= 2) wait_vm<(NS >= 2 ? NS - 2 : 0) * R * NI>();
        else if (ahead == NS - 3 && NS >= 3) wait_vm<(NS >= 3 ? NS - 3 : 0) * R * NI>();
        else wait_vm<0>();
        typename T::raw w[R];
#pragma unroll
        for (int r = 0; r < R; ++r) T::fetch_lds(ring + slot * SLOT + r * NI * 1024, tt - 64 * wsub, w[r]);
        float acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = wsum(active ? T::dotr(w[r], tt, x) : 0.0f);
        if constexpr (WPR > 1) {
            if (lane == 0) for (int r = 0; r < R; ++r) red[par][wave][r] = acc[r];
            __syncthreads();
            if (wsub == 0) for (int r = 0; r < R; ++r) { float s = red[par][wave][r]; for (int k = 1; k < WPR; ++k) s += red[par][wave + k][r]; acc[r] = s; }
        }
        if (wsub == 0 && lane < R) {
            const int64_t row0 = g * RPG + (wave / WPR) * R;
            float v = acc[0];
#pragma unroll
            for (int r = 1; r < R; ++r) v = lane == r ? acc[r] : v;
            if (row0 + lane < p.M) p.dst[row0 + lane] = v;
        }
        slot = (slot + 1) % NS;
    }
}

// one-shot with the group staged through LDS by LDS-DMA: each wave copies its R row slices
// (contiguous 1 KiB per instruction) at entry, loads the activation, waits, then reads its
// task slices from LDS.  The dispatcher's WG turnover provides the pipelining.
template <class T, int R, int WPR, bool NT>
__global__ __launch_bounds__(256) void k_oneshot_lds(const args p) {
    constexpr int SEG = 16 * T::BB;
    constexpr int NI = (SEG + 1023) / 1024;
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * R * NI * 1024];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wsub = wave % WPR;
    const int t = wsub * 64 + lane;
    const bool active = t < p.ntasks;
    const int tt = active ? t : 0;
    const int nt_w = min(64, p.ntasks - 64 * wsub);
    const int seg = (nt_w / 4) * T::BB;
    uint8_t * mine = lds + wave * R * NI * 1024;
    const int64_t row0 = (int64_t) blockIdx.x * (4 / WPR) * R + (wave / WPR) * R;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint8_t * src = p.W + min(row0 + r, p.M - 1) * p.nb01 + (int64_t) wsub * SEG;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int off = min(i * 1024 + 16 * lane, seg - 16);
            __builtin_amdgcn_global_load_lds((const void *) (src + off), (lds_ptr_t) (mine + r * NI * 1024 + i * 1024), 16, 0, NT ? 2 : 0);
        }
    }
    typename T::act x;
    T::load(p.A, tt, x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    typename T::raw w[R];
#pragma unroll
    for (int r = 0; r < R; ++r) T::fetch_lds(mine + r * NI * 1024, tt - 64 * wsub, w[r]);
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = wsum(active ? T::dotr(w[r], tt, x) : 0.0f);
    if constexpr (WPR > 1) {
        __shared__ float red[4][R];
        if (lane == 0) for (int r = 0; r < R; ++r) red[wave][r] = acc[r];
        __syncthreads();
        if (wsub == 0) for (int r = 0; r < R; ++r) { float s = red[wave][r]; for (int k = 1; k < WPR; ++k) s += red[wave + k][r]; acc[r] = s; }
    }
    if (wsub == 0 && lane < R) {
        float v = acc[0];
#pragma unroll
        for (int r = 1; r < R; ++r) v = lane == r ? acc[r] : v;
        if (row0 + lane < p.M) p.dst[row0 + lane] = v;
    }
}

#ifdef LAB_EXACT
// the product's one-shot body (k_gemv.hip gemv_os_body, MODE 0 without epilogues): LDS-DMA
// weights, records in LDS, the CPU-order walker.  STAGE < 3 cuts it short for attribution:
// 0 = stop after the DMA wait, 1 = + rec (records), 2 = + walker
template <class T, int R, int WPR, int STAGE>
__global__ __launch_bounds__(256) void k_os_exact(const uint8_t * W, int64_t nb01, int64_t M, float * dst, mi355x::gemv_act Aa,
                                                   int ntasks) {
    using namespace mi355x;
    constexpr int RPG = (4 / WPR) * R;
    constexpr int SEG = (64 / T::per_block) * T::blk_bytes, NI = (SEG + 1023) / 1024, SLICE = NI * 1024;
    extern __shared__ __attribute__((aligned(16))) uint32_t xr[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wsub = wave % WPR;
    const int t = wsub * 64 + lane;
    const bool active = t < ntasks;
    const int tt = active ? t : 0;
    const int nb = ntasks / T::per_block;
    const int rowl0 = (wave / WPR) * R;
    const int64_t row0 = (int64_t) blockIdx.x * RPG + rowl0;
    uint8_t * mine = (uint8_t *) xr + 8192 + (size_t) wave * R * SLICE;
    const int nt_w = min(64, ntasks - 64 * wsub);
    const int seg = (nt_w / T::per_block) * T::blk_bytes;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint8_t * src = W + min(row0 + r, M - 1) * nb01 + (int64_t) wsub * SEG;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int off = min(i * 1024 + 16 * lane, seg - 16);
            __builtin_amdgcn_global_load_lds((const void *) (src + off), (lds_ptr_t) (mine + r * SLICE + i * 1024), 16, 0, 2);
        }
    }
    typename T::act x;
    T::load(Aa, tt, x);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (STAGE == 0) {
        if (lane == 0 && row0 < M) dst[row0] = (float) mine[lane];
        return;
    }
    uint32_t * xb = xr;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        typename T::raw w;
        T::template fetch<ld_lds>(mine + r * SLICE - (int64_t) wsub * SEG, tt, w);
        T::rec(w, tt, x, active, xb + (size_t) (rowl0 + r) * nb * T::RS);
    }
    if constexpr (WPR > 1) __syncthreads();
    else wave_lds_sync();
    if (STAGE == 1) {
        if (lane == 0 && row0 < M) dst[row0] = __uint_as_float(xb[(size_t) rowl0 * nb * T::RS + 1]);
        return;
    }
    const int wr = lane / T::LPR, ws = lane % T::LPR;
    const int wrc = wr < R ? wr : 0;
    if (wsub == 0) {
        const float v = T::walk(xb + (size_t) (rowl0 + wrc) * nb * T::RS, nb, ws);
        if (wr < R && ws == 0 && row0 + wr < M) dst[row0 + wr] = v;
    }
}

#endif

__global__ __launch_bounds__(256) void k_read(const uint4 * __restrict__ p, size_t n16, unsigned * __restrict__ out) {
    unsigned acc = 0;
    const size_t stride = (size_t) gridDim.x * blockDim.x;
    size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n16; i += 8 * stride) {
        v4u v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load((const v4u *) (p + i + u * stride));
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) { const uint4 v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678u) out[0] = acc;
}

static hipStream_t S;
static hipEvent_t E0, E1;
static uint8_t * POOL;
static const size_t POOLB = 3ull << 30;

template <class F>
static double time_us(size_t bytes, F && launch) {
    const int nslots = (int) (POOLB / ((bytes + 4095) / 4096 * 4096));
    for (int i = 0; i < 4; ++i) launch(i % nslots);
    const int N = 40;
    CK(hipEventRecord(E0, S));
    for (int i = 0; i < N; ++i) launch((i + 4) % nslots);
    CK(hipEventRecord(E1, S));
    CK(hipEventSynchronize(E1));
    float ms;
    CK(hipEventElapsedTime(&ms, E0, E1));
    return ms * 1000.0 / N;
}

template <class T, int R, int WPR, bool NT>
static void run_variant(const char * shape, int64_t K, int64_t M, act_t A, float * dst, int mode, int wgs) {
    const int64_t nb01 = K / 256 * T::BB;
    const size_t bytes = (size_t) nb01 * M;
    const size_t slot = (bytes + 4095) / 4096 * 4096;
    args a = {nullptr, nb01, M, dst, A, (int) (K / 64), 0};
    constexpr int RPG = (4 / WPR) * R;
    a.ngroups = (M + RPG - 1) / RPG;
    const double us = time_us(bytes, [&](int s) {
        a.W = POOL + (size_t) s * slot;
        if (mode == 0) hipLaunchKernelGGL((k_oneshot<T, R, WPR, NT>), dim3((unsigned) a.ngroups), dim3(256), 0, S, a);
        else if (mode == 3) hipLaunchKernelGGL((k_oneshot_lds<T, R, WPR, NT>), dim3((unsigned) a.ngroups), dim3(256), 0, S, a);
        else hipLaunchKernelGGL((k_pipe<T, R, WPR, NT>), dim3((unsigned) std::min<int64_t>(a.ngroups, wgs)), dim3(256), 0, S, a);
    });
    printf("%-14s %s R=%d WPR=%d NT=%d %-7s wgs=%5d  %8.2f us  %5.2f TB/s\n", shape, T::BB == 144 ? "q4K" : "q6K", R, WPR, (int) NT,
           mode == 0 ? "oneshot" : (mode == 3 ? "os_lds" : "pipe"), mode == 0 || mode == 3 ? (int) a.ngroups : wgs, us, bytes / us / 1e6);
}

template <class T, int R, int WPR, int NS, bool NT>
static void run_ring(const char * shape, int64_t K, int64_t M, act_t A, float * dst, int wgs) {
    const int64_t nb01 = K / 256 * T::BB;
    const size_t bytes = (size_t) nb01 * M;
    const size_t slot = (bytes + 4095) / 4096 * 4096;
    args a = {nullptr, nb01, M, dst, A, (int) (K / 64), 0};
    constexpr int RPG = (4 / WPR) * R;
    a.ngroups = (M + RPG - 1) / RPG;
    constexpr int SEG = 16 * T::BB, NI = (SEG + 1023) / 1024;
    const size_t lds = (size_t) 4 * NS * R * NI * 1024;
    if (lds > 144 * 1024) return;
    static bool attr = false;
    if (!attr) { CK(hipFuncSetAttribute((const void *) k_ring<T, R, WPR, NS, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds)); attr = true; }
    const double us = time_us(bytes, [&](int s) {
        a.W = POOL + (size_t) s * slot;
        hipLaunchKernelGGL((k_ring<T, R, WPR, NS, NT>), dim3((unsigned) std::min<int64_t>(a.ngroups, wgs)), dim3(256), lds, S, a);
    });
    printf("%-14s %s R=%d WPR=%d NT=%d ring%d   wgs=%5d  %8.2f us  %5.2f TB/s  (lds %zu KB/wg)\n", shape, T::BB == 144 ? "q4K" : "q6K", R, WPR,
           (int) NT, NS, wgs, us, bytes / us / 1e6, lds / 1024);
}

#ifdef LAB_EXACT
template <class T, int R, int WPR, int STAGE>
static void run_exact(const char * shape, int64_t K, int64_t M, act_t A, float * dst) {
    const int64_t nb01 = K / 256 * T::blk_bytes * (T::per_block == 4 ? 1 : 8);
    const size_t bytes = (size_t) nb01 * M;
    const size_t slot = (bytes + 4095) / 4096 * 4096;
    constexpr int RPG = (4 / WPR) * R;
    const int64_t ng = (M + RPG - 1) / RPG;
    constexpr int SEG = (64 / T::per_block) * T::blk_bytes, NI = (SEG + 1023) / 1024;
    const size_t lds = 8192 + (size_t) 4 * R * NI * 1024;   // (records: 8 KiB, more than any of these)
    const int ntasks = (int) (K / 64);
    mi355x::gemv_act Aa = {A.qs, A.d, A.s};
    const double us = time_us(bytes, [&](int s) {
        hipLaunchKernelGGL((k_os_exact<T, R, WPR, STAGE>), dim3((unsigned) ng), dim3(256), lds, S, POOL + (size_t) s * slot, nb01, M, dst,
                           Aa, ntasks);
    });
    printf("%-14s exact R=%d WPR=%d stage%d wgs=%5d  %8.2f us  %5.2f TB/s\n", shape, R, WPR, STAGE, (int) ng, us, bytes / us / 1e6);
}
#endif

template <class T, int WPR>
static void sweep(const char * shape, int64_t K, int64_t M, act_t A, float * dst) {
    run_variant<T, 1, WPR, false>(shape, K, M, A, dst, 0, 0);
    run_variant<T, 2, WPR, false>(shape, K, M, A, dst, 0, 0);
    run_variant<T, 2, WPR, true>(shape, K, M, A, dst, 0, 0);
    run_variant<T, 1, WPR, true>(shape, K, M, A, dst, 3, 0);
    run_variant<T, 2, WPR, true>(shape, K, M, A, dst, 3, 0);
    run_variant<T, 2, WPR, false>(shape, K, M, A, dst, 3, 0);
    run_variant<T, 4, WPR, true>(shape, K, M, A, dst, 3, 0);
    for (int wgs : {1024, 2048}) run_variant<T, 2, WPR, true>(shape, K, M, A, dst, 1, wgs);
    for (int wgs : {768, 1024}) run_ring<T, 1, WPR, 3, true>(shape, K, M, A, dst, wgs);
}

int main() {
    CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
    CK(hipEventCreate(&E0));
    CK(hipEventCreate(&E1));
    CK(hipMalloc(&POOL, POOLB));
    CK(hipMemset(POOL, 0x11, POOLB));
    int8_t * qs; float * d; int16_t * s; float * dst; unsigned * o;
    CK(hipMalloc(&qs, 1 << 16)); CK(hipMalloc(&d, 4096)); CK(hipMalloc(&s, 8192)); CK(hipMalloc(&dst, 1 << 20)); CK(hipMalloc(&o, 64));
    CK(hipMemset(qs, 3, 1 << 16)); CK(hipMemset(d, 0, 4096)); CK(hipMemset(s, 0, 8192));
    act_t A = {qs, d, s};
    // streaming-read floor for each size
    for (size_t bytes : {9437184ul, 14155776ul, 33030144ul, 48168960ul, 66060288ul, 440000000ul}) {
        for (int blocks : {2048}) {
            const size_t slot = (bytes + 4095) / 4096 * 4096;
            const double us = time_us(bytes, [&](int sl) {
                hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, S, (const uint4 *) (POOL + (size_t) sl * slot), bytes / 16, o);
            });
            printf("read %7.2f MB blocks %5d  %8.2f us  %5.2f TB/s\n", bytes / 1e6, blocks, us, bytes / us / 1e6);
        }
    }
#ifdef LAB_EXACT
    for (int st = 0; st < 4; ++st) {
        auto go = [&](auto stc) {
            constexpr int ST = decltype(stc)::value;
            run_exact<mi355x::g_q4_K, 1, 1, ST>("gu 4096x28672", 4096, 28672, A, dst);
            run_exact<mi355x::g_q4_K, 2, 4, ST>("dn 14336x4096", 14336, 4096, A, dst);
            run_exact<mi355x::g_q6_K, 1, 4, ST>("dn6 14336x4096", 14336, 4096, A, dst);
            run_exact<mi355x::g_q6_K, 1, 1, ST>("out 4096x128256", 4096, 128256, A, dst);
        };
        if (st == 0) go(std::integral_constant<int, 0>());
        if (st == 1) go(std::integral_constant<int, 1>());
        if (st == 2) go(std::integral_constant<int, 2>());
        if (st == 3) go(std::integral_constant<int, 3>());
    }
    run_variant<q4K, 1, 1, true>("gu 4096x28672", 4096, 28672, A, dst, 3, 0);
    run_variant<q4K, 2, 4, true>("dn 14336x4096", 14336, 4096, A, dst, 3, 0);
    run_variant<q6K, 1, 4, true>("dn6 14336x4096", 14336, 4096, A, dst, 3, 0);
    run_variant<q6K, 1, 1, true>("out 4096x128256", 4096, 128256, A, dst, 3, 0);
    return 0;
#endif
    sweep<q4K, 1>("qkv 4096x6144", 4096, 6144, A, dst);
    sweep<q4K, 1>("o 4096x4096", 4096, 4096, A, dst);
    sweep<q4K, 1>("gu 4096x28672", 4096, 28672, A, dst);
    sweep<q4K, 4>("dn 14336x4096", 14336, 4096, A, dst);
    sweep<q6K, 4>("dn6 14336x4096", 14336, 4096, A, dst);
    sweep<q6K, 1>("out 4096x128256", 4096, 128256, A, dst);
    return 0;
}
