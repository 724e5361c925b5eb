// common.h — shared definitions for the MI355X (gfx950, CDNA4) ggml backend.
//
// The backend is compiled against the reference's public ggml ABI headers
// (ggml/include/ggml.h, ggml-backend.h and ggml/src/ggml-backend-impl.h); nothing
// from ggml-cuda / ggml-hip is used.  Quant block layouts are restated here with
// static_asserts against the sizes fixed in ggml/src/ggml-common.h:167-334.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstddef>
#include <cstring>

#include "ggml.h"
#include "ggml-backend.h"
#include "libm_exact.h"

extern "C" void ggml_log_internal(enum ggml_log_level level, const char * format, ...);

#define MI_LOG_INFO(...)  ggml_log_internal(GGML_LOG_LEVEL_INFO,  __VA_ARGS__)
#define MI_LOG_WARN(...)  ggml_log_internal(GGML_LOG_LEVEL_WARN,  __VA_ARGS__)
#define MI_LOG_ERROR(...) ggml_log_internal(GGML_LOG_LEVEL_ERROR, __VA_ARGS__)
#define MI_LOG_DEBUG(...) ggml_log_internal(GGML_LOG_LEVEL_DEBUG, __VA_ARGS__)

// Fatal HIP error: mirrors the reference's CUDA_CHECK -> ggml_cuda_error -> abort
// (ggml/src/ggml-cuda/ggml-cuda.cu:70-81) with the HIP error string.
#define MI_CHECK(expr)                                                                      \
    do {                                                                                    \
        hipError_t mi_err_ = (expr);                                                        \
        if (mi_err_ != hipSuccess) {                                                        \
            ggml_abort(__FILE__, __LINE__, "MI355X: %s failed: %s", #expr,                 \
                       hipGetErrorString(mi_err_));                                         \
        }                                                                                   \
    } while (0)

namespace mi355x {

constexpr int WAVE = 64;   // CDNA wavefront width
constexpr int QK_K = 256;  // K-quant super-block

// ---- quant blocks (byte-exact restatement of ggml-common.h) ------------------------------
struct blk_q4_0 { uint16_t d; uint8_t qs[16]; };
struct blk_q8_0 { uint16_t d; int8_t qs[32]; };
struct blk_q4_K { uint16_t d; uint16_t dmin; uint8_t scales[12]; uint8_t qs[128]; };
struct blk_q5_K { uint16_t d; uint16_t dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; };
struct blk_q6_K { uint8_t ql[128]; uint8_t qh[64]; int8_t scales[16]; uint16_t d; };
struct blk_q8_K { float d; int8_t qs[256]; int16_t bsums[16]; };

static_assert(sizeof(blk_q4_0) == 18,  "q4_0");
static_assert(sizeof(blk_q8_0) == 34,  "q8_0");
static_assert(sizeof(blk_q4_K) == 144, "q4_K");
static_assert(sizeof(blk_q5_K) == 176, "q5_K");
static_assert(sizeof(blk_q6_K) == 210, "q6_K");
static_assert(sizeof(blk_q8_K) == 292, "q8_K");

// ---- device helpers ------------------------------------------------------------------------
__device__ __forceinline__ float h2f(uint16_t h) { return __half2float(__ushort_as_half(h)); }
__device__ __forceinline__ uint16_t f2h(float f) { return __half_as_ushort(__float2half_rn(f)); }

// 16/8/4-byte loads from arbitrarily aligned addresses.  gfx950 under ROCm runs in
// unaligned-access mode, so the compiler lowers these to single dwordx4/x2/dword loads.
__device__ __forceinline__ uint4 ld16(const void * p) { uint4 v; __builtin_memcpy(&v, p, 16); return v; }
__device__ __forceinline__ uint2 ld8(const void * p)  { uint2 v; __builtin_memcpy(&v, p, 8);  return v; }
__device__ __forceinline__ uint32_t ld4(const void * p) { uint32_t v; __builtin_memcpy(&v, p, 4); return v; }
__device__ __forceinline__ uint16_t ld2(const void * p) { uint16_t v; __builtin_memcpy(&v, p, 2); return v; }

__device__ __forceinline__ int dot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

// In-graph kernel timeline (profiling only, exec_ctx::kt_take): per workgroup the chip-wide
// 100 MHz realtime counter at entry (slot 0) and at each wave's exit (slots 1 .. waves), so the
// host can rebuild every instrumented launch's start, dispatch ramp, end and the gaps between
// launches inside a REPLAYED hipGraph (rocprofv3 cannot trace replayed graphs on ROCm 7.2).
__device__ __forceinline__ unsigned kt_wg() { return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); }
// stride: the region's slots per workgroup (exec_ctx::kt_take's 1 + threads / 64), passed in by the
// kernel: blockDim is a 16-bit load from the dispatch packet, a memory round trip that held wave 0
// of every traced workgroup at its entry
__device__ __forceinline__ void kt_enter(unsigned long long * kt, unsigned stride) {
    if (kt && threadIdx.x == 0) kt[stride * kt_wg()] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void kt_exit(unsigned long long * kt, unsigned stride) {
    if (kt && (threadIdx.x & 63) == 0) kt[stride * kt_wg() + 1 + threadIdx.x / 64] = __builtin_amdgcn_s_memrealtime();
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
    return v;
}

// DPP lane exchanges (VALU, no LDS round trip): within quads (xor 1, xor 2), half-row mirror
// (lane i <-> 7-i of each 8) and row mirror (i <-> 15-i of each 16).  Every pairing is total,
// so a commutative reduction over them leaves each group's result in all of its lanes.
template <int CTRL>
__device__ __forceinline__ int dpp(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HMIRROR = 0x141, DPP_MIRROR = 0x140;
__device__ __forceinline__ int quad_sum(int v) { v += dpp<DPP_XOR1>(v); return v + dpp<DPP_XOR2>(v); }
__device__ __forceinline__ float dppf_xor1(float v) { return __int_as_float(dpp<DPP_XOR1>(__float_as_int(v))); }
__device__ __forceinline__ float dppf_xor2(float v) { return __int_as_float(dpp<DPP_XOR2>(__float_as_int(v))); }
// lane i <- lane i^4: row_shr:4 for lanes with bit 2 set, row_shl:4 for the others
__device__ __forceinline__ float dppf_xor4(float v) {
    const int up = dpp<0x114>(__float_as_int(v)), dn = dpp<0x104>(__float_as_int(v));
    return __int_as_float((threadIdx.x & 4) ? up : dn);
}
__device__ __forceinline__ int oct_sum(int v) { v = quad_sum(v); return v + dpp<DPP_HMIRROR>(v); }
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = (uint64_t) __double_as_longlong(v);
    const uint32_t lo = (uint32_t) dpp<CTRL>((int) (uint32_t) b), hi = (uint32_t) dpp<CTRL>((int) (uint32_t) (b >> 32));
    return __longlong_as_double((long long) (((uint64_t) hi << 32) | lo));
}
// a wave-uniform double sum (all 64 lanes active) in a fixed order that is NOT the shuffle
// tree's: rows by DPP, then the four row sums by readlane.  For sums whose result is decided
// against the CPU's own order afterwards (rms_mean_decided)
__device__ __forceinline__ double wave_sum_rows_f64(double v) {
    v = __dadd_rn(v, dpp_f64<DPP_XOR1>(v));
    v = __dadd_rn(v, dpp_f64<DPP_XOR2>(v));
    v = __dadd_rn(v, dpp_f64<DPP_HMIRROR>(v));
    v = __dadd_rn(v, dpp_f64<DPP_MIRROR>(v));
    auto rl = [&](int l) {
        const uint64_t b = (uint64_t) __double_as_longlong(v);
        const uint32_t lo = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) b, l);
        const uint32_t hi = (uint32_t) __builtin_amdgcn_readlane((int) (uint32_t) (b >> 32), l);
        return __longlong_as_double((long long) (((uint64_t) hi << 32) | lo));
    };
    return __dadd_rn(__dadd_rn(rl(0), rl(16)), __dadd_rn(rl(32), rl(48)));
}
// the sum of a 16-lane row by DPP (every lane of the row holds it); same caveat on the order
__device__ __forceinline__ double row_sum16_f64(double v) {
    v = __dadd_rn(v, dpp_f64<DPP_XOR1>(v));
    v = __dadd_rn(v, dpp_f64<DPP_XOR2>(v));
    v = __dadd_rn(v, dpp_f64<DPP_HMIRROR>(v));
    return __dadd_rn(v, dpp_f64<DPP_MIRROR>(v));
}
// wave-uniform max / min of unsigned 32-bit values (all 64 lanes active): rows by DPP, then
// the four row results by readlane
__device__ __forceinline__ uint32_t wave_umax(uint32_t v) {
    v = max(v, (uint32_t) dpp<DPP_XOR1>((int) v));
    v = max(v, (uint32_t) dpp<DPP_XOR2>((int) v));
    v = max(v, (uint32_t) dpp<DPP_HMIRROR>((int) v));
    v = max(v, (uint32_t) dpp<DPP_MIRROR>((int) v));
    const uint32_t a = (uint32_t) __builtin_amdgcn_readlane((int) v, 0), b = (uint32_t) __builtin_amdgcn_readlane((int) v, 16);
    const uint32_t c = (uint32_t) __builtin_amdgcn_readlane((int) v, 32), d = (uint32_t) __builtin_amdgcn_readlane((int) v, 48);
    return max(max(a, b), max(c, d));
}
__device__ __forceinline__ uint32_t wave_umin(uint32_t v) {
    v = min(v, (uint32_t) dpp<DPP_XOR1>((int) v));
    v = min(v, (uint32_t) dpp<DPP_XOR2>((int) v));
    v = min(v, (uint32_t) dpp<DPP_HMIRROR>((int) v));
    v = min(v, (uint32_t) dpp<DPP_MIRROR>((int) v));
    const uint32_t a = (uint32_t) __builtin_amdgcn_readlane((int) v, 0), b = (uint32_t) __builtin_amdgcn_readlane((int) v, 16);
    const uint32_t c = (uint32_t) __builtin_amdgcn_readlane((int) v, 32), d = (uint32_t) __builtin_amdgcn_readlane((int) v, 48);
    return min(min(a, b), min(c, d));
}

// ggml_v_expf of the AVX-512 CPU backend (ggml-cpu/vec.h:731-756), bit-exact: the
// reference's SiLU and soft_max use it, not libm expf.
__device__ __forceinline__ float v_expf_avx512(float x) {
    const float r = 0x1.8p23f;
    const float z = fmaf(x, 0x1.715476p+0f, r);
    const float n = __fsub_rn(z, r);
    const float b = fmaf(-n, 0x1.7f7d1cp-20f, fmaf(-n, 0x1.62e4p-1f, x));
    const float u = __fmul_rn(b, b);
    const float j = fmaf(fmaf(fmaf(0x1.0e4020p-7f, b, 0x1.573e2ep-5f), u, fmaf(0x1.555e66p-3f, b, 0x1.fffdb6p-2f)), u,
                         fmaf(0x1.ffffecp-1f, b, 1.0f));
    if (fabsf(n) > 192.0f) return n <= 0.0f ? 0.0f : INFINITY;
    return ldexpf(j, (int) n);  // _mm512_scalef_ps(j, n)
}

// glibc expf as the CPU backend's scalar paths call it (libm_exact.h restates its algorithm
// bit for bit; a correctly rounded exp differs from it on a small fraction of inputs)
__device__ __forceinline__ float expf_cr(float x) { return lx_expf(x); }

// the _mm512_reduce_add_ps tree (GCC avx512fintrin.h) over 16 lane values
__device__ __forceinline__ float reduce16_avx512(const float (&w)[16]) {
    float t3[8], t6[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) t3[i] = __fadd_rn(w[8 + i], w[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) t6[i] = __fadd_rn(t3[4 + i], t3[i]);
    return __fadd_rn(__fadd_rn(t6[0], t6[2]), __fadd_rn(t6[1], t6[3]));
}

// 6-bit scale/min unpack of Q4_K/Q5_K (ggml-quants.c:625 get_scale_min_k4)
__device__ __forceinline__ void scale_min_k4(int j, const uint8_t * q, int & d, int & m) {
    if (j < 4) {
        d = q[j] & 63;
        m = q[j + 4] & 63;
    } else {
        d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

// ---- host helpers ----------------------------------------------------------------------------
static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace mi355x
