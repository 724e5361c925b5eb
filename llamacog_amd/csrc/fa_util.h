// fa_util.h — device helpers of the CPU-exact flash-attention kernels (k_fattn_exact.hip) shared
// with the Q/K/V launch that carries the short-context decode attention (k_gemv.hip, fa_dsh4.h).
#pragma once
#include "common.h"
#include <hip/hip_fp16.h>

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

// lane q of a quad reads lane (q | 2) / (q | 1): quad_perm [2,3,2,3] / [1,1,3,3]
__device__ __forceinline__ float quad_from_plus2(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xEE, 0xf, 0xf, false));
}
__device__ __forceinline__ float quad_from_plus1(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xF5, 0xf, 0xf, false));
}

typedef __attribute__((address_space(3))) void * lds_ptr_t;

// LDS-DMA of 16 B per lane issued as inline asm: the compiler then sees no LDS write in flight
// and does not drain vmcnt before the issuing wave's next LDS read (with the builtin it waited
// for the V stage — and for the next chunk's K loads issued after it — before every score
// write / coefficient read of k_fattn_dec2's producers).  The caller waits for the data itself.
__device__ __forceinline__ void lds_dma16(const void * src, const void * lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (lds_ptr_t) lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m), "v"(src) : "memory", "m0");
}

// the same for 4 B per lane (global_load_lds_dword): rows that are not 16-B granular (q8_0 / q4_0
// cache rows of 136 / 72 B) packed in LDS
__device__ __forceinline__ void lds_dma4(const void * src, const void * lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (lds_ptr_t) lds);
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dword %1, off" ::"s"(m), "v"(src) : "memory", "m0");
}

// s_waitcnt vmcnt(n) for a runtime n (an immediate operand: one case per count, up to 63)
__device__ __forceinline__ void eng_vm_wait_fa(int n) {
#define FW(k) case k: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(k) : "memory"); break;
#define FW8(k) FW(k) FW(k + 1) FW(k + 2) FW(k + 3) FW(k + 4) FW(k + 5) FW(k + 6) FW(k + 7)
    switch (n) {
        FW8(0) FW8(8) FW8(16) FW8(24) FW8(32) FW8(40) FW8(48) FW(56) FW(57) FW(58) FW(59) FW(60) FW(61) FW(62) FW(63)
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
#undef FW8
#undef FW
}

// one step of the f16 accumulation, y = f16(fma(v, vs, y)) with v and y as f16 bits in the low
// halves: v_fma_mix_f32 converts both exactly and rounds the fma once to f32, v_cvt_f16_f32
// rounds that to f16 — the CPU's cvtph_ps / fmadd_ps / cvtps_ph sequence, two dependent
// instructions (written out so the compiler neither fuses the two roundings into
// v_fma_mixlo_f16 nor re-packs y between steps)
__device__ __forceinline__ uint32_t f16_mad(uint32_t vbits, float vs, uint32_t ybits) {
    float t;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(vbits), "v"(vs), "v"(ybits));
    uint32_t r;
    asm("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}

// y = f16(f32(y) * ms): v_fma_mix_f32 with a -0 addend is the product rounded once to f32 (as
// the CPU's _mm512_mul_ps of the converted halves), then the f16 rounding (vec_scale_f16)
// (the -0 addend comes in a register: -0.0 is not an inline constant, and a +0 addend would turn
// a -0 product into +0)
__device__ __forceinline__ uint32_t f16_scale(uint32_t ybits, float ms, float nz) {
    float t;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(t) : "v"(ybits), "v"(ms), "v"(nz));
    uint32_t r;
    asm("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}

// dot_f16_avx512_q4 with the f16 -> f32 conversions folded into v_fma_mix_f32 (exact: the
// conversion is exact and the fma rounds once; the first product is fma(k, q, -0) = k·q
// rounded, as _mm512_mul_ps)
template <int SEL>
__device__ __forceinline__ float mixfma(uint32_t kbits, float q, float acc) {
    float r;
    if constexpr (SEL == 0) asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(kbits), "v"(q), "v"(acc));
    else asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(kbits), "v"(q), "v"(acc));
    return r;
}

__device__ __forceinline__ float dot_f16_mix_d128(const uint2 (&kh)[8], const float (&qf)[8][4], float nz) {
    float w[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float acc[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const uint32_t k0 = c < 2 ? kh[jj].x : kh[jj].y, k1 = c < 2 ? kh[4 + jj].x : kh[4 + jj].y;
            float t = (c & 1) ? mixfma<1>(k0, qf[jj][c], nz) : mixfma<0>(k0, qf[jj][c], nz);
            acc[jj] = (c & 1) ? mixfma<1>(k1, qf[4 + jj][c], t) : mixfma<0>(k1, qf[4 + jj][c], t);
        }
        w[c] = __fadd_rn(__fadd_rn(acc[0], acc[2]), __fadd_rn(acc[1], acc[3]));
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = __fadd_rn(w[c], quad_from_plus2(w[c]));
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = __fadd_rn(w[c], quad_from_plus1(w[c]));
    return __fadd_rn(__fadd_rn(w[0], w[2]), __fadd_rn(w[1], w[3]));
}

// mixfma with q as well held as an f16 half: fma(f32(k half SK), f32(q half SQ), acc), one rounding
template <int SK, int SQ>
__device__ __forceinline__ float mixfma_h(uint32_t kbits, uint32_t qbits, float acc) {
    float r;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[%4,%5,0] op_sel_hi:[1,1,0]" : "=v"(r) : "v"(kbits), "v"(qbits), "v"(acc), "n"(SK), "n"(SQ));
    return r;
}

// dot_f16_mix_d128 with q as packed f16 pairs: qh[m][h] = (q[16m + 4qd + 2h], q[16m + 4qd + 2h + 1]) rounded to
// f16 (the CPU's Q conversion), half the registers of the f32 copy; the same products and order
__device__ __forceinline__ float dot_f16_mix_d128_h(const uint2 (&kh)[8], const uint32_t (&qh)[8][2], float nz) {
    float w[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float acc[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const uint32_t k0 = c < 2 ? kh[jj].x : kh[jj].y, k1 = c < 2 ? kh[4 + jj].x : kh[4 + jj].y;
            float t = (c & 1) ? mixfma_h<1, 1>(k0, qh[jj][c >> 1], nz) : mixfma_h<0, 0>(k0, qh[jj][c >> 1], nz);
            acc[jj] = (c & 1) ? mixfma_h<1, 1>(k1, qh[4 + jj][c >> 1], t) : mixfma_h<0, 0>(k1, qh[4 + jj][c >> 1], t);
        }
        w[c] = __fadd_rn(__fadd_rn(acc[0], acc[2]), __fadd_rn(acc[1], acc[3]));
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = __fadd_rn(w[c], quad_from_plus2(w[c]));
#pragma unroll
    for (int c = 0; c < 4; ++c) w[c] = __fadd_rn(w[c], quad_from_plus1(w[c]));
    return __fadd_rn(__fadd_rn(w[0], w[2]), __fadd_rn(w[1], w[3]));
}

// wave-wide inclusive max-scan by DPP (rows by row_shr 1/2/4/8, then row_bcast:15 / :31 —
// GFX9 DPP), and the exclusive shift by one lane (wave_shr:1); absent sources read -inf
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp_ninf(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp((int) 0xff800000u, __float_as_int(v), CTRL, ROWS, 0xf, false));
}
__device__ __forceinline__ float wave_scan_max(float x) {
    x = fmaxf(x, dpp_ninf<0x111>(x));
    x = fmaxf(x, dpp_ninf<0x112>(x));
    x = fmaxf(x, dpp_ninf<0x114>(x));
    x = fmaxf(x, dpp_ninf<0x118>(x));
    x = fmaxf(x, dpp_ninf<0x142, 0xa>(x));
    x = fmaxf(x, dpp_ninf<0x143, 0xc>(x));
    return x;
}

// LDS written by lanes of this wave and read back by other lanes of it: LDS instructions of one
// wave execute in order, so only the compiler must not reorder them (wave_lds_sync's release
// fence would also wait for this wave's outstanding LDS-DMA and global loads)
__device__ __forceinline__ void dc_wave_lds_order() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// the producers' LDS hand-off words as relaxed workgroup-scope atomics: they compile to ds_read /
// ds_write (a volatile access through a generic pointer became a flat access, which counts in
// vmcnt — the compiler then drained the next chunk's K loads right after issuing them)
template <class V> __device__ __forceinline__ V lds_ld(V * p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
template <class V> __device__ __forceinline__ void lds_st(V * p, V v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// a bounded LDS spin: a hand-off that never completes ends the wait (wrong output, which the
// parity tests see) instead of faulting the GPU
__device__ __forceinline__ void ds_wait_flag(int * f) {
    int guard = 0;
    while (lds_ld(f) == 0) {
        __builtin_amdgcn_s_sleep(1);
        if (++guard > (1 << 24)) break;   // a lost flag shows as wrong output, never as a fault
    }
    asm volatile("" ::: "memory");
}

// the mask word of position j (0xfc00 = -inf past the cache) as an asm load: the caller waits
__device__ __forceinline__ uint32_t ds_mask_ld(const char * mask, int j, int n_kv) {
    uint32_t v = 0xfc00;
    if (j < n_kv) {
        if (mask) asm volatile("global_load_ushort %0, %1, off" : "=v"(v) : "v"(mask + 2 * j) : "memory");
        else v = 0;
    }
    return v;
}

}  // namespace mi355x
