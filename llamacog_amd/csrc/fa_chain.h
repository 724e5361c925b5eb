// fa_chain.h — the f16 VKQ recurrence's fast batch (k_fattn_exact.hip k_fattn_dec2), shared with
// its microbenchmark (tools/ubench_dc.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mi355x {

// One fast batch of the chain: DC_U positions of y = f16(fma(v, vs, y)), S += vs, with the next
// batch's V values and coefficients read from LDS in the shadow of the first dependent steps
// (in-order issue: reads placed in front of the chain would delay it; issued early, they have
// landed by the batch's end, where the block waits for them so its outputs are ready when the
// compiler sees them).  v / s: this batch; vn / sn*: the next one; va / sa: LDS byte addresses
// of this batch's V element and coefficients.
__device__ __forceinline__ void dc_fast_batch(uint32_t & y, float & S, const uint32_t (&v)[8], const float (&s)[8],
                                              uint32_t (&vn)[8], float4 & sn0, float4 & sn1, uint32_t va, uint32_t sa) {
    float t;
    asm volatile(
        "v_fma_mix_f32 %[t], %[v0], %[s0], %[y] op_sel_hi:[1,0,1]\n"
        "ds_read_u16 %[n0], %[va] offset:2048\n"
        "ds_read_u16 %[n1], %[va] offset:2304\n"
        "v_add_f32 %[S], %[S], %[s0]\n"
        "s_nop 0\n"
        "v_cvt_f16_f32 %[y], %[t]\n"
        "s_nop 0\n"
        "v_fma_mix_f32 %[t], %[v1], %[s1], %[y] op_sel_hi:[1,0,1]\n"
        "ds_read_u16 %[n2], %[va] offset:2560\n"
        "ds_read_u16 %[n3], %[va] offset:2816\n"
        "v_add_f32 %[S], %[S], %[s1]\n"
        "s_nop 0\n"
        "v_cvt_f16_f32 %[y], %[t]\n"
        "s_nop 0\n"
        "v_fma_mix_f32 %[t], %[v2], %[s2], %[y] op_sel_hi:[1,0,1]\n"
        "ds_read_u16 %[n4], %[va] offset:3072\n"
        "ds_read_u16 %[n5], %[va] offset:3328\n"
        "v_add_f32 %[S], %[S], %[s2]\n"
        "s_nop 0\n"
        "v_cvt_f16_f32 %[y], %[t]\n"
        "s_nop 0\n"
        "v_fma_mix_f32 %[t], %[v3], %[s3], %[y] op_sel_hi:[1,0,1]\n"
        "ds_read_u16 %[n6], %[va] offset:3584\n"
        "ds_read_u16 %[n7], %[va] offset:3840\n"
        "v_add_f32 %[S], %[S], %[s3]\n"
        "s_nop 0\n"
        "v_cvt_f16_f32 %[y], %[t]\n"
        "s_nop 0\n"
        "v_fma_mix_f32 %[t], %[v4], %[s4], %[y] op_sel_hi:[1,0,1]\n"
        "ds_read_b128 %[c0], %[sa] offset:32\n"
        "ds_read_b128 %[c1], %[sa] offset:48\n"
        "v_add_f32 %[S], %[S], %[s4]\n"
        "s_nop 0\n"
        "v_cvt_f16_f32 %[y], %[t]\n"
        "s_nop 0\n"
        "v_fma_mix_f32 %[t], %[v5], %[s5], %[y] op_sel_hi:[1,0,1]\n"
        "v_add_f32 %[S], %[S], %[s5]\n"
        "s_nop 0\n"
        "v_cvt_f16_f32 %[y], %[t]\n"
        "s_nop 0\n"
        "v_fma_mix_f32 %[t], %[v6], %[s6], %[y] op_sel_hi:[1,0,1]\n"
        "v_add_f32 %[S], %[S], %[s6]\n"
        "s_nop 0\n"
        "v_cvt_f16_f32 %[y], %[t]\n"
        "s_nop 0\n"
        "v_fma_mix_f32 %[t], %[v7], %[s7], %[y] op_sel_hi:[1,0,1]\n"
        "v_add_f32 %[S], %[S], %[s7]\n"
        "s_nop 0\n"
        "v_cvt_f16_f32 %[y], %[t]\n"
        "s_nop 0\n"
        "s_waitcnt lgkmcnt(0)\n"
        : [t] "=&v"(t), [y] "+v"(y), [S] "+v"(S),
          [n0] "=&v"(vn[0]), [n1] "=&v"(vn[1]), [n2] "=&v"(vn[2]), [n3] "=&v"(vn[3]),
          [n4] "=&v"(vn[4]), [n5] "=&v"(vn[5]), [n6] "=&v"(vn[6]), [n7] "=&v"(vn[7]),
          [c0] "=&v"(sn0), [c1] "=&v"(sn1)
        : [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]),
          [v4] "v"(v[4]), [v5] "v"(v[5]), [v6] "v"(v[6]), [v7] "v"(v[7]),
          [s0] "v"(s[0]), [s1] "v"(s[1]), [s2] "v"(s[2]), [s3] "v"(s[3]),
          [s4] "v"(s[4]), [s5] "v"(s[5]), [s6] "v"(s[6]), [s7] "v"(s[7]),
          [va] "v"(va), [sa] "v"(sa)
        : "memory");
}

}  // namespace mi355x
