// rope.h — RoPE arithmetic shared by the ROPE kernel (k_elem.hip) and the fused GEMV
// epilogue (k_gemv.hip), so fused and unfused graphs produce the same bits.
//
// RoPE follows ops.cpp:5080-5362: theta for pair i is built like ggml_rope_cache_init —
// theta_0 = p, theta_{i+1} = theta_i * theta_scale (fp32, sequential) — then rope_yarn.
#pragma once

#include "common.h"

namespace mi355x {

struct rope_params {
    int n_dims; int mode; float freq_scale, ext_factor, attn_factor; float corr0, corr1; float theta_scale;
    int has_ff;
};

// host: parameters of a ROPE node (op_params layout of ggml_rope_ext, ggml.c)
bool rope_params_of(const ggml_tensor * dst, rope_params & rp);

__device__ __forceinline__ void rope_yarn_dev(float theta_extrap, float freq_scale, float corr0, float corr1, int64_t i0,
                                              float ext_factor, float mscale, float & c, float & s) {
    const float theta_interp = freq_scale * theta_extrap;
    float theta = theta_interp;
    if (ext_factor != 0.0f) {
        const float y = (i0 / 2 - corr0) / fmaxf(0.001f, corr1 - corr0);
        const float ramp_mix = (1.0f - fminf(1.0f, fmaxf(0.0f, y))) * ext_factor;
        theta = theta_interp * (1 - ramp_mix) + theta_extrap * ramp_mix;
        mscale *= 1.0f + 0.1f * logf(1.0f / freq_scale);
    }
    // glibc cosf / sinf of the CPU backend, restated bit for bit (libm_exact.h)
    c = __fmul_rn(lx_cosf(theta), mscale);
    s = __fmul_rn(lx_sinf(theta), mscale);
}

// cos/sin of pair ip (dims 2ip, 2ip+1) at position p
__device__ __forceinline__ void rope_cs(const rope_params & rp, float p, int64_t ip, const float * ff, float & c, float & s) {
    float theta = p;
    for (int64_t k = 0; k < ip; ++k) theta *= rp.theta_scale;
    const float f = rp.has_ff ? ff[ip] : 1.0f;
    rope_yarn_dev(theta / f, rp.freq_scale, rp.corr0, rp.corr1, 2 * ip, rp.ext_factor, rp.attn_factor, c, s);
}

// the rotation; the reference's x86-64-v4 build contracts it as below (bit-exact vs
// tests/golden/rope.npz)
__device__ __forceinline__ void rope_rotate(float x0, float x1, float c, float s, float & o0, float & o1) {
    o0 = fmaf(x0, c, -__fmul_rn(x1, s));
    o1 = fmaf(x0, s, __fmul_rn(x1, c));
}

struct exec_ctx;
// the graph's cos/sin table [ntok][n_dims/2] of a ROPE node's positions (k_elem.hip), built on
// first use and shared by the graph's ROPE kernels and fused GEMV rope epilogues
const float2 * rope_table(exec_ctx & ctx, const ggml_tensor * r, const rope_params & rp, const int32_t * pos,
                          const float * ff, int64_t ntok);

}  // namespace mi355x
