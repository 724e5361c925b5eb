/*
 * ggml_oracle.c — CPU restatement of the reference's quantized LLaMA hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libggml-mi355x.so, bench.py's GPU
 * leg) links, loads or calls this file; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may.  It is the parity checker for the HIP kernels.
 *
 * Every function restates the reference's scalar arithmetic (file:line in the reference
 * tree /root/reference) so the integer parts are bit-exact with the CPU backend and the
 * float parts follow the same operation order.  Pinned against golden vectors produced by
 * the reference CPU backend itself (oracle/gen_golden.c, tests/golden/*.npz).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define QK_K 256
#define MAXF(a, b) ((a) > (b) ? (a) : (b))
#define MINF(a, b) ((a) < (b) ? (a) : (b))

/* ggml_type ids, ggml/include/ggml.h:351-392 */
enum { T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q8_0 = 8, T_Q4_K = 12, T_Q5_K = 13, T_Q6_K = 14, T_Q8_K = 15 };

/* ---- fp16 <-> fp32, round-to-nearest-even (F16C _cvtss_sh(x, 0) / _cvtsh_ss) ---------------- */
static inline float fp32_from_bits(uint32_t w) { float f; memcpy(&f, &w, 4); return f; }
static inline uint32_t fp32_to_bits(float f) { uint32_t w; memcpy(&w, &f, 4); return w; }

float orc_fp16_to_fp32(uint16_t h) {
    const uint32_t sign = (uint32_t) (h & 0x8000) << 16;
    uint32_t exp = (h >> 10) & 0x1f, man = h & 0x3ff;
    if (exp == 0) {
        if (man == 0) return fp32_from_bits(sign);
        /* subnormal */
        float v = ldexpf((float) man, -24);
        return sign ? -v : v;
    }
    if (exp == 31) return fp32_from_bits(sign | 0x7f800000u | (man << 13));
    return fp32_from_bits(sign | ((exp + 112) << 23) | (man << 13));
}

uint16_t orc_fp32_to_fp16(float f) {
    const uint32_t x = fp32_to_bits(f);
    const uint32_t sign = (x >> 16) & 0x8000;
    const uint32_t ax = x & 0x7fffffff;
    if (ax >= 0x7f800000u) return (uint16_t) (sign | (ax > 0x7f800000u ? 0x7e00 : 0x7c00)); /* nan/inf */
    if (ax >= 0x477ff000u) return (uint16_t) (sign | 0x7c00);                               /* overflow */
    if (ax < 0x38800000u) {
        /* subnormal half: value = ax_float / 2^-24 rounded to nearest even */
        const float v = fp32_from_bits(ax);
        const float s = v * 16777216.0f; /* exact scaling by 2^24 */
        float r = rintf(s);              /* RNE */
        return (uint16_t) (sign | (uint32_t) r);
    }
    /* normal: round mantissa 23 -> 10 bits, RNE */
    uint32_t m = ax + 0xfffu + ((ax >> 13) & 1);
    m -= 0x38000000u; /* rebias 127 -> 15 */
    return (uint16_t) (sign | (m >> 13));
}

/* ---- x86-64-v4 (AVX-512) arithmetic of the CPU backend the reference selects on the
 * MI355X host (refhost libggml-cpu-x64v4.so) ---------------------------------------------- */
/* _mm512_reduce_add_ps (GCC avx512fintrin.h): 8 / 4 / 2 / 1 tree */
static float reduce16(const float * w) {
    float t3[8], t6[4];
    for (int i = 0; i < 8; ++i) t3[i] = w[8 + i] + w[i];
    for (int i = 0; i < 4; ++i) t6[i] = t3[4 + i] + t3[i];
    return (t6[0] + t6[2]) + (t6[1] + t6[3]);
}

/* ggml_vec_dot_f16 / ggml_vec_dot_f32 with GGML_F16_STEP 64, EPR 16 (vec.cpp:191-231,
 * simd-mappings.h AVX512F): 4 accumulators x 16 lanes of f32 FMAs, REDUCE, double leftovers */
static float dot_avx512(const float * x, const float * y, int64_t n) {
    float acc[64];
    const int64_t np = n & ~(int64_t) 63;
    for (int s = 0; s < 64; ++s) acc[s] = 0.0f;
    for (int64_t i = 0; i < np; i += 64)
        for (int s = 0; s < 64; ++s) acc[s] = fmaf(x[i + s], y[i + s], acc[s]);
    float w[16];
    for (int l = 0; l < 16; ++l) w[l] = (acc[l] + acc[32 + l]) + (acc[16 + l] + acc[48 + l]);
    double sumf = reduce16(w);
    for (int64_t i = np; i < n; ++i) sumf += (double) (x[i] * y[i]);
    return (float) sumf;
}

float orc_dot_cpu(int type, int64_t n, const void * vx, const void * vy, int repack);

/* K·Q of the CPU flash-attention for an f16 cache: Q rounded to f16, ggml_vec_dot_f16 */
void orc_fa_scores(const float * q, const uint16_t * k, int64_t n, int64_t D, float * s);

/* ggml_v_expf, AVX-512 variant (ggml-cpu/vec.h:731-756) */
float orc_v_expf(float x) {
    const float r = 0x1.8p23f;
    const float z = fmaf(x, 0x1.715476p+0f, r);
    const float n = z - r;
    const float b = fmaf(-n, 0x1.7f7d1cp-20f, fmaf(-n, 0x1.62e4p-1f, x));
    const float u = b * b;
    const float j = fmaf(fmaf(fmaf(0x1.0e4020p-7f, b, 0x1.573e2ep-5f), u, fmaf(0x1.555e66p-3f, b, 0x1.fffdb6p-2f)), u,
                         fmaf(0x1.ffffecp-1f, b, 1.0f));
    if (fabsf(n) > 192.0f) return n <= 0.0f ? 0.0f : INFINITY;
    return ldexpf(j, (int) n);
}

/* ggml_vec_silu_f32 (vec.cpp:233-255): AVX-512 body x / (1 + v_expf(-x)) in 16-wide
 * chunks, libm expf for the tail (ggml_silu_f32, vec.h) */
void orc_silu(const float * x, int64_t n, float * y) {
    const int64_t nv = n & ~(int64_t) 15;
    for (int64_t i = 0; i < n; ++i) {
        const float e = i < nv ? orc_v_expf(0.0f - x[i]) : expf(-x[i]);
        y[i] = x[i] / (1.0f + e);
    }
}

/* ---- block layouts, ggml/src/ggml-common.h:167-334 -------------------------------------------- */
typedef struct { uint16_t d; uint8_t qs[16]; } b_q4_0;
typedef struct { uint16_t d; int8_t qs[32]; } b_q8_0;
typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; } b_q4_K;
typedef struct { uint16_t d, dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; } b_q5_K;
typedef struct { uint8_t ql[128]; uint8_t qh[64]; int8_t scales[16]; uint16_t d; } b_q6_K;
typedef struct { float d; int8_t qs[256]; int16_t bsums[16]; } b_q8_K;

int orc_block_size(int type) {
    switch (type) {
        case T_Q4_0: return 32; case T_Q8_0: return 32;
        case T_Q4_K: case T_Q5_K: case T_Q6_K: case T_Q8_K: return 256;
        default: return 1;
    }
}
int orc_type_size(int type) {
    switch (type) {
        case T_F32: return 4; case T_F16: return 2;
        case T_Q4_0: return 18; case T_Q8_0: return 34; case T_Q4_K: return 144; case T_Q5_K: return 176;
        case T_Q6_K: return 210; case T_Q8_K: return 292;
        default: return 0;
    }
}

/* nearest_int, ggml-quants.c:366-371 (round half to even via the 1.5*2^23 trick) */
static inline int nearest_int(float fval) {
    float val = fval + 12582912.f;
    int i; memcpy(&i, &val, sizeof(int));
    return (i & 0x007fffff) - 0x00400000;
}

/* quantize_row_q8_K_ref, ggml-quants.c:2471-2508 (the x86 CPU backend uses it verbatim,
 * ggml-cpu/arch/x86/quants.c:481-484) */
void orc_quantize_row_q8_K(const float * x, void * vy, int64_t k) {
    b_q8_K * y = (b_q8_K *) vy;
    const int64_t nb = k / QK_K;
    for (int64_t i = 0; i < nb; i++) {
        float max = 0, amax = 0;
        for (int j = 0; j < QK_K; ++j) {
            const float ax = fabsf(x[j]);
            if (ax > amax) { amax = ax; max = x[j]; }
        }
        if (!amax) {
            y[i].d = 0;
            memset(y[i].qs, 0, QK_K);
            memset(y[i].bsums, 0, sizeof(y[i].bsums));
            x += QK_K;
            continue;
        }
        const float iscale = -127.f / max;
        for (int j = 0; j < QK_K; ++j) {
            const volatile float prod = iscale * x[j];  /* no contraction into the rounding add */
            const int v = nearest_int(prod);
            y[i].qs[j] = (int8_t) MINF(127, v);
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = (int16_t) sum;
        }
        y[i].d = 1 / iscale;
        x += QK_K;
    }
}

/* x86 quantize_row_q8_0, ggml-cpu/arch/x86/quants.c:278-372: d = max/127, id = 127/max,
 * round-half-even of x*id (_mm256_round_ps(_MM_ROUND_NEAREST)), d stored as fp16 (F16C RNE). */
void orc_quantize_row_q8_0(const float * x, void * vy, int64_t k) {
    b_q8_0 * y = (b_q8_0 *) vy;
    const int64_t nb = k / 32;
    for (int64_t i = 0; i < nb; i++) {
        float amax = 0.0f;
        for (int j = 0; j < 32; ++j) amax = MAXF(amax, fabsf(x[i * 32 + j]));
        const float d = amax / 127.f;
        y[i].d = orc_fp32_to_fp16(d);
        const float id = amax != 0.0f ? 127.f / amax : 0.0f;
        for (int j = 0; j < 32; ++j) {
            const volatile float v = x[i * 32 + j] * id;
            float r = rintf(v);
            if (r > 127.f) r = 127.f;
            if (r < -128.f) r = -128.f;
            y[i].qs[j] = (int8_t) r;
        }
    }
}

/* quantize_row_q4_0_ref, ggml-quants.c:25-60 (the CPU's from_float for a q4_0 KV cache): d = the
 * signed value of largest magnitude / -8, nibbles MIN(15, (int8_t)(x * id + 8.5f)) */
void orc_quantize_row_q4_0(const float * x, void * vy, int64_t k) {
    b_q4_0 * y = (b_q4_0 *) vy;
    for (int64_t i = 0; i < k / 32; i++) {
        float amax = 0.0f, mx = 0.0f;
        for (int j = 0; j < 32; j++) {
            const float v = x[i * 32 + j];
            if (amax < fabsf(v)) { amax = fabsf(v); mx = v; }
        }
        const float d = mx / -8;
        const float id = d ? 1.0f / d : 0.0f;
        y[i].d = orc_fp32_to_fp16(d);
        for (int j = 0; j < 16; ++j) {
            const float x0 = x[i * 32 + j] * id, x1 = x[i * 32 + 16 + j] * id;
            const int8_t a0 = (int8_t) (x0 + 8.5f), a1 = (int8_t) (x1 + 8.5f);
            const uint8_t xi0 = a0 < 15 ? (uint8_t) a0 : 15, xi1 = a1 < 15 ? (uint8_t) a1 : 15;
            y[i].qs[j] = xi0 | (uint8_t) (xi1 << 4);
        }
    }
}

/* get_scale_min_k4, ggml-quants.c:625-633 */
static inline void get_scale_min_k4(int j, const uint8_t * q, uint8_t * d, uint8_t * m) {
    if (j < 4) {
        *d = q[j] & 63; *m = q[j + 4] & 63;
    } else {
        *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
        *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4);
    }
}

/* dequantize_row_* , ggml-quants.c:249 (q4_0), 343 (q8_0), 1274 (q4_K), 1476 (q5_K), 1684 (q6_K) */
void orc_dequantize_row(int type, const void * vx, float * y, int64_t k) {
    if (type == T_Q4_0) {
        const b_q4_0 * x = (const b_q4_0 *) vx;
        for (int64_t i = 0; i < k / 32; i++) {
            const float d = orc_fp16_to_fp32(x[i].d);
            for (int j = 0; j < 16; ++j) {
                y[i * 32 + j] = ((x[i].qs[j] & 0x0F) - 8) * d;
                y[i * 32 + j + 16] = ((x[i].qs[j] >> 4) - 8) * d;
            }
        }
    } else if (type == T_Q8_0) {
        const b_q8_0 * x = (const b_q8_0 *) vx;
        for (int64_t i = 0; i < k / 32; i++) {
            const float d = orc_fp16_to_fp32(x[i].d);
            for (int j = 0; j < 32; ++j) y[i * 32 + j] = x[i].qs[j] * d;
        }
    } else if (type == T_Q4_K) {
        const b_q4_K * x = (const b_q4_K *) vx;
        for (int64_t i = 0; i < k / QK_K; i++) {
            const uint8_t * q = x[i].qs;
            const float d = orc_fp16_to_fp32(x[i].d), min = orc_fp16_to_fp32(x[i].dmin);
            int is = 0; uint8_t sc, m;
            for (int j = 0; j < QK_K; j += 64) {
                get_scale_min_k4(is + 0, x[i].scales, &sc, &m);
                const float d1 = d * sc, m1 = min * m;
                get_scale_min_k4(is + 1, x[i].scales, &sc, &m);
                const float d2 = d * sc, m2 = min * m;
                for (int l = 0; l < 32; ++l) *y++ = d1 * (q[l] & 0xF) - m1;
                for (int l = 0; l < 32; ++l) *y++ = d2 * (q[l] >> 4) - m2;
                q += 32; is += 2;
            }
        }
    } else if (type == T_Q5_K) {
        const b_q5_K * x = (const b_q5_K *) vx;
        for (int64_t i = 0; i < k / QK_K; i++) {
            const uint8_t * ql = x[i].qs; const uint8_t * qh = x[i].qh;
            const float d = orc_fp16_to_fp32(x[i].d), min = orc_fp16_to_fp32(x[i].dmin);
            int is = 0; uint8_t sc, m; uint8_t u1 = 1, u2 = 2;
            for (int j = 0; j < QK_K; j += 64) {
                get_scale_min_k4(is + 0, x[i].scales, &sc, &m);
                const float d1 = d * sc, m1 = min * m;
                get_scale_min_k4(is + 1, x[i].scales, &sc, &m);
                const float d2 = d * sc, m2 = min * m;
                for (int l = 0; l < 32; ++l) *y++ = d1 * ((ql[l] & 0xF) + (qh[l] & u1 ? 16 : 0)) - m1;
                for (int l = 0; l < 32; ++l) *y++ = d2 * ((ql[l] >> 4) + (qh[l] & u2 ? 16 : 0)) - m2;
                ql += 32; is += 2; u1 <<= 2; u2 <<= 2;
            }
        }
    } else if (type == T_Q6_K) {
        const b_q6_K * x = (const b_q6_K *) vx;
        for (int64_t i = 0; i < k / QK_K; i++) {
            const float d = orc_fp16_to_fp32(x[i].d);
            const uint8_t * ql = x[i].ql; const uint8_t * qh = x[i].qh; const int8_t * sc = x[i].scales;
            for (int n = 0; n < QK_K; n += 128) {
                for (int l = 0; l < 32; ++l) {
                    const int is = l / 16;
                    const int8_t q1 = (int8_t) ((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                    const int8_t q2 = (int8_t) ((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                    const int8_t q3 = (int8_t) ((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                    const int8_t q4 = (int8_t) ((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
                    y[l + 0] = d * sc[is + 0] * q1;
                    y[l + 32] = d * sc[is + 2] * q2;
                    y[l + 64] = d * sc[is + 4] * q3;
                    y[l + 96] = d * sc[is + 6] * q4;
                }
                y += 128; ql += 64; qh += 32; sc += 8;
            }
        }
    } else if (type == T_F16) {
        const uint16_t * x = (const uint16_t *) vx;
        for (int64_t i = 0; i < k; ++i) y[i] = orc_fp16_to_fp32(x[i]);
    } else if (type == T_F32) {
        memcpy(y, vx, sizeof(float) * k);
    }
}

/* Integer parts of the vec_dot kernels (ggml-cpu/quants.c:110-144, 269-297, 514-722):
 * per-block integer sums returned in isum[b] (and min-sums in msum[b] for q4_K/q5_K) so
 * tests can check them bit-exactly; the float result follows the generic kernels'
 * combination d_x*d_y*isum - dmin_x*d_y*msum. */
float orc_vec_dot(int type, int64_t n, const void * vx, const void * vy, int32_t * isum, int32_t * msum) {
    float sumf = 0.0f;
    if (type == T_Q4_0 || type == T_Q8_0) {
        const b_q8_0 * y = (const b_q8_0 *) vy;
        for (int64_t ib = 0; ib < n / 32; ++ib) {
            int s = 0;
            float dx;
            if (type == T_Q4_0) {
                const b_q4_0 * x = (const b_q4_0 *) vx + ib;
                for (int j = 0; j < 16; ++j) {
                    s += ((x->qs[j] & 0x0F) - 8) * y[ib].qs[j];
                    s += ((x->qs[j] >> 4) - 8) * y[ib].qs[j + 16];
                }
                dx = orc_fp16_to_fp32(x->d);
            } else {
                const b_q8_0 * x = (const b_q8_0 *) vx + ib;
                for (int j = 0; j < 32; ++j) s += x->qs[j] * y[ib].qs[j];
                dx = orc_fp16_to_fp32(x->d);
            }
            if (isum) isum[ib] = s;
            sumf += s * (dx * orc_fp16_to_fp32(y[ib].d));
        }
        return sumf;
    }
    const b_q8_K * y = (const b_q8_K *) vy;
    for (int64_t i = 0; i < n / QK_K; ++i) {
        int8_t a[QK_K];
        int sumi = 0, summ = 0;
        float dx, dmx = 0.0f;
        if (type == T_Q4_K || type == T_Q5_K) {
            const uint8_t * sc12;
            const uint8_t * q4;
            const uint8_t * hm = NULL;
            if (type == T_Q4_K) {
                const b_q4_K * x = (const b_q4_K *) vx + i;
                sc12 = x->scales; q4 = x->qs; dx = orc_fp16_to_fp32(x->d); dmx = orc_fp16_to_fp32(x->dmin);
            } else {
                const b_q5_K * x = (const b_q5_K *) vx + i;
                sc12 = x->scales; q4 = x->qs; hm = x->qh; dx = orc_fp16_to_fp32(x->d); dmx = orc_fp16_to_fp32(x->dmin);
            }
            uint8_t m = 1;
            for (int j = 0; j < QK_K / 64; ++j) {
                for (int l = 0; l < 32; ++l) a[64 * j + l] = (int8_t) ((q4[32 * j + l] & 0xF) + (hm && (hm[l] & m) ? 16 : 0));
                m <<= 1;
                for (int l = 0; l < 32; ++l) a[64 * j + 32 + l] = (int8_t) ((q4[32 * j + l] >> 4) + (hm && (hm[l] & m) ? 16 : 0));
                m <<= 1;
            }
            for (int j = 0; j < 8; ++j) {
                uint8_t sc, mn;
                get_scale_min_k4(j, sc12, &sc, &mn);
                int dot = 0;
                for (int l = 0; l < 32; ++l) dot += a[32 * j + l] * y[i].qs[32 * j + l];
                sumi += sc * dot;
                summ += mn * (y[i].bsums[2 * j] + y[i].bsums[2 * j + 1]);
            }
        } else { /* Q6_K */
            const b_q6_K * x = (const b_q6_K *) vx + i;
            dx = orc_fp16_to_fp32(x->d);
            const uint8_t * ql = x->ql; const uint8_t * qh = x->qh;
            for (int h = 0; h < 2; ++h) {
                for (int l = 0; l < 32; ++l) {
                    a[128 * h + l + 0] = (int8_t) ((ql[64 * h + l] & 0xF) | (((qh[32 * h + l] >> 0) & 3) << 4)) - 32;
                    a[128 * h + l + 32] = (int8_t) ((ql[64 * h + l + 32] & 0xF) | (((qh[32 * h + l] >> 2) & 3) << 4)) - 32;
                    a[128 * h + l + 64] = (int8_t) ((ql[64 * h + l] >> 4) | (((qh[32 * h + l] >> 4) & 3) << 4)) - 32;
                    a[128 * h + l + 96] = (int8_t) ((ql[64 * h + l + 32] >> 4) | (((qh[32 * h + l] >> 6) & 3) << 4)) - 32;
                }
            }
            for (int j = 0; j < 16; ++j) {
                int dot = 0;
                for (int l = 0; l < 16; ++l) dot += a[16 * j + l] * y[i].qs[16 * j + l];
                sumi += x->scales[j] * dot;
            }
        }
        if (isum) isum[i] = sumi;
        if (msum) msum[i] = summ;
        sumf += (dx * y[i].d) * (float) sumi - (dmx * y[i].d) * (float) summ;
    }
    return sumf;
}

/* ggml_compute_forward_mul_mat for quantized src0 (ggml-cpu/ggml-cpu.c:1192-1384): every
 * src1 row is first converted with the weight type's from_float (vec_dot_type), then
 * Y[t][m] = vec_dot(W[m], Xq[t]).  W: M rows of K; X: T rows of K; Y: T rows of M. */
void orc_mul_mat(int type, const void * W, int64_t K, int64_t M, const float * X, int64_t T, float * Y) {
    const size_t wrow = (size_t) (K / orc_block_size(type)) * orc_type_size(type);
    if (type == T_F16 || type == T_F32) {
        float * w = (float *) malloc(sizeof(float) * K);
        for (int64_t m = 0; m < M; ++m) {
            orc_dequantize_row(type, (const char *) W + m * wrow, w, K);
            for (int64_t t = 0; t < T; ++t) {
                double s = 0;
                for (int64_t k = 0; k < K; ++k) s += (double) w[k] * X[t * K + k];
                Y[t * M + m] = (float) s;
            }
        }
        free(w);
        return;
    }
    const int kq = type == T_Q4_K || type == T_Q5_K || type == T_Q6_K;
    const size_t arow = kq ? (size_t) (K / 256) * sizeof(b_q8_K) : (size_t) (K / 32) * sizeof(b_q8_0);
    char * xq = (char *) malloc(arow * T);
    for (int64_t t = 0; t < T; ++t) {
        if (kq) orc_quantize_row_q8_K(X + t * K, xq + t * arow, K);
        else orc_quantize_row_q8_0(X + t * K, xq + t * arow, K);
    }
    for (int64_t t = 0; t < T; ++t)
        for (int64_t m = 0; m < M; ++m)
            Y[t * M + m] = orc_vec_dot(type, K, (const char *) W + m * wrow, xq + t * arow, NULL, NULL);
    free(xq);
}

/* ==== The CPU backend's float combination orders (x86-64-v4 build, the variant the
 * reference's loader picks on the build container and on the MI355X host) =====================
 * Integer parts are exact in any order; what these restate is where the CPU rounds.  Every
 * kernel keeps per-block integer sums in int32 SIMD lanes and accumulates them into f32 lanes
 * with one FMA per block, so the float result is a set of per-lane FMA chains over the blocks
 * in order, then a fixed horizontal reduction.  In all the 256-bit kernels below a 32-bit lane
 * holds the 4-byte group (e % 32) / 4 of every 32-element chunk: "class" c of element e. */

/* hsum_float_8 (ggml-cpu/arch/x86/quants.c:27-58): ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7)) */
static float hsum8(const float * a) {
    float r[4];
    for (int i = 0; i < 4; ++i) r[i] = a[i + 4] + a[i];
    return (r[0] + r[2]) + (r[1] + r[3]);
}

/* unpacked weight quants of one 256-block (value per element, before the -32 of q6_K) */
static void unpack_k(int type, const void * blk, int8_t * a) {
    if (type == T_Q6_K) {
        const b_q6_K * x = (const b_q6_K *) blk;
        for (int h = 0; h < 2; ++h)
            for (int l = 0; l < 32; ++l) {
                const uint8_t * ql = x->ql + 64 * h; const uint8_t * qh = x->qh + 32 * h;
                a[128 * h + l + 0]  = (int8_t) ((ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
                a[128 * h + l + 32] = (int8_t) ((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
                a[128 * h + l + 64] = (int8_t) ((ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
                a[128 * h + l + 96] = (int8_t) ((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
            }
        return;
    }
    const uint8_t * q4 = type == T_Q4_K ? ((const b_q4_K *) blk)->qs : ((const b_q5_K *) blk)->qs;
    const uint8_t * hm = type == T_Q5_K ? ((const b_q5_K *) blk)->qh : NULL;
    uint8_t m = 1;
    for (int j = 0; j < 4; ++j) {
        for (int l = 0; l < 32; ++l) a[64 * j + l] = (int8_t) ((q4[32 * j + l] & 0xF) + (hm && (hm[l] & m) ? 16 : 0));
        m <<= 1;
        for (int l = 0; l < 32; ++l) a[64 * j + 32 + l] = (int8_t) ((q4[32 * j + l] >> 4) + (hm && (hm[l] & m) ? 16 : 0));
        m <<= 1;
    }
}

/* The per-class integers of one block: cls[c] = sum over elements e of class c of
 * scale(e) * q(e) * y(e); min = sum_s m_s * (bsums[2s] + bsums[2s+1]) for q4_K / q5_K.
 * Exposed for the GPU tests (the kernels produce the same integers). */
void orc_block_classes(int type, const void * blk, const void * yblk, int32_t * cls, int32_t * imin) {
    for (int c = 0; c < 8; ++c) cls[c] = 0;
    if (imin) *imin = 0;
    if (type == T_Q8_0) {
        const b_q8_0 * x = (const b_q8_0 *) blk; const b_q8_0 * y = (const b_q8_0 *) yblk;
        for (int e = 0; e < 32; ++e) cls[e / 4] += x->qs[e] * y->qs[e];
        return;
    }
    if (type == T_Q4_0) {
        const b_q4_0 * x = (const b_q4_0 *) blk; const b_q8_0 * y = (const b_q8_0 *) yblk;
        for (int j = 0; j < 16; ++j) {
            cls[j / 4] += ((x->qs[j] & 0xF) - 8) * y->qs[j];
            cls[4 + j / 4] += ((x->qs[j] >> 4) - 8) * y->qs[j + 16];
        }
        return;
    }
    const b_q8_K * y = (const b_q8_K *) yblk;
    int8_t a[QK_K];
    unpack_k(type, blk, a);
    if (type == T_Q6_K) {
        const b_q6_K * x = (const b_q6_K *) blk;
        for (int e = 0; e < QK_K; ++e) cls[(e % 32) / 4] += x->scales[e / 16] * a[e] * y->qs[e];
        return;
    }
    const uint8_t * sc12 = type == T_Q4_K ? ((const b_q4_K *) blk)->scales : ((const b_q5_K *) blk)->scales;
    int mn_sum = 0;
    for (int s = 0; s < 8; ++s) {
        uint8_t sc, mn;
        get_scale_min_k4(s, sc12, &sc, &mn);
        for (int l = 0; l < 32; ++l) cls[l / 4] += sc * a[32 * s + l] * y->qs[32 * s + l];
        mn_sum += mn * (y->bsums[2 * s] + y->bsums[2 * s + 1]);
    }
    if (imin) *imin = mn_sum;
}

/* One output element of the CPU's mul_mat, weight row wx (n elements) against the activation
 * row vy already in the vec_dot_type, in the order the x64-v4 CPU backend computes it:
 *   repack = 0: the vec_dot kernels (ggml-cpu/arch/x86/quants.c):
 *     q8_0  :965   acc[c] = fma(dx*dy, I[c], acc[c]) per 32-block;       hsum8(acc)
 *               (llamafile tinyBLAS_Q0_AVX for T >= 2, sgemm.cpp:914-961, has the same order)
 *     q4_K  :1837  acc[c] = fma(dy*dx, I[c], acc[c]); acc_m[k] = fma(-dy*dmin, P[k], acc_m[k])
 *               with P[k] the min products of sub-blocks 2k, 2k+1; hsum8(acc) + ((m0+m2)+(m1+m3))
 *     q5_K  :2062  acc[c] = fma(dy*dx, I[c], acc[c]); summs = fma(Imin, -dy*dmin, summs);
 *               hsum8(acc) + summs
 *     q6_K  :2324  acc[c] = fma(dy*dx, I[c], acc[c]);                       hsum8(acc)
 *   repack = 1: weights in the CPU_REPACK buffer (ggml-cpu/repack.cpp:1416-1458, AVX2, rows % 8):
 *     q4_K  ggml_gemv/gemm_q4_K_8x8_q8_K (arch/x86/repack.cpp:718, 1771):
 *               A = fma(Iacc, dx*dy, A); B = fma(Imin, dmin*dy, B); A - B
 *     q4_0  ggml_gemv/gemm_q4_0_8x8_q8_0 (arch/x86/repack.cpp:579, 992): A = fma(I, dx*dy, A)
 */
float orc_dot_cpu(int type, int64_t n, const void * vx, const void * vy, int repack) {
    int32_t cls[8], imin;
    if (type == T_Q8_0 || type == T_Q4_0) {
        const int64_t nb = n / 32;
        float acc[8] = {0}, A = 0.0f;
        for (int64_t b = 0; b < nb; ++b) {
            const b_q8_0 * y = (const b_q8_0 *) vy + b;
            const void * xb = type == T_Q8_0 ? (const void *) ((const b_q8_0 *) vx + b) : (const void *) ((const b_q4_0 *) vx + b);
            const uint16_t xd16 = type == T_Q8_0 ? ((const b_q8_0 *) xb)->d : ((const b_q4_0 *) xb)->d;
            orc_block_classes(type, xb, y, cls, NULL);
            const float d = orc_fp16_to_fp32(xd16) * orc_fp16_to_fp32(y->d);
            if (type == T_Q4_0 && repack) {
                int I = 0;
                for (int c = 0; c < 8; ++c) I += cls[c];
                A = fmaf((float) I, d, A);
            } else {
                for (int c = 0; c < 8; ++c) acc[c] = fmaf(d, (float) cls[c], acc[c]);
            }
        }
        return (type == T_Q4_0 && repack) ? A : hsum8(acc);
    }
    const int64_t nb = n / QK_K;
    const int bsz = orc_type_size(type);
    float acc[8] = {0}, accm[4] = {0}, A = 0.0f, B = 0.0f, summs = 0.0f;
    for (int64_t b = 0; b < nb; ++b) {
        const char * xb = (const char *) vx + b * bsz;
        const b_q8_K * y = (const b_q8_K *) vy + b;
        orc_block_classes(type, xb, y, cls, &imin);
        if (type == T_Q6_K) {
            const float d = y->d * orc_fp16_to_fp32(((const b_q6_K *) xb)->d);
            for (int c = 0; c < 8; ++c) acc[c] = fmaf(d, (float) cls[c], acc[c]);
            continue;
        }
        const uint16_t d16 = type == T_Q4_K ? ((const b_q4_K *) xb)->d : ((const b_q5_K *) xb)->d;
        const uint16_t m16 = type == T_Q4_K ? ((const b_q4_K *) xb)->dmin : ((const b_q5_K *) xb)->dmin;
        if (type == T_Q4_K && repack == 1) {
            int I = 0;
            for (int c = 0; c < 8; ++c) I += cls[c];
            A = fmaf((float) I, orc_fp16_to_fp32(d16) * y->d, A);
            B = fmaf((float) imin, orc_fp16_to_fp32(m16) * y->d, B);
            continue;
        }
        if (type == T_Q4_K && repack == 2) {
            /* the gemm accumulates once per PAIR of sub-blocks (arch/x86/repack.cpp:2155-2168) */
            const uint8_t * sc12 = ((const b_q4_K *) xb)->scales;
            int8_t a[QK_K];
            unpack_k(type, xb, a);
            const float dd = orc_fp16_to_fp32(d16) * y->d, dm = orc_fp16_to_fp32(m16) * y->d;
            for (int sb = 0; sb < 4; ++sb) {
                int I = 0, Mn = 0;
                for (int u = 0; u < 2; ++u) {
                    const int s = 2 * sb + u;
                    uint8_t sc, mn;
                    get_scale_min_k4(s, sc12, &sc, &mn);
                    int dot = 0;
                    for (int l = 0; l < 32; ++l) dot += a[32 * s + l] * y->qs[32 * s + l];
                    I += sc * dot;
                    Mn += mn * (y->bsums[2 * s] + y->bsums[2 * s + 1]);
                }
                A = fmaf((float) I, dd, A);
                B = fmaf((float) Mn, dm, B);
            }
            continue;
        }
        const float d = y->d * orc_fp16_to_fp32(d16);
        const float dmin = -y->d * orc_fp16_to_fp32(m16);
        for (int c = 0; c < 8; ++c) acc[c] = fmaf(d, (float) cls[c], acc[c]);
        if (type == T_Q5_K) {
            summs = fmaf((float) imin, dmin, summs);
        } else {
            const uint8_t * sc12 = ((const b_q4_K *) xb)->scales;
            for (int k = 0; k < 4; ++k) {
                uint8_t sc, m0, m1;
                get_scale_min_k4(2 * k, sc12, &sc, &m0);
                get_scale_min_k4(2 * k + 1, sc12, &sc, &m1);
                const int P = m0 * (y->bsums[4 * k] + y->bsums[4 * k + 1]) + m1 * (y->bsums[4 * k + 2] + y->bsums[4 * k + 3]);
                accm[k] = fmaf(dmin, (float) P, accm[k]);
            }
        }
    }
    if (type == T_Q4_K && repack) return A - B;   /* 1: gemv, 2: gemm */
    if (type == T_Q5_K) return hsum8(acc) + summs;
    if (type == T_Q4_K) return hsum8(acc) + ((accm[0] + accm[2]) + (accm[1] + accm[3]));
    return hsum8(acc);
}

/* ggml_quantize_mat_q8_K_4x8 (arch/x86/repack.cpp:315-530), the activation quantizer of the
 * repacked Q4_K gemm for every group of 4 rows: the values of quantize_row_q8_K_ref except
 * for the sign of iscale, which is -127/amax whenever +amax occurs in the block (the scalar
 * reference takes the sign of the FIRST element of largest magnitude). */
void orc_quantize_row_q8_K_4x8(const float * x, void * vy, int64_t k) {
    b_q8_K * y = (b_q8_K *) vy;
    for (int64_t i = 0; i < k / QK_K; i++, x += QK_K) {
        float amax = 0.0f;
        for (int j = 0; j < QK_K; ++j) amax = MAXF(amax, fabsf(x[j]));
        int pos = 0;
        for (int j = 0; j < QK_K; ++j) pos |= x[j] == amax;
        const float iscale = amax != 0.0f ? (pos ? -127.f / amax : 127.f / amax) : 0.0f;
        for (int j = 0; j < QK_K; ++j) {
            const volatile float prod = x[j] * iscale;
            y[i].qs[j] = (int8_t) rintf(prod);
        }
        for (int j = 0; j < QK_K / 16; ++j) {
            int sum = 0;
            for (int ii = 0; ii < 16; ++ii) sum += y[i].qs[j * 16 + ii];
            y[i].bsums[j] = (int16_t) sum;
        }
        y[i].d = amax != 0.0f ? 1 / iscale : 0.0f;
    }
}

/* tinyBLAS<16, __m512> (llamafile/sgemm.cpp:331-427): per output one 16-lane FMA chain over K
 * in steps of 16, then _mm512_reduce_add_ps — the CPU's f32 mul_mat for T >= 2 when
 * K % 16 == 0 and M % 4 == 0 (sgemm.cpp:3324-3345) */
static float dot_tinyblas16(const float * a, const float * b, int64_t n) {
    float acc[16] = {0};
    for (int64_t l = 0; l < n; l += 16)
        for (int i = 0; i < 16; ++i) acc[i] = fmaf(a[l + i], b[l + i], acc[i]);
    return reduce16(acc);
}

/* The CPU backend's mul_mat as libllama runs it (ggml-cpu/ggml-cpu.c:1192-1384, with the
 * repack and llamafile paths).  repack = 1: Q4_K / Q4_0 weights with M % 8 == 0 sit in the
 * CPU_REPACK buffer (libllama's default).  W: M rows of K; X: T rows of K; Y: T rows of M. */
void orc_mul_mat_cpu(int type, const void * W, int64_t K, int64_t M, const float * X, int64_t T, float * Y, int repack) {
    const size_t wrow = (size_t) (K / orc_block_size(type)) * orc_type_size(type);
    if (type == T_F32) {
        const int tiny = T >= 2 && K % 16 == 0 && M % 4 == 0;
        for (int64_t t = 0; t < T; ++t)
            for (int64_t m = 0; m < M; ++m) {
                const float * w = (const float *) ((const char *) W + m * wrow);
                Y[t * M + m] = tiny ? dot_tinyblas16(w, X + t * K, K) : dot_avx512(w, X + t * K, K);
            }
        return;
    }
    repack = repack && (type == T_Q4_K || type == T_Q4_0) && M % 8 == 0;
    const int kq = type == T_Q4_K || type == T_Q5_K || type == T_Q6_K;
    const size_t arow = kq ? (size_t) (K / 256) * sizeof(b_q8_K) : (size_t) (K / 32) * sizeof(b_q8_0);
    char * xq = (char *) malloc(arow * T);
    for (int64_t t = 0; t < T; ++t) {
        if (!kq) orc_quantize_row_q8_0(X + t * K, xq + t * arow, K);
        else if (repack && type == T_Q4_K && t < T - T % 4) orc_quantize_row_q8_K_4x8(X + t * K, xq + t * arow, K);
        else orc_quantize_row_q8_K(X + t * K, xq + t * arow, K);
    }
    for (int64_t t = 0; t < T; ++t) {
        const int mode = repack && type == T_Q4_K && t < T - T % 4 ? 2 : repack;
        for (int64_t m = 0; m < M; ++m)
            Y[t * M + m] = orc_dot_cpu(type, K, (const char *) W + m * wrow, xq + t * arow, mode);
    }
    free(xq);
}

/* ggml_compute_forward_mul_mat_id (ggml-cpu/ggml-cpu.c:1466-1600): for token t and slot e,
 * Y[t][e][:] = mul_mat(As[ids[t][e]], X[t][e % ne11]) with the mat-vec's per-row arithmetic
 * (the activation row quantized to the vec_dot_type, vec_dot per weight row).  As: n_as
 * matrices of M rows; ids: T rows of ids_row int32 (first n_used used); X: [T][ne11][K]. */
void orc_mul_mat_id(int type, const void * As, int64_t K, int64_t M, int64_t n_as, const int32_t * ids, int64_t ids_row,
                    int64_t n_used, const float * X, int64_t ne11, int64_t T, float * Y) {
    const size_t wmat = (size_t) (K / orc_block_size(type)) * orc_type_size(type) * (size_t) M;
    for (int64_t t = 0; t < T; ++t) {
        for (int64_t e = 0; e < n_used; ++e) {
            const int32_t ex = ids[t * ids_row + e];
            if (ex < 0 || ex >= n_as) continue;
            orc_mul_mat(type, (const char *) As + (size_t) ex * wmat, K, M, X + (t * ne11 + e % ne11) * K, 1,
                        Y + (t * n_used + e) * M);
        }
    }
}

/* mul_mat_id in the CPU backend's exact float order as libllama runs it: each routed pair is one
 * mat-vec (T = 1) of orc_mul_mat_cpu — repacked gemv for Q4_K / Q4_0 stacks with M % 8 == 0
 * (repack.cpp:1277-1405 forward_mul_mat_id), the vec_dot order otherwise (ggml-cpu.c:1466) */
void orc_mul_mat_id_cpu(int type, const void * As, int64_t K, int64_t M, int64_t n_as, const int32_t * ids, int64_t ids_row,
                        int64_t n_used, const float * X, int64_t ne11, int64_t T, float * Y, int repack) {
    const size_t wmat = (size_t) (K / orc_block_size(type)) * orc_type_size(type) * (size_t) M;
    for (int64_t t = 0; t < T; ++t) {
        for (int64_t e = 0; e < n_used; ++e) {
            const int32_t ex = ids[t * ids_row + e];
            if (ex < 0 || ex >= n_as) continue;
            orc_mul_mat_cpu(type, (const char *) As + (size_t) ex * wmat, K, M, X + (t * ne11 + e % ne11) * K, 1,
                            Y + (t * n_used + e) * M, repack);
        }
    }
}

/* ggml_compute_forward_argsort_f32 (ggml-cpu/ops.cpp:6956-6993): the exchange sort per row;
 * order 0 ascending, 1 descending */
void orc_argsort(const float * x, int64_t ne0, int64_t nrows, int order, int32_t * dst) {
    for (int64_t r = 0; r < nrows; ++r) {
        const float * s = x + r * ne0;
        int32_t * d = dst + r * ne0;
        for (int64_t j = 0; j < ne0; ++j) d[j] = (int32_t) j;
        for (int64_t j = 0; j < ne0; ++j) {
            for (int64_t k = j + 1; k < ne0; ++k) {
                if ((order == 0 && s[d[j]] > s[d[k]]) || (order == 1 && s[d[j]] < s[d[k]])) {
                    const int32_t tmp = d[j];
                    d[j] = d[k];
                    d[k] = tmp;
                }
            }
        }
    }
}

/* ggml_compute_forward_sum_rows_f32 (ggml-cpu/ops.cpp:1956-1986) with ggml_vec_sum_f32
 * (ggml-cpu/vec.h:908-918): sequential double sum, rounded once */
void orc_sum_rows(const float * x, int64_t ne0, int64_t nrows, float * y) {
    for (int64_t r = 0; r < nrows; ++r) {
        double s = 0.0;
        for (int64_t i = 0; i < ne0; ++i) s += (double) x[r * ne0 + i];
        y[r] = (float) s;
    }
}

/* ggml_compute_forward_rms_norm_f32, ggml-cpu/ops.cpp:3270-3316 (sum in double) */
void orc_rms_norm(const float * x, int64_t ne0, int64_t nrows, float eps, float * y) {
    for (int64_t r = 0; r < nrows; ++r) {
        double sum = 0.0;
        for (int64_t i = 0; i < ne0; ++i) sum += (double) (x[r * ne0 + i] * x[r * ne0 + i]);
        const float mean = (float) (sum / ne0);
        const float scale = 1.0f / sqrtf(mean + eps);
        for (int64_t i = 0; i < ne0; ++i) y[r * ne0 + i] = x[r * ne0 + i] * scale;
    }
}

/* ggml_rope_yarn_corr_dims, ggml.c:3772-3784 */
static float corr_dim(int n_dims, int n_ctx_orig, float n_rot, float base) {
    return n_dims * logf(n_ctx_orig / (n_rot * 2 * (float) M_PI)) / (2 * logf(base));
}

/* ggml_compute_forward_rope_f32 + ggml_rope_cache_init + rope_yarn, ops.cpp:5080-5362.
 * x: [n_tok][n_head][ne0] (contiguous ggml [ne0, n_head, n_tok]); mode 0 = NORM, 2 = NEOX */
void orc_rope(const float * x, int64_t ne0, int64_t n_head, int64_t n_tok, const int32_t * pos, int n_dims, int mode,
              int n_ctx_orig, float freq_base, float freq_scale, float ext_factor, float attn_factor, float beta_fast,
              float beta_slow, const float * ff, float * y) {
    const float theta_scale = powf(freq_base, -2.0f / n_dims);
    float corr[2];
    corr[0] = MAXF(0, floorf(corr_dim(n_dims, n_ctx_orig, beta_fast, freq_base)));
    corr[1] = MINF(n_dims - 1, ceilf(corr_dim(n_dims, n_ctx_orig, beta_slow, freq_base)));
    float * cache = (float *) malloc(sizeof(float) * ne0);
    for (int64_t t = 0; t < n_tok; ++t) {
        float theta = (float) pos[t];
        for (int64_t i0 = 0; i0 < ne0; i0 += 2) {
            const float f = ff ? ff[i0 / 2] : 1.0f;
            const float theta_extrap = theta / f;
            const float theta_interp = freq_scale * theta_extrap;
            float th = theta_interp, mscale = attn_factor;
            if (ext_factor != 0.0f) {
                const float yy = (i0 / 2 - corr[0]) / MAXF(0.001f, corr[1] - corr[0]);
                const float ramp_mix = (1 - MINF(1, MAXF(0, yy))) * ext_factor;
                th = theta_interp * (1 - ramp_mix) + theta_extrap * ramp_mix;
                mscale *= 1.0f + 0.1f * logf(1.0f / freq_scale);
            }
            cache[i0] = cosf(th) * mscale;
            cache[i0 + 1] = sinf(th) * mscale;
            theta *= theta_scale;
        }
        for (int64_t h = 0; h < n_head; ++h) {
            const float * src = x + (t * n_head + h) * ne0;
            float * dst = y + (t * n_head + h) * ne0;
            for (int64_t i0 = 0; i0 < ne0; ++i0) dst[i0] = src[i0];
            for (int64_t i0 = 0; i0 < n_dims; i0 += 2) {
                const float c = cache[i0], s = cache[i0 + 1];
                int64_t a0, a1;
                if (mode & 2) { a0 = i0 / 2; a1 = i0 / 2 + n_dims / 2; }
                else { a0 = i0; a1 = i0 + 1; }
                const float x0 = src[a0], x1 = src[a1];
                /* the x86-64-v4 build contracts ops.cpp:5245-5246 as fma(x0, c, -(x1*s)) and
                 * fma(x0, s, x1*c) (bit-exact against tests/golden/rope.npz) */
                dst[a0] = fmaf(x0, c, -(x1 * s));
                dst[a1] = fmaf(x0, s, x1 * c);
            }
        }
    }
    free(cache);
}

/* ggml_compute_forward_soft_max_f32, ops.cpp:4731-4827 (no ALiBi); mask rows broadcast
 * with row index r % mask_rows; sum in double */
void orc_soft_max(const float * x, int64_t nc, int64_t nr, const float * mask, int64_t mask_rows, float scale, float * y) {
    for (int64_t r = 0; r < nr; ++r) {
        float mx = -INFINITY;
        for (int64_t i = 0; i < nc; ++i) {
            float w = x[r * nc + i] * scale;
            if (mask) w += mask[(r % mask_rows) * nc + i];
            y[r * nc + i] = w;
            mx = MAXF(mx, w);
        }
        /* ggml_vec_soft_max_f32 (vec.cpp:257-300): 16-wide ggml_v_expf chunks reduced by
         * _mm512_reduce_add_ps and summed in double; libm expf for the tail */
        double sum = 0.0;
        int64_t i = 0;
        for (; i + 15 < nc; i += 16) {
            float w[16];
            for (int k = 0; k < 16; ++k) { w[k] = orc_v_expf(y[r * nc + i + k] - mx); y[r * nc + i + k] = w[k]; }
            sum += (double) reduce16(w);
        }
        for (; i < nc; ++i) {
            const float e = expf(y[r * nc + i] - mx);
            y[r * nc + i] = e;
            sum += (double) e;
        }
        const float inv = (float) (1.0 / sum);
        for (int64_t i = 0; i < nc; ++i) y[r * nc + i] *= inv;
    }
}

#ifndef FA_S_UPDATE
/* S = S*ms + vs is NOT contracted in the reference build (measured: the unfused form is
 * 99.97% bit-exact on tests/golden/flash_attn.npz, the fused one 98%) */
#define FA_S_UPDATE(S, ms, vs) ((S) * (ms) + (vs))
#endif
/* ggml_compute_forward_flash_attn_ext_f16, ops.cpp:7015-7232, for K/V f16, q8_0 or q4_0.
 * q: [n_q][H][D] f32, k/v: [n_kv][Hkv][D] in kv_type, mask: [n_q][n_kv] f16 (may be NULL),
 * out: [n_q][H][D].  f16 V accumulates VKQ in f16 exactly like the CPU (ops.cpp:7147-7171). */
void orc_flash_attn(const float * q, const void * k, const void * v, const uint16_t * mask, int kv_type, int64_t D,
                    int64_t n_q, int64_t H, int64_t n_kv, int64_t Hkv, float scale, float softcap, float * out) {
    const int64_t gqa = H / Hkv;
    const size_t row = kv_type == T_F16 ? D * 2 : (D / 32) * (kv_type == T_Q4_0 ? sizeof(b_q4_0) : sizeof(b_q8_0));
    if (softcap != 0) scale /= softcap;
    float * vkq32 = (float *) malloc(sizeof(float) * D);
    uint16_t * vkq16 = (uint16_t *) malloc(sizeof(uint16_t) * D);
    float * v32 = (float *) malloc(sizeof(float) * D);
    uint16_t * q16 = (uint16_t *) malloc(sizeof(uint16_t) * D);
    b_q8_0 * q8 = (b_q8_0 *) malloc(sizeof(b_q8_0) * (D / 32 + 1));
    float * qf = (float *) malloc(sizeof(float) * D);
    float * kf = (float *) malloc(sizeof(float) * D);
    for (int64_t iq = 0; iq < n_q; ++iq) {
        for (int64_t h = 0; h < H; ++h) {
            const float * pq = q + (iq * H + h) * D;
            if (kv_type == T_F16) {
                for (int64_t d = 0; d < D; ++d) { q16[d] = orc_fp32_to_fp16(pq[d]); qf[d] = orc_fp16_to_fp32(q16[d]); }
            } else {
                orc_quantize_row_q8_0(pq, q8, D);
            }
            float S = 0.0f, M = -INFINITY;
            if (kv_type == T_F16) memset(vkq16, 0, sizeof(uint16_t) * D);
            else memset(vkq32, 0, sizeof(float) * D);
            const int64_t hk = h / gqa;
            for (int64_t ic = 0; ic < n_kv; ++ic) {
                const float mv = mask ? orc_fp16_to_fp32(mask[iq * n_kv + ic]) : 0.0f;
                if (mv == -INFINITY) continue;
                const char * kd = (const char *) k + (ic * Hkv + hk) * row;
                const char * vd = (const char *) v + (ic * Hkv + hk) * row;
                float s;
                if (kv_type == T_F16) {
                    for (int64_t d = 0; d < D; ++d) kf[d] = orc_fp16_to_fp32(((const uint16_t *) kd)[d]);
                    s = dot_avx512(kf, qf, D);
                } else {
                    s = orc_dot_cpu(kv_type, D, kd, q8, 0);   /* ggml_vec_dot_q8_0_q8_0 / _q4_0_q8_0 order */
                }
                s = s * scale;
                if (softcap != 0.0f) s = softcap * tanhf(s);
                s += mv;
                const float Mold = M;
                float ms = 1.0f, vs = 1.0f;
                if (kv_type == T_F16) {
                    if (s > M) {
                        M = s;
                        ms = expf(Mold - M);
                        for (int64_t d = 0; d < D; ++d) vkq16[d] = orc_fp32_to_fp16(orc_fp16_to_fp32(vkq16[d]) * ms);
                    } else {
                        vs = expf(s - M);
                    }
                    /* ggml_vec_mad_f16, AVX-512: GGML_F16_VEC_FMA = _mm512_fmadd_ps (vec.h:262-291) */
                    for (int64_t d = 0; d < D; ++d)
                        vkq16[d] = orc_fp32_to_fp16(fmaf(orc_fp16_to_fp32(((const uint16_t *) vd)[d]), vs, orc_fp16_to_fp32(vkq16[d])));
                } else {
                    if (s > M) {
                        M = s;
                        ms = expf(Mold - M);
                        for (int64_t d = 0; d < D; ++d) vkq32[d] *= ms;
                    } else {
                        vs = expf(s - M);
                    }
                    orc_dequantize_row(kv_type, vd, v32, D);
                    for (int64_t d = 0; d < D; ++d) vkq32[d] = fmaf(v32[d], vs, vkq32[d]);   /* ggml_vec_mad_f32 */
                }
                S = FA_S_UPDATE(S, ms, vs);
            }
            if (kv_type == T_F16) for (int64_t d = 0; d < D; ++d) vkq32[d] = orc_fp16_to_fp32(vkq16[d]);
            const float S_inv = 1.0f / S;
            for (int64_t d = 0; d < D; ++d) out[(iq * H + h) * D + d] = vkq32[d] * S_inv;
        }
    }
    free(vkq32); free(vkq16); free(v32); free(q16); free(q8); free(qf); free(kf);
}

void orc_fa_scores(const float * q, const uint16_t * k, int64_t n, int64_t D, float * s) {
    float * qf = (float *) malloc(sizeof(float) * D);
    float * kf = (float *) malloc(sizeof(float) * D);
    for (int64_t d = 0; d < D; ++d) qf[d] = orc_fp16_to_fp32(orc_fp32_to_fp16(q[d]));
    for (int64_t j = 0; j < n; ++j) {
        for (int64_t d = 0; d < D; ++d) kf[d] = orc_fp16_to_fp32(k[j * D + d]);
        s[j] = dot_avx512(kf, qf, D);
    }
    free(qf); free(kf);
}
