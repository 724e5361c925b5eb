// The exact FA recurrence's inner loop in isolation (one wave per SIMD, D = 128 dims on 2 waves
// like k_fattn_exact phase 3): V from LDS [pos][D] u16 per position, vs coefficients by b128
// broadcast per 4 positions, y = f16(fma(v, vs, y)) and S += vs.  Variants:
//   0: batches of U = 8, next batch prefetched (the kernel's structure);
//   1: V transposed in LDS [D][pos]: one ds_read_b64 carries 4 positions of a dim;
//   2: variant 1 with b128 reads (8 positions per read).
// s_memtime ticks per position, printed per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t f16_mad(uint32_t vbits, float vs, uint32_t ybits) {
    float t;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(vbits), "v"(vs), "v"(ybits));
    uint32_t r;
    asm("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}
__device__ __forceinline__ uint32_t f16_mad_hi(uint32_t vbits, float vs, uint32_t ybits) {
    float t;
    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,1]" : "=v"(t) : "v"(vbits), "v"(vs), "v"(ybits));
    uint32_t r;
    asm("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(t));
    return r;
}

constexpr int D = 128, CH = 256, U = 8;

template <int MODE>
__global__ __launch_bounds__(256) void k_rec(const uint16_t * vg, const float * sg, float * out, unsigned long long * cyc, int reps) {
    __shared__ __attribute__((aligned(16))) uint16_t vl[CH * D];
    __shared__ __attribute__((aligned(16))) float sc[CH + 64];
    const int tid = threadIdx.x;
    for (int i = tid; i < CH * D; i += 256) {
        const int pos = i / D, d = i % D;
        vl[MODE == 0 ? i : d * CH + pos] = vg[i];
    }
    for (int i = tid; i < CH + 64; i += 256) sc[i] = i < CH ? sg[i] : 0.0f;
    __syncthreads();
    uint32_t y = 0;
    float S = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (tid < D) {
        for (int rep = 0; rep < reps; ++rep) {
            if constexpr (MODE == 0) {
                uint32_t va[U], vb[U];
                float sa[U], sb[U];
                auto ldb = [&](int j, uint32_t (&vv)[U], float (&vs)[U]) {
                    const uint16_t * vp = vl + j * D + tid;
#pragma unroll
                    for (int u = 0; u < U; ++u) vv[u] = vp[u * D];
#pragma unroll
                    for (int u = 0; u < U; u += 4) {
                        const float4 t = *(const float4 *) (sc + j + u);
                        vs[u] = t.x; vs[u + 1] = t.y; vs[u + 2] = t.z; vs[u + 3] = t.w;
                    }
                };
                auto run = [&](const uint32_t (&vv)[U], const float (&vs)[U]) {
#pragma unroll
                    for (int u = 0; u < U; ++u) { y = f16_mad(vv[u], vs[u], y); S = __fadd_rn(S, vs[u]); }
                };
                ldb(0, va, sa);
                for (int j = 0; j < CH; j += 2 * U) {
                    ldb(j + U, vb, sb);
                    run(va, sa);
                    if (j + 2 * U < CH) ldb(j + 2 * U, va, sa);
                    run(vb, sb);
                }
            } else {
                constexpr int PR = MODE == 1 ? 4 : 8;   // positions per read
                typedef uint32_t vt __attribute__((ext_vector_type(PR / 2)));
                const vt * vp = (const vt *) (vl + tid * CH);
                vt a = vp[0], b;
                float sa[PR], sb[PR];
                auto lds = [&](int j, float (&vs)[PR]) {
#pragma unroll
                    for (int u = 0; u < PR; u += 4) {
                        const float4 t = *(const float4 *) (sc + j + u);
                        vs[u] = t.x; vs[u + 1] = t.y; vs[u + 2] = t.z; vs[u + 3] = t.w;
                    }
                };
                auto run = [&](const vt & v, const float (&vs)[PR]) {
#pragma unroll
                    for (int u = 0; u < PR; u += 2) {
                        y = f16_mad(v[u / 2], vs[u], y); S = __fadd_rn(S, vs[u]);
                        y = f16_mad_hi(v[u / 2], vs[u + 1], y); S = __fadd_rn(S, vs[u + 1]);
                    }
                };
                lds(0, sa);
                for (int j = 0; j < CH; j += 2 * PR) {
                    b = vp[(j + PR) / PR]; lds(j + PR, sb);
                    run(a, sa);
                    if (j + 2 * PR < CH) { a = vp[(j + 2 * PR) / PR]; lds(j + 2 * PR, sa); }
                    run(b, sb);
                }
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid < D) out[tid] = (float) y + S;
    if (tid == 0) cyc[0] = t1 - t0;
}

int main() {
    uint16_t * vg; float * sg, * out; unsigned long long * cyc;
    hipMalloc(&vg, CH * D * 2); hipMemset(vg, 0x1c, CH * D * 2);
    hipMalloc(&sg, CH * 4); hipMemset(sg, 0x3c, CH * 4);
    hipMalloc(&out, 256 * 4); hipMalloc(&cyc, 8);
    const int reps = 64;
    const char * names[] = {"row-major u16 per position (kernel)", "transposed, b64 = 4 positions", "transposed, b128 = 8 positions"};
    for (int m = 0; m < 3; ++m) {
        for (int rep = 0; rep < 2; ++rep) {
            if (m == 0) hipLaunchKernelGGL(k_rec<0>, dim3(1), dim3(256), 0, 0, vg, sg, out, cyc, reps);
            if (m == 1) hipLaunchKernelGGL(k_rec<1>, dim3(1), dim3(256), 0, 0, vg, sg, out, cyc, reps);
            if (m == 2) hipLaunchKernelGGL(k_rec<2>, dim3(1), dim3(256), 0, 0, vg, sg, out, cyc, reps);
            (void) hipDeviceSynchronize();
        }
        unsigned long long c;
        (void) hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-40s %.2f ticks/position\n", names[m], (double) c / (reps * CH));
    }
    return 0;
}
