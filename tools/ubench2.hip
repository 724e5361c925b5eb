// ubench2.hip — where does a single-row RMS-norm kernel spend its time on MI355X?
// Variants of the decode-time norm (4096 floats, one workgroup), timed back to back.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int NV, bool DBL, bool W, bool PREF>
__global__ __launch_bounds__(1024) void k_norm(const float * __restrict__ a, const float * __restrict__ w, float * __restrict__ y,
                                               float * __restrict__ yw) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nthr = blockDim.x;
    float4 v[NV], ww[NV];
    if (PREF && W) {
#pragma unroll
        for (int k = 0; k < NV; ++k) ww[k] = *(const float4 *) (w + 4 * (tid + nthr * k));
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = *(const float4 *) (a + 4 * (tid + nthr * k));
    __shared__ double part[16];
    double sum = 0.0;
    float sf = 0.0f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        if (DBL) {
            sum += (double) (v[k].x * v[k].x); sum += (double) (v[k].y * v[k].y);
            sum += (double) (v[k].z * v[k].z); sum += (double) (v[k].w * v[k].w);
        } else {
            sf += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
        }
    }
    if (!DBL) sum = sf;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) part[wave] = sum;
    __syncthreads();
    sum = 0;
    for (int i = 0; i < nthr / 64; ++i) sum += part[i];
    const float scale = 1.0f / sqrtf((float) (sum / 4096.0) + 1e-5f);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        float4 r = v[k];
        r.x *= scale; r.y *= scale; r.z *= scale; r.w *= scale;
        *(float4 *) (y + 4 * (tid + nthr * k)) = r;
        if (W) {
            const float4 m = PREF ? ww[k] : *(const float4 *) (w + 4 * (tid + nthr * k));
            r.x *= m.x; r.y *= m.y; r.z *= m.z; r.w *= m.w;
            *(float4 *) (yw + 4 * (tid + nthr * k)) = r;
        }
    }
}

__global__ void k_empty() {}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float *a, *w, *y, *yw;
    CK(hipMalloc(&a, 1 << 20)); CK(hipMalloc(&w, 1 << 20)); CK(hipMalloc(&y, 1 << 20)); CK(hipMalloc(&yw, 1 << 20));
    CK(hipMemset(a, 0, 1 << 20)); CK(hipMemset(w, 0, 1 << 20));
    const int N = 2000;
    auto run = [&](const char * name, auto launch) -> int {
        for (int i = 0; i < 50; ++i) launch();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < N; ++i) launch();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-48s %.2f us/kernel\n", name, ms * 1000.0 / N);
        return 0;
    };
    run("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); });
    run("norm 256thr dbl", [&] { hipLaunchKernelGGL((k_norm<4, true, false, false>), dim3(1), dim3(256), 0, s, a, w, y, yw); });
    run("norm 256thr float", [&] { hipLaunchKernelGGL((k_norm<4, false, false, false>), dim3(1), dim3(256), 0, s, a, w, y, yw); });
    run("norm 256thr dbl +w", [&] { hipLaunchKernelGGL((k_norm<4, true, true, false>), dim3(1), dim3(256), 0, s, a, w, y, yw); });
    run("norm 256thr dbl +w prefetch", [&] { hipLaunchKernelGGL((k_norm<4, true, true, true>), dim3(1), dim3(256), 0, s, a, w, y, yw); });
    run("norm 1024thr dbl +w prefetch", [&] { hipLaunchKernelGGL((k_norm<1, true, true, true>), dim3(1), dim3(1024), 0, s, a, w, y, yw); });
    run("norm 1024thr float +w prefetch", [&] { hipLaunchKernelGGL((k_norm<1, false, true, true>), dim3(1), dim3(1024), 0, s, a, w, y, yw); });
    return 0;
}
