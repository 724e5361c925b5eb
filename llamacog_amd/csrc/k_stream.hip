// k_stream.hip — the measured HBM read ceiling that bench.py prices the decode path against
// ("peak bandwidth must be measured on the box with the in-repo STREAM-read
// kernel").  A non-temporal 16-B-per-lane read of 440 MB slices rotated over a 4 GiB pool, so
// no launch hits the 256 MB Infinity Cache; best grid of a few; same kernel as tools/ubench3.hip.
#include "ops.h"
#include "../../include/ggml-mi355x.h"

namespace mi355x {

typedef unsigned sv4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream_read(const sv4u * __restrict__ p, size_t n16, unsigned * __restrict__ out) {
    constexpr int U = 8;
    unsigned acc = 0;
    const size_t stride = (size_t) gridDim.x * blockDim.x;
    size_t i = (size_t) blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        sv4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) { const sv4u v = p[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678u) out[0] = acc;   // keeps the loads; never true for the fill below
}

}  // namespace mi355x

extern "C" GGML_BACKEND_API double ggml_backend_mi355x_hbm_read_gbs(int device) {
    using namespace mi355x;
    if (hipSetDevice(device) != hipSuccess) return -1.0;
    const size_t pool = 4ull << 30, bytes = 440ull << 20;
    void * p = nullptr;
    unsigned * o = nullptr;
    if (hipMalloc(&p, pool) != hipSuccess) { (void) hipGetLastError(); return -1.0; }
    MI_CHECK(hipMalloc(&o, 64));
    MI_CHECK(hipMemset(p, 1, pool));
    hipStream_t s;
    hipEvent_t e0, e1;
    MI_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    MI_CHECK(hipEventCreate(&e0));
    MI_CHECK(hipEventCreate(&e1));
    const int nslots = (int) (pool / bytes);
    const size_t n16 = bytes / 16;
    double best = 0.0;
    for (int blocks : {2048, 4096, 8192}) {
        auto launch = [&](int it) {
            const sv4u * base = (const sv4u *) p + (size_t) (it % nslots) * n16;
            hipLaunchKernelGGL(k_stream_read, dim3(blocks), dim3(256), 0, s, base, n16, o);
        };
        for (int i = 0; i < 4; ++i) launch(i);
        const int N = 20;
        MI_CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < N; ++i) launch(i + 4);
        MI_CHECK(hipEventRecord(e1, s));
        MI_CHECK(hipEventSynchronize(e1));
        float ms = 0.0f;
        MI_CHECK(hipEventElapsedTime(&ms, e0, e1));
        best = std::max(best, (double) bytes * N / (ms * 1e-3) / 1e9);
    }
    MI_CHECK(hipEventDestroy(e0));
    MI_CHECK(hipEventDestroy(e1));
    MI_CHECK(hipStreamDestroy(s));
    MI_CHECK(hipFree(o));
    MI_CHECK(hipFree(p));
    return best;
}
