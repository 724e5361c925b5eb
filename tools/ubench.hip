// ubench.hip — launch-floor microbenchmarks on MI355X: how long a back-to-back chain of
// tiny kernels takes per kernel (stream launches vs one hipGraph), for sizing the decode
// graph's kernel count.  Build: hipcc --offload-arch=gfx950 -O3 ubench.hip -o ubench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty() {}

__global__ void k_touch(const float * __restrict__ x, float * __restrict__ y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = x[i] + 1.0f;
}

// dependent chain: y = f(x) where x was just written by the previous kernel
__global__ void k_chain(float * __restrict__ a, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = a[i] * 0.5f + 1.0f;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float * x; float * y;
    CK(hipMalloc(&x, 64 << 20));
    CK(hipMalloc(&y, 64 << 20));
    CK(hipMemset(x, 0, 64 << 20));
    const int N = 2000;
    auto run = [&](const char * name, auto launch) -> int {
        for (int i = 0; i < 50; ++i) launch();
        CK(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < N; ++i) launch();
        CK(hipEventRecord(e1, s));
        auto t1 = std::chrono::steady_clock::now();
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-40s gpu %.2f us/kernel  host-enqueue %.2f us/kernel\n", name, ms * 1000.0 / N,
               std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
        return 0;
    };
    run("empty <<<1,64>>>", [&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); });
    run("empty <<<1024,256>>>", [&] { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s); });
    run("touch 4096 floats <<<16,256>>>", [&] { hipLaunchKernelGGL(k_touch, dim3(16), dim3(256), 0, s, x, y, 4096); });
    run("chain 4096 floats <<<16,256>>>", [&] { hipLaunchKernelGGL(k_chain, dim3(16), dim3(256), 0, s, x, 4096); });
    run("chain 4096 floats <<<1,256>>>x16/thr", [&] { hipLaunchKernelGGL(k_chain, dim3(1), dim3(256), 0, s, x, 256); });

    // the same chain captured once into a graph of N/10 kernels, replayed 10 times
    for (int variant = 0; variant < 2; ++variant) {
        hipGraph_t g;
        hipGraphExec_t ge;
        const int K = 200;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        for (int i = 0; i < K; ++i) {
            if (variant == 0) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
            else hipLaunchKernelGGL(k_chain, dim3(16), dim3(256), 0, s, x, 4096);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        auto t1 = std::chrono::steady_clock::now();
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("graph of %d %-26s gpu %.2f us/kernel  host-enqueue %.2f us/kernel\n", K,
               variant == 0 ? "empty" : "chain", ms * 1000.0 / (10 * K),
               std::chrono::duration<double, std::micro>(t1 - t0).count() / (10 * K));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    return 0;
}
