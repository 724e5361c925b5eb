// graph_probe.hip — host cost of replaying a captured hipGraph of N small kernels on MI355X:
// host time inside hipGraphLaunch, and device time of the replay, for graphs of kernels only
// and of kernels plus one memset node (a non-kernel node may take the replay off the
// pre-recorded packet path).  Compare with N eager hipLaunchKernelGGL calls.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/graph_probe tools/graph_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_spin(float * p, int iters) {
    float v = p[threadIdx.x];
    for (int i = 0; i < iters; ++i) v = v * 1.0001f + 0.5f;
    if (v == 12345.f) p[threadIdx.x] = v;
}

static double now_us() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char ** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;   // kernel length
    float * d;
    CK(hipMalloc(&d, 1 << 20));
    CK(hipMemset(d, 0, 1 << 20));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int memset_node = 0; memset_node < 2; ++memset_node) {
        for (int n : {50, 100, 200, 400}) {
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
            for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, st, d, iters);
            if (memset_node) CK(hipMemsetAsync(d + 4096, 0, 4096, st));
            CK(hipStreamEndCapture(st, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, st));
            CK(hipStreamSynchronize(st));
            const int reps = 20;
            double host = 0;
            float dev = 0;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, st));
                const double t0 = now_us();
                CK(hipGraphLaunch(ge, st));
                host += now_us() - t0;
                CK(hipEventRecord(e1, st));
                CK(hipStreamSynchronize(st));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                dev += ms;
            }
            printf("graph n=%3d memset=%d: hipGraphLaunch host %8.1f us (%.2f us/node), replay device %8.1f us\n", n, memset_node,
                   host / reps, host / reps / n, 1e3 * dev / reps);
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
        }
    }
    for (int n : {100, 200}) {
        double host = 0;
        float dev = 0;
        const int reps = 10;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, st));
            const double t0 = now_us();
            for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, st, d, iters);
            host += now_us() - t0;
            CK(hipEventRecord(e1, st));
            CK(hipStreamSynchronize(st));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            dev += ms;
        }
        printf("eager n=%3d: launch host %8.1f us (%.2f us/launch), device %8.1f us\n", n, host / reps, host / reps / n, 1e3 * dev / reps);
    }
    // one kernel alone, for its duration
    CK(hipEventRecord(e0, st));
    hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, st, d, iters);
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("single kernel: %.1f us\n", 1e3 * ms);
    return 0;
}
