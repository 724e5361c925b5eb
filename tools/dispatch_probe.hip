// Workgroup dispatch-rate probe: back-to-back launches of a near-empty kernel (each workgroup
// touches its dynamic LDS and writes one word) over the grid sizes and LDS footprints of the
// decode mat-vecs, to separate the dispatcher's workgroup rate from the GEMV's own work.
//   hipcc --offload-arch=gfx950 -O3 tools/dispatch_probe.hip -o tools/bin/dispatch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_touch(unsigned * out, int waves_work) {
    extern __shared__ unsigned lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    unsigned v = lds[(threadIdx.x + 1) & (blockDim.x - 1)];
    for (int i = 0; i < waves_work; ++i) v = v * 1664525u + 1013904223u;
    if (v == 0x9e3779b9u) out[blockIdx.x] = v;
}

int main() {
    unsigned * out;
    hipMalloc(&out, 1 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("%8s %6s %8s %8s %10s\n", "grid", "block", "lds KB", "us", "WG/us");
    for (int block : {256, 512, 1024}) {
        for (int lds_kb : {4, 16, 32}) {
            for (int grid : {1024, 2048, 4096, 7168, 14336}) {
                const size_t lds = (size_t) lds_kb * 1024;
                for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_touch, dim3(grid), dim3(block), lds, 0, out, 0);
                const int N = 50;
                hipEventRecord(e0, 0);
                for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_touch, dim3(grid), dim3(block), lds, 0, out, 0);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                const double us = ms * 1e3 / N;
                printf("%8d %6d %8d %8.2f %10.1f\n", grid, block, lds_kb, us, grid / us);
            }
        }
    }
    return 0;
}
