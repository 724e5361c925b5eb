// lds_dma_probe.hip — where does buffer_load_dwordx4 ... lds put each lane's 16 bytes on gfx950,
// and does the instruction offset move the LDS destination too?  (global_load_lds_dwordx4 beside
// it as the known layout.)  Source: bytes i -> i & 0xff pattern as dwords.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef int rs4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void * ldsp;

template <int MODE>
__global__ void k(const uint32_t * src, uint32_t * out) {
    __shared__ uint32_t lds[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = 0xdeadbeef;
    __syncthreads();
    const uint64_t a = (uint64_t) src;
    rs4 r;
    r.x = __builtin_amdgcn_readfirstlane((int) (uint32_t) a);
    r.y = __builtin_amdgcn_readfirstlane((int) ((uint32_t) (a >> 32) & 0xffffu));
    r.z = -1; r.w = 0x00020000;
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t) (uintptr_t) (ldsp) lds);
    const uint32_t vo = 16u * threadIdx.x;
    if (MODE == 0) {
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen offset:0 nt lds" ::"v"(vo), "s"(r), "s"(m) : "memory", "m0");
    } else if (MODE == 1) {
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen offset:1024 nt lds" ::"v"(vo), "s"(r), "s"(m) : "memory", "m0");
    } else {
        const uint32_t * p = src + 4 * threadIdx.x;
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(p), "s"(m) : "memory", "m0");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += 64) out[i] = lds[i];
}

int main() {
    std::vector<uint32_t> h(2048);
    for (int i = 0; i < 2048; ++i) h[i] = i;
    uint32_t *s, *o;
    hipMalloc(&s, 8192); hipMalloc(&o, 8192);
    hipMemcpy(s, h.data(), 8192, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 3; ++mode) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, s, o);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, s, o);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, s, o);
        std::vector<uint32_t> r(2048);
        hipMemcpy(r.data(), o, 8192, hipMemcpyDeviceToHost);
        printf("mode %d (%s):", mode, mode == 0 ? "buffer off 0" : mode == 1 ? "buffer off 1024" : "global");
        int first = -1, last = -1;
        for (int i = 0; i < 2048; ++i) if (r[i] != 0xdeadbeef) { if (first < 0) first = i; last = i; }
        printf(" written dwords [%d, %d]; lds[first..first+8] =", first, last);
        for (int i = first; i < first + 8 && i >= 0; ++i) printf(" %u", r[i]);
        printf("; lds[first+4*16..] = %u %u\n", first >= 0 ? r[first + 64] : 0, first >= 0 ? r[first + 65] : 0);
    }
    return 0;
}
