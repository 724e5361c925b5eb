// p2p_check.cpp — the split-layer stage hand-off of the MI355X plugin through the reference's
// own scheduler entry point, ggml_backend_tensor_copy_async (ggml-backend.cpp), which calls the
// destination backend's cpy_tensor_async:
//   p2p_check <plugin.so> <src device> <dst device> <floats> [repeats]
// Two backend instances (the same device twice is the same-device path), a tensor in each
// one's buffer, a seeded fill, the async copy, a sync on the destination, and a bit compare.
// Prints the hand-off counters (RCCL send/recv vs peer copy) and exits non-zero on mismatch.
#include "ggml.h"
#include "ggml-alloc.h"
#include "ggml-backend.h"

#include <dlfcn.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char ** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s plugin.so src_dev dst_dev n_floats [repeats]\n", argv[0]);
        return 2;
    }
    const int ds = atoi(argv[2]), dd = atoi(argv[3]);
    const int64_t n = atoll(argv[4]);
    const int reps = argc > 5 ? atoi(argv[5]) : 3;
    ggml_backend_reg_t reg = ggml_backend_load(argv[1]);
    if (!reg) { fprintf(stderr, "plugin did not load\n"); return 2; }
    const int ndev = (int) ggml_backend_reg_dev_count(reg);
    if (ds >= ndev || dd >= ndev) { fprintf(stderr, "need devices %d and %d, have %d\n", ds, dd, ndev); return 3; }
    ggml_backend_t bs = ggml_backend_dev_init(ggml_backend_reg_dev_get(reg, ds), nullptr);
    ggml_backend_t bd = ggml_backend_dev_init(ggml_backend_reg_dev_get(reg, dd), nullptr);
    ggml_init_params ip = {ggml_tensor_overhead() * 4, nullptr, true};
    ggml_context * cs = ggml_init(ip), * cd = ggml_init(ip);
    ggml_tensor * a = ggml_new_tensor_1d(cs, GGML_TYPE_F32, n);
    ggml_tensor * b = ggml_new_tensor_1d(cd, GGML_TYPE_F32, n);
    ggml_backend_buffer_t bufs = ggml_backend_alloc_ctx_tensors(cs, bs);
    ggml_backend_buffer_t bufd = ggml_backend_alloc_ctx_tensors(cd, bd);
    std::vector<float> h(n), o(n);
    int bad = 0;
    for (int r = 0; r < reps; ++r) {
        uint32_t x = 12345u + 977u * r;
        for (int64_t i = 0; i < n; ++i) { x = x * 1664525u + 1013904223u; h[i] = (float) (int32_t) x * 1e-9f; }
        ggml_backend_tensor_set(a, h.data(), 0, n * sizeof(float));
        ggml_backend_tensor_copy_async(bs, bd, a, b);
        ggml_backend_synchronize(bd);
        ggml_backend_tensor_get(b, o.data(), 0, n * sizeof(float));
        bad += memcmp(h.data(), o.data(), n * sizeof(float)) != 0;
    }
    long rccl = -1, peer = -1;
    void * hnd = dlopen(argv[1], RTLD_NOW | RTLD_NOLOAD);
    if (hnd) {
        auto fn = (void (*)(long *, long *)) dlsym(hnd, "ggml_backend_mi355x_p2p_stats");
        if (fn) fn(&rccl, &peer);
    }
    printf("p2p_check src=%d dst=%d n=%lld reps=%d: mismatches %d, hand-offs rccl=%ld peer=%ld\n", ds, dd, (long long) n, reps,
           bad, rccl, peer);
    ggml_backend_buffer_free(bufs);
    ggml_backend_buffer_free(bufd);
    ggml_free(cs);
    ggml_free(cd);
    ggml_backend_free(bs);
    ggml_backend_free(bd);
    return bad ? 1 : 0;
}
