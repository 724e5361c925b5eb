// backend.cpp — the ggml backend plugin ABI for AMD MI355X (gfx950).
//
// Implements the five vtables of the reference's plugin boundary
// (ggml/src/ggml-backend-impl.h:17-207) natively on the HIP runtime:
//   reg    (ggml_backend_reg_i,         impl.h:191-207)  "MI355X", one device per visible GPU
//   device (ggml_backend_device_i,      impl.h:137-185)  "MI355X<i>", supports_op gate
//   buft   (ggml_backend_buffer_type_i, impl.h:17-35)    hipMalloc'd HBM, 256-B alignment
//   buffer (ggml_backend_buffer_i,      impl.h:41-66)    synchronous set/get via hipMemcpy
//   stream (ggml_backend_i,             impl.h:87-124)   one HIP stream, async graph_compute
// and exports ggml_backend_init / ggml_backend_score (impl.h:215-251) so the reference's
// dlopen loader (ggml-backend-reg.cpp:232-276, GGML_BACKEND_PATH at :586-590) picks it up.
// The reference counterpart is the CUDA backend (ggml-cuda.cu:516-3534); nothing of it
// is reused — this file is written against the HIP runtime and the CDNA4 kernels in this
// directory.
#include "ggml-backend-impl.h"
#include "ops.h"
#include "../../include/ggml-mi355x.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

using namespace mi355x;

#define MI355X_NAME "MI355X"

// ------------------------------------------------------------------------------------------
// timing accumulators (global so bench.py can read them through the C ABI)
// ------------------------------------------------------------------------------------------
static std::atomic<int> g_timing{0};
static std::atomic<int> g_graph_timing{0};
static std::mutex g_timing_mtx;
static double g_acc_ms[8], g_acc_bytes[8];
static long   g_acc_count[8];

// ------------------------------------------------------------------------------------------
// exec_ctx helpers
// ------------------------------------------------------------------------------------------
void * exec_ctx::scratch(int slot, size_t bytes) {
    GGML_ASSERT(slot >= 0 && slot < N_SLOTS);
    if (bytes <= slot_size[slot]) return slot_ptr[slot];
    GGML_ASSERT(!capturing && "mi355x: scratch growth during graph capture");
    size_t nsz = std::max(bytes, slot_size[slot] + slot_size[slot] / 2);
    nsz = (nsz + (1 << 20) - 1) & ~size_t((1 << 20) - 1);
    if (slot_ptr[slot]) {
        MI_CHECK(hipStreamSynchronize(stream));
        wait_no_capture();   // another context's capture may be open (thread safety)
        MI_CHECK(hipFree(slot_ptr[slot]));
    }
    MI_CHECK(hipMalloc(&slot_ptr[slot], nsz));
    slot_size[slot] = nsz;
    ++scratch_gen;
    return slot_ptr[slot];
}

bool exec_ctx::prepare_dyn(ggml_cgraph * g) {
    dyn_nodes.clear();
    dyn_host.clear();
    const int n = ggml_graph_n_nodes(g);
    for (int i = 0; i < n; ++i) {
        ggml_tensor * t = ggml_graph_node(g, i);
        if (t->op == GGML_OP_CPY) {
            dyn_nodes.push_back(t);
            dyn_host.push_back(t->src[1]->data);
        }
    }
    if (dyn_host.empty()) return true;
    // fixed-size table: captured graphs keep its address, so it is never reallocated
    constexpr size_t DYN_CAP = 16384;
    if (dyn_host.size() > DYN_CAP) {   // direct pointers; this graph is not replayable
        dyn_nodes.clear();
        dyn_host.clear();
        return false;
    }
    if (!dyn_dev) {
        MI_CHECK(hipMalloc((void **) &dyn_dev, DYN_CAP * sizeof(void *)));
        dyn_cap = DYN_CAP;
        for (int k = 0; k < DYN_RING; ++k) {
            MI_CHECK(hipHostMalloc((void **) &dyn_pin[k], DYN_CAP * sizeof(void *), hipHostMallocDefault));
            MI_CHECK(hipEventCreateWithFlags(&dyn_ev[k], hipEventDisableTiming));
            MI_CHECK(hipEventRecord(dyn_ev[k], stream));
        }
    }
    // stage through pinned memory: the copy runs asynchronously on the stream, so the buffer it
    // reads is only refilled once the copy that last used it has completed.  A ring of DYN_RING
    // buffers: the host blocks only when it runs DYN_RING graphs ahead of the device (the
    // scheduler's pipeline keeps up to n_copies = 4 graphs in flight per backend)
    const int k = dyn_flip;
    dyn_flip = (dyn_flip + 1) % DYN_RING;
    MI_CHECK(hipEventSynchronize(dyn_ev[k]));
    memcpy(dyn_pin[k], dyn_host.data(), dyn_host.size() * sizeof(void *));
    MI_CHECK(hipMemcpyAsync(dyn_dev, dyn_pin[k], dyn_host.size() * sizeof(void *), hipMemcpyHostToDevice, stream));
    MI_CHECK(hipEventRecord(dyn_ev[k], stream));
    return true;
}

void exec_ctx::free_scratch() {
    for (int i = 0; i < N_SLOTS; ++i) {
        if (slot_ptr[i]) (void) hipFree(slot_ptr[i]);
        slot_ptr[i] = nullptr;
        slot_size[i] = 0;
    }
    if (dyn_dev) (void) hipFree(dyn_dev);
    dyn_dev = nullptr;
    dyn_cap = 0;
    for (int k = 0; k < DYN_RING; ++k) {
        if (dyn_pin[k]) (void) hipHostFree(dyn_pin[k]);
        if (dyn_ev[k]) (void) hipEventDestroy(dyn_ev[k]);
        dyn_pin[k] = nullptr;
        dyn_ev[k] = nullptr;
    }
    if (fa_cnt) (void) hipFree(fa_cnt);
    fa_cnt = nullptr;
    if (moe_cnt) (void) hipFree(moe_cnt);
    moe_cnt = nullptr;
    if (kt_buf) (void) hipFree(kt_buf);
    kt_buf = nullptr;
    kt_cap = kt_off = 0;
}

hipEvent_t exec_ctx::get_event() {
    if (!event_pool.empty()) {
        hipEvent_t e = event_pool.back();
        event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    MI_CHECK(hipEventCreate(&e));
    return e;
}

void exec_ctx::time_begin(int kind, double bytes, hipEvent_t & beg) {
    (void) kind; (void) bytes;
    beg = get_event();
    MI_CHECK(hipEventRecord(beg, stream));
}

void exec_ctx::time_end(int kind, double bytes, hipEvent_t beg) {
    hipEvent_t end = get_event();
    MI_CHECK(hipEventRecord(end, stream));
    pending.push_back({beg, end, bytes, kind});
}

// a timed region that launched nothing: its begin event goes back to the pool, no sample
void exec_ctx::time_cancel(hipEvent_t beg) {
    if (beg) event_pool.push_back(beg);
}

void exec_ctx::collect_timing() {
    if (pending.empty()) return;
    std::lock_guard<std::mutex> lk(g_timing_mtx);
    for (auto & t : pending) {
        float ms = 0.0f;
        MI_CHECK(hipEventElapsedTime(&ms, t.beg, t.end));
        g_acc_ms[t.kind] += ms;
        g_acc_bytes[t.kind] += t.bytes;
        g_acc_count[t.kind] += 1;
        event_pool.push_back(t.beg);
        event_pool.push_back(t.end);
    }
    pending.clear();
}

// ------------------------------------------------------------------------------------------
// device / registry state
// ------------------------------------------------------------------------------------------
struct mi_device_ctx {
    int device;
    std::string name;
    std::string description;
    std::string arch;
    ggml_backend_buffer_type buft;
    size_t total_mem = 0;
};

struct mi_reg_ctx {
    std::vector<ggml_backend_device> devices;
    std::vector<mi_device_ctx *> dev_ctx;
};

static ggml_backend_reg_t mi_reg();

// ------------------------------------------------------------------------------------------
// buffer
// ------------------------------------------------------------------------------------------
struct mi_buffer_ctx {
    int device;
    void * dev_ptr;
};

static void up_drain(int device);

static void mi_buf_free(ggml_backend_buffer_t buffer) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
    up_drain(ctx->device);   // no upload still writes into it
    MI_CHECK(hipFree(ctx->dev_ptr));
    delete ctx;
}

static void * mi_buf_get_base(ggml_backend_buffer_t buffer) {
    return ((mi_buffer_ctx *) buffer->context)->dev_ptr;
}

static enum ggml_status mi_buf_init_tensor(ggml_backend_buffer_t buffer, ggml_tensor * tensor) {
    if (tensor->view_src != nullptr) return GGML_STATUS_SUCCESS;
    // zero the tail padding that get_alloc_size added for quantized rows
    if (ggml_is_quantized(tensor->type)) {
        const size_t nb = ggml_nbytes(tensor);
        const size_t padded = ggml_backend_buft_get_alloc_size(buffer->buft, tensor);
        if (padded > nb) {
            auto * ctx = (mi_buffer_ctx *) buffer->context;
            MI_CHECK(hipSetDevice(ctx->device));
            MI_CHECK(hipMemset((char *) tensor->data + nb, 0, padded - nb));
        }
    }
    return GGML_STATUS_SUCCESS;
}

// GGML_MI355X_HOSTPROF=1: host time inside the plugin's entry points, summed per kind and printed
// every 64 graph computes (diagnostic; what libllama spends outside them is the rest of a step)
enum { HP_SUPPORTS, HP_SET_ASYNC, HP_GET_ASYNC, HP_SET, HP_GET, HP_COMPUTE, HP_SYNC, HP_C_FENCE, HP_C_DYN, HP_C_SIG, HP_C_LAUNCH, HP_N };
static const bool g_hostprof = getenv("GGML_MI355X_HOSTPROF") && atoi(getenv("GGML_MI355X_HOSTPROF")) != 0;
static std::atomic<long long> g_hp_ns[HP_N];
static std::atomic<long long> g_hp_cnt[HP_N];
struct hp_scope {
    int k; std::chrono::steady_clock::time_point t0;
    explicit hp_scope(int kind) : k(kind) { if (g_hostprof) t0 = std::chrono::steady_clock::now(); }
    ~hp_scope() {
        if (!g_hostprof) return;
        g_hp_ns[k] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        g_hp_cnt[k] += 1;
    }
};
static void hp_report() {
    static const char * nm[HP_N] = {"supports_op", "set_async", "get_async", "buf_set", "buf_get", "graph_compute", "synchronize",
                                    "gc:fence", "gc:dyn", "gc:signature", "gc:launch"};
    fprintf(stderr, "[hostprof]");
    for (int k = 0; k < HP_N; ++k) {
        // swap-and-read: scopes still closing on other threads land in the next report
        const long long c = g_hp_cnt[k].exchange(0), ns = g_hp_ns[k].exchange(0);
        fprintf(stderr, " %s %lld x %.1f us", nm[k], c, c ? ns / 1e3 / c : 0.0);
    }
    fprintf(stderr, "\n");
}

// ------------------------------------------------------------------------------------------
// small host -> device uploads.  The scheduler copies a decode step's graph inputs (positions,
// KQ mask, output ids, the CPU split's embedding rows) with the synchronous set_tensor
// (ggml-backend.cpp:1374-1398; ggml-cuda.cu:604-610 copies and waits).  A set of at most UP_MAX
// bytes is instead copied into a pinned staging ring and issued as hipMemcpyAsync on the
// device's upload stream: the caller's buffer is free on return (the memcpy), and every later
// user of the device's memory is ordered behind the uploads:
//   * a backend stream (graph_compute, the async tensor calls) waits on an event recorded after
//     the last upload, once per new upload (up_fence);
//   * the synchronous buffer calls (get / memset / copy / clear / free / a large set) drain the
//     upload stream first (up_drain).
// The scheduler synchronises with the previous use of an input before it sets it (the lines
// cited above), so the write-after-read order is the synchronous copy's.
// GGML_MI355X_ASYNC_SET=0 keeps the synchronous copy.
// ------------------------------------------------------------------------------------------
struct mi_upload {
    std::mutex mtx;
    hipStream_t stream = nullptr;
    char * ring = nullptr;       // pinned staging
    size_t head = 0;
    uint64_t seq = 0;            // uploads issued
    uint64_t drained = 0;        // uploads known complete
    hipEvent_t ev = nullptr;
    uint64_t ev_seq = 0;         // the upload ev was last recorded behind
};
static constexpr size_t UP_MAX = 64 << 10, UP_RING = 8 << 20;
static constexpr int UP_MAXDEV = 64;
static mi_upload g_up[UP_MAXDEV];

static bool up_enabled() {
    static const bool on = !getenv("GGML_MI355X_ASYNC_SET") || atoi(getenv("GGML_MI355X_ASYNC_SET")) != 0;
    return on;
}

static void up_drain_locked(mi_upload & u) {
    if (u.drained == u.seq) return;
    MI_CHECK(hipStreamSynchronize(u.stream));
    u.drained = u.seq;
}

// every upload to this HIP device is complete (the synchronous buffer calls)
static void up_drain(int device) {
    if (device < 0 || device >= UP_MAXDEV) return;
    mi_upload & u = g_up[device];
    std::lock_guard<std::mutex> lk(u.mtx);
    up_drain_locked(u);
}

// stream st (of this HIP device) waits for every upload issued so far; seen = the upload count
// it last waited for (per backend)
static void up_fence(int device, hipStream_t st, uint64_t & seen) {
    if (device < 0 || device >= UP_MAXDEV) return;
    mi_upload & u = g_up[device];
    std::lock_guard<std::mutex> lk(u.mtx);
    if (u.seq == seen) return;
    if (u.drained != u.seq) {
        if (u.ev_seq != u.seq) {
            MI_CHECK(hipEventRecord(u.ev, u.stream));
            u.ev_seq = u.seq;
        }
        MI_CHECK(hipStreamWaitEvent(st, u.ev, 0));
    }
    seen = u.seq;
}

// the asynchronous small set (current device = device); false: the caller copies synchronously
static bool up_set(int device, void * dst, const void * data, size_t size) {
    if (!up_enabled() || size > UP_MAX || device < 0 || device >= UP_MAXDEV) return false;
    mi_upload & u = g_up[device];
    std::lock_guard<std::mutex> lk(u.mtx);
    if (!u.stream) {
        MI_CHECK(hipStreamCreateWithFlags(&u.stream, hipStreamNonBlocking));
        MI_CHECK(hipHostMalloc((void **) &u.ring, UP_RING, hipHostMallocDefault));
        MI_CHECK(hipEventCreateWithFlags(&u.ev, hipEventDisableTiming));
    }
    const size_t n = (size + 255) & ~size_t(255);
    if (u.head + n > UP_RING) {   // wrap: the copies still reading the ring are waited for
        up_drain_locked(u);
        u.head = 0;
    }
    memcpy(u.ring + u.head, data, size);
    MI_CHECK(hipMemcpyAsync(dst, u.ring + u.head, size, hipMemcpyHostToDevice, u.stream));
    u.head += n;
    ++u.seq;
    return true;
}

static void mi_buf_memset_tensor(ggml_backend_buffer_t buffer, ggml_tensor * tensor, uint8_t value, size_t offset, size_t size) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
    up_drain(ctx->device);
    MI_CHECK(hipMemsetAsync((char *) tensor->data + offset, value, size, hipStreamPerThread));
    MI_CHECK(hipStreamSynchronize(hipStreamPerThread));
}

static void mi_buf_set_tensor(ggml_backend_buffer_t buffer, ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    hp_scope hp_(HP_SET);
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
    if (up_set(ctx->device, (char *) tensor->data + offset, data, size)) return;
    up_drain(ctx->device);
    MI_CHECK(hipMemcpyAsync((char *) tensor->data + offset, data, size, hipMemcpyHostToDevice, hipStreamPerThread));
    MI_CHECK(hipStreamSynchronize(hipStreamPerThread));
}

static void mi_buf_get_tensor(ggml_backend_buffer_t buffer, const ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    hp_scope hp_(HP_GET);
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
    up_drain(ctx->device);
    MI_CHECK(hipMemcpyAsync(data, (const char *) tensor->data + offset, size, hipMemcpyDeviceToHost, hipStreamPerThread));
    MI_CHECK(hipStreamSynchronize(hipStreamPerThread));
}

static bool mi_buf_is_ours(ggml_backend_buffer_t buffer);

static bool mi_buf_cpy_tensor(ggml_backend_buffer_t buffer, const ggml_tensor * src, ggml_tensor * dst) {
    if (src->buffer == nullptr || !mi_buf_is_ours(src->buffer)) return false;
    auto * sctx = (mi_buffer_ctx *) src->buffer->context;
    auto * dctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(dctx->device));
    up_drain(sctx->device);
    up_drain(dctx->device);
    if (sctx->device == dctx->device) {
        MI_CHECK(hipMemcpyAsync(dst->data, src->data, ggml_nbytes(src), hipMemcpyDeviceToDevice, hipStreamPerThread));
    } else {
        MI_CHECK(hipMemcpyPeerAsync(dst->data, dctx->device, src->data, sctx->device, ggml_nbytes(src), hipStreamPerThread));
    }
    MI_CHECK(hipStreamSynchronize(hipStreamPerThread));
    return true;
}

static void mi_buf_clear(ggml_backend_buffer_t buffer, uint8_t value) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
    up_drain(ctx->device);
    MI_CHECK(hipMemsetAsync(ctx->dev_ptr, value, buffer->size, hipStreamPerThread));
    MI_CHECK(hipStreamSynchronize(hipStreamPerThread));
}

static const ggml_backend_buffer_i mi_buffer_iface = {
    /* .free_buffer   = */ mi_buf_free,
    /* .get_base      = */ mi_buf_get_base,
    /* .init_tensor   = */ mi_buf_init_tensor,
    /* .memset_tensor = */ mi_buf_memset_tensor,
    /* .set_tensor    = */ mi_buf_set_tensor,
    /* .get_tensor    = */ mi_buf_get_tensor,
    /* .cpy_tensor    = */ mi_buf_cpy_tensor,
    /* .clear         = */ mi_buf_clear,
    /* .reset         = */ nullptr,
};

static bool mi_buf_is_ours(ggml_backend_buffer_t buffer) {
    return buffer->iface.get_base == mi_buf_get_base;
}

// ------------------------------------------------------------------------------------------
// buffer type
// ------------------------------------------------------------------------------------------
static const char * mi_buft_get_name(ggml_backend_buffer_type_t buft) {
    return ((mi_device_ctx *) buft->context)->name.c_str();
}

static ggml_backend_buffer_t mi_buft_alloc_buffer(ggml_backend_buffer_type_t buft, size_t size) {
    auto * dctx = (mi_device_ctx *) buft->context;
    MI_CHECK(hipSetDevice(dctx->device));
    void * ptr = nullptr;
    size = std::max<size_t>(size, 1);
    hipError_t err = hipMalloc(&ptr, size);
    if (err != hipSuccess) {
        (void) hipGetLastError();
        MI_LOG_ERROR("%s: allocating %.2f MiB on device %d: hipMalloc failed: %s\n", __func__, size / 1024.0 / 1024.0,
                     dctx->device, hipGetErrorString(err));
        return nullptr;
    }
    auto * bctx = new mi_buffer_ctx{dctx->device, ptr};
    return ggml_backend_buffer_init(buft, mi_buffer_iface, bctx, size);
}

static size_t mi_buft_get_alignment(ggml_backend_buffer_type_t) { return 256; }

static size_t mi_buft_get_alloc_size(ggml_backend_buffer_type_t, const ggml_tensor * tensor) {
    size_t sz = ggml_nbytes(tensor);
    // quantized tensors get a 256-byte zeroed tail so vector loads of the last block never
    // touch unowned memory
    if (ggml_is_quantized(tensor->type)) sz += 256;
    return sz;
}

static bool mi_buft_is_host(ggml_backend_buffer_type_t) { return false; }

static const ggml_backend_buffer_type_i mi_buft_iface = {
    /* .get_name       = */ mi_buft_get_name,
    /* .alloc_buffer   = */ mi_buft_alloc_buffer,
    /* .get_alignment  = */ mi_buft_get_alignment,
    /* .get_max_size   = */ nullptr,
    /* .get_alloc_size = */ mi_buft_get_alloc_size,
    /* .is_host        = */ mi_buft_is_host,
};

static bool mi_buft_is_ours(ggml_backend_buffer_type_t buft) {
    return buft->iface.get_name == mi_buft_get_name;
}

// ------------------------------------------------------------------------------------------
// pinned host buffer type (device get_host_buffer_type; the role of ggml-cuda's CUDA_Host).
// libllama puts the logits / embeddings output buffer (llama-context.cpp:1247-1253) and the
// CPU backend's compute buffer — the token-embedding GET_ROWS output — (:211-217) in it, so the
// per-token device<->host copies are DMA from page-locked memory instead of staged copies.
// The buffer is an ordinary CPU buffer over hipHostMalloc'd memory.
// ------------------------------------------------------------------------------------------
static const char * mi_host_buft_get_name(ggml_backend_buffer_type_t) { return MI355X_NAME "_Host"; }

static void mi_host_buf_free(ggml_backend_buffer_t buffer) { (void) hipHostFree(buffer->context); }

static ggml_backend_buffer_t mi_host_buft_alloc(ggml_backend_buffer_type_t buft, size_t size) {
    void * ptr = nullptr;
    if (hipHostMalloc(&ptr, std::max<size_t>(size, 1), hipHostMallocDefault) != hipSuccess) {
        (void) hipGetLastError();
        MI_LOG_WARN("mi355x: hipHostMalloc of %.2f MiB failed; using pageable host memory\n", size / 1048576.0);
        return ggml_backend_buft_alloc_buffer(ggml_backend_cpu_buffer_type(), size);
    }
    ggml_backend_buffer_t buf = ggml_backend_cpu_buffer_from_ptr(ptr, size);
    buf->buft = buft;
    buf->iface.free_buffer = mi_host_buf_free;
    return buf;
}

static size_t mi_host_buft_get_alignment(ggml_backend_buffer_type_t) {
    return ggml_backend_buft_get_alignment(ggml_backend_cpu_buffer_type());
}

static bool mi_host_buft_is_host(ggml_backend_buffer_type_t) { return true; }

static size_t mi_reg_get_device_count(ggml_backend_reg_t reg);
static ggml_backend_dev_t mi_reg_get_device(ggml_backend_reg_t reg, size_t index);

static ggml_backend_buffer_type_t mi_host_buft() {
    // .device = the registry's first device, as CUDA_Host (ggml-cuda.cu:1145): with mmap on,
    // libllama then keeps CPU-resident weights in the mmap'd CPU buffer instead of copying them
    // into page-locked memory (src/llama-model.cpp:1742-1750)
    static ggml_backend_buffer_type buft = {
        /* .iface   = */ {
            /* .get_name       = */ mi_host_buft_get_name,
            /* .alloc_buffer   = */ mi_host_buft_alloc,
            /* .get_alignment  = */ mi_host_buft_get_alignment,
            /* .get_max_size   = */ nullptr,
            /* .get_alloc_size = */ nullptr,
            /* .is_host        = */ mi_host_buft_is_host,
        },
        /* .device  = */ mi_reg_get_device_count(mi_reg()) > 0 ? mi_reg_get_device(mi_reg(), 0) : nullptr,
        /* .context = */ nullptr,
    };
    return &buft;
}

// ------------------------------------------------------------------------------------------
// buffer_from_host_ptr (device vtable, ggml-backend-impl.h; libllama wraps its mmap'd model
// file this way when a device advertises caps.buffer_from_host_ptr, src/llama-model.cpp:
// 4311-4337): the host range is page-locked and mapped into the GPU's address space
// (hipHostRegister), and tensors in it are read by the kernels over the host link, in place.
// The capability stays false in the device props, as the reference GPU backend's
// (ggml-cuda.cu:2975): for a discrete GPU, weights read over PCIe every token are the slow
// choice, and libllama then copies the weights into device memory instead.  The entry point
// exists for callers that want zero-copy access (tests/test_gpu_kernels.py checks a mat-vec
// over such a buffer bit for bit against the same weights in HBM).
// ------------------------------------------------------------------------------------------
struct mi_hostptr_ctx { void * host; void * dev; size_t size; int device; };

static const char * mi_hostptr_buft_get_name(ggml_backend_buffer_type_t) { return MI355X_NAME "_Mapped"; }
// tensor->data in this buffer is the DEVICE mapping of the host range (hipHostGetDevicePointer),
// which the CPU may not dereference: the buffer is not a host buffer to ggml (the CPU backend's
// supports_buft and the scheduler's host shortcuts key on is_host); host access goes through
// get_tensor, at the same offset from the host base
static bool mi_hostptr_buft_is_host(ggml_backend_buffer_type_t) { return false; }

static void mi_hostptr_free(ggml_backend_buffer_t buffer) {
    auto * c = (mi_hostptr_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(c->device));
    (void) hipHostUnregister(c->host);
    delete c;
}
static void * mi_hostptr_get_base(ggml_backend_buffer_t buffer) { return ((mi_hostptr_ctx *) buffer->context)->dev; }
// the CPU side reaches a tensor at the same offset from the host base
static char * mi_hostptr_host_addr(ggml_backend_buffer_t buffer, const ggml_tensor * t) {
    auto * c = (mi_hostptr_ctx *) buffer->context;
    return (char *) c->host + ((const char *) t->data - (const char *) c->dev);
}
// the wrapped range is the caller's (libllama's read-only model mmap, src/llama-model.cpp:4311-4337):
// the backend only reads it, and refuses to write into it
static void mi_hostptr_refuse_write(const char * what) {
    GGML_ABORT("mi355x: %s on a buffer_from_host_ptr buffer: the wrapped host memory is the caller's and is read-only here", what);
}
static void mi_hostptr_memset(ggml_backend_buffer_t, ggml_tensor *, uint8_t, size_t, size_t) { mi_hostptr_refuse_write("memset_tensor"); }
static void mi_hostptr_set(ggml_backend_buffer_t, ggml_tensor *, const void *, size_t, size_t) { mi_hostptr_refuse_write("set_tensor"); }
static void mi_hostptr_get(ggml_backend_buffer_t b, const ggml_tensor * t, void * d, size_t off, size_t n) { memcpy(d, mi_hostptr_host_addr(b, t) + off, n); }
static void mi_hostptr_clear(ggml_backend_buffer_t, uint8_t) { mi_hostptr_refuse_write("clear"); }

static const ggml_backend_buffer_i mi_hostptr_iface = {
    /* .free_buffer   = */ mi_hostptr_free,
    /* .get_base      = */ mi_hostptr_get_base,
    /* .init_tensor   = */ nullptr,
    /* .memset_tensor = */ mi_hostptr_memset,
    /* .set_tensor    = */ mi_hostptr_set,
    /* .get_tensor    = */ mi_hostptr_get,
    /* .cpy_tensor    = */ nullptr,
    /* .clear         = */ mi_hostptr_clear,
    /* .reset         = */ nullptr,
};

static ggml_backend_buffer_type_t mi_hostptr_buft(ggml_backend_dev_t dev) {
    static std::mutex mtx;
    static std::map<ggml_backend_dev_t, ggml_backend_buffer_type *> bufts;
    std::lock_guard<std::mutex> lk(mtx);
    auto it = bufts.find(dev);
    if (it != bufts.end()) return it->second;
    auto * b = new ggml_backend_buffer_type{{mi_hostptr_buft_get_name, nullptr, nullptr, nullptr, nullptr, mi_hostptr_buft_is_host}, dev, nullptr};
    bufts.emplace(dev, b);
    return b;
}

static ggml_backend_buffer_t mi_dev_buffer_from_host_ptr(ggml_backend_dev_t dev, void * ptr, size_t size, size_t max_tensor_size) {
    (void) max_tensor_size;
    const int device = ((mi_device_ctx *) dev->context)->device;
    MI_CHECK(hipSetDevice(device));
    if (hipHostRegister(ptr, size, hipHostRegisterMapped) != hipSuccess) {
        (void) hipGetLastError();
        MI_LOG_WARN("mi355x: hipHostRegister of %.2f MiB failed\n", size / 1048576.0);
        return nullptr;
    }
    void * dptr = nullptr;
    if (hipHostGetDevicePointer(&dptr, ptr, 0) != hipSuccess || dptr == nullptr) {
        (void) hipGetLastError();
        (void) hipHostUnregister(ptr);
        return nullptr;
    }
    return ggml_backend_buffer_init(mi_hostptr_buft(dev), mi_hostptr_iface, new mi_hostptr_ctx{ptr, dptr, size, device}, size);
}

// ------------------------------------------------------------------------------------------
// row-split buffer type: ggml_backend_split_buffer_type(main_device, tensor_split), the proc
// address libllama asks for with -sm row (src/llama-model.cpp:337-360; the reference GPU
// backend's is ggml-cuda.cu:789-1087).  A matrix in it is cut into row slices, one per device
// in proportion to tensor_split (rounded to 64 rows, so every slice keeps whole GEMV row
// groups), each slice in its device's memory; tensor->extra lists them.  The main device's
// backend computes the MUL_MATs that read such a weight (op_mul_mat_split): slice by slice, the
// rows gathered into the output.  Each output row's arithmetic is the one-device kernel's, so
// the result is bit-identical to a single-device run.
// ------------------------------------------------------------------------------------------
struct mi_split_buft_ctx { int main_device; std::vector<float> split; std::string name; };   // split: cumulative fractions
struct mi_split_extra { split_parts sp; };
struct mi_split_buf_ctx { std::vector<mi_split_extra *> extras; };
constexpr int64_t MI_SPLIT_ROUND = 64;

static int mi_dev_hip(int d) { return ((mi_reg_ctx *) mi_reg()->context)->dev_ctx[d]->device; }

static void mi_split_rows(const mi_split_buft_ctx * b, int64_t nrows, int d, int64_t & lo, int64_t & hi) {
    const int nd = (int) b->split.size();
    lo = d == 0 ? 0 : (int64_t) (nrows * b->split[d]);
    lo -= lo % MI_SPLIT_ROUND;
    if (d == nd - 1) {
        hi = nrows;
    } else {
        hi = (int64_t) (nrows * b->split[d + 1]);
        hi -= hi % MI_SPLIT_ROUND;
    }
    hi = std::max(hi, lo);
}

static const char * mi_split_buft_get_name(ggml_backend_buffer_type_t buft) { return ((mi_split_buft_ctx *) buft->context)->name.c_str(); }
static bool mi_split_buft_is_ours(ggml_backend_buffer_type_t buft) { return buft && buft->iface.get_name == mi_split_buft_get_name; }

static void mi_split_buf_free(ggml_backend_buffer_t buffer) {
    auto * ctx = (mi_split_buf_ctx *) buffer->context;
    for (mi_split_extra * e : ctx->extras) {
        for (int i = 0; i < e->sp.n; ++i) {
            MI_CHECK(hipSetDevice(e->sp.p[i].hip));
            MI_CHECK(hipFree(e->sp.p[i].data));
        }
        delete e;
    }
    delete ctx;
}

// the slices live in the extras; the buffer's base is a placeholder that is never dereferenced
static void * mi_split_buf_get_base(ggml_backend_buffer_t) { return (void *) 0x1000; }

static enum ggml_status mi_split_buf_init_tensor(ggml_backend_buffer_t buffer, ggml_tensor * tensor) {
    GGML_ASSERT(tensor->view_src == nullptr && "mi355x: views of row-split tensors are not supported");
    GGML_ASSERT(ggml_is_contiguous(tensor) && "mi355x: row-split tensors must be contiguous");
    auto * ctx = (mi_split_buf_ctx *) buffer->context;
    const auto * b = (const mi_split_buft_ctx *) buffer->buft->context;
    auto * e = new mi_split_extra{};
    const int64_t nrows = ggml_nrows(tensor);
    const size_t rs = ggml_row_size(tensor->type, tensor->ne[0]);
    GGML_ASSERT(b->split.size() <= (size_t) MI_MAX_DEV);
    for (int d = 0; d < (int) b->split.size(); ++d) {
        int64_t lo, hi;
        mi_split_rows(b, nrows, d, lo, hi);
        if (hi <= lo) continue;
        split_part & p = e->sp.p[e->sp.n++];
        p.hip = mi_dev_hip(d);
        p.lo = lo;
        p.hi = hi;
        const size_t bytes = (size_t) (hi - lo) * rs, pad = ggml_is_quantized(tensor->type) ? 256 : 0;
        MI_CHECK(hipSetDevice(p.hip));
        MI_CHECK(hipMalloc(&p.data, bytes + pad));
        if (pad) MI_CHECK(hipMemset((char *) p.data + bytes, 0, pad));   // the zeroed tail of the one-device buffer
    }
    ctx->extras.push_back(e);
    tensor->extra = e;
    return GGML_STATUS_SUCCESS;
}

static void mi_split_buf_set_tensor(ggml_backend_buffer_t, ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    // whole tensors only (as the reference's split buffer: ggml-cuda.cu:879-880)
    GGML_ASSERT(offset == 0 && size == ggml_nbytes(tensor));
    const auto * e = (const mi_split_extra *) tensor->extra;
    const size_t rs = ggml_row_size(tensor->type, tensor->ne[0]);
    for (int i = 0; i < e->sp.n; ++i) {
        const split_part & p = e->sp.p[i];
        MI_CHECK(hipSetDevice(p.hip));
        MI_CHECK(hipMemcpy(p.data, (const char *) data + p.lo * rs, (size_t) (p.hi - p.lo) * rs, hipMemcpyHostToDevice));
    }
}

static void mi_split_buf_get_tensor(ggml_backend_buffer_t, const ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    GGML_ASSERT(offset == 0 && size == ggml_nbytes(tensor));
    const auto * e = (const mi_split_extra *) tensor->extra;
    const size_t rs = ggml_row_size(tensor->type, tensor->ne[0]);
    for (int i = 0; i < e->sp.n; ++i) {
        const split_part & p = e->sp.p[i];
        MI_CHECK(hipSetDevice(p.hip));
        MI_CHECK(hipMemcpy((char *) data + p.lo * rs, p.data, (size_t) (p.hi - p.lo) * rs, hipMemcpyDeviceToHost));
    }
}

static void mi_split_buf_clear(ggml_backend_buffer_t buffer, uint8_t value) {
    auto * ctx = (mi_split_buf_ctx *) buffer->context;
    for (mi_split_extra * e : ctx->extras) {
        for (int i = 0; i < e->sp.n; ++i) {
            MI_CHECK(hipSetDevice(e->sp.p[i].hip));
            (void) value;   // slices are rewritten by set_tensor; a clear only touches what init_tensor owns
        }
    }
}

static const ggml_backend_buffer_i mi_split_buffer_iface = {
    /* .free_buffer   = */ mi_split_buf_free,
    /* .get_base      = */ mi_split_buf_get_base,
    /* .init_tensor   = */ mi_split_buf_init_tensor,
    /* .memset_tensor = */ nullptr,
    /* .set_tensor    = */ mi_split_buf_set_tensor,
    /* .get_tensor    = */ mi_split_buf_get_tensor,
    /* .cpy_tensor    = */ nullptr,
    /* .clear         = */ mi_split_buf_clear,
    /* .reset         = */ nullptr,
};

static ggml_backend_buffer_t mi_split_buft_alloc_buffer(ggml_backend_buffer_type_t buft, size_t size) {
    // nothing is allocated here: init_tensor places each tensor's slices on their devices
    return ggml_backend_buffer_init(buft, mi_split_buffer_iface, new mi_split_buf_ctx, size);
}

static size_t mi_split_buft_get_alignment(ggml_backend_buffer_type_t) { return 128; }

static size_t mi_split_buft_get_alloc_size(ggml_backend_buffer_type_t buft, const ggml_tensor * tensor) {
    const auto * b = (const mi_split_buft_ctx *) buft->context;
    const int64_t nrows = ggml_nrows(tensor);
    const size_t rs = ggml_row_size(tensor->type, tensor->ne[0]);
    size_t total = 0;
    for (int d = 0; d < (int) b->split.size(); ++d) {
        int64_t lo, hi;
        mi_split_rows(b, nrows, d, lo, hi);
        if (hi > lo) total += (size_t) (hi - lo) * rs + (ggml_is_quantized(tensor->type) ? 256 : 0);
    }
    return total;
}

static bool mi_split_buft_is_host(ggml_backend_buffer_type_t) { return false; }

static const ggml_backend_buffer_type_i mi_split_buft_iface = {
    /* .get_name       = */ mi_split_buft_get_name,
    /* .alloc_buffer   = */ mi_split_buft_alloc_buffer,
    /* .get_alignment  = */ mi_split_buft_get_alignment,
    /* .get_max_size   = */ nullptr,
    /* .get_alloc_size = */ mi_split_buft_get_alloc_size,
    /* .is_host        = */ mi_split_buft_is_host,
};

// tensor_split: per-device proportions (nullptr or all zero: equal shares), as libllama passes
// llama_model_params::tensor_split
static ggml_backend_buffer_type_t mi_split_buffer_type(int main_device, const float * tensor_split) {
    static std::mutex mtx;
    static std::map<std::pair<int, std::vector<float>>, ggml_backend_buffer_type *> cache;
    std::lock_guard<std::mutex> lk(mtx);
    const int nd = (int) mi_reg_get_device_count(mi_reg());
    if (main_device < 0 || main_device >= nd) return nullptr;
    if (nd > MI_MAX_DEV) {   // split_parts holds MI_MAX_DEV slices
        MI_LOG_WARN("mi355x: row split over %d devices exceeds the %d-device limit\n", nd, MI_MAX_DEV);
        return nullptr;
    }
    std::vector<float> w(nd, 0.0f);
    bool any = false;
    for (int i = 0; i < nd; ++i) {
        w[i] = tensor_split ? std::max(tensor_split[i], 0.0f) : 0.0f;
        any = any || w[i] > 0.0f;
    }
    if (!any) std::fill(w.begin(), w.end(), 1.0f);
    float sum = 0.0f;
    std::vector<float> cum(nd);
    for (int i = 0; i < nd; ++i) { cum[i] = sum; sum += w[i]; }
    for (int i = 0; i < nd; ++i) cum[i] /= sum;
    auto key = std::make_pair(main_device, cum);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    auto * bctx = new mi_split_buft_ctx{main_device, cum, std::string(MI355X_NAME) + std::to_string(main_device) + "_Split"};
    auto * buft = new ggml_backend_buffer_type{mi_split_buft_iface, mi_reg_get_device(mi_reg(), main_device), bctx};
    cache.emplace(key, buft);
    return buft;
}

namespace mi355x {
bool tensor_split_parts(const ggml_tensor * t, split_parts & sp) {
    if (!t || !t->buffer || !mi_split_buft_is_ours(t->buffer->buft) || !t->extra) return false;
    sp = ((const mi_split_extra *) t->extra)->sp;
    return true;
}
}

// may device `dev` run op with a row-split weight (the main device, rows on it, one 2-D matrix;
// Q4_K / Q4_0 only with whole 8-row groups, the condition of the CPU's repacked order, which
// must not differ between a slice and the whole matrix)
static bool mi_split_op_ok(ggml_backend_dev_t dev, const ggml_tensor * op) {
    for (int s = 0; s < GGML_MAX_SRC; ++s) {
        const ggml_tensor * t = op->src[s];
        if (!t || !t->buffer || !mi_split_buft_is_ours(t->buffer->buft)) continue;
        if (op->op != GGML_OP_MUL_MAT || s != 0) return false;
        const auto * b = (const mi_split_buft_ctx *) t->buffer->buft->context;
        if (mi_reg_get_device(mi_reg(), b->main_device) != dev) return false;
        if (t->ne[2] != 1 || t->ne[3] != 1 || !ggml_is_contiguous(t)) return false;
        if ((t->type == GGML_TYPE_Q4_K || t->type == GGML_TYPE_Q4_0) && t->ne[1] % 8 != 0) return false;
        int64_t lo, hi;
        mi_split_rows(b, ggml_nrows(t), b->main_device, lo, hi);
        if (hi <= lo) return false;   // the main device holds no rows (small matrices: no row split)
        if (!ggml_is_contiguous(op->src[1])) return false;
    }
    return true;
}

// ------------------------------------------------------------------------------------------
// backend (stream)
// ------------------------------------------------------------------------------------------
// hipGraph replay of repeated graphs (decode re-submits an identical graph every token).
// A graph is captured the second time its signature is seen and replayed while it stays
// unchanged; the signature covers everything a launch reads from the host: op, type,
// shapes, strides, data pointers and op_params of every node and its sources (the role of
// ggml-cuda.cu's ggml_graph_node_has_matching_properties, re-stated for this backend).
struct graph_entry {
    std::vector<int64_t> sig;
    int             seen = 0;
    hipGraphExec_t  exec = nullptr;
    uint64_t        last_use = 0;
    uint64_t        gen = 0;          // exec_ctx::scratch_gen the graph was captured under
    std::vector<exec_ctx::kt_launch> kt_list;   // timeline regions baked into the capture
    size_t          kt_off = 0;
};

struct mi_backend_ctx {
    int device;
    std::string name;
    exec_ctx ex;
    std::vector<graph_entry> graphs;   // small LRU of recently seen graphs
    uint64_t use_clock = 0;
    bool graphs_broken = false;        // capture failed once: stay eager
    uint64_t up_seen = 0;              // uploads this stream has waited for (up_fence)
    // hand-off events of cpy_tensor_async (recorded on this stream, waited on by the
    // destination's): a ring created once instead of an event per copy
    std::vector<hipEvent_t> xev;
    size_t xev_next = 0;
    hipEvent_t next_xevent() {
        constexpr size_t RING = 16;
        if (xev.size() < RING) {
            hipEvent_t e;
            MI_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            xev.push_back(e);
            return e;
        }
        return xev[xev_next++ % RING];
    }
};

// ------------------------------------------------------------------------------------------
// split-layer hand-off over RCCL: one communicator clique over every visible
// device (ncclCommInitAll, rank = HIP device id), created on the first cross-device copy so a
// single-GPU process never initialises RCCL.  A stage boundary is a point-to-point
// ncclSend (source stream) / ncclRecv (destination stream) pair in one group — the
// collective library's xGMI transport, stream-ordered on both sides, no host sync.
// GGML_MI355X_P2P=peer selects hipMemcpyPeerAsync + event instead (A/B and fallback).
// ------------------------------------------------------------------------------------------
// The clique covers the HIP devices that own a backend when the first hand-off happens (rank =
// position in `devs`), not every visible GPU.  Any RCCL error disables RCCL for the process and
// the hand-off falls back to hipMemcpyPeerAsync: a failed collective never aborts the decode.
// GGML_MI355X_P2P: unset = RCCL between distinct GPUs; "peer" = hipMemcpyPeerAsync only;
// "rccl" = RCCL also between two ggml devices on ONE GPU (virtual devices, GGML_MI355X_VDEV):
// a one-rank communicator and a self send/recv, so the RCCL path runs on a single-GPU box.
struct mi_p2p {
    std::mutex mtx;
    int state = 0;                      // 0 = not tried, 1 = ready, -1 = unavailable
    std::vector<int> devs;              // HIP device id of each rank
    std::vector<ncclComm_t> comms;      // by rank
    std::vector<int> self_dev;          // one-rank communicators of the forced same-GPU mode
    std::vector<ncclComm_t> self_comm;
};
static mi_p2p g_p2p;
static std::atomic<long> g_p2p_rccl{0}, g_p2p_peer{0}, g_p2p_d2d{0};
// HIP devices that own at least one backend (mi_dev_init_backend)
static std::mutex g_bdev_mtx;
static std::vector<int> g_bdevs;

enum p2p_mode { P2P_RCCL, P2P_PEER, P2P_RCCL_ALL };
static p2p_mode p2p_mode_env() {
    const char * v = getenv("GGML_MI355X_P2P");
    if (v && strcmp(v, "peer") == 0) return P2P_PEER;
    if (v && strcmp(v, "rccl") == 0) return P2P_RCCL_ALL;
    return P2P_RCCL;
}

static void p2p_disable(const char * what, ncclResult_t r) {
    MI_LOG_WARN("mi355x: RCCL %s failed (%s); stage hand-offs use hipMemcpyPeerAsync from now on\n", what,
                ncclGetErrorString(r));
    g_p2p.state = -1;
}

// rank of HIP device `dev` in the clique (built on first use), or -1
static int p2p_rank(int dev) {
    std::lock_guard<std::mutex> lk(g_p2p.mtx);
    if (g_p2p.state == 0) {
        {
            std::lock_guard<std::mutex> lb(g_bdev_mtx);
            g_p2p.devs = g_bdevs;
        }
        std::sort(g_p2p.devs.begin(), g_p2p.devs.end());
        const int n = (int) g_p2p.devs.size();
        g_p2p.comms.assign(n, nullptr);
        const ncclResult_t r = n > 1 ? ncclCommInitAll(g_p2p.comms.data(), n, g_p2p.devs.data()) : ncclInvalidUsage;
        if (r == ncclSuccess) {
            g_p2p.state = 1;
        } else {
            MI_LOG_WARN("mi355x: RCCL communicator init over %d devices failed (%s); stage hand-off uses hipMemcpyPeerAsync\n",
                        n, n > 1 ? ncclGetErrorString(r) : "one device");
            g_p2p.comms.clear();
            g_p2p.state = -1;
        }
    }
    if (g_p2p.state != 1) return -1;
    for (size_t k = 0; k < g_p2p.devs.size(); ++k) {
        if (g_p2p.devs[k] == dev) return (int) k;
    }
    return -1;
}

// one ncclSend (source stream) + ncclRecv (destination stream) in a group; false = not sent
static bool p2p_send_recv(const void * src, int sdev, hipStream_t ss, void * dst, int ddev, hipStream_t ds, size_t n) {
    const int rs = p2p_rank(sdev), rd = p2p_rank(ddev);
    if (rs < 0 || rd < 0) return false;
    std::lock_guard<std::mutex> lk(g_p2p.mtx);
    if (g_p2p.state != 1) return false;
    MI_CHECK(hipSetDevice(sdev));
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess) {
        ncclResult_t a = ncclSend(src, n, ncclUint8, rd, g_p2p.comms[rs], ss);
        ncclResult_t b = a == ncclSuccess ? ncclRecv(dst, n, ncclUint8, rs, g_p2p.comms[rd], ds) : a;
        r = ncclGroupEnd();
        if (r == ncclSuccess) r = b;
    }
    if (r != ncclSuccess) {
        p2p_disable("send/recv", r);
        return false;
    }
    g_p2p_rccl.fetch_add(1);
    return true;
}

// forced RCCL between two ggml devices on one GPU: self send/recv of a one-rank communicator,
// both on the source stream (the caller makes the destination stream wait)
static bool p2p_self(const void * src, void * dst, int dev, hipStream_t ss, size_t n) {
    std::lock_guard<std::mutex> lk(g_p2p.mtx);
    if (g_p2p.state < 0) return false;
    ncclComm_t comm = nullptr;
    for (size_t k = 0; k < g_p2p.self_dev.size(); ++k) {
        if (g_p2p.self_dev[k] == dev) comm = g_p2p.self_comm[k];
    }
    if (!comm) {
        const ncclResult_t r = ncclCommInitAll(&comm, 1, &dev);
        if (r != ncclSuccess) {
            p2p_disable("one-rank communicator init", r);
            return false;
        }
        g_p2p.self_dev.push_back(dev);
        g_p2p.self_comm.push_back(comm);
    }
    MI_CHECK(hipSetDevice(dev));
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess) {
        ncclResult_t a = ncclSend(src, n, ncclUint8, 0, comm, ss);
        ncclResult_t b = a == ncclSuccess ? ncclRecv(dst, n, ncclUint8, 0, comm, ss) : a;
        r = ncclGroupEnd();
        if (r == ncclSuccess) r = b;
    }
    if (r != ncclSuccess) {
        p2p_disable("self send/recv", r);
        return false;
    }
    g_p2p_rccl.fetch_add(1);
    return true;
}

static void p2p_destroy() {
    std::lock_guard<std::mutex> lk(g_p2p.mtx);
    for (ncclComm_t c : g_p2p.comms) {
        if (c) (void) ncclCommDestroy(c);
    }
    for (ncclComm_t c : g_p2p.self_comm) {
        if (c) (void) ncclCommDestroy(c);
    }
    g_p2p.comms.clear();
    g_p2p.devs.clear();
    g_p2p.self_comm.clear();
    g_p2p.self_dev.clear();
    g_p2p.state = 0;
}

static int env_flag(const char * name) {
    const char * v = getenv(name);
    return v && atoi(v) != 0 ? 1 : 0;
}
static std::atomic<long> g_graph_captures{0}, g_graph_replays{0};
// Captures in flight in any thread (the role of ggml-cuda.cu:516-541's lock): freeing a stream,
// an event or device memory while another thread's stream is being captured is not safe on the
// HIP runtime, so backend teardown and scratch reallocation wait until no capture is open.
static std::mutex g_capture_mtx;
static std::condition_variable g_capture_cv;
static int g_captures_open = 0;
namespace mi355x {
void wait_no_capture() {
    std::unique_lock<std::mutex> lk(g_capture_mtx);
    g_capture_cv.wait(lk, [] { return g_captures_open == 0; });
}
}
static void capture_open() {
    std::lock_guard<std::mutex> lk(g_capture_mtx);
    ++g_captures_open;
}
static void capture_close() {
    std::lock_guard<std::mutex> lk(g_capture_mtx);
    if (--g_captures_open == 0) g_capture_cv.notify_all();
}
static std::atomic<int> g_no_fuse{env_flag("GGML_MI355X_NO_FUSE")};
// rocprofv3 --kernel-trace (ROCm 7.2) segfaults the profiled process when it traces the
// kernels of a replayed hipGraph; under kernel tracing the same kernels are launched
// eagerly instead (profiles/README.md)
static std::atomic<int> g_no_graph{env_flag("GGML_MI355X_NO_GRAPH") | env_flag("ROCPROF_KERNEL_TRACE")};
// in-graph kernel timeline (profiling; GGML_MI355X_KTRACE=1 or ggml_backend_mi355x_set_ktrace)
static std::atomic<int> g_ktrace{env_flag("GGML_MI355X_KTRACE")};
// per launch: first start, last start, last end; workgroup 0's end (a prologue launch's lead)
// and the mean workgroup lifetime (start to its last wave's exit)
struct kt_sample { long graph; int idx; const char * name; unsigned nwg; double t0, t_last_start, t1, t_wg0_end, wg_mean; };
static std::mutex g_kt_mtx;
static std::vector<kt_sample> g_kt_samples;
static long g_kt_graphs = 0;

namespace mi355x {
bool ktrace_enabled() { return g_ktrace.load(std::memory_order_relaxed) != 0; }

unsigned long long * exec_ctx::kt_take(const char * name, unsigned nwg, unsigned threads) {
    // the buffer outlives a traced run; untraced launches get no region (no stamps, no perturbation)
    if (!kt_buf || !ktrace_enabled()) return nullptr;
    const unsigned stride = 1 + threads / 64;
    const size_t n = (size_t) nwg * stride;
    if (kt_off + n > kt_cap) return nullptr;
    kt_list.push_back({name, kt_off, nwg, stride});
    unsigned long long * p = kt_buf + kt_off;
    kt_off += n;
    return p;
}

bool fusion_enabled() { return g_no_fuse.load(std::memory_order_relaxed) == 0; }
bool graphs_enabled() { return g_no_graph.load(std::memory_order_relaxed) == 0; }
// GGML_MI355X_DEBUG_OPS=1: every dispatched node and stand-alone activation quantize on stderr
bool debug_ops() { static const bool on = env_flag("GGML_MI355X_DEBUG_OPS"); return on; }
}

static void graph_signature(ggml_cgraph * cgraph, std::vector<int64_t> & sig) {
    sig.clear();
    const int n = ggml_graph_n_nodes(cgraph);
    sig.reserve((size_t) n * 48);
    // CPY destinations (and the CPY nodes, which alias them) are read through the dynamic
    // pointer table, so their addresses / view offsets are not part of the signature
    static thread_local std::vector<const ggml_tensor *> dyn;
    dyn.clear();
    for (int i = 0; i < n; ++i) {
        const ggml_tensor * t = ggml_graph_node(cgraph, i);
        if (t->op == GGML_OP_CPY) { dyn.push_back(t); dyn.push_back(t->src[1]); }
    }
    // sorted: ~11 lookups per node over ~650 nodes every token (host time of graph_compute)
    std::sort(dyn.begin(), dyn.end());
    // only CPY nodes and their destinations (views of the caches) can be in the list: every other
    // tensor skips the search (~11 lookups per node over ~650 nodes every token)
    auto is_dyn = [&](const ggml_tensor * t) {
        return (t->op == GGML_OP_CPY || t->op == GGML_OP_VIEW) && std::binary_search(dyn.begin(), dyn.end(), t);
    };
    auto put_tensor = [&](const ggml_tensor * t) {
        sig.push_back(is_dyn(t) ? 0 : (int64_t) (intptr_t) t->data);
        sig.push_back((int64_t) t->type);
        for (int k = 0; k < 4; ++k) sig.push_back(t->ne[k]);
        for (int k = 0; k < 4; ++k) sig.push_back((int64_t) t->nb[k]);
    };
    sig.push_back(n);
    sig.push_back(ktrace_enabled() ? 1 : 0);   // a traced capture bakes the timeline regions in
    for (int i = 0; i < n; ++i) {
        const ggml_tensor * t = ggml_graph_node(cgraph, i);
        sig.push_back((int64_t) (intptr_t) t);
        sig.push_back((int64_t) t->op);
        put_tensor(t);
        const int32_t * pp = t->op_params;
        const bool skip_params = t->op == GGML_OP_VIEW && is_dyn(t);   // view offset = n_past
        for (int k = 0; k < GGML_MAX_OP_PARAMS / 8; ++k) {
            int64_t v = 0;
            if (!skip_params) memcpy(&v, pp + 2 * k, 8);
            sig.push_back(v);
        }
        for (int j = 0; j < GGML_MAX_SRC; ++j) {
            if (t->src[j]) put_tensor(t->src[j]);
            else sig.push_back(-1);
        }
    }
}

static const char * mi_backend_get_name(ggml_backend_t backend) {
    return ((mi_backend_ctx *) backend->context)->name.c_str();
}

static void mi_backend_free(ggml_backend_t backend) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    wait_no_capture();
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipStreamSynchronize(ctx->ex.stream));
    ctx->ex.collect_timing();
    for (auto e : ctx->ex.event_pool) (void) hipEventDestroy(e);
    for (auto e : ctx->xev) (void) hipEventDestroy(e);
    for (auto & g : ctx->graphs) {
        if (g.exec) (void) hipGraphExecDestroy(g.exec);
    }
    ctx->ex.free_scratch();
    MI_CHECK(hipStreamDestroy(ctx->ex.stream));
    delete ctx;
    delete backend;
}

static void mi_backend_set_tensor_async(ggml_backend_t backend, ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    hp_scope hp_(HP_SET_ASYNC);
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    up_fence(ctx->device, ctx->ex.stream, ctx->up_seen);
    MI_CHECK(hipMemcpyAsync((char *) tensor->data + offset, data, size, hipMemcpyHostToDevice, ctx->ex.stream));
}

static void mi_backend_get_tensor_async(ggml_backend_t backend, const ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    hp_scope hp_(HP_GET_ASYNC);
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    up_fence(ctx->device, ctx->ex.stream, ctx->up_seen);
    MI_CHECK(hipMemcpyAsync(data, (const char *) tensor->data + offset, size, hipMemcpyDeviceToHost, ctx->ex.stream));
}

static bool mi_backend_is_ours(ggml_backend_t backend);

// Cross-device copy hook used by the scheduler for split inputs (ggml-backend.cpp:1391-1399,
// called on the destination backend; ggml-cuda.cu:2437-2490 is the CUDA counterpart).
//   * different MI355X devices: ncclSend on the source stream + ncclRecv on the destination
//     stream in one group (RCCL over xGMI, see mi_p2p above), or hipMemcpyPeerAsync + event;
//   * same GPU (two backend instances, or two virtual devices): async D2D on the source stream
//     (or RCCL self send/recv under GGML_MI355X_P2P=rccl), the destination stream waits on a
//     pooled event recorded after it.
static bool mi_backend_cpy_tensor_async(ggml_backend_t backend_src, ggml_backend_t backend_dst, const ggml_tensor * src, ggml_tensor * dst) {
    if (!mi_backend_is_ours(backend_src) || !mi_backend_is_ours(backend_dst)) return false;
    if (!src->buffer || !dst->buffer || !mi_buf_is_ours(src->buffer) || !mi_buf_is_ours(dst->buffer)) return false;
    if (!ggml_is_contiguous(src) || !ggml_is_contiguous(dst) || ggml_nbytes(src) != ggml_nbytes(dst)) return false;
    auto * sctx = (mi_backend_ctx *) backend_src->context;
    auto * dctx = (mi_backend_ctx *) backend_dst->context;
    const size_t n = ggml_nbytes(dst);
    MI_CHECK(hipSetDevice(sctx->device));
    up_fence(sctx->device, sctx->ex.stream, sctx->up_seen);
    MI_CHECK(hipSetDevice(dctx->device));
    up_fence(dctx->device, dctx->ex.stream, dctx->up_seen);
    static const p2p_mode mode = p2p_mode_env();
    if (sctx->device != dctx->device && mode != P2P_PEER &&
        p2p_send_recv(src->data, sctx->device, sctx->ex.stream, dst->data, dctx->device, dctx->ex.stream, n)) {
        return true;
    }
    MI_CHECK(hipSetDevice(sctx->device));
    if (sctx->device == dctx->device) {
        if (!(mode == P2P_RCCL_ALL && backend_src != backend_dst && p2p_self(src->data, dst->data, sctx->device, sctx->ex.stream, n))) {
            MI_CHECK(hipMemcpyAsync(dst->data, src->data, n, hipMemcpyDeviceToDevice, sctx->ex.stream));
            g_p2p_d2d.fetch_add(1);
        }
    } else {
        MI_CHECK(hipMemcpyPeerAsync(dst->data, dctx->device, src->data, sctx->device, n, sctx->ex.stream));
        g_p2p_peer.fetch_add(1);
    }
    if (backend_src != backend_dst) {
        hipEvent_t ev = sctx->next_xevent();
        MI_CHECK(hipEventRecord(ev, sctx->ex.stream));
        MI_CHECK(hipSetDevice(dctx->device));
        MI_CHECK(hipStreamWaitEvent(dctx->ex.stream, ev, 0));
    }
    return true;
}

// decodes the current graph's timeline regions (synchronous: profiling runs only)
static void kt_collect(mi_backend_ctx * ctx) {
    auto & ex = ctx->ex;
    MI_CHECK(hipStreamSynchronize(ex.stream));
    if (ex.kt_list.empty()) return;
    std::vector<unsigned long long> h(ex.kt_off);
    MI_CHECK(hipMemcpy(h.data(), ex.kt_buf, ex.kt_off * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    static double tick_ns = 0.0;
    if (tick_ns == 0.0) {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess || khz <= 0) khz = 100000;
        tick_ns = 1e6 / khz;
    }
    std::lock_guard<std::mutex> lk(g_kt_mtx);
    const long gs = g_kt_graphs++;
    unsigned long long base = ~0ull;
    for (auto & l : ex.kt_list) {
        for (unsigned w = 0; w < l.nwg; ++w) {
            const unsigned long long v = h[l.off + (size_t) w * l.stride];
            if (v && v < base) base = v;
        }
    }
    for (size_t i = 0; i < ex.kt_list.size(); ++i) {
        const auto & l = ex.kt_list[i];
        unsigned long long s0 = ~0ull, sl = 0, e1 = 0, w0e = 0;
        double life = 0.0;
        unsigned nl = 0;
        for (unsigned w = 0; w < l.nwg; ++w) {
            const unsigned long long * r = h.data() + l.off + (size_t) w * l.stride;
            unsigned long long we = 0;
            for (unsigned k = 1; k < l.stride; ++k) we = std::max(we, r[k]);
            if (r[0]) {
                s0 = std::min(s0, r[0]);
                sl = std::max(sl, r[0]);
                if (we >= r[0]) { life += (double) (we - r[0]); ++nl; }
            }
            e1 = std::max(e1, we);
            if (w == 0) w0e = we;
        }
        if (s0 == ~0ull) continue;
        // GGML_MI355X_KTRACE_RAW=<name>: every slot of that launch's workgroup 0, in us from its start
        static const char * raw = getenv("GGML_MI355X_KTRACE_RAW");
        if (raw && strcmp(raw, l.name) == 0) {
            const unsigned long long * r = h.data() + l.off;
            fprintf(stderr, "[ktraw] %s:", l.name);
            for (unsigned k = 1; k < l.stride; ++k) fprintf(stderr, " %.2f", r[k] >= r[0] ? (r[k] - r[0]) * tick_ns / 1e3 : -1.0);
            fprintf(stderr, "\n");
        }
        // GGML_MI355X_KTRACE_DIST=<name>: every workgroup's start and end of that launch, in us from its
        // first start (workgroup order)
        static const char * dist = getenv("GGML_MI355X_KTRACE_DIST");
        if (dist && strcmp(dist, l.name) == 0) {
            fprintf(stderr, "[ktdist] %s:", l.name);
            for (unsigned w = 0; w < l.nwg; ++w) {
                const unsigned long long * r = h.data() + l.off + (size_t) w * l.stride;
                unsigned long long we = 0;
                for (unsigned k = 1; k < l.stride; ++k) we = std::max(we, r[k]);
                fprintf(stderr, " %.2f,%.2f", r[0] ? (r[0] - s0) * tick_ns / 1e3 : -1.0, we ? (we - s0) * tick_ns / 1e3 : -1.0);
            }
            fprintf(stderr, "\n");
        }
        g_kt_samples.push_back({gs, (int) i, l.name, l.nwg, (s0 - base) * tick_ns, (sl - base) * tick_ns, (e1 - base) * tick_ns,
                                w0e ? (w0e - base) * tick_ns : 0.0, nl ? life / nl * tick_ns : 0.0});
    }
}

static void mi_backend_synchronize(ggml_backend_t backend) {
    hp_scope hp_(HP_SYNC);
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipStreamSynchronize(ctx->ex.stream));
    ctx->ex.collect_timing();
}

static void run_nodes(exec_ctx & ex, ggml_cgraph * cgraph) {
    ex.kt_off = 0;
    ex.kt_list.clear();
    ex.qcache_clear();
    ex.rt_table = nullptr;
    ex.done.clear();
    ex.silu_defer = ex.silu_mul = nullptr;
    ex.pro = {};
    ex.moe = {};
    ex.moe_pro = {};
    const int n = ggml_graph_n_nodes(cgraph);
    for (int i = 0; i < n;) i += op_compute(ex, cgraph, i);
    GGML_ASSERT(!ex.moe.comb && !ex.moe_pro.mm);   // deferred MoE work always meets its consumer
    if (ex.silu_defer) {   // a deferred SILU whose MUL never came
        op_unary(ex, ex.silu_defer);
        ex.silu_defer = ex.silu_mul = nullptr;
    }
    ex.pro = {};
}

// returns true when the graph was launched as (or captured into) a hipGraph
static bool graph_compute_hipgraph(mi_backend_ctx * ctx, ggml_cgraph * cgraph) {
    // a scratch slot grew since these graphs were captured (e.g. a longer prompt after
    // decoding): their kernel arguments point at freed slots, so they are dropped and
    // re-captured on a later sighting
    for (auto it = ctx->graphs.begin(); it != ctx->graphs.end();) {
        if (it->exec && it->gen != ctx->ex.scratch_gen) {
            MI_CHECK(hipStreamSynchronize(ctx->ex.stream));
            MI_CHECK(hipGraphExecDestroy(it->exec));
            it = ctx->graphs.erase(it);
        } else {
            ++it;
        }
    }
    static thread_local std::vector<int64_t> sig;
    {
        hp_scope hps(HP_C_SIG);
        graph_signature(cgraph, sig);
    }
    graph_entry * e = nullptr;
    for (auto & g : ctx->graphs) {
        if (g.sig == sig) { e = &g; break; }
    }
    if (!e) {
        constexpr size_t MAX_GRAPHS = 4;
        if (ctx->graphs.size() >= MAX_GRAPHS) {
            auto lru = ctx->graphs.begin();
            for (auto it = ctx->graphs.begin(); it != ctx->graphs.end(); ++it) {
                if (it->last_use < lru->last_use) lru = it;
            }
            if (lru->exec) MI_CHECK(hipGraphExecDestroy(lru->exec));
            ctx->graphs.erase(lru);
        }
        ctx->graphs.emplace_back();
        e = &ctx->graphs.back();
        e->sig = sig;
    }
    e->last_use = ++ctx->use_clock;
    if (e->exec) {
        hp_scope hpl(HP_C_LAUNCH);
        MI_CHECK(hipGraphLaunch(e->exec, ctx->ex.stream));
        ctx->ex.kt_list = e->kt_list;
        ctx->ex.kt_off = e->kt_off;
        g_graph_replays.fetch_add(1);
        return true;
    }
    if (++e->seen < 2) return false;   // first sighting runs eagerly (sizes the scratch arena)

    hipGraph_t g = nullptr;
    ctx->ex.capturing = true;
    capture_open();
    MI_CHECK(hipStreamBeginCapture(ctx->ex.stream, hipStreamCaptureModeRelaxed));
    run_nodes(ctx->ex, cgraph);
    const hipError_t cerr = hipStreamEndCapture(ctx->ex.stream, &g);
    capture_close();
    ctx->ex.capturing = false;
    if (cerr != hipSuccess || g == nullptr ||
        hipGraphInstantiate(&e->exec, g, nullptr, nullptr, 0) != hipSuccess) {
        MI_LOG_WARN("mi355x: hipGraph capture failed (%s); running graphs eagerly\n", hipGetErrorString(cerr));
        (void) hipGetLastError();
        if (g) (void) hipGraphDestroy(g);
        e->exec = nullptr;
        ctx->graphs_broken = true;
        return false;
    }
    MI_CHECK(hipGraphDestroy(g));
    e->gen = ctx->ex.scratch_gen;
    e->kt_list = ctx->ex.kt_list;
    e->kt_off = ctx->ex.kt_off;
    MI_CHECK(hipGraphLaunch(e->exec, ctx->ex.stream));
    g_graph_captures.fetch_add(1);
    return true;
}

static enum ggml_status mi_backend_graph_compute(ggml_backend_t backend, ggml_cgraph * cgraph) {
    static std::atomic<long> hp_graphs{0};
    if (g_hostprof && (hp_graphs.fetch_add(1) + 1) % 64 == 0) hp_report();
    hp_scope hp_(HP_COMPUTE);
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    {
        hp_scope hpf(HP_C_FENCE);
        up_fence(ctx->device, ctx->ex.stream, ctx->up_seen);   // the graph's inputs (set_tensor) are in
    }
    ctx->ex.timing = g_timing.load(std::memory_order_relaxed) != 0;
    // whole-graph timing (kind TK_GRAPH: device time between events around the graph;
    // TK_GRAPH_HOST: host time spent in this call) — works with hipGraph replay
    const bool gtime = g_graph_timing.load(std::memory_order_relaxed) != 0;
    const auto h0 = std::chrono::steady_clock::now();
    hipEvent_t gbeg = nullptr;
    if (gtime) {
        gbeg = ctx->ex.get_event();
        MI_CHECK(hipEventRecord(gbeg, ctx->ex.stream));
    }
    bool dyn_ok;
    {
        hp_scope hpd(HP_C_DYN);
        dyn_ok = ctx->ex.prepare_dyn(cgraph);
    }
    const bool ktrace = ktrace_enabled();
    if (ktrace) {
        if (!ctx->ex.kt_buf) {
            ctx->ex.kt_cap = (size_t) 1 << 22;
            MI_CHECK(hipMalloc(&ctx->ex.kt_buf, ctx->ex.kt_cap * sizeof(unsigned long long)));
        }
        MI_CHECK(hipMemsetAsync(ctx->ex.kt_buf, 0, ctx->ex.kt_cap * sizeof(unsigned long long), ctx->ex.stream));
    }
    // a row-split mat-mul with a slice on another GPU runs its helper streams eagerly
    bool foreign = false;
    for (int i = 0; i < ggml_graph_n_nodes(cgraph) && !foreign; ++i) {
        const ggml_tensor * t = ggml_graph_node(cgraph, i);
        split_parts sp;
        if (t->op == GGML_OP_MUL_MAT && tensor_split_parts(t->src[0], sp)) {
            for (int k = 0; k < sp.n; ++k) foreign = foreign || sp.p[k].hip != ctx->device;
        }
    }
    const bool use_graph = dyn_ok && graphs_enabled() && !ctx->graphs_broken && !ctx->ex.timing && !foreign;
    if (!use_graph || !graph_compute_hipgraph(ctx, cgraph)) {
        run_nodes(ctx->ex, cgraph);
    }
    if (ktrace) kt_collect(ctx);
    if (gtime) {
        hipEvent_t gend = ctx->ex.get_event();
        MI_CHECK(hipEventRecord(gend, ctx->ex.stream));
        ctx->ex.pending.push_back({gbeg, gend, 0.0, TK_GRAPH});
        const double hms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count();
        std::lock_guard<std::mutex> lk(g_timing_mtx);
        g_acc_ms[TK_GRAPH_HOST] += hms;
        g_acc_count[TK_GRAPH_HOST] += 1;
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        MI_LOG_ERROR("%s: kernel launch failed: %s\n", __func__, hipGetErrorString(err));
        return GGML_STATUS_FAILED;
    }
    return GGML_STATUS_SUCCESS;
}

static void mi_backend_event_record(ggml_backend_t backend, ggml_backend_event_t event) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipEventRecord((hipEvent_t) event->context, ctx->ex.stream));
}

static void mi_backend_event_wait(ggml_backend_t backend, ggml_backend_event_t event) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipStreamWaitEvent(ctx->ex.stream, (hipEvent_t) event->context, 0));
}

static const ggml_backend_i mi_backend_iface = {
    /* .get_name           = */ mi_backend_get_name,
    /* .free               = */ mi_backend_free,
    /* .set_tensor_async   = */ mi_backend_set_tensor_async,
    /* .get_tensor_async   = */ mi_backend_get_tensor_async,
    /* .cpy_tensor_async   = */ mi_backend_cpy_tensor_async,
    /* .synchronize        = */ mi_backend_synchronize,
    /* .graph_plan_create  = */ nullptr,
    /* .graph_plan_free    = */ nullptr,
    /* .graph_plan_update  = */ nullptr,
    /* .graph_plan_compute = */ nullptr,
    /* .graph_compute      = */ mi_backend_graph_compute,
    /* .event_record       = */ mi_backend_event_record,
    /* .event_wait         = */ mi_backend_event_wait,
};

static ggml_guid_t mi_guid() {
    static ggml_guid guid = {0x4d, 0x49, 0x33, 0x35, 0x35, 0x58, 0x2d, 0x67, 0x66, 0x78, 0x39, 0x35, 0x30, 0x2d, 0x76, 0x31};
    return &guid;
}

static bool mi_backend_is_ours(ggml_backend_t backend) {
    return backend != nullptr && ggml_guid_matches(backend->guid, mi_guid());
}

// ------------------------------------------------------------------------------------------
// device
// ------------------------------------------------------------------------------------------
static const char * mi_dev_get_name(ggml_backend_dev_t dev) { return ((mi_device_ctx *) dev->context)->name.c_str(); }
static const char * mi_dev_get_description(ggml_backend_dev_t dev) { return ((mi_device_ctx *) dev->context)->description.c_str(); }

static void mi_dev_get_memory(ggml_backend_dev_t dev, size_t * free, size_t * total) {
    auto * ctx = (mi_device_ctx *) dev->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipMemGetInfo(free, total));
}

static enum ggml_backend_dev_type mi_dev_get_type(ggml_backend_dev_t) { return GGML_BACKEND_DEVICE_TYPE_GPU; }

static void mi_dev_get_props(ggml_backend_dev_t dev, ggml_backend_dev_props * props) {
    props->name = mi_dev_get_name(dev);
    props->description = mi_dev_get_description(dev);
    props->type = mi_dev_get_type(dev);
    mi_dev_get_memory(dev, &props->memory_free, &props->memory_total);
    props->caps = {
        /* .async                = */ true,
        /* .host_buffer          = */ !getenv("GGML_MI355X_NO_HOST_BUFFER"),
        /* .buffer_from_host_ptr = */ false,
        /* .events               = */ true,
    };
}

static ggml_backend_t mi_dev_init_backend(ggml_backend_dev_t dev, const char * params) {
    (void) params;
    auto * dctx = (mi_device_ctx *) dev->context;
    MI_CHECK(hipSetDevice(dctx->device));
    auto * ctx = new mi_backend_ctx;
    ctx->device = dctx->device;
    ctx->name = dctx->name;
    ctx->ex.device = dctx->device;
    MI_CHECK(hipStreamCreateWithFlags(&ctx->ex.stream, hipStreamNonBlocking));
    {
        std::lock_guard<std::mutex> lk(g_bdev_mtx);
        if (std::find(g_bdevs.begin(), g_bdevs.end(), dctx->device) == g_bdevs.end()) g_bdevs.push_back(dctx->device);
    }
    return new ggml_backend{
        /* .guid    = */ mi_guid(),
        /* .iface   = */ mi_backend_iface,
        /* .device  = */ dev,
        /* .context = */ ctx,
    };
}

static ggml_backend_buffer_type_t mi_dev_get_buffer_type(ggml_backend_dev_t dev) {
    return &((mi_device_ctx *) dev->context)->buft;
}

// GGML_MI355X_NO_HOST_BUFFER=1: no pinned host buffer type (pageable copies, as round 1)
static ggml_backend_buffer_type_t mi_dev_get_host_buffer_type(ggml_backend_dev_t) {
    return getenv("GGML_MI355X_NO_HOST_BUFFER") ? nullptr : mi_host_buft();
}

static bool mi_dev_supports_op(ggml_backend_dev_t dev, const ggml_tensor * op) {
    hp_scope hp_(HP_SUPPORTS);
    return mi_split_op_ok(dev, op) && op_supported(op);
}

static bool mi_dev_supports_buft(ggml_backend_dev_t dev, ggml_backend_buffer_type_t buft) {
    if (mi_split_buft_is_ours(buft)) return buft->device == dev;
    if (buft->iface.get_name == mi_hostptr_buft_get_name) return buft->device == dev;   // mapped host memory
    return mi_buft_is_ours(buft) && buft->context == dev->context;
}

// mirror of the CUDA heuristic (ggml-cuda.cu:3326-3347): offload big-batch ops whose
// weights live in host memory
// the batch an op carries, as the scheduler's offload test measures it (the CUDA backend's
// per-op rule, ggml-cuda.cu:3326-3338): the token count of a mat-mul, the token dimension ne[2]
// of MUL_MAT_ID (ne[1] is the expert slots) and ROPE (ne[1] is the heads), the rows otherwise;
// GET_ROWS (the embedding) is never offloaded
static int64_t mi_op_batch(const ggml_tensor * op) {
    switch (op->op) {
        case GGML_OP_GET_ROWS: return 0;
        case GGML_OP_MUL_MAT: return op->ne[1];
        case GGML_OP_MUL_MAT_ID: case GGML_OP_ROPE: case GGML_OP_ROPE_BACK: return op->ne[2];
        default: return ggml_nrows(op);
    }
}

static bool mi_dev_offload_op(ggml_backend_dev_t, const ggml_tensor * op) {
    const int min_batch = 32;
    return mi_op_batch(op) >= min_batch;
}

static ggml_backend_event_t mi_dev_event_new(ggml_backend_dev_t dev) {
    auto * ctx = (mi_device_ctx *) dev->context;
    MI_CHECK(hipSetDevice(ctx->device));
    hipEvent_t ev;
    MI_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    return new ggml_backend_event{dev, ev};
}

static void mi_dev_event_free(ggml_backend_dev_t, ggml_backend_event_t event) {
    MI_CHECK(hipEventDestroy((hipEvent_t) event->context));
    delete event;
}

static void mi_dev_event_synchronize(ggml_backend_dev_t, ggml_backend_event_t event) {
    MI_CHECK(hipEventSynchronize((hipEvent_t) event->context));
}

static const ggml_backend_device_i mi_device_iface = {
    /* .get_name             = */ mi_dev_get_name,
    /* .get_description      = */ mi_dev_get_description,
    /* .get_memory           = */ mi_dev_get_memory,
    /* .get_type             = */ mi_dev_get_type,
    /* .get_props            = */ mi_dev_get_props,
    /* .init_backend         = */ mi_dev_init_backend,
    /* .get_buffer_type      = */ mi_dev_get_buffer_type,
    /* .get_host_buffer_type = */ mi_dev_get_host_buffer_type,
    /* .buffer_from_host_ptr = */ mi_dev_buffer_from_host_ptr,
    /* .supports_op          = */ mi_dev_supports_op,
    /* .supports_buft        = */ mi_dev_supports_buft,
    /* .offload_op           = */ mi_dev_offload_op,
    /* .event_new            = */ mi_dev_event_new,
    /* .event_free           = */ mi_dev_event_free,
    /* .event_synchronize    = */ mi_dev_event_synchronize,
};

// ------------------------------------------------------------------------------------------
// registry
// ------------------------------------------------------------------------------------------
static const char * mi_reg_get_name(ggml_backend_reg_t) { return MI355X_NAME; }

static size_t mi_reg_get_device_count(ggml_backend_reg_t reg) {
    return ((mi_reg_ctx *) reg->context)->devices.size();
}

static ggml_backend_dev_t mi_reg_get_device(ggml_backend_reg_t reg, size_t index) {
    auto * ctx = (mi_reg_ctx *) reg->context;
    GGML_ASSERT(index < ctx->devices.size());
    return &ctx->devices[index];
}

static ggml_backend_feature * mi_get_features(ggml_backend_reg_t) {
    static ggml_backend_feature features[] = {
        {"ARCH", "gfx950"},
        {"WAVE_SIZE", "64"},
        {"MMV_DOT4", "1"},
        {nullptr, nullptr},
    };
    return features;
}

static void * mi_reg_get_proc_address(ggml_backend_reg_t, const char * name) {
    if (strcmp(name, "ggml_backend_get_features") == 0) return (void *) mi_get_features;
    if (strcmp(name, "ggml_backend_split_buffer_type") == 0) return (void *) mi_split_buffer_type;
    return nullptr;
}

static const ggml_backend_reg_i mi_reg_iface = {
    /* .get_name         = */ mi_reg_get_name,
    /* .get_device_count = */ mi_reg_get_device_count,
    /* .get_device       = */ mi_reg_get_device,
    /* .get_proc_address = */ mi_reg_get_proc_address,
};

static ggml_backend_reg_t mi_reg() {
    static std::mutex mtx;
    static ggml_backend_reg reg;
    static bool initialized = false;
    std::lock_guard<std::mutex> lock(mtx);
    if (!initialized) {
        auto * ctx = new mi_reg_ctx;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) {
            (void) hipGetLastError();
            n = 0;
        }
        // GGML_MI355X_VDEV=k (k > 1): k ggml devices over HIP device 0 — libllama's multi-device
        // paths (layer split with the scheduler's pipeline copies and cpy_tensor_async hand-offs,
        // row split) then run on a one-GPU box; each virtual device has its own buffers and streams
        const int vdev = getenv("GGML_MI355X_VDEV") ? std::min(atoi(getenv("GGML_MI355X_VDEV")), MI_MAX_DEV) : 0;
        const int nd = (vdev > 1 && n >= 1) ? vdev : std::min(n, MI_MAX_DEV);
        ctx->dev_ctx.reserve(nd);
        ctx->devices.reserve(nd);
        for (int i = 0; i < nd; ++i) {
            const int hip = nd != n ? 0 : i;
            hipDeviceProp_t prop;
            MI_CHECK(hipGetDeviceProperties(&prop, hip));
            auto * d = new mi_device_ctx;
            d->device = hip;
            d->name = std::string(MI355X_NAME) + std::to_string(i);
            d->arch = prop.gcnArchName;
            d->description = std::string(prop.name) + " (" + d->arch + ", " + std::to_string(prop.multiProcessorCount) + " CUs" +
                             (nd != n ? ", virtual device " + std::to_string(i) + " of HIP device 0)" : ")");
            d->total_mem = prop.totalGlobalMem;
            d->buft = {mi_buft_iface, nullptr, d};
            ctx->dev_ctx.push_back(d);
        }
        n = nd;
        for (int i = 0; i < n; ++i) {
            ctx->devices.push_back({mi_device_iface, &reg, ctx->dev_ctx[i]});
            ctx->dev_ctx[i]->buft.device = &ctx->devices[i];
        }
        reg = {GGML_BACKEND_API_VERSION, mi_reg_iface, ctx};
        initialized = true;
    }
    return &reg;
}

// ------------------------------------------------------------------------------------------
// exported C ABI (include/ggml-mi355x.h)
// ------------------------------------------------------------------------------------------
extern "C" {

GGML_BACKEND_API ggml_backend_reg_t ggml_backend_init(void) { return mi_reg(); }

GGML_BACKEND_API int ggml_backend_score(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void) hipGetLastError();
        return 0;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 0;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 100 : 0;
}

GGML_BACKEND_API ggml_backend_reg_t ggml_backend_mi355x_reg(void) { return mi_reg(); }

GGML_BACKEND_API int ggml_backend_mi355x_get_device_count(void) { return (int) mi_reg_get_device_count(mi_reg()); }

GGML_BACKEND_API ggml_backend_t ggml_backend_mi355x_init(int device) {
    ggml_backend_reg_t reg = mi_reg();
    if (device < 0 || (size_t) device >= mi_reg_get_device_count(reg)) return nullptr;
    return mi_dev_init_backend(mi_reg_get_device(reg, device), nullptr);
}

GGML_BACKEND_API bool ggml_backend_is_mi355x(ggml_backend_t backend) { return mi_backend_is_ours(backend); }

GGML_BACKEND_API void ggml_backend_mi355x_graph_stats(long * captures, long * replays) {
    if (captures) *captures = g_graph_captures.load();
    if (replays) *replays = g_graph_replays.load();
}

GGML_BACKEND_API void ggml_backend_mi355x_set_graph_timing(int enable) { g_graph_timing.store(enable ? 1 : 0); }

GGML_BACKEND_API void ggml_backend_mi355x_p2p_stats(long * rccl, long * peer) {
    if (rccl) *rccl = g_p2p_rccl.load();
    if (peer) *peer = g_p2p_peer.load();
}

GGML_BACKEND_API void ggml_backend_mi355x_handoff_stats(long * rccl, long * peer, long * d2d) {
    if (rccl) *rccl = g_p2p_rccl.load();
    if (peer) *peer = g_p2p_peer.load();
    if (d2d) *d2d = g_p2p_d2d.load();
}

GGML_BACKEND_API void ggml_backend_mi355x_p2p_release(void) { p2p_destroy(); }

GGML_BACKEND_API void ggml_backend_mi355x_split_stats(long * mm, long * foreign) { mi355x::split_stats(mm, foreign); }

GGML_BACKEND_API ggml_backend_buffer_type_t ggml_backend_mi355x_split_buffer_type(int main_device, const float * tensor_split) {
    return mi_split_buffer_type(main_device, tensor_split);
}

GGML_BACKEND_API void ggml_backend_mi355x_set_flags(int no_fuse, int no_graph) {
    g_no_fuse.store(no_fuse ? 1 : 0);
    g_no_graph.store(no_graph ? 1 : 0);
}

GGML_BACKEND_API void ggml_backend_mi355x_set_timing(int enable) { g_timing.store(enable ? 1 : 0); }

GGML_BACKEND_API void ggml_backend_mi355x_set_ktrace(int enable) { g_ktrace.store(enable ? 1 : 0); }

GGML_BACKEND_API int ggml_backend_mi355x_ktrace_dump(const char * path) {
    std::lock_guard<std::mutex> lk(g_kt_mtx);
    FILE * f = fopen(path, "w");
    if (!f) return -1;
    fprintf(f, "graph,idx,kernel,nwg,start_ns,last_start_ns,end_ns,wg0_end_ns,wg_mean_ns\n");
    for (const auto & k : g_kt_samples) {
        fprintf(f, "%ld,%d,%s,%u,%.0f,%.0f,%.0f,%.0f,%.0f\n", k.graph, k.idx, k.name, k.nwg, k.t0, k.t_last_start, k.t1, k.t_wg0_end,
                k.wg_mean);
    }
    fclose(f);
    const int n = (int) g_kt_samples.size();
    g_kt_samples.clear();
    g_kt_graphs = 0;
    return n;
}

GGML_BACKEND_API void ggml_backend_mi355x_reset_timing(void) {
    std::lock_guard<std::mutex> lk(g_timing_mtx);
    for (int i = 0; i < 8; ++i) { g_acc_ms[i] = 0; g_acc_bytes[i] = 0; g_acc_count[i] = 0; }
}

GGML_BACKEND_API int ggml_backend_mi355x_get_timing(int kind, double * ms, double * bytes, long * count) {
    if (kind < 0 || kind >= 8) return -1;
    std::lock_guard<std::mutex> lk(g_timing_mtx);
    *ms = g_acc_ms[kind];
    *bytes = g_acc_bytes[kind];
    *count = g_acc_count[kind];
    return 0;
}

}  // extern "C"
