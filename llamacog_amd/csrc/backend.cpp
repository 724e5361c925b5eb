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

#include <atomic>
#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

using namespace mi355x;

#define MI355X_NAME "MI355X"

// ------------------------------------------------------------------------------------------
// timing accumulators (global so bench.py can read them through the C ABI)
// ------------------------------------------------------------------------------------------
static std::atomic<int> g_timing{0};
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
        MI_CHECK(hipFree(slot_ptr[slot]));
    }
    MI_CHECK(hipMalloc(&slot_ptr[slot], nsz));
    slot_size[slot] = nsz;
    return slot_ptr[slot];
}

void exec_ctx::free_scratch() {
    for (int i = 0; i < N_SLOTS; ++i) {
        if (slot_ptr[i]) (void) hipFree(slot_ptr[i]);
        slot_ptr[i] = nullptr;
        slot_size[i] = 0;
    }
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

static void mi_buf_free(ggml_backend_buffer_t buffer) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
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

static void mi_buf_memset_tensor(ggml_backend_buffer_t buffer, ggml_tensor * tensor, uint8_t value, size_t offset, size_t size) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipMemsetAsync((char *) tensor->data + offset, value, size, hipStreamPerThread));
    MI_CHECK(hipStreamSynchronize(hipStreamPerThread));
}

static void mi_buf_set_tensor(ggml_backend_buffer_t buffer, ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipMemcpyAsync((char *) tensor->data + offset, data, size, hipMemcpyHostToDevice, hipStreamPerThread));
    MI_CHECK(hipStreamSynchronize(hipStreamPerThread));
}

static void mi_buf_get_tensor(ggml_backend_buffer_t buffer, const ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    auto * ctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipMemcpyAsync(data, (const char *) tensor->data + offset, size, hipMemcpyDeviceToHost, hipStreamPerThread));
    MI_CHECK(hipStreamSynchronize(hipStreamPerThread));
}

static bool mi_buf_is_ours(ggml_backend_buffer_t buffer);

static bool mi_buf_cpy_tensor(ggml_backend_buffer_t buffer, const ggml_tensor * src, ggml_tensor * dst) {
    if (src->buffer == nullptr || !mi_buf_is_ours(src->buffer)) return false;
    auto * sctx = (mi_buffer_ctx *) src->buffer->context;
    auto * dctx = (mi_buffer_ctx *) buffer->context;
    MI_CHECK(hipSetDevice(dctx->device));
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
// backend (stream)
// ------------------------------------------------------------------------------------------
struct mi_backend_ctx {
    int device;
    std::string name;
    exec_ctx ex;
};

static const char * mi_backend_get_name(ggml_backend_t backend) {
    return ((mi_backend_ctx *) backend->context)->name.c_str();
}

static void mi_backend_free(ggml_backend_t backend) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipStreamSynchronize(ctx->ex.stream));
    ctx->ex.collect_timing();
    for (auto e : ctx->ex.event_pool) (void) hipEventDestroy(e);
    ctx->ex.free_scratch();
    MI_CHECK(hipStreamDestroy(ctx->ex.stream));
    delete ctx;
    delete backend;
}

static void mi_backend_set_tensor_async(ggml_backend_t backend, ggml_tensor * tensor, const void * data, size_t offset, size_t size) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipMemcpyAsync((char *) tensor->data + offset, data, size, hipMemcpyHostToDevice, ctx->ex.stream));
}

static void mi_backend_get_tensor_async(ggml_backend_t backend, const ggml_tensor * tensor, void * data, size_t offset, size_t size) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipMemcpyAsync(data, (const char *) tensor->data + offset, size, hipMemcpyDeviceToHost, ctx->ex.stream));
}

static bool mi_backend_is_ours(ggml_backend_t backend);

// Cross-device copy hook used by the scheduler for split inputs (ggml-backend.cpp:1391).
// Same device: async D2D on the source stream; different MI355X devices: peer copy over
// xGMI.  The destination stream waits on an event recorded after the copy.
static bool mi_backend_cpy_tensor_async(ggml_backend_t backend_src, ggml_backend_t backend_dst, const ggml_tensor * src, ggml_tensor * dst) {
    if (!mi_backend_is_ours(backend_src) || !mi_backend_is_ours(backend_dst)) return false;
    if (!src->buffer || !dst->buffer || !mi_buf_is_ours(src->buffer) || !mi_buf_is_ours(dst->buffer)) return false;
    auto * sctx = (mi_backend_ctx *) backend_src->context;
    auto * dctx = (mi_backend_ctx *) backend_dst->context;
    const size_t n = ggml_nbytes(dst);
    MI_CHECK(hipSetDevice(sctx->device));
    if (sctx->device == dctx->device) {
        MI_CHECK(hipMemcpyAsync(dst->data, src->data, n, hipMemcpyDeviceToDevice, sctx->ex.stream));
    } else {
        MI_CHECK(hipMemcpyPeerAsync(dst->data, dctx->device, src->data, sctx->device, n, sctx->ex.stream));
    }
    if (backend_src != backend_dst) {
        hipEvent_t ev;
        MI_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        MI_CHECK(hipEventRecord(ev, sctx->ex.stream));
        MI_CHECK(hipSetDevice(dctx->device));
        MI_CHECK(hipStreamWaitEvent(dctx->ex.stream, ev, 0));
        MI_CHECK(hipEventDestroy(ev));
    }
    return true;
}

static void mi_backend_synchronize(ggml_backend_t backend) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    MI_CHECK(hipStreamSynchronize(ctx->ex.stream));
    ctx->ex.collect_timing();
}

static enum ggml_status mi_backend_graph_compute(ggml_backend_t backend, ggml_cgraph * cgraph) {
    auto * ctx = (mi_backend_ctx *) backend->context;
    MI_CHECK(hipSetDevice(ctx->device));
    ctx->ex.timing = g_timing.load(std::memory_order_relaxed) != 0;
    const int n = ggml_graph_n_nodes(cgraph);
    for (int i = 0; i < n;) {
        i += op_compute(ctx->ex, cgraph, i);
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
        /* .host_buffer          = */ false,
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

static bool mi_dev_supports_op(ggml_backend_dev_t dev, const ggml_tensor * op) {
    (void) dev;
    return op_supported(op);
}

static bool mi_dev_supports_buft(ggml_backend_dev_t dev, ggml_backend_buffer_type_t buft) {
    return mi_buft_is_ours(buft) && buft->context == dev->context;
}

// mirror of the CUDA heuristic (ggml-cuda.cu:3326-3347): offload big-batch ops whose
// weights live in host memory
static bool mi_dev_offload_op(ggml_backend_dev_t, const ggml_tensor * op) {
    const int min_batch = 32;
    return op->ne[1] >= min_batch && op->op != GGML_OP_GET_ROWS;
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
    /* .get_host_buffer_type = */ nullptr,
    /* .buffer_from_host_ptr = */ nullptr,
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
        ctx->dev_ctx.reserve(n);
        ctx->devices.reserve(n);
        for (int i = 0; i < n; ++i) {
            hipDeviceProp_t prop;
            MI_CHECK(hipGetDeviceProperties(&prop, i));
            auto * d = new mi_device_ctx;
            d->device = i;
            d->name = std::string(MI355X_NAME) + std::to_string(i);
            d->arch = prop.gcnArchName;
            d->description = std::string(prop.name) + " (" + d->arch + ", " + std::to_string(prop.multiProcessorCount) + " CUs)";
            d->total_mem = prop.totalGlobalMem;
            d->buft = {mi_buft_iface, nullptr, d};
            ctx->dev_ctx.push_back(d);
        }
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

GGML_BACKEND_API void ggml_backend_mi355x_set_timing(int enable) { g_timing.store(enable ? 1 : 0); }

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
