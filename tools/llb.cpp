// llb.cpp — a thin C-ABI driver over the reference's UNCHANGED libllama (include/llama.h)
// used by bench.py, the greedy-parity tests and smoke().  It reproduces llama-bench's
// measurement loops (tools/llama-bench/llama-bench.cpp:1747-1795, test_prompt/test_gen)
// so the timed region is exactly what llama-bench times, while letting Python own the
// warmup/step/barrier protocol of the bench contract.
//
// Backends are loaded explicitly: the score-selected CPU backend from refhost/build
// (libllama requires it for the token-embedding GET_ROWS, src/llama-model.cpp:1572) and
// optionally the MI355X plugin via ggml_backend_load (same path as GGML_BACKEND_PATH).
#include "ggml-backend.h"
#include "llama.h"

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

std::mutex g_log_mtx;
std::string g_log;
bool g_log_echo = false;

void log_cb(enum ggml_log_level level, const char * text, void *) {
    std::lock_guard<std::mutex> lk(g_log_mtx);
    g_log += text;
    if (g_log.size() > (1u << 20)) g_log.erase(0, g_log.size() - (1u << 19));
    if (g_log_echo || level == GGML_LOG_LEVEL_ERROR) fputs(text, stderr);
}

struct dump_rec {
    std::string name;
    int op;
    int64_t ne[4];
    std::vector<float> data;
};

struct llb {
    bool dump = false;
    std::vector<dump_rec> recs;
    llama_model * model = nullptr;
    llama_context * ctx = nullptr;
    const llama_vocab * vocab = nullptr;
    int n_vocab = 0;
    int n_batch = 0;
    llama_context_params cparams;
    std::vector<ggml_backend_dev_t> devs;
};

// scheduler eval callback (cf. examples/eval-callback): keep a copy of every f32 node
bool dump_cb(struct ggml_tensor * t, bool ask, void * ud) {
    auto * h = (llb *) ud;
    if (ask) return h->dump;
    dump_rec r;
    r.name = t->name;
    r.op = (int) t->op;
    for (int i = 0; i < 4; ++i) r.ne[i] = t->ne[i];
    if (t->type != GGML_TYPE_F32 || ggml_nelements(t) > (1 << 22)) {   // order only, no data
        h->recs.push_back(std::move(r));
        return true;
    }
    r.data.resize(ggml_nelements(t));
    if (ggml_is_contiguous(t)) {
        ggml_backend_tensor_get(t, r.data.data(), 0, ggml_nbytes(t));
    } else {
        r.data.clear();
    }
    h->recs.push_back(std::move(r));
    return true;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" {

// Load backends once: cpu_dir = directory holding libggml-cpu-*.so; plugin may be NULL.
int llb_load_backends(const char * cpu_dir, const char * plugin_path, int echo_log) {
    g_log_echo = echo_log != 0;
    llama_log_set(log_cb, nullptr);
    ggml_log_set(log_cb, nullptr);
    // LLB_CPU_LIB pins one CPU variant (e.g. libggml-cpu-x64v3.so) instead of the
    // score-selected best one — used to measure the reference's own cross-ISA spread
    const char * cpu_lib = getenv("LLB_CPU_LIB");
    if (cpu_lib && cpu_lib[0]) {
        ggml_backend_load(cpu_lib);
    } else {
        ggml_backend_load_all_from_path(cpu_dir);
    }
    if (plugin_path && plugin_path[0]) {
        if (!ggml_backend_load(plugin_path)) return -1;
    }
    llama_backend_init();
    return (int) ggml_backend_dev_count();
}

int llb_dev_count(void) { return (int) ggml_backend_dev_count(); }

const char * llb_dev_name(int i) { return ggml_backend_dev_name(ggml_backend_dev_get(i)); }

int llb_dev_type(int i) { return (int) ggml_backend_dev_type(ggml_backend_dev_get(i)); }

// gpu_mask: bit i selects registry device i as a model device; 0 = CPU only.
void * llb_open(const char * path, unsigned long long gpu_mask, int n_gpu_layers, int flash_attn, int n_ctx,
                int n_batch, int n_ubatch, int type_k, int type_v, int n_threads, int split_mode, int dump) {
    auto * h = new llb;
    h->dump = dump != 0;
    for (size_t i = 0; i < ggml_backend_dev_count(); ++i) {
        if (gpu_mask & (1ull << i)) h->devs.push_back(ggml_backend_dev_get(i));
    }
    h->devs.push_back(nullptr);
    llama_model_params mp = llama_model_default_params();
    mp.devices = h->devs.data();
    mp.n_gpu_layers = gpu_mask ? n_gpu_layers : 0;
    mp.split_mode = (enum llama_split_mode) split_mode;
    mp.use_mmap = true;
    h->model = llama_model_load_from_file(path, mp);
    if (!h->model) { delete h; return nullptr; }
    llama_context_params cp = llama_context_default_params();
    cp.n_ctx = n_ctx;
    cp.n_batch = n_batch;
    cp.n_ubatch = n_ubatch;
    cp.flash_attn = flash_attn != 0;
    cp.type_k = (enum ggml_type) type_k;
    cp.type_v = (enum ggml_type) type_v;
    cp.n_threads = n_threads;
    cp.n_threads_batch = n_threads;
    cp.no_perf = true;
    cp.op_offload = gpu_mask != 0;
    if (h->dump) {
        cp.cb_eval = dump_cb;
        cp.cb_eval_user_data = h;
    }
    h->cparams = cp;
    h->ctx = llama_init_from_model(h->model, cp);
    if (!h->ctx) { llama_model_free(h->model); delete h; return nullptr; }
    h->vocab = llama_model_get_vocab(h->model);
    h->n_vocab = llama_vocab_n_tokens(h->vocab);
    h->n_batch = n_batch;
    return h;
}

void llb_close(void * hp) {
    auto * h = (llb *) hp;
    if (!h) return;
    llama_free(h->ctx);
    llama_model_free(h->model);
    delete h;
}

int llb_n_vocab(void * hp) { return ((llb *) hp)->n_vocab; }

void llb_clear(void * hp) { llama_memory_clear(llama_get_memory(((llb *) hp)->ctx), false); }

// decode n tokens as one batch (chunks of n_batch); returns 0 on success
int llb_decode(void * hp, const int32_t * toks, int n) {
    auto * h = (llb *) hp;
    for (int i = 0; i < n; i += h->n_batch) {
        const int nb = std::min(h->n_batch, n - i);
        int r = llama_decode(h->ctx, llama_batch_get_one(const_cast<int32_t *>(toks + i), nb));
        if (r != 0) return r;
    }
    llama_synchronize(h->ctx);
    return 0;
}

// logits of the last decoded token (n_vocab floats)
const float * llb_logits(void * hp) { return llama_get_logits_ith(((llb *) hp)->ctx, -1); }

// llama-bench test_prompt: n_prompt random tokens, returns wall seconds
double llb_time_prompt(void * hp, int n_prompt) {
    auto * h = (llb *) hp;
    std::vector<int32_t> toks(n_prompt);
    toks[0] = llama_vocab_get_add_bos(h->vocab) ? llama_vocab_bos(h->vocab) : std::rand() % h->n_vocab;
    for (int i = 1; i < n_prompt; ++i) toks[i] = std::rand() % h->n_vocab;
    const double t0 = now_s();
    if (llb_decode(hp, toks.data(), n_prompt) != 0) return -1.0;
    return now_s() - t0;
}

// llama-bench test_gen: n_gen single-token decodes, returns wall seconds
double llb_time_gen(void * hp, int n_gen) {
    auto * h = (llb *) hp;
    int32_t tok = llama_vocab_get_add_bos(h->vocab) ? llama_vocab_bos(h->vocab) : std::rand() % h->n_vocab;
    const double t0 = now_s();
    for (int i = 0; i < n_gen; ++i) {
        if (llama_decode(h->ctx, llama_batch_get_one(&tok, 1)) != 0) return -1.0;
        llama_synchronize(h->ctx);
        tok = std::rand() % h->n_vocab;
    }
    return now_s() - t0;
}

// test_gen with the host time split: seconds inside llama_decode (graph build, scheduling,
// input upload, launch) and inside llama_synchronize (waiting for the device)
double llb_time_gen_split(void * hp, int n_gen, double * t_decode, double * t_sync) {
    auto * h = (llb *) hp;
    int32_t tok = llama_vocab_get_add_bos(h->vocab) ? llama_vocab_bos(h->vocab) : std::rand() % h->n_vocab;
    double td = 0, ts = 0;
    const double t0 = now_s();
    for (int i = 0; i < n_gen; ++i) {
        const double a = now_s();
        if (llama_decode(h->ctx, llama_batch_get_one(&tok, 1)) != 0) return -1.0;
        const double b = now_s();
        llama_synchronize(h->ctx);
        const double c = now_s();
        td += b - a;
        ts += c - b;
        tok = std::rand() % h->n_vocab;
    }
    *t_decode = td;
    *t_sync = ts;
    return now_s() - t0;
}

// greedy decoding: feeds prompt, then n_gen argmax tokens; writes ids and (optionally) all
// logits [n_gen][n_vocab] of each step
int llb_greedy(void * hp, const int32_t * prompt, int n_prompt, int n_gen, int32_t * out_ids, float * out_logits) {
    auto * h = (llb *) hp;
    if (llb_decode(hp, prompt, n_prompt) != 0) return -1;
    for (int s = 0; s < n_gen; ++s) {
        const float * lg = llama_get_logits_ith(h->ctx, -1);
        if (out_logits) memcpy(out_logits + (size_t) s * h->n_vocab, lg, sizeof(float) * h->n_vocab);
        int best = 0;
        for (int i = 1; i < h->n_vocab; ++i) if (lg[i] > lg[best]) best = i;
        out_ids[s] = best;
        int32_t t = best;
        if (s + 1 < n_gen && llb_decode(hp, &t, 1) != 0) return -2;
    }
    return 0;
}

// tests/test-thread-safety.cpp's pattern (several contexts of one model, each decoding in its own
// thread at the same time): n_contexts extra contexts on h's model, each greedy-decodes the same
// prompt concurrently; ids [c][n_gen], logits [c][n_gen][n_vocab].  Returns 0, or -(1 + c) for
// the first context that failed
int llb_greedy_threads(void * hp, int n_contexts, const int32_t * prompt, int n_prompt, int n_gen, int32_t * out_ids,
                       float * out_logits) {
    auto * h = (llb *) hp;
    std::vector<llama_context *> ctxs(n_contexts, nullptr);
    for (int c = 0; c < n_contexts; ++c) {
        ctxs[c] = llama_init_from_model(h->model, h->cparams);
        if (!ctxs[c]) {
            for (auto * x : ctxs) if (x) llama_free(x);
            return -(1 + c);
        }
    }
    std::atomic<int> failed{0};
    std::vector<std::thread> th;
    for (int c = 0; c < n_contexts; ++c) {
        th.emplace_back([&, c]() {
            llama_context * ctx = ctxs[c];
            std::vector<int32_t> p(prompt, prompt + n_prompt);
            if (llama_decode(ctx, llama_batch_get_one(p.data(), n_prompt)) != 0) { failed = 1 + c; return; }
            for (int s = 0; s < n_gen; ++s) {
                llama_synchronize(ctx);
                const float * lg = llama_get_logits_ith(ctx, -1);
                float * dst = out_logits + ((size_t) c * n_gen + s) * h->n_vocab;
                memcpy(dst, lg, sizeof(float) * h->n_vocab);
                int best = 0;
                for (int i = 1; i < h->n_vocab; ++i) if (lg[i] > lg[best]) best = i;
                out_ids[(size_t) c * n_gen + s] = best;
                int32_t t = best;
                if (s + 1 < n_gen && llama_decode(ctx, llama_batch_get_one(&t, 1)) != 0) { failed = 1 + c; return; }
            }
        });
    }
    for (auto & t : th) t.join();
    for (auto * x : ctxs) llama_free(x);
    return failed ? -failed.load() : 0;
}

// copy (a tail of) the captured log; returns its full length
int llb_log(char * buf, int cap) {
    std::lock_guard<std::mutex> lk(g_log_mtx);
    const int n = (int) g_log.size();
    if (buf && cap > 0) {
        const int k = std::min(cap - 1, n);
        memcpy(buf, g_log.data() + (n - k), k);
        buf[k] = 0;
    }
    return n;
}

int llb_dump_n(void * hp) { return (int) ((llb *) hp)->recs.size(); }
const char * llb_dump_name(void * hp, int i) { return ((llb *) hp)->recs[i].name.c_str(); }
int llb_dump_op(void * hp, int i) { return ((llb *) hp)->recs[i].op; }
long long llb_dump_size(void * hp, int i) { return (long long) ((llb *) hp)->recs[i].data.size(); }
void llb_dump_data(void * hp, int i, float * out) {
    auto & r = ((llb *) hp)->recs[i];
    memcpy(out, r.data.data(), r.data.size() * sizeof(float));
}
void llb_dump_clear(void * hp) { ((llb *) hp)->recs.clear(); }

void llb_log_clear(void) {
    std::lock_guard<std::mutex> lk(g_log_mtx);
    g_log.clear();
}

}  // extern "C"
