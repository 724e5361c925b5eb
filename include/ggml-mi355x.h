// ggml-mi355x.h — C ABI of libggml-mi355x.so, the MI355X (gfx950) ggml backend plugin.
//
// The plugin boundary is the reference's ggml backend interface
// (ggml/src/ggml-backend-impl.h:17-251); the two entry points the reference's dlopen
// loader binds are:
//   ggml_backend_init   — ggml-backend-reg.cpp:249  (dlsym "ggml_backend_init")
//   ggml_backend_score  — ggml-backend-reg.cpp:239  (dlsym "ggml_backend_score"); 0 = unusable
// and replace, for this device, the CUDA/HIP backend's ggml_backend_cuda_reg()
// (ggml/src/ggml-cuda/ggml-cuda.cu:3499-3534, GGML_BACKEND_DL_IMPL at :3548).
// The remaining functions mirror ggml-cuda.h's public helpers (ggml/include/ggml-cuda.h)
// plus kernel-timing hooks used by bench.py for the roofline figure.
#pragma once

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ggml_backend_reg * ggml_backend_reg_t;
typedef struct ggml_backend *     ggml_backend_t;

// plugin entry points (GGML_BACKEND_DL)
ggml_backend_reg_t ggml_backend_init(void);
int                ggml_backend_score(void);

// direct use (cf. ggml-cuda.h: ggml_backend_cuda_reg / _init / ggml_backend_is_cuda /
// ggml_backend_cuda_get_device_count)
ggml_backend_reg_t ggml_backend_mi355x_reg(void);
int                ggml_backend_mi355x_get_device_count(void);
ggml_backend_t     ggml_backend_mi355x_init(int device);
bool               ggml_backend_is_mi355x(ggml_backend_t backend);

// kernel timing with HIP events recorded on the backend stream around each launch of the
// mat-vec (kind 0), MFMA mat-mul (1) and flash-attention (2) kernels; bytes are the
// algorithmic bytes of each launch
void ggml_backend_mi355x_set_timing(int enable);
void ggml_backend_mi355x_reset_timing(void);
int  ggml_backend_mi355x_get_timing(int kind, double * ms, double * bytes, long * count);
// whole-graph timing: kind 5 = device time of each graph_compute (events around it, works
// with hipGraph replay), kind 6 = host time spent inside graph_compute
void ggml_backend_mi355x_set_graph_timing(int enable);

// in-graph kernel timeline (profiling): each instrumented launch (the decode mat-vecs and the
// exact flash attention) stamps the chip's realtime counter per workgroup at entry and per wave
// at exit, also inside replayed hipGraphs; graph_compute then synchronises and decodes the
// stamps.  ktrace_dump writes "graph,idx,kernel,nwg,start_ns,last_start_ns,end_ns" rows (times
// from the graph's first stamp), clears them and returns the row count (-1: file error)
void ggml_backend_mi355x_set_ktrace(int enable);
int  ggml_backend_mi355x_ktrace_dump(const char * path);

// run-time switches (default from GGML_MI355X_NO_FUSE / GGML_MI355X_NO_GRAPH): no_fuse = one
// kernel per ggml node, no_graph = no hipGraph replay of repeated graphs
void ggml_backend_mi355x_set_flags(int no_fuse, int no_graph);
// hipGraph statistics since load: graphs captured, replays launched
void ggml_backend_mi355x_graph_stats(long * captures, long * replays);
// split-layer stage hand-offs since load (cpy_tensor_async between two MI355X devices): sent
// over RCCL (ncclSend/ncclRecv, the default) / as hipMemcpyPeerAsync (GGML_MI355X_P2P=peer or
// RCCL unavailable).  Replaces the peer-copy path of ggml-cuda.cu:2437-2490.
void ggml_backend_mi355x_p2p_stats(long * rccl, long * peer);
// the same plus the hand-offs between two ggml devices on ONE GPU (two backends, or the virtual
// devices of GGML_MI355X_VDEV) that went as an async device-to-device copy (d2d); with
// GGML_MI355X_P2P=rccl those go as an RCCL self send/recv and count under rccl
void ggml_backend_mi355x_handoff_stats(long * rccl, long * peer, long * d2d);
// destroys the RCCL communicators (re-created on the next cross-device copy)
void ggml_backend_mi355x_p2p_release(void);
// row split (-sm row): the buffer type libllama obtains through
// ggml_backend_reg_get_proc_address(reg, "ggml_backend_split_buffer_type") (src/llama-model.cpp:
// 337-360; ggml-cuda.cu:1047 is the reference GPU backend's): matrices cut into per-device row
// slices in proportion to tensor_split (nullptr: equal shares)
ggml_backend_buffer_type_t ggml_backend_mi355x_split_buffer_type(int main_device, const float * tensor_split);
// row-split mat-muls executed, and slices of them computed on another GPU than the main device's
void ggml_backend_mi355x_split_stats(long * mm, long * foreign);
// measured HBM read ceiling of a device in GB/s (STREAM-style non-temporal read of 440 MB
// slices of a 4 GiB pool, best of three grids; llamacog_amd/csrc/k_stream.hip): the peak
// bench.py reports its roofline fractions against beside the 8 TB/s nominal.  -1 on failure.
double ggml_backend_mi355x_hbm_read_gbs(int device);

// ---- flat kernel ABI (llamacog_amd/csrc/capi.cpp) ---------------------------------------------
// Plain device pointers + sizes + a HIP stream (NULL = private stream, synchronised on
// return).  Each call builds the ggml node the reference graph would contain and runs the
// same launcher graph_compute runs.  Layouts are row-major, outermost index first.
void * mi355x_dev_alloc(size_t bytes);
void   mi355x_dev_free(void * p);
void   mi355x_h2d(void * dst, const void * src, size_t n);
void   mi355x_d2h(void * dst, const void * src, size_t n);
void   mi355x_memset(void * dst, int v, size_t n);
void   mi355x_sync(void);

// activation quantization (replaces ggml-cpu's from_float for the vec_dot_type,
// ggml-cpu/ggml-cpu.c:1254-1289): vdt = 15 (Q8_K) or 8 (Q8_0); output is SoA:
// qs[nrows][k] int8, d[nrows][k/blk] f32, s[nrows][k/16 (Q8_K) | k/32 (Q8_0)] int16
int mi355x_quantize_rows(int vdt, const float * x, int64_t k, int64_t nrows, void * qs, void * d, void * s, void * stream);
// MUL_MAT (ggml-cpu/ggml-cpu.c:1192-1384): y[T][M] = W[M][K] . X[T][K]
int mi355x_mul_mat(int wtype, const void * w, int64_t K, int64_t M, const float * x, int64_t T, float * y, void * stream);
// RMS_NORM (ops.cpp:3270-3316), optionally fused with the following MUL by w[ne0]
int mi355x_rms_norm(const float * x, int64_t ne0, int64_t nrows, float eps, const float * w, float * y, float * y_mul,
                    void * stream);
// ROPE (ops.cpp:5178-5362), x [n_tok][n_head][ne0]
int mi355x_rope(const float * x, int64_t ne0, int64_t n_head, int64_t n_tok, const int32_t * pos, int n_dims, int mode,
                int n_ctx_orig, float freq_base, float freq_scale, float ext_factor, float attn_factor, float beta_fast,
                float beta_slow, const float * ff, float * y, void * stream);
// SOFT_MAX (ops.cpp:4731-4827), x viewed as [nr/mask_rows][mask_rows][nc]
int mi355x_soft_max(const float * x, int64_t nc, int64_t nr, const float * mask, int64_t mask_rows, float scale, float * y,
                    void * stream);
// UNARY SILU (ops.cpp:2902, vec.cpp:233)
int mi355x_silu(const float * x, int64_t ne0, int64_t nrows, float * y, void * stream);
// MUL_MAT_ID (ggml-cpu/ggml-cpu.c:1466, the MoE expert mat-mul): as [n_as][M][K] rows of wtype,
// ids [T][ids_row] int32 (first n_used per token used), x [T][ne11][K] f32, y [T][n_used][M]
int mi355x_mul_mat_id(int wtype, const void * as, int64_t K, int64_t M, int64_t n_as, const int32_t * ids, int64_t ids_row,
                      int64_t n_used, const float * x, int64_t ne11, int64_t T, float * y, void * stream);
// ARGSORT (ops.cpp:6956-6993, ggml_top_k): order 0 ascending, 1 descending; out [nrows][ne0] int32
int mi355x_argsort(const float * x, int64_t ne0, int64_t nrows, int order, int32_t * out, void * stream);
// SUM_ROWS (ops.cpp:1956-1986): y [nrows]
int mi355x_sum_rows(const float * x, int64_t ne0, int64_t nrows, float * y, void * stream);
// FLASH_ATTN_EXT (ops.cpp:7015-7232): q [n_q][H][D] f32, k/v [n_kv][Hkv][D] f16 (1) or q8_0 (8),
// mask [n_q][n_kv] f16 or NULL, out [n_q][H][D]
// test hook: phase-1 scores of the CPU-exact flash attention (q [128] f32, k [n][128] f16)
int mi355x_fa_scores_d128(const float * q, const uint16_t * k, int64_t n, float * s, void * stream);
int mi355x_flash_attn(const float * q, const void * k, const void * v, const uint16_t * mask, int kv_type, int64_t D,
                      int64_t n_q, int64_t H, int64_t n_kv, int64_t Hkv, float scale, float softcap, float * out,
                      void * stream);

// microbenchmark hook: average device time (us) of one decode GEMV launch over nmat M x K
// matrices of type wtype sharing one activation row, weights rotating over `copies` copies
double mi355x_bench_gemv(int wtype, int64_t K, int64_t M, int nmat, int copies, int iters);
// microbenchmark hook: which = 0 decode flash attention (D 128, H 32, Hkv 8, a cache
// positions, b unmasked), 1 fused ADD+RMS_NORM+MUL+Q8_K of a floats; device us per launch
double mi355x_bench_op(int which, int64_t a, int64_t b, int iters);

#ifdef __cplusplus
}
#endif
