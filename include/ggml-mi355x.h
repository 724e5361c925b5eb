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

#ifdef __cplusplus
}
#endif
