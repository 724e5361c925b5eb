"""ctypes view of oracle/build/liboracle.so — the CPU restatement (oracle/ggml_oracle.c).
Test infrastructure only (tests/, smoke, bench cpu_baseline may use it)."""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "oracle", "build", "liboracle.so")

F32, F16, Q4_0, Q8_0, Q4_K, Q5_K, Q6_K, Q8_K = 0, 1, 2, 8, 12, 13, 14, 15
BLK = {Q4_0: (32, 18), Q8_0: (32, 34), Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210), Q8_K: (256, 292),
       F16: (1, 2), F32: (1, 4)}
P = ctypes.c_void_p
I64 = ctypes.c_int64
_lib = None


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "build/liboracle.so"], check=True)
        L = ctypes.CDLL(LIB)
        L.orc_fp16_to_fp32.argtypes = [ctypes.c_uint16]
        L.orc_fp16_to_fp32.restype = ctypes.c_float
        L.orc_fp32_to_fp16.argtypes = [ctypes.c_float]
        L.orc_fp32_to_fp16.restype = ctypes.c_uint16
        L.orc_quantize_row_q8_K.argtypes = [P, P, I64]
        L.orc_quantize_row_q8_0.argtypes = [P, P, I64]
        L.orc_quantize_row_q4_0.argtypes = [P, P, I64]
        L.orc_dequantize_row.argtypes = [ctypes.c_int, P, P, I64]
        L.orc_vec_dot.argtypes = [ctypes.c_int, I64, P, P, P, P]
        L.orc_vec_dot.restype = ctypes.c_float
        L.orc_mul_mat.argtypes = [ctypes.c_int, P, I64, I64, P, I64, P]
        L.orc_rms_norm.argtypes = [P, I64, I64, ctypes.c_float, P]
        L.orc_rope.argtypes = [P, I64, I64, I64, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                               ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, P, P]
        L.orc_soft_max.argtypes = [P, I64, I64, P, I64, ctypes.c_float, P]
        L.orc_flash_attn.argtypes = [P, P, P, P, ctypes.c_int, I64, I64, I64, I64, I64, ctypes.c_float, ctypes.c_float, P]
        L.orc_mul_mat_id.argtypes = [ctypes.c_int, P, I64, I64, I64, P, I64, I64, P, I64, I64, P]
        L.orc_argsort.argtypes = [P, I64, I64, ctypes.c_int, P]
        L.orc_sum_rows.argtypes = [P, I64, I64, P]
        L.orc_mul_mat_cpu.argtypes = [ctypes.c_int, P, I64, I64, P, I64, P, ctypes.c_int]
        L.orc_block_classes.argtypes = [ctypes.c_int, P, P, P, P]
        L.orc_mul_mat_id_cpu.argtypes = [ctypes.c_int, P, I64, I64, I64, P, I64, I64, P, I64, I64, P, ctypes.c_int]
        _lib = L
    return _lib


def nbytes(t, n):
    b, s = BLK[t]
    return n // b * s


def quantize_rows(t, x):
    """Q8_K / Q8_0 / Q4_0 quantization of each row (CPU from_float semantics)."""
    assert t in (Q8_K, Q8_0, Q4_0), t
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.zeros((x.shape[0], nbytes(t, x.shape[1])), dtype=np.uint8)
    f = {Q8_K: lib().orc_quantize_row_q8_K, Q8_0: lib().orc_quantize_row_q8_0, Q4_0: lib().orc_quantize_row_q4_0}[t]
    for r in range(x.shape[0]):
        f(ptr(x[r]), ptr(out[r]), x.shape[1])
    return out


def dequantize_rows(t, q, k):
    out = np.zeros((q.shape[0], k), dtype=np.float32)
    for r in range(q.shape[0]):
        lib().orc_dequantize_row(t, ptr(np.ascontiguousarray(q[r])), ptr(out[r]), k)
    return out


def vec_dot(t, k, wrow, arow):
    nb = k // BLK[t][0]
    isum = np.zeros(nb, dtype=np.int32)
    msum = np.zeros(nb, dtype=np.int32)
    v = lib().orc_vec_dot(t, k, ptr(np.ascontiguousarray(wrow)), ptr(np.ascontiguousarray(arow)), ptr(isum), ptr(msum))
    return v, isum, msum


def mul_mat(t, wq, K, M, x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros((x.shape[0], M), dtype=np.float32)
    lib().orc_mul_mat(t, ptr(np.ascontiguousarray(wq)), K, M, ptr(x), x.shape[0], ptr(y))
    return y


def mul_mat_cpu(t, wq, K, M, x, repack=True):
    """mul_mat in the CPU backend's exact float order as libllama runs it (orc_mul_mat_cpu):
    Q4_K / Q4_0 weights repacked (rows % 8), the vec_dot / tinyBLAS orders otherwise."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros((x.shape[0], M), dtype=np.float32)
    lib().orc_mul_mat_cpu(t, ptr(np.ascontiguousarray(wq)), K, M, ptr(x), x.shape[0], ptr(y), 1 if repack else 0)
    return y


def rms_norm(x, eps):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros_like(x)
    lib().orc_rms_norm(ptr(x), x.shape[1], x.shape[0], eps, ptr(y))
    return y


def rope(x, pos, n_dims, mode, base, ff=None, n_ctx_orig=8192, freq_scale=1.0, ext_factor=0.0, attn_factor=1.0,
         beta_fast=32.0, beta_slow=1.0):
    x = np.ascontiguousarray(x, dtype=np.float32)
    ntok, nh, ne0 = x.shape
    y = np.zeros_like(x)
    lib().orc_rope(ptr(x), ne0, nh, ntok, ptr(np.ascontiguousarray(pos, dtype=np.int32)), n_dims, mode, n_ctx_orig,
                   base, freq_scale, ext_factor, attn_factor, beta_fast, beta_slow,
                   ptr(np.ascontiguousarray(ff, dtype=np.float32)) if ff is not None else None, ptr(y))
    return y


def soft_max(x, mask, scale):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros_like(x)
    m = np.ascontiguousarray(mask, dtype=np.float32) if mask is not None else None
    lib().orc_soft_max(ptr(x), x.shape[1], x.shape[0], ptr(m), m.shape[0] if m is not None else 1, scale, ptr(y))
    return y


def flash_attn(q, k, v, mask_u16, kv_type, D, H, Hkv, n_kv, scale, softcap=0.0):
    q = np.ascontiguousarray(q, dtype=np.float32)
    n_q = q.shape[0]
    out = np.zeros((n_q, H, D), dtype=np.float32)
    lib().orc_flash_attn(ptr(q), ptr(np.ascontiguousarray(k)), ptr(np.ascontiguousarray(v)),
                         ptr(np.ascontiguousarray(mask_u16)) if mask_u16 is not None else None, kv_type, D, n_q, H,
                         n_kv, Hkv, scale, softcap, ptr(out))
    return out


def silu(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros_like(x)
    L = lib()
    L.orc_silu.argtypes = [P, I64, P]
    for r in range(x.reshape(-1, x.shape[-1]).shape[0]):
        xr = x.reshape(-1, x.shape[-1])[r]
        yr = np.zeros_like(xr)
        L.orc_silu(ptr(np.ascontiguousarray(xr)), xr.size, ptr(yr))
        y.reshape(-1, x.shape[-1])[r] = yr
    return y


def v_expf(x):
    L = lib()
    L.orc_v_expf.argtypes = [ctypes.c_float]
    L.orc_v_expf.restype = ctypes.c_float
    return np.array([L.orc_v_expf(float(v)) for v in np.ravel(x)], dtype=np.float32).reshape(np.shape(x))


def split_q8(t, blocks, k):
    """AoS Q8_K / Q8_0 blocks (ggml-common.h) -> the plugin's SoA (qs, d, sums)."""
    n = blocks.shape[0]
    if t == Q8_K:
        b = blocks.reshape(n, k // 256, 292)
        d = b[:, :, 0:4].copy().view(np.float32).reshape(n, k // 256)
        qs = b[:, :, 4:260].copy().view(np.int8).reshape(n, k)
        s = b[:, :, 260:292].copy().view(np.int16).reshape(n, k // 16)
        return qs, d, s
    b = blocks.reshape(n, k // 32, 34)
    d16 = b[:, :, 0:2].copy().view(np.float16).reshape(n, k // 32)
    qs = b[:, :, 2:34].copy().view(np.int8).reshape(n, k)
    s = qs.reshape(n, k // 32, 32).astype(np.int32).sum(axis=2).astype(np.int16)
    return qs, d16.astype(np.float32), s


def mul_mat_id(t, wq, K, M, n_as, ids, n_used, x):
    """MUL_MAT_ID: wq [n_as*M] rows, ids [T][ids_row] (first n_used used), x [T][ne11][K] -> [T][n_used][M]."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    T, ne11 = x.shape[0], x.shape[1]
    y = np.zeros((T, n_used, M), dtype=np.float32)
    lib().orc_mul_mat_id(t, ptr(np.ascontiguousarray(wq)), K, M, n_as, ptr(ids), ids.shape[1], n_used, ptr(x), ne11, T,
                         ptr(y))
    return y


def mul_mat_id_cpu(t, wq, K, M, n_as, ids, n_used, x, repack=True):
    """MUL_MAT_ID in the CPU backend's exact float order as libllama runs it (orc_mul_mat_id_cpu)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    T, ne11 = x.shape[0], x.shape[1]
    y = np.zeros((T, n_used, M), dtype=np.float32)
    lib().orc_mul_mat_id_cpu(t, ptr(np.ascontiguousarray(wq)), K, M, n_as, ptr(ids), ids.shape[1], n_used, ptr(x), ne11,
                             T, ptr(y), 1 if repack else 0)
    return y


def argsort(x, order):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.zeros(x.shape, dtype=np.int32)
    lib().orc_argsort(ptr(x), x.shape[1], x.shape[0], order, ptr(out))
    return out


def sum_rows(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    y = np.zeros(x.shape[0], dtype=np.float32)
    lib().orc_sum_rows(ptr(x), x.shape[1], x.shape[0], ptr(y))
    return y
