"""ctypes binding of the plugin's flat kernel ABI (include/ggml-mi355x.h, csrc/capi.cpp).

Host numpy arrays in, host numpy arrays out; device buffers come from the plugin's own
mi355x_dev_alloc (no other HIP binding needed).  Every function fails loudly when the
plugin is missing or no MI355X is visible — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import plugin_lib, BackendMissing

P = ctypes.c_void_p
I64 = ctypes.c_int64
F = ctypes.c_float

_lib = None

Q8_K, Q8_0, F16, F32 = 15, 8, 1, 0


def lib():
    global _lib
    if _lib is None:
        L = plugin_lib()
        if L.ggml_backend_mi355x_get_device_count() <= 0:
            raise BackendMissing("no MI355X visible to the plugin")
        L.mi355x_dev_alloc.restype = P
        L.mi355x_dev_alloc.argtypes = [ctypes.c_size_t]
        L.mi355x_dev_free.argtypes = [P]
        L.mi355x_h2d.argtypes = [P, P, ctypes.c_size_t]
        L.mi355x_d2h.argtypes = [P, P, ctypes.c_size_t]
        L.mi355x_memset.argtypes = [P, ctypes.c_int, ctypes.c_size_t]
        L.mi355x_quantize_rows.argtypes = [ctypes.c_int, P, I64, I64, P, P, P, P]
        L.mi355x_mul_mat.argtypes = [ctypes.c_int, P, I64, I64, P, I64, P, P]
        L.mi355x_rms_norm.argtypes = [P, I64, I64, F, P, P, P, P]
        L.mi355x_rope.argtypes = [P, I64, I64, I64, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, F, F, F, F, F, F, P, P, P]
        L.mi355x_soft_max.argtypes = [P, I64, I64, P, I64, F, P, P]
        L.mi355x_silu.argtypes = [P, I64, I64, P, P]
        L.mi355x_flash_attn.argtypes = [P, P, P, P, ctypes.c_int, I64, I64, I64, I64, I64, F, F, P, P]
        L.mi355x_mul_mat_id.argtypes = [ctypes.c_int, P, I64, I64, I64, P, I64, I64, P, I64, I64, P, P]
        L.mi355x_argsort.argtypes = [P, I64, I64, ctypes.c_int, P, P]
        L.mi355x_sum_rows.argtypes = [P, I64, I64, P, P]
        _lib = L
    return _lib


class Dev:
    """A device buffer holding a copy of a host array (or an uninitialised one)."""

    def __init__(self, arr: np.ndarray | None = None, nbytes: int | None = None, fill: int | None = 0xFF):
        L = lib()
        self.nbytes = arr.nbytes if arr is not None else int(nbytes)
        self.ptr = L.mi355x_dev_alloc(max(self.nbytes, 1))
        if not self.ptr:
            raise MemoryError(f"mi355x_dev_alloc({self.nbytes})")
        if arr is not None:
            a = np.ascontiguousarray(arr)
            L.mi355x_h2d(self.ptr, a.ctypes.data_as(P), self.nbytes)
        elif fill is not None:
            L.mi355x_memset(self.ptr, fill, self.nbytes)  # poison: unwritten outputs show up

    def get(self, dtype, shape) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        assert out.nbytes <= self.nbytes
        lib().mi355x_d2h(out.ctypes.data_as(P), self.ptr, out.nbytes)
        return out

    def free(self):
        if self.ptr:
            lib().mi355x_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _chk(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} returned {rc} (unsupported shape/type)")


def quantize_rows(vdt: int, x: np.ndarray):
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, k = x.shape
    blk, grp = (256, 16) if vdt == Q8_K else (32, 32)
    dx = Dev(x)
    qs, d, s = Dev(nbytes=n * k), Dev(nbytes=n * (k // blk) * 4), Dev(nbytes=n * (k // grp) * 2)
    _chk(lib().mi355x_quantize_rows(vdt, dx.ptr, k, n, qs.ptr, d.ptr, s.ptr, None), "quantize_rows")
    return qs.get(np.int8, (n, k)), d.get(np.float32, (n, k // blk)), s.get(np.int16, (n, k // grp))


def mul_mat(wtype: int, wq: np.ndarray, K: int, M: int, x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    T = x.shape[0]
    dw, dx, dy = Dev(wq), Dev(x), Dev(nbytes=T * M * 4)
    _chk(lib().mi355x_mul_mat(wtype, dw.ptr, K, M, dx.ptr, T, dy.ptr, None), "mul_mat")
    return dy.get(np.float32, (T, M))


def rms_norm(x: np.ndarray, eps: float, w: np.ndarray | None = None):
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, ne0 = x.shape
    dx, dy = Dev(x), Dev(nbytes=x.nbytes)
    dw = Dev(np.ascontiguousarray(w, dtype=np.float32)) if w is not None else None
    dm = Dev(nbytes=x.nbytes) if w is not None else None
    _chk(lib().mi355x_rms_norm(dx.ptr, ne0, n, eps, dw.ptr if dw else None, dy.ptr, dm.ptr if dm else None, None),
         "rms_norm")
    y = dy.get(np.float32, x.shape)
    return (y, dm.get(np.float32, x.shape)) if w is not None else y


def rope(x, pos, n_dims, mode, base, ff=None, n_ctx_orig=8192, freq_scale=1.0, ext_factor=0.0, attn_factor=1.0,
         beta_fast=32.0, beta_slow=1.0):
    x = np.ascontiguousarray(x, dtype=np.float32)
    ntok, nh, ne0 = x.shape
    dx, dp, dy = Dev(x), Dev(np.ascontiguousarray(pos, dtype=np.int32)), Dev(nbytes=x.nbytes)
    df = Dev(np.ascontiguousarray(ff, dtype=np.float32)) if ff is not None else None
    _chk(lib().mi355x_rope(dx.ptr, ne0, nh, ntok, dp.ptr, n_dims, mode, n_ctx_orig, base, freq_scale, ext_factor,
                           attn_factor, beta_fast, beta_slow, df.ptr if df else None, dy.ptr, None), "rope")
    return dy.get(np.float32, x.shape)


def soft_max(x, mask, scale):
    x = np.ascontiguousarray(x, dtype=np.float32)
    nr, nc = x.shape
    dx, dy = Dev(x), Dev(nbytes=x.nbytes)
    dm = Dev(np.ascontiguousarray(mask, dtype=np.float32)) if mask is not None else None
    _chk(lib().mi355x_soft_max(dx.ptr, nc, nr, dm.ptr if dm else None, mask.shape[0] if mask is not None else 1, scale,
                               dy.ptr, None), "soft_max")
    return dy.get(np.float32, x.shape)


def silu(x):
    x = np.ascontiguousarray(x, dtype=np.float32)
    x2 = x.reshape(-1, x.shape[-1])
    dx, dy = Dev(x2), Dev(nbytes=x2.nbytes)
    _chk(lib().mi355x_silu(dx.ptr, x2.shape[1], x2.shape[0], dy.ptr, None), "silu")
    return dy.get(np.float32, x.shape)


def flash_attn(q, k, v, mask_u16, kv_type, D, H, Hkv, n_kv, scale, softcap=0.0):
    q = np.ascontiguousarray(q, dtype=np.float32)
    n_q = q.shape[0]
    dq, dk, dv, do = Dev(q), Dev(np.ascontiguousarray(k)), Dev(np.ascontiguousarray(v)), Dev(nbytes=n_q * H * D * 4)
    dm = Dev(np.ascontiguousarray(mask_u16, dtype=np.uint16)) if mask_u16 is not None else None
    _chk(lib().mi355x_flash_attn(dq.ptr, dk.ptr, dv.ptr, dm.ptr if dm else None, kv_type, D, n_q, H, n_kv, Hkv, scale,
                                 softcap, do.ptr, None), "flash_attn")
    return do.get(np.float32, (n_q, H, D))


def mul_mat_id(wtype: int, wq: np.ndarray, K: int, M: int, n_as: int, ids: np.ndarray, n_used: int, x: np.ndarray):
    """MUL_MAT_ID: wq [n_as*M][row bytes], ids [T][ids_row] int32 (first n_used used), x [T][ne11][K].
    Returns y [T][n_used][M]."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    T, ne11 = x.shape[0], x.shape[1]
    dw, di, dx, dy = Dev(wq), Dev(ids), Dev(x), Dev(nbytes=T * n_used * M * 4)
    _chk(lib().mi355x_mul_mat_id(wtype, dw.ptr, K, M, n_as, di.ptr, ids.shape[1], n_used, dx.ptr, ne11, T, dy.ptr, None),
         "mul_mat_id")
    return dy.get(np.float32, (T, n_used, M))


def argsort(x: np.ndarray, order: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, ne0 = x.shape
    dx, do = Dev(x), Dev(nbytes=x.nbytes)
    _chk(lib().mi355x_argsort(dx.ptr, ne0, n, order, do.ptr, None), "argsort")
    return do.get(np.int32, x.shape)


def sum_rows(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    n, ne0 = x.shape
    dx, dy = Dev(x), Dev(nbytes=n * 4)
    _chk(lib().mi355x_sum_rows(dx.ptr, ne0, n, dy.ptr, None), "sum_rows")
    return dy.get(np.float32, (n,))
