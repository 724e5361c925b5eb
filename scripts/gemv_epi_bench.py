"""Decode GEMV cost of each fused epilogue / prologue kind (capi mi355x_bench_gemv2), on the
Llama-3-8B Q4_K_M shapes, back-to-back launches over cold weights."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

Q4_K, Q6_K = 12, 14
BB = {Q4_K: 144, Q6_K: 210}
KINDS = ["plain", "silu", "f16", "rope+f16", "pro-norm", "pro-mul"]
lib = la.plugin_lib()
f = lib.mi355x_bench_gemv2
f.restype = ctypes.c_double
f.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
shapes = [("Wq", Q4_K, 4096, 4096, 1, [0, 2, 3, 4]), ("Wk", Q4_K, 4096, 1024, 1, [0, 3]),
          ("gate+up", Q4_K, 4096, 14336, 2, [0, 1, 4]), ("down q4K", Q4_K, 14336, 4096, 1, [0, 5]),
          ("down q6K", Q6_K, 14336, 4096, 1, [0, 5]), ("Wv q6K", Q6_K, 4096, 1024, 1, [0, 2])]
for name, t, K, M, nm, kinds in shapes:
    mb = K // 256 * BB[t] * M * nm
    copies = max(2, -(-(1 << 30) // mb))
    for k in kinds:
        us = f(t, K, M, nm, copies, 50, k)
        print(f"{name:9s} K={K:6d} M={M:6d} x{nm} {KINDS[k]:9s} {mb / 1e6:7.1f} MB {us:8.2f} us {mb / us / 1e6:5.2f} TB/s", flush=True)
