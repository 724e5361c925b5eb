"""Decode GEMV per weight type on the Mixtral / Llama FFN shapes, cold weights (mi355x_bench_gemv2)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

BB = {12: 144, 13: 176, 14: 210}
NM = {12: "q4_K", 13: "q5_K", 14: "q6_K"}
lib = la.plugin_lib()
g = lib.mi355x_bench_gemv2
g.restype = ctypes.c_double
g.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
for t, K, M, nm in [(12, 4096, 14336, 2), (13, 4096, 14336, 2), (12, 14336, 4096, 1), (13, 14336, 4096, 1), (14, 14336, 4096, 1)]:
    mb = K // 256 * BB[t] * M * nm
    us = g(t, K, M, nm, max(2, -(-(1 << 30) // mb)), 50, 0)
    print(f"{NM[t]} K={K} M={M} x{nm}: {mb / 1e6:6.1f} MB {us:7.2f} us {mb / us / 1e6:5.2f} TB/s", flush=True)
