"""Dense decode GEMV paths on the FFN shapes, cold weights: the pipelined grouped GEMV (kind 0)
vs the general one-row-per-wave mat-vec k_mmv_q (kind 7).  Run with GGML_MI355X_GEMV_PIPE=0 to
see the one-shot grouped kernel instead of the pipelined one."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

BB = {12: 144, 13: 176, 14: 210}
lib = la.plugin_lib()
g = lib.mi355x_bench_gemv2
g.restype = ctypes.c_double
g.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
tag = os.environ.get("GGML_MI355X_GEMV_PIPE", "1")
for t, K, M in [(12, 14336, 4096), (14, 14336, 4096), (12, 4096, 4096), (12, 4096, 14336), (14, 4096, 128256)]:
    mb = K // 256 * BB[t] * M
    cp = max(2, -(-(1 << 30) // mb))
    a = g(t, K, M, 1, cp, 30, 0)
    b = g(t, K, M, 1, cp, 30, 7)
    print(f"[pipe={tag}] type {t} K={K} M={M}: grouped {a:7.2f} us ({mb / a / 1e6:4.2f} TB/s)  k_mmv_q {b:7.2f} us "
          f"({mb / b / 1e6:4.2f} TB/s)", flush=True)
