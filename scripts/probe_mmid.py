"""MUL_MAT_ID decode (2 of 8 experts, shared activation) vs the dense grouped GEMV on the same
shape, cold weights (mi355x_bench_gemv2 kind 6 vs kind 0)."""
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
for t, K, M, nm in [(13, 4096, 14336, 2), (13, 14336, 4096, 1), (12, 4096, 14336, 2)]:
    mb = K // 256 * BB[t] * M * nm
    dense = g(t, K, M, nm, max(2, -(-(1 << 30) // mb)), 30, 0)
    mid = g(t, K, M, nm, 4, 30, 6)
    print(f"type {t} K={K} M={M} x{nm}: dense {dense:7.2f} us ({mb / dense / 1e6:4.2f} TB/s)  mul_mat_id {mid:7.2f} us "
          f"({mb / mid / 1e6:4.2f} TB/s) [{os.environ.get('GGML_MI355X_MMID_PIPE', '1')}]", flush=True)
