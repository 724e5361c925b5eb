"""Decode microbenchmarks on MI355X (capi hooks): the decode GEMV with its weights cold
(rotating copies > Infinity Cache) vs Infinity-Cache resident (one copy), the CPU-exact flash
attention's phase split at three fill levels of a 256-cell cache, the fused norm, and the
streaming-read reference cold vs resident."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

Q4_K, Q6_K = 12, 14
BB = {Q4_K: 144, Q6_K: 210}
lib = la.plugin_lib()
g = lib.mi355x_bench_gemv2
g.restype = ctypes.c_double
g.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
op = lib.mi355x_bench_op
op.restype = ctypes.c_double
op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for name, t, K, M, nm, epi in [("Wo", Q4_K, 4096, 4096, 1, 0), ("Wq rope", Q4_K, 4096, 4096, 1, 3),
                               ("gate+up", Q4_K, 4096, 14336, 2, 0), ("gate+up silu", Q4_K, 4096, 14336, 2, 1),
                               ("down q4K", Q4_K, 14336, 4096, 1, 0), ("down q6K", Q6_K, 14336, 4096, 1, 0)]:
    mb = K // 256 * BB[t] * M * nm
    cold = g(t, K, M, nm, max(2, -(-(1 << 30) // mb)), 50, epi)
    warm = g(t, K, M, nm, 1, 50, epi)
    print(f"{name:13s} {mb / 1e6:6.1f} MB cold {cold:7.2f} us {mb / cold / 1e6:5.2f} TB/s | resident {warm:7.2f} us "
          f"{mb / warm / 1e6:5.2f} TB/s", flush=True)
for n in (16, 136, 256):
    us = op(2, 256, n, 30)   # FA phase split goes to stderr
    print(f"fa n_kv=256 valid={n}: {us:.2f} us", flush=True)
print(f"fused add+norm+mul+q8K 4096: {op(1, 4096, 0, 50):.2f} us", flush=True)
for copies in (16, 1):
    for grid in (16, 32, 64):
        us = op(100 + grid, 64 << 20, copies, 20)
        print(f"stream read 64 MiB copies={copies} grid={grid * 64}: {us:.2f} us {64 * 1.048576 / us:.2f} TB/s", flush=True)
