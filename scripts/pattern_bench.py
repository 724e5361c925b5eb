"""GEMV access pattern vs contiguous reads vs the GEMV itself (q4_K rows, K = 4096)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
lib.mi355x_bench_op.restype = ctypes.c_double
lib.mi355x_bench_op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
lib.mi355x_bench_gemv.restype = ctypes.c_double
lib.mi355x_bench_gemv.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
for M in (4096, 14336, 28672, 128256):
    nbytes = M * 2304
    copies = max(2, (1 << 30) // nbytes + 1)
    t0 = lib.mi355x_bench_op(200, nbytes, copies, 50)
    t1 = lib.mi355x_bench_op(201, nbytes, copies, 50)
    ts = lib.mi355x_bench_op(164, nbytes, copies, 50)
    tg = lib.mi355x_bench_gemv(12, 4096, M, 1, copies, 50)
    print(f"M={M:6d} {nbytes / 1e6:6.1f} MB  gemv-pattern {t0:7.2f}us {nbytes / t0 / 1e6:4.2f}TB/s  "
          f"contig-rows {t1:7.2f}us {nbytes / t1 / 1e6:4.2f}TB/s  stream {ts:7.2f}us {nbytes / ts / 1e6:4.2f}TB/s  "
          f"gemv {tg:7.2f}us {nbytes / tg / 1e6:4.2f}TB/s", flush=True)
