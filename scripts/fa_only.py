"""One flash-attention microbenchmark configuration (for counter collection)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
lib.mi355x_bench_op.restype = ctypes.c_double
lib.mi355x_bench_op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
print(f"FA exact n_kv={n} valid={n - 24}: {lib.mi355x_bench_op(0, n, n - 24, 20):.2f} us")
