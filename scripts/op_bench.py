"""Microbenchmarks of the decode-step small ops (flash attention, fused norm) on MI355X."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
lib.mi355x_bench_op.restype = ctypes.c_double
lib.mi355x_bench_op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for n_kv, nv in ((256, 1), (256, 40), (256, 256), (512, 300), (1024, 1000), (4096, 4000)):
    print(f"FA exact  n_kv={n_kv:5d} valid={nv:5d}  {lib.mi355x_bench_op(0, n_kv, nv, 200):8.2f} us")
for n in (4096, 8192):
    print(f"norm fused ne0={n}  {lib.mi355x_bench_op(1, n, 0, 500):8.2f} us")
