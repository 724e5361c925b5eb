"""Per-phase cycle breakdown of the CPU-exact flash-attention kernel (s_memtime, wg 0)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
lib.mi355x_bench_op.restype = ctypes.c_double
lib.mi355x_bench_op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for n_kv, nv in ((256, 1), (256, 64), (256, 256), (1024, 1000), (4096, 4000)):
    t = lib.mi355x_bench_op(2, n_kv, nv, 50)
    print(f"FA exact  n_kv={n_kv:5d} valid={nv:5d}  {t:8.2f} us", flush=True)
