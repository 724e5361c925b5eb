"""Phase split of the CPU-exact decode flash attention (mi355x_bench_op 2, s_memtime cycles of
workgroup 0 to stderr) at three fill levels of a 256-cell cache, plus the fused norm."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
op = lib.mi355x_bench_op
op.restype = ctypes.c_double
op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for n in (16, 136, 256):
    print(f"fa n_kv=256 valid={n}: {op(2, 256, n, 30):.2f} us", flush=True)
print(f"fused add+norm+mul+q8K 4096: {op(1, 4096, 0, 50):.2f} us", flush=True)
