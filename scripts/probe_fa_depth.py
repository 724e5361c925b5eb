"""Phase split of the CPU-exact decode flash attention at depth (mi355x_bench_op 2: s_memtime
ticks of workgroup 0 per phase, to stderr), 32 query heads over 8 KV heads, D = 128."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
op = lib.mi355x_bench_op
op.restype = ctypes.c_double
op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for n in [int(x) for x in (sys.argv[1:] or ["136", "1024", "4096"])]:
    print(f"fa n_kv={n} valid={n}: {op(2, n, n, 10):.2f} us", flush=True)
