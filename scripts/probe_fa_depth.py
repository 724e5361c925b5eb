"""Phase split of the CPU-exact decode flash attention at depth (mi355x_bench_op 2: s_memtime
ticks of workgroup 0 per phase, to stderr), 32 query heads over 8 KV heads, D = 128.
Arguments: n_kv:valid pairs (a cache of n_kv positions, the first `valid` unmasked)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
op = lib.mi355x_bench_op
op.restype = ctypes.c_double
op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for arg in (sys.argv[1:] or ["256:16", "256:136", "1024:1024", "4096:4096"]):
    n, v = (int(x) for x in arg.split(":")) if ":" in arg else (int(arg), int(arg))
    t0 = op(0, n, v, 50)
    print(f"fa n_kv={n} valid={v}: {t0:.2f} us (plain)", flush=True)
    print(f"fa n_kv={n} valid={v}: {op(2, n, v, 10):.2f} us (phase counters)", flush=True)
