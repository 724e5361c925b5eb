"""Phase split of the decode flash attention (mi355x_bench_op 2: s_memtime cycles of workgroup 0
from the start to each phase's end, to stderr) at fill levels of a 256-cell cache: the
short-context kernel k_fattn_dsh, and with GGML_MI355X_FA_DSH=0 k_fattn_dec2."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
op = lib.mi355x_bench_op
op.restype = ctypes.c_double
op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for n in (16, 72, 136, 256):
    print(f"fa n_kv=256 valid={n}: {op(2, 256, n, 30):.2f} us", flush=True)
