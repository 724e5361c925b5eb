"""Prefill flash-attention kernel time (mi355x_bench_op 302: D 128, 32/8 heads, causal, random
data) for a few prompt lengths; the second pass prints the per-phase cycles of workgroup (0, 0)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
f = lib.mi355x_bench_op
f.restype = ctypes.c_double
f.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
tag = " ".join(f"{k[12:]}={v}" for k, v in os.environ.items() if k.startswith("GGML_MI355X_FA") or k.startswith("GGML_MI355X_PF")) or "default"
out = [f"n{n} {f(302, n, 0, 10):7.1f}us" for n in (128, 512, 2048)]
print(f"[{tag}] " + " | ".join(out), flush=True)
f(302, 512, 1, 3)
