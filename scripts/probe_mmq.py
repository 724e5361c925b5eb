"""Prefill MUL_MAT kernel time on the Llama-3-8B shapes (mi355x_bench_op 300 = Q4_K, 301 = Q6_K;
K = 4096, M rows, T tokens), with the environment's GGML_MI355X_MMQ_* knobs."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
f = lib.mi355x_bench_op
f.restype = ctypes.c_double
f.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
tag = " ".join(f"{k[12:]}={v}" for k, v in os.environ.items() if k.startswith("GGML_MI355X_MMQ")) or "default"
out = []
for w, M, T in [(300, 4096, 512), (300, 14336, 512), (300, 1024, 512), (301, 4096, 512)]:
    us = f(w, M, T, 20)
    out.append(f"{'q4K' if w == 300 else 'q6K'} M{M} T{T} {us:7.1f}us {2 * 4096 * M * T / us / 1e6:6.1f}TF")
print(f"[{tag}] " + " | ".join(out), flush=True)
