"""Decode GEMV geometry on the Llama-3-8B FFN shapes (cold weights, mi355x_bench_gemv2 kind 0):
one launch per shape, timed with HIP events; under `rocprofv3 --pmc FETCH_SIZE` it is the
traffic calibration run (scripts/pmc_calib.py)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

BB = {12: 144, 13: 176, 14: 210}
lib = la.plugin_lib()
g = lib.mi355x_bench_gemv2
g.restype = ctypes.c_double
g.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
tag = " ".join(f"{k[13:]}={v}" for k, v in os.environ.items() if k.startswith("GGML_MI355X_GEMV") or k.startswith("GGML_MI355X_OS")) or "default"
out = []
for t, K, M, nm in [(12, 14336, 4096, 1), (14, 14336, 4096, 1), (12, 4096, 14336, 2), (12, 4096, 28672, 1), (12, 4096, 4096, 1), (12, 4096, 6144, 1), (14, 4096, 128256, 1)]:
    mb = K // 256 * BB[t] * M * nm
    cp = max(2, -(-(1 << 30) // mb))
    a = g(t, K, M, nm, cp, 40, 0)
    out.append(f"t{t} {K}x{M}x{nm} {a:6.2f}us {mb / a / 1e6:4.2f}TB/s")
print(f"[{tag}] " + " | ".join(out), flush=True)
