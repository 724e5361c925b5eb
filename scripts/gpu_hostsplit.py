"""Host/device split of the decode step: time inside llama_decode vs llama_synchronize."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import llamacog_amd as la
from llamacog_amd import gguf_synth as gs

path = gs.ensure("llama3-8b-q4km")
m = la.Model(path, gpu=True, n_ctx=512, n_threads=16)
lib = m.lib
lib.llb_time_gen_split.restype = ctypes.c_double
lib.llb_time_gen_split.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
m.time_gen(8)
pl = la.plugin_lib()
pl.ggml_backend_mi355x_set_graph_timing(1)
pl.ggml_backend_mi355x_reset_timing()
for n in (64,):
    td, ts = ctypes.c_double(), ctypes.c_double()
    t = lib.llb_time_gen_split(m.h, n, ctypes.byref(td), ctypes.byref(ts))
    print(f"n={n} total {t / n * 1e3:.3f} ms/tok  decode-call {td.value / n * 1e3:.3f} ms  sync {ts.value / n * 1e3:.3f} ms")
print("graph stats", la.graph_stats())
for k, name in ((5, "device time per graph_compute"), (6, "host time in graph_compute")):
    ms, _, cnt = la.kernel_timing(pl, k)
    print(f"{name}: {ms / max(cnt, 1):.3f} ms x {cnt}")
