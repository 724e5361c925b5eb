"""HBM streaming-read reference (k_stream_read) and the decode GEMV at several grid sizes."""
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
lib.mi355x_bench_op.restype = ctypes.c_double
lib.mi355x_bench_op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for mb in (2.4, 9.4, 14.2, 33.0, 48.2, 66.1, 431.0):
    nbytes = int(mb * 1e6) // 4096 * 4096
    copies = max(2, (1 << 30) // nbytes + 1)
    row = []
    for g in (4, 8, 16, 32, 64):
        us = lib.mi355x_bench_op(100 + g, nbytes, copies, 50)
        row.append(f"g{g * 64}:{us:7.2f}us {nbytes / us / 1e6:4.2f}TB/s")
    print(f"stream {mb:6.1f} MB  " + "  ".join(row), flush=True)
