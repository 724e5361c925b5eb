"""Decode-GEMV weight access pattern vs contiguous reads, no arithmetic (capi.cpp k_pattern_read):
MODE 0 = the q4_K task pattern (header + two 16-B quant chunks per lane per row), MODE 1 = the same
bytes as contiguous 16-B chunks; k_stream_read for reference.  GB/s per launch size."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

lib = la.plugin_lib()
op = lib.mi355x_bench_op
op.restype = ctypes.c_double
op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
for mb in (9.4, 33.0, 66.0, 432.0):
    nb = int(mb * 1e6) // 2304 * 2304
    t0 = op(200, nb, 4, 20)
    t1 = op(201, nb, 4, 20)
    ts = op(100 + 32, nb // 16 * 16, 4, 20)
    print(f"{mb:6.1f} MB: task pattern {t0:8.2f} us {nb / t0 / 1e3:7.0f} GB/s | contiguous {t1:8.2f} us {nb / t1 / 1e3:7.0f} GB/s | stream(2048 wg) {ts:8.2f} us {nb / ts / 1e3:7.0f} GB/s", flush=True)
