"""Decode GEMV microbenchmark (k_gemv.hip) on the Llama-3-8B Q4_K_M shapes: device time per
launch and effective HBM bandwidth (weights rotate over > 1 GB so no launch hits the MALL)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la

Q4_K, Q6_K, Q8_0, Q4_0, Q5_K = 12, 14, 8, 2, 13
BLK = {Q4_K: (256, 144), Q6_K: (256, 210), Q8_0: (32, 34), Q4_0: (32, 18), Q5_K: (256, 176)}
lib = la.plugin_lib()
lib.mi355x_bench_gemv.restype = ctypes.c_double
lib.mi355x_bench_gemv.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int]
shapes = [("Wq q4_K", Q4_K, 4096, 4096, 1), ("Wk q4_K", Q4_K, 4096, 1024, 1), ("Wv q6_K", Q6_K, 4096, 1024, 1),
          ("gate+up q4_K x2", Q4_K, 4096, 14336, 2), ("gate q4_K", Q4_K, 4096, 14336, 1),
          ("down q6_K", Q6_K, 14336, 4096, 1), ("down q4_K", Q4_K, 14336, 4096, 1), ("output q6_K", Q6_K, 4096, 128256, 1),
          ("Wq q8_0", Q8_0, 4096, 4096, 1), ("gate q8_0", Q8_0, 4096, 14336, 1)]
for name, t, K, M, nm in shapes:
    blk, bs = BLK[t]
    mb = K // blk * bs * M * nm
    copies = max(2, -(-(1 << 30) // mb))
    us = lib.mi355x_bench_gemv(t, K, M, nm, copies, 50)
    print(f"{name:18s} K={K:6d} M={M:6d} x{nm}  {mb / 1e6:7.1f} MB  {us:8.2f} us  {mb / us / 1e6:5.2f} TB/s")
