"""Decode GEMV from HBM vs from the Infinity Cache: the one-shot kernel on the Llama-3-8B FFN /
attention shapes, back-to-back launches over rotating copies larger than the 256 MiB cache
(cold: every byte from HBM) and over ONE copy (warm: a layer's matrices fit the cache, every
byte from it after the first launch).  Decides whether prefetching a layer's FFN weights into the
cache during attention (when HBM is idle) can shorten the FFN mat-vecs.
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

Q4_K, Q6_K = 12, 14
BB = {Q4_K: (144, 256), Q6_K: (210, 256)}
SHAPES = [("O-proj q4K", Q4_K, 4096, 4096, 1), ("QK q4K", Q4_K, 4096, 5120, 1), ("gate+up q4K", Q4_K, 4096, 14336, 2),
          ("down q4K", Q4_K, 14336, 4096, 1), ("down q6K", Q6_K, 14336, 4096, 1), ("head q6K", Q6_K, 4096, 128256, 1)]


def main():
    import llamacog_amd as la
    g = la.plugin_lib().mi355x_bench_gemv2
    g.restype = ctypes.c_double
    g.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    for name, t, K, M, nm in SHAPES:
        bb, qk = BB[t]
        mb = K // qk * bb * M * nm
        cold = g(t, K, M, nm, max(2, -(-(3 << 30) // mb)), 40, 0)
        warm = g(t, K, M, nm, 1, 40, 0)
        print(f"{name:14s} {mb / 1e6:7.1f} MB  cold {cold:7.2f} us {mb / cold / 1e6:5.2f} TB/s   "
              f"cache {warm:7.2f} us {mb / warm / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
