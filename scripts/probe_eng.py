"""Decode GEMV microbenchmark: the persistent loader/consumer engine (k_gemv_eng) against the
one-shot kernel (k_gemv_os) on the Llama-3-8B / 70B decode shapes, weights cold (rotating copies
larger than the Infinity Cache), back-to-back launches (capi mi355x_bench_gemv2).

Each configuration runs in its own process (the plugin reads its switches once):
  python scripts/probe_eng.py            -> table of every variant
  python scripts/probe_eng.py --child    -> one variant, from the environment
"""
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

Q4_K, Q6_K, Q8_0 = 12, 14, 8
BB = {Q4_K: (144, 256), Q6_K: (210, 256), Q8_0: (34, 32)}
SHAPES = [("O-proj q4K", Q4_K, 4096, 4096, 1), ("QK q4K", Q4_K, 4096, 5120, 1), ("gate+up q4K", Q4_K, 4096, 14336, 2),
          ("down q4K", Q4_K, 14336, 4096, 1), ("down q6K", Q6_K, 14336, 4096, 1), ("head q6K", Q6_K, 4096, 128256, 1),
          ("70B gate+up", Q4_K, 8192, 28672, 2), ("q8_0 4096", Q8_0, 4096, 4096, 1)]


def child():
    import llamacog_amd as la
    lib = la.plugin_lib()
    g = lib.mi355x_bench_gemv2
    g.restype = ctypes.c_double
    g.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    for name, t, K, M, nm in SHAPES:
        bb, qk = BB[t]
        mb = K // qk * bb * M * nm
        copies = max(2, -(-(3 << 30) // mb))
        us = g(t, K, M, nm, copies, 40, 0)
        print(f"{name:14s} {mb / 1e6:7.1f} MB {us:8.2f} us {mb / us / 1e6:5.2f} TB/s", flush=True)


def main():
    if "--child" in sys.argv:
        return child()
    variants = [("one-shot", {"GGML_MI355X_GEMV_ENG": "0"})] + [
        (f"eng {c}", {"GGML_MI355X_GEMV_ENG": "1", "GGML_MI355X_ENG_CFG": c}) for c in ("214", "412")] + [
        ("eng 412 prof", {"GGML_MI355X_GEMV_ENG": "1", "GGML_MI355X_ENG_CFG": "412", "GGML_MI355X_ENG_PROF": "1"})]
    for label, env in variants:
        print(f"== {label}", flush=True)
        e = dict(os.environ)
        e.update(env)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=e, capture_output=True, text=True,
                           timeout=240)
        print(r.stdout, end="", flush=True)
        for line in r.stderr.splitlines():
            if "[eng-prof]" in line:
                print("   ", line, flush=True)
        if r.returncode != 0:
            print(f"[rc={r.returncode}] {r.stderr[-600:]}", flush=True)
            return r.returncode


if __name__ == "__main__":
    sys.exit(main() or 0)
