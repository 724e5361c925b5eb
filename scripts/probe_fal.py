"""Decode flash attention at depth (32 query heads over 8 KV heads, D = 128, mi355x_bench_op 0 /
3): the long-context pair (k_fal_scores + k_fal_chain) against the per-head kernels (f16:
k_fattn_dec2, q8_0: k_fattn_exact), each variant in its own process (GGML_MI355X_FA_LONG is read
once).  Prints us per layer-call for n_kv:valid pairs."""
import ctypes
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(which):
    import llamacog_amd as la
    op = la.plugin_lib().mi355x_bench_op
    op.restype = ctypes.c_double
    op.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    for n, v in ((256, 136), (512, 512), (768, 700), (1024, 1024), (2048, 2048), (4352, 4096), (8192, 8192)):
        print(f"  n_kv={n:5d} valid={v:5d}: {op(which, n, v, 30):8.2f} us", flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        return child(int(sys.argv[2]))
    for kv, which in (("f16", 0), ("q8_0", 3)):
        for label, env in (("per-head kernels", {"GGML_MI355X_FA_LONG": "0"}), ("long pair", {"GGML_MI355X_FA_LONG": "256"})):
            print(f"== {kv} cache, {label}", flush=True)
            e = dict(os.environ)
            e.update(env)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", str(which)], env=e,
                               capture_output=True, text=True, timeout=240)
            print(r.stdout, end="", flush=True)
            if r.returncode != 0:
                print(f"[rc={r.returncode}] {r.stderr[-800:]}", flush=True)
                return r.returncode


if __name__ == "__main__":
    sys.exit(main() or 0)
