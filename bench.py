#!/usr/bin/env python3
"""bench.py — llama-bench tg128 (+ pp512) tok/s of Llama-3-8B Q4_K_M on MI355X.

Drives the reference's unchanged libllama (refhost/build, via tools/llb.cpp which repeats
llama-bench's test_gen/test_prompt loops, tools/llama-bench/llama-bench.cpp:1747-1795) with
the MI355X plugin loaded.  A "step" is one single-token llama_decode (n_batch = 1, the
BASELINE.json configs[1] decode workload); K timed steps are bracketed by a barrier and a
device synchronisation, the max over ranks is taken, and rank 0 prints one JSON line.

Multi-GPU: the decode path of one stream does not shard (layer split is sequential,
SURVEY.md §8(e)), so --gpus N runs N independent replicas, one process per GPU
("replicas only", weak scaling); value = N*K / max-rank time.

Extra objects on the line: "roofline" (the dominant kernel — the quantized mat-vec —
timed with HIP events on the plugin's stream) and "cpu_baseline" (the reference's own
llama-bench on the CPU backend, a bounded tg sample on the same host).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
MFMA_I8_PEAK_TOPS = 2500.0   # dense int8 MFMA, no sparsity (MI355X_MICROARCH.md)
# algorithmic work of one pp512 of Llama-3-8B: 2*6.98e9*512 layer matmuls +
# output (last token) + attention
PP512_FLOP = 7.22e12
TRAFFIC_FILE = os.path.join(REPO, "profiles", "r01", "pmc_traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="llama3-8b-q4km")
    ap.add_argument("--layers", type=int, default=None, help="override layer count (debug only)")
    ap.add_argument("--pp", type=int, default=512, help="prompt length for the pp figure (0 = skip)")
    ap.add_argument("--fa", type=int, default=1)
    ap.add_argument("--kv", default="f16")
    ap.add_argument("--roofline-steps", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-gen", type=int, default=16)
    ap.add_argument("--model-dir", default=os.environ.get("LLAMACOG_MODEL_DIR", "/tmp/llamacog_amd_models"))
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, lrank


class Dist:
    """Barrier / max-reduction over ranks (gloo on host memory; the timed work itself runs
    on the plugin's HIP stream and is synchronised by llama_synchronize)."""

    def __init__(self, ws: int):
        self.ws = ws
        self.pg = None
        if ws > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.ws > 1:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if self.ws == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.ws > 1:
            self.dist.destroy_process_group()


def cpu_baseline(model: str, threads: int, n_gen: int, fa: int) -> dict:
    """The reference's ggml-cpu path (refhost/build/llama-bench, score-selected CPU variant,
    our plugin NOT loaded) on a bounded tg sample of the same model on this host."""
    exe = os.path.join(REPO, "refhost", "build", "llama-bench")
    env = {k: v for k, v in os.environ.items() if k != "GGML_BACKEND_PATH"}
    cmd = [exe, "-m", model, "-p", "0", "-n", str(n_gen), "-r", "1", "-t", str(threads), "-fa", str(fa), "-o", "json"]
    t0 = time.time()
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    if out.returncode != 0:
        return {"value": None, "unit": "tok/s", "cores": threads, "kind": "reference",
                "sample": f"llama-bench failed rc={out.returncode}: {out.stderr[-300:]}"}
    rows = json.loads(out.stdout)
    r = rows[0]
    return {"value": round(float(r["avg_ts"]), 3), "unit": "tok/s", "cores": threads, "kind": "reference",
            "sample": f"reference llama-bench (ggml-cpu, {r.get('cpu_info', '?')}) tg{n_gen} x1 rep, -t {threads}, "
                      f"-fa {fa}, same synthetic GGUF; wall {time.time() - t0:.1f}s incl. load"}


def main():
    a = parse()
    ws, rank, lrank = dist_env()
    if ws > 1:
        # one process per GPU: restrict this rank's HIP runtime (and so the plugin's
        # device list) to its own GPU before anything touches HIP
        os.environ["HIP_VISIBLE_DEVICES"] = str(lrank)
    dist = Dist(ws)

    import llamacog_amd as la
    from llamacog_amd import gguf_synth

    cfg = gguf_synth.CONFIGS[a.config]
    suffix = f"-{a.layers}l" if a.layers else ""
    path = os.path.join(a.model_dir, f"{a.config}{suffix}-s0.gguf")
    if lrank == 0 and not os.path.exists(path):
        t0 = time.time()
        gguf_synth.ensure(a.config, path, seed=0, n_layer=a.layers)
        if rank == 0:
            print(f"[bench] wrote {path} in {time.time() - t0:.1f}s", file=sys.stderr)
    dist.barrier()

    n_ctx = ((a.warmup + a.steps + max(a.pp, 0) + a.roofline_steps + 255) // 256 + 1) * 256
    m = la.Model(path, gpu=True, n_ctx=n_ctx, flash_attn=bool(a.fa), kv_type=a.kv, n_gpus=1)
    plugin = la.plugin_lib()
    if a.verbose and rank == 0:
        print(la.log_tail(m.lib)[-4000:], file=sys.stderr)

    # pp figure (one ubatch of a.pp tokens, as llama-bench pp512)
    pp_tps = None
    if a.pp > 0:
        m.clear()
        m.time_prompt(min(a.pp, 64))  # warm
        m.clear()
        tpp = m.time_prompt(a.pp)
        pp_tps = a.pp / tpp

    # tg: W untimed decode steps, then exactly K timed steps
    m.clear()
    if a.warmup > 0:
        m.time_gen(a.warmup)
    dist.barrier()
    t_local = m.time_gen(a.steps)   # each step ends in llama_synchronize (device sync)
    dist.barrier()
    t = dist.max(t_local)
    value = ws * a.steps / t

    # where a step's wall time goes: host work inside llama_decode (libllama graph build,
    # scheduling, input upload, our graph_compute and launch) vs waiting in llama_synchronize
    m.clear()
    m.time_gen(4)
    plugin.ggml_backend_mi355x_reset_timing()
    plugin.ggml_backend_mi355x_set_graph_timing(1)
    t_sp, t_dec, t_syn = m.time_gen_split(a.steps)
    plugin.ggml_backend_mi355x_set_graph_timing(0)
    g_ms, _, g_n = la.kernel_timing(plugin, 5)    # device time of each graph_compute (events around it)
    gh_ms, _, gh_n = la.kernel_timing(plugin, 6)  # host time inside graph_compute

    # roofline pass: HIP events around every mat-vec launch on the plugin stream
    m.clear()
    m.time_gen(4)
    plugin.ggml_backend_mi355x_reset_timing()
    plugin.ggml_backend_mi355x_set_timing(1)
    t_rf = m.time_gen(a.roofline_steps)
    plugin.ggml_backend_mi355x_set_timing(0)
    mv_ms, mv_bytes, mv_n = la.kernel_timing(plugin, 0)
    fa_ms, fa_bytes, fa_n = la.kernel_timing(plugin, 2)
    achieved = (mv_bytes / (mv_ms * 1e-3)) / 1e9 if mv_ms > 0 else None
    # HBM bytes per GEMV launch from the PMC pass (rocprofv3 --pmc FETCH_SIZE, x2 gfx950
    # correction), committed with its command under profiles/ (scripts/gpu_final.sh, scripts/pmc_traffic.py)
    traffic = None
    if os.path.exists(TRAFFIC_FILE):
        try:
            traffic = json.load(open(TRAFFIC_FILE)).get("gemv_bytes_per_launch")
        except Exception:
            traffic = None
    wbytes = gguf_synth.weight_bytes_per_token(
        gguf_synth.ModelConfig(**{**cfg.__dict__, "n_layer": a.layers or cfg.n_layer}))

    gstats = la.graph_stats()
    m.close()
    cpu = None
    if rank == 0 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(path, a.cpu_threads, a.cpu_gen, a.fa)
        except Exception as e:  # the baseline must never hide the GPU result
            cpu = {"value": None, "unit": "tok/s", "cores": a.cpu_threads, "kind": "reference", "sample": f"error: {e}"}

    if rank == 0:
        out = {
            "metric": "llama-bench tg128 + pp512 tok/s, Llama-3-8B Q4_K_M; 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "tok/s",
            "n_gpus": ws,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * t / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "i8",
            "data": "synthetic",
            "config": {
                "workload": f"{cfg.name} ({a.config}{suffix}) tg: n_batch=1 single-token llama_decode, "
                            f"fa={a.fa}, kv={a.kv}, n_ctx={n_ctx}; random-but-valid Q4_K/Q6_K blocks",
                "model": a.config + suffix,
                "global_batch": ws,
                "seq_len": a.warmup + a.steps,
                "parallelism": f"replicas x{ws}" if ws > 1 else "single GPU",
            },
            "pp_tok_s": round(pp_tps, 2) if pp_tps else None,
            "pp_tokens": a.pp,
            "pp_roofline": ({"bound": "mfma", "unit": "TFLOP/s", "peak": MFMA_I8_PEAK_TOPS,
                             "achieved": round(PP512_FLOP / (a.pp / pp_tps) / 1e12, 2),
                             "frac": round(PP512_FLOP / (a.pp / pp_tps) / 1e12 / MFMA_I8_PEAK_TOPS, 4),
                             "note": "whole pp512 (all kernels), Llama-3-8B algorithmic FLOPs"}
                            if (pp_tps and a.pp == 512 and a.config == "llama3-8b-q4km" and not a.layers) else None),
            "weight_bytes_per_token": wbytes,
            "model_bw_GBs": round(wbytes * (a.steps / t_local) / 1e9, 1),
            "model_bw_frac_of_8TBs": round(wbytes * (a.steps / t_local) / 1e9 / HBM_PEAK_GBS, 4),
            "roofline": {
                "bound": "hbm",
                "kernel": "k_gemv_pipe (quantized decode GEMV, every decode MUL_MAT)",
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": "profiles/r01/pmc_traffic.json" if traffic else None,
                "launches": mv_n,
                "avg_launch_us": round(1e3 * mv_ms / mv_n, 3) if mv_n else None,
                "algorithmic_bytes_per_launch": round(mv_bytes / mv_n) if mv_n else None,
                "measured_over_steps": a.roofline_steps,
                "fattn_avg_us": round(1e3 * fa_ms / fa_n, 3) if fa_n else None,
                "timed_pass_tok_s": round(a.roofline_steps / t_rf, 2),
            },
            # wall = one llama_decode + llama_synchronize; device_graph = GPU time of the graph
            # (events before/after graph_compute's launches); graph_compute_host = host time in
            # our graph_compute (signature, KV-slot table upload, hipGraph launch); the rest of the
            # wall is libllama's host work (graph build, scheduling, input upload, logits copy)
            "step_split_ms": {"wall": round(1e3 * t_sp / a.steps, 4),
                              "device_graph": round(g_ms / g_n, 4) if g_n else None,
                              "graph_compute_host": round(gh_ms / gh_n, 4) if gh_n else None,
                              "llama_decode_call": round(1e3 * t_dec / a.steps, 4),
                              "llama_synchronize_call": round(1e3 * t_syn / a.steps, 4)},
            "cpu_baseline": cpu,
            "hipgraph": dict(zip(("captures", "replays"), gstats)),
        }
        print(json.dumps(out))
    dist.close()


if __name__ == "__main__":
    main()
