#!/usr/bin/env python3
"""bench.py — llama-bench tg128 (+ pp512) tok/s of Llama-3-8B Q4_K_M on MI355X.

Drives the reference's unchanged libllama (refhost/build, via tools/llb.cpp which repeats
llama-bench's test_gen/test_prompt loops, tools/llama-bench/llama-bench.cpp:1747-1795) with
the MI355X plugin loaded.  A "step" is one single-token llama_decode (n_batch = 1, the
BASELINE.json configs[1] decode workload); K timed steps are bracketed by a barrier and a
device synchronisation, the max over ranks is taken, and rank 0 prints one JSON line.

Multi-GPU.  `value` is the same workload at every N: under
torch.distributed.run (one process per GPU, as the driver launches it) every rank decodes its
own Llama-3-8B replica on its own GPU, and value = N streams x K steps / the slowest rank's time
("weak": fixed work per GPU).  Beside it, `split_series` is BASELINE.json configs[3] at the same
N: Llama-3-70B Q4_K_M split by layers over the N GPUs in ONE process (libllama -sm layer, the
scheduler's pipeline copies, stage hand-offs through backend.cpp cpy_tensor_async = RCCL
ncclSend/ncclRecv between GPUs), run by rank 0 in a child process that sees every GPU while the
other ranks wait at a barrier; N = 1 gives the 70B's one-GPU point of the same series.
--cpu runs the harness on the CPU backend (tests only).

Extra objects on the line: "roofline" (the dominant kernel — the quantized mat-vec — timed
with HIP events on the plugin's stream; fractions against the measured STREAM-read peak and
the 8 TB/s nominal) and "cpu_baseline" (the reference's own llama-bench on the CPU backend,
BASELINE.md §3: physical cores of this process's CPU set, -r 5, tg128 and pp512).
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
# dense int8 MFMA, no sparsity: 2x the dense BF16 2.5 PFLOP/s (MI355X_MICROARCH.md, matrix cores)
MFMA_I8_PEAK_TOPS = 5000.0
# algorithmic work of one pp512 of Llama-3-8B: 2*6.98e9*512 layer matmuls +
# output (last token) + attention
PP512_FLOP = 7.22e12
# HBM bytes per decode-GEMV launch from a separate rocprofv3 --pmc FETCH_SIZE pass of the SAME
# model (scripts/gpu_r06_pmc.sh, scripts/pmc_traffic.py), one file per --config
TRAFFIC_DIR = os.path.join("profiles", "r06", "pmc")


def traffic_file(config):
    return os.path.join(TRAFFIC_DIR, f"pmc_traffic_{config}.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="llama3-8b-q4km")
    ap.add_argument("--layers", type=int, default=None, help="override layer count (debug only)")
    ap.add_argument("--pp", type=int, default=512, help="prompt length for the pp figure (0 = skip)")
    ap.add_argument("--pp-reps", type=int, default=3, help="timed pp runs after the warmup run (mean tok/s)")
    ap.add_argument("--fa", type=int, default=1)
    ap.add_argument("--kv", default="f16")
    ap.add_argument("--depth", type=int, default=0, help="KV depth before the timed steps (llama-bench -d)")
    ap.add_argument("--roofline-steps", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = physical cores of this process's CPU set")
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--cpu", action="store_true", help="run the harness on the CPU backend (tests)")
    ap.add_argument("--model-dir", default=os.environ.get("LLAMACOG_MODEL_DIR", "/tmp/llamacog_amd_models"))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--no-split-series", action="store_true", help="skip the 70B layer-split series")
    ap.add_argument("--split-config", default="llama3-70b-q4km")
    ap.add_argument("--split-steps", type=int, default=32)
    ap.add_argument("--split-warmup", type=int, default=4)
    # the driver bounds the whole bench (600 s): a stuck split child must cost only the series
    ap.add_argument("--split-timeout", type=int, default=240, help="seconds before the split child is killed")
    ap.add_argument("--split-pp", type=int, default=512, help="prompt length of the split series' pp figure (0 = skip)")
    ap.add_argument("--split-only", action="store_true", help=argparse.SUPPRESS)   # the series' child process
    return ap.parse_args()


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, lrank


class Dist:
    """Barrier / max-reduction over ranks (gloo on host memory; the timed work itself runs
    on the plugin's HIP streams and is synchronised by llama_synchronize)."""

    def __init__(self, ws: int):
        self.ws = ws
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


def physical_cores() -> tuple[int, str]:
    """Physical cores of this process's CPU set (SMT siblings counted once), capped by the
    thread budget the box grants (OMP_NUM_THREADS), and the lscpu topology for the record."""
    cpus = sorted(os.sched_getaffinity(0))
    cores = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                core = f.read().strip()
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                pkg = f.read().strip()
            cores.add((pkg, core))
        except OSError:
            cores.add(("?", str(c)))
    n = len(cores)
    budget = os.environ.get("OMP_NUM_THREADS")
    if budget and budget.isdigit():
        n = min(n, int(budget))
    topo = "?"
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = dict(l.split(":", 1) for l in out.splitlines() if ":" in l)
        topo = (f"{kv.get('Model name', '?').strip()}: {kv.get('Socket(s)', '?').strip()} sockets x "
                f"{kv.get('Core(s) per socket', '?').strip()} cores x {kv.get('Thread(s) per core', '?').strip()} threads; "
                f"this process: {len(cpus)} CPUs = {len(cores)} physical cores")
    except Exception:
        pass
    return max(n, 1), topo


def cpu_baseline(model: str, threads: int, reps: int, fa: int) -> dict:
    """The reference's ggml-cpu path (refhost/build/llama-bench, score-selected CPU variant,
    our plugin NOT loaded) on the same model: pp512 and tg128, -r reps."""
    exe = os.path.join(REPO, "refhost", "build", "llama-bench")
    env = {k: v for k, v in os.environ.items() if k != "GGML_BACKEND_PATH"}
    cores, topo = physical_cores()
    threads = threads or cores
    cmd = [exe, "-m", model, "-p", "512", "-n", "128", "-r", str(reps), "-t", str(threads), "-fa", str(fa), "-o", "json"]
    t0 = time.time()
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=1200)
    if out.returncode != 0:
        return {"value": None, "unit": "tok/s", "cores": threads, "kind": "reference",
                "sample": f"llama-bench failed rc={out.returncode}: {out.stderr[-300:]}"}
    rows = json.loads(out.stdout)
    tg = next(r for r in rows if r.get("n_gen", 0) > 0)
    pp = next((r for r in rows if r.get("n_prompt", 0) > 0), None)
    return {"value": round(float(tg["avg_ts"]), 3), "unit": "tok/s", "cores": threads, "kind": "reference",
            "tg_stddev": round(float(tg.get("stddev_ts", 0.0)), 3),
            "pp512_tok_s": round(float(pp["avg_ts"]), 2) if pp else None,
            "sample": f"reference llama-bench (ggml-cpu, {tg.get('cpu_info', '?')}) -p 512 -n 128 -r {reps} -t {threads} "
                      f"-fa {fa}, same synthetic GGUF; {topo}; wall {time.time() - t0:.1f}s incl. load"}


def main():
    a = parse()
    if a.split_only:
        return split_only(a)
    ws, rank, lrank = dist_env()
    visible = os.environ.get("HIP_VISIBLE_DEVICES")   # the job's GPUs (the split series' child sees all)
    if ws > 1:
        # replicas: restrict each rank's HIP runtime to its own GPU before anything touches HIP
        os.environ["HIP_VISIBLE_DEVICES"] = visible.split(",")[lrank] if visible else str(lrank)
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

    gpu = not a.cpu
    n_ctx = ((a.warmup + a.steps + a.depth + max(a.pp, 0) + a.roofline_steps + 255) // 256 + 1) * 256
    res = run_worker(a, la, path, gpu, n_ctx, dist)
    # the 70B layer-split series at this N: rank 0's child process over every GPU of the job
    dist.barrier()
    if rank == 0 and not a.no_split_series:
        res["split_series"] = split_child(a, max(a.gpus, ws), visible)
    dist.barrier()
    if rank == 0:
        emit(a, la, gguf_synth, cfg, suffix, ws, gpu, n_ctx, res)
    dist.close()


def split_child(a, n: int, visible) -> dict:
    """runs bench.py --split-only in a child process (all of the job's GPUs visible, no rank
    environment) and returns its JSON object"""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                            "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK", "ROLE_RANK")}
    env.pop("HIP_VISIBLE_DEVICES", None)
    if visible:
        env["HIP_VISIBLE_DEVICES"] = visible
    cmd = [sys.executable, os.path.abspath(__file__), "--split-only", "--gpus", str(n), "--config", a.split_config,
           "--steps", str(a.split_steps), "--warmup", str(a.split_warmup), "--model-dir", a.model_dir, "--fa", str(a.fa),
           "--kv", a.kv, "--split-pp", str(a.split_pp)] + (["--cpu"] if a.cpu else [])
    t0 = time.time()
    try:
        # bounded: a stuck split child (e.g. a hand-off that never completes) costs the series,
        # never the replica line this process prints afterwards
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=a.split_timeout, env=env)
    except subprocess.TimeoutExpired as e:
        err = e.stderr.decode(errors="replace") if isinstance(e.stderr, bytes) else (e.stderr or "")
        return {"error": f"timed out after {a.split_timeout} s: {err[-400:]}"}
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if out.returncode != 0 or not lines:
        return {"error": f"rc={out.returncode}: {out.stderr[-400:]}"}
    d = json.loads(lines[-1])
    d["wall_s"] = round(time.time() - t0, 1)
    return d


def split_only(a):
    """the split series' child: the layer split of a.config over a.gpus devices in this process"""
    import llamacog_amd as la
    from llamacog_amd import gguf_synth
    path = os.path.join(a.model_dir, f"{a.config}-s0.gguf")
    t0 = time.time()
    if not os.path.exists(path):
        gguf_synth.ensure(a.config, path, seed=0)
    t_write = time.time() - t0
    gpu = not a.cpu
    n_ctx = ((a.warmup + a.steps + max(a.split_pp, 0) + 255) // 256 + 1) * 256
    m = la.Model(path, gpu=gpu, n_ctx=n_ctx, flash_attn=bool(a.fa), kv_type=a.kv,
                 n_gpus=a.gpus if gpu else None, split_mode=1)
    devs = [n for _, n, t in la.devices(m.lib) if n.startswith("MI355X")][:a.gpus] if gpu else ["CPU"]
    h0 = la.handoff_stats() if gpu else (0, 0, 0)
    if a.warmup > 0:
        m.time_gen(a.warmup)
    t = m.time_gen(a.steps)
    # pp at this N (one ubatch of split_pp tokens through the layer pipeline, after one warm run)
    pp_tps = None
    if a.split_pp > 0:
        m.clear()
        m.time_prompt(a.split_pp)
        m.clear()
        pp_tps = a.split_pp / m.time_prompt(a.split_pp)
    h1 = la.handoff_stats() if gpu else (0, 0, 0)
    m.close()
    cfg = gguf_synth.CONFIGS[a.config]
    wb = gguf_synth.weight_bytes_per_token(cfg)
    tg = a.steps / t
    print(json.dumps({
        "model": a.config, "n_devices": len(devs), "devices": devs, "steps": a.steps, "warmup": a.warmup,
        "tg_tok_s": round(tg, 3), "ms_per_token": round(1e3 * t / a.steps, 4),
        "pp_tok_s": round(pp_tps, 2) if pp_tps else None, "pp_tokens": a.split_pp,
        "weight_bytes_per_token": wb,
        # decode reads every weight byte once per token, one stage after another: the fraction of
        # ONE GPU's 8 TB/s the pipeline's byte rate reaches (the stages do not stream concurrently)
        "tg_frac_of_8TBs": round(wb * tg / 8e12, 4),
        "stage_handoffs": dict(zip(("rccl", "peer", "d2d"), (h1[i] - h0[i] for i in range(3)))),
        "gguf_write_s": round(t_write, 1),
        "partition": f"libllama -sm layer over {len(devs)} device(s): contiguous layer ranges, output on the last",
    }))


def run_worker(a, la, path, gpu, n_ctx, dist) -> dict:
    r = {}
    m = la.Model(path, gpu=gpu, n_ctx=n_ctx, flash_attn=bool(a.fa), kv_type=a.kv, n_gpus=1 if gpu else None)
    plugin = la.plugin_lib() if gpu else None
    if a.verbose:
        print(la.log_tail(m.lib)[-4000:], file=sys.stderr)

    # pp figure (one ubatch of a.pp tokens, as llama-bench pp512: one warmup prompt of the same
    # length, tools/llama-bench/llama-bench.cpp:1933-1945, then the mean of --pp-reps runs' tok/s)
    r["pp_tps"] = None
    if a.pp > 0:
        m.clear()
        m.time_prompt(a.pp)  # warm
        tps = []
        for _ in range(max(1, a.pp_reps)):
            m.clear()
            tps.append(a.pp / m.time_prompt(a.pp))
        r["pp_tps"] = sum(tps) / len(tps)

    # tg: W untimed decode steps (after a.depth prompt tokens), then exactly K timed steps
    def fill():
        m.clear()
        if a.depth > 0:
            m.time_prompt(a.depth)
    fill()
    if a.warmup > 0:
        m.time_gen(a.warmup)
    dist.barrier()
    t_local = m.time_gen(a.steps)   # each step ends in llama_synchronize (device sync)
    dist.barrier()
    r["t"] = dist.max(t_local)
    r["t_local"] = t_local

    r["split"] = r["roof"] = None
    if gpu:
        # where a step's wall time goes: host work inside llama_decode (libllama graph build,
        # scheduling, input upload, our graph_compute and launch) vs waiting in llama_synchronize
        fill()
        m.time_gen(4)
        plugin.ggml_backend_mi355x_reset_timing()
        plugin.ggml_backend_mi355x_set_graph_timing(1)
        t_sp, t_dec, t_syn = m.time_gen_split(a.steps)
        plugin.ggml_backend_mi355x_set_graph_timing(0)
        g_ms, _, g_n = la.kernel_timing(plugin, 5)    # device time of each graph_compute (events around it)
        gh_ms, _, gh_n = la.kernel_timing(plugin, 6)  # host time inside graph_compute
        r["split"] = {"wall": round(1e3 * t_sp / a.steps, 4),
                      "device_graph": round(g_ms / a.steps, 4) if g_n else None,
                      "graph_compute_host": round(gh_ms / a.steps, 4) if gh_n else None,
                      "llama_decode_call": round(1e3 * t_dec / a.steps, 4),
                      "llama_synchronize_call": round(1e3 * t_syn / a.steps, 4)}

        # roofline pass: HIP events around every mat-vec launch on the plugin streams
        fill()
        m.time_gen(4)
        plugin.ggml_backend_mi355x_reset_timing()
        plugin.ggml_backend_mi355x_set_timing(1)
        t_rf = m.time_gen(a.roofline_steps) if a.roofline_steps > 0 else 0.0
        plugin.ggml_backend_mi355x_set_timing(0)
        mv_ms, mv_bytes, mv_n = la.kernel_timing(plugin, 0)
        fa_ms, _, fa_n = la.kernel_timing(plugin, 2)
        r["roof"] = (mv_ms, mv_bytes, mv_n, fa_ms, fa_n, t_rf)
        r["gstats"] = la.graph_stats()
    m.close()
    if gpu:
        # the measured STREAM-read ceiling of device 0 (k_stream.hip), after the model is gone
        r["hbm_gbs"] = la.hbm_read_gbs(0)
    r["cpu"] = None
    if not a.no_cpu_baseline and not a.cpu and int(os.environ.get("RANK", "0")) == 0:
        try:
            r["cpu"] = cpu_baseline(path, a.cpu_threads, a.cpu_reps, a.fa)
        except Exception as e:  # the baseline must never hide the GPU result
            r["cpu"] = {"value": None, "unit": "tok/s", "cores": a.cpu_threads, "kind": "reference", "sample": f"error: {e}"}
    return r


def emit(a, la, gguf_synth, cfg, suffix, ws, gpu, n_ctx, r):
    t = r["t"]
    n_units = ws                               # GPUs in the job, one replica each
    streams = ws                               # independent decode streams
    value = streams * a.steps / t
    wbytes = gguf_synth.weight_bytes_per_token(
        gguf_synth.ModelConfig(**{**cfg.__dict__, "n_layer": a.layers or cfg.n_layer}))
    roof = None
    if r.get("roof"):
        mv_ms, mv_bytes, mv_n, fa_ms, fa_n, t_rf = r["roof"]
        achieved = (mv_bytes / (mv_ms * 1e-3)) / 1e9 if mv_ms > 0 else None
        hbm = r.get("hbm_gbs") or 0.0
        # HBM bytes per GEMV launch from the PMC pass (rocprofv3 --pmc FETCH_SIZE, x2 gfx950
        # correction), committed with its command under profiles/ (scripts/gpu_final.sh, scripts/pmc_traffic.py)
        traffic = None
        tf = traffic_file(a.config) if not a.layers else None
        if tf and os.path.exists(os.path.join(REPO, tf)):
            try:
                traffic = json.load(open(os.path.join(REPO, tf))).get("gemv_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {
            "bound": "hbm",
            "kernel": "k_gemv_os / k_gemv_os2 (one-shot LDS-DMA quantized decode GEMV, every decode MUL_MAT)",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "peak_measured": round(hbm, 1) if hbm > 0 else None,
            "frac_of_measured": round(achieved / hbm, 4) if achieved and hbm > 0 else None,
            "traffic": traffic,
            "traffic_source": f"{tf}: a separate rocprofv3 --pmc FETCH_SIZE pass of {a.config} (scripts/gpu_r06_pmc.sh), not this run" if traffic else None,
            # the event-timed pass runs eagerly (hipGraph replay off, so every GEMV launch carries
            # its own events); the replayed product path's per-launch times are in the in-graph
            # timeline (scripts/ktrace.py, profiles/r04/ktrace_base.txt)
            "timing": "eager pass, graphs off (per-launch HIP events)",
            "launches": mv_n,
            "avg_launch_us": round(1e3 * mv_ms / mv_n, 3) if mv_n else None,
            "algorithmic_bytes_per_launch": round(mv_bytes / mv_n) if mv_n else None,
            "measured_over_steps": a.roofline_steps,
            "fattn_avg_us": round(1e3 * fa_ms / fa_n, 3) if fa_n else None,
            "timed_pass_tok_s": round(a.roofline_steps / t_rf, 2) if t_rf > 0 else None,
        }
    pp_tps = r.get("pp_tps")
    hbm = r.get("hbm_gbs") or 0.0
    tok_s_stream = a.steps / r["t_local"]
    depth0, depth1 = a.depth + a.warmup + 1, a.depth + a.warmup + a.steps
    out = {
        "metric": "llama-bench tg128 + pp512 tok/s, Llama-3-8B Q4_K_M; 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "tok/s",
        "n_gpus": n_units,
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
                        f"fa={a.fa}, kv={a.kv}, n_ctx={n_ctx}, KV depth {depth0}..{depth1} over the timed steps; "
                        f"random-but-valid quant blocks" + ("; CPU backend (harness test)" if not gpu else ""),
            "model": a.config + suffix,
            "global_batch": streams,
            "seq_len": depth1,
            "parallelism": f"replicas x{ws} (one Llama-3-8B decode stream per GPU)" if ws > 1 else "single GPU",
        },
        "pp_tok_s": round(pp_tps, 2) if pp_tps else None,
        "pp_tokens": a.pp,
        "pp_roofline": ({"bound": "mfma", "unit": "TFLOP/s", "peak": MFMA_I8_PEAK_TOPS,
                         "achieved": round(PP512_FLOP / (a.pp / pp_tps) / 1e12, 2),
                         "frac": round(PP512_FLOP / (a.pp / pp_tps) / 1e12 / MFMA_I8_PEAK_TOPS, 4),
                         "note": "whole pp512 (all kernels), Llama-3-8B algorithmic FLOPs, int8 dense peak"}
                        if (pp_tps and gpu and a.pp == 512 and a.config == "llama3-8b-q4km" and not a.layers) else None),
        "weight_bytes_per_token": wbytes,
        "model_bw_GBs": round(wbytes * tok_s_stream / 1e9, 1),
        "model_bw_frac_of_8TBs": round(wbytes * tok_s_stream / 1e9 / HBM_PEAK_GBS, 4),
        "model_bw_frac_of_measured": round(wbytes * tok_s_stream / 1e9 / hbm, 4) if hbm > 0 else None,
        "roofline": roof,
        # wall = one llama_decode + llama_synchronize; device_graph = GPU time of the graph(s)
        # per step (events around graph_compute); graph_compute_host = host time in our
        # graph_compute per step (signature, KV-slot table upload, hipGraph launch); the rest of
        # the wall is libllama's host work (graph build, scheduling, input upload, logits copy)
        "step_split_ms": r.get("split"),
        "cpu_baseline": r.get("cpu"),
        "hipgraph": dict(zip(("captures", "replays"), r["gstats"])) if r.get("gstats") else None,
        # BASELINE.json configs[3] at this N: the 70B split by layers over the job's GPUs
        "split_series": r.get("split_series"),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
