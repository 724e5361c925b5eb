"""In-graph kernel timeline of Llama-3-8B decode (backend.cpp kt_collect): every decode mat-vec
and exact flash-attention launch stamps the chip's realtime counter per workgroup at entry and
per wave at exit INSIDE the replayed hipGraph; this script decodes N tokens with the timeline
on and prints, per launch label, the mean duration, dispatch ramp and the gap that precedes it,
plus the per-token span split into instrumented kernel time and gaps.

usage: python scripts/ktrace.py [--config llama3-8b-q4km] [--tokens 16] [--depth 0] [--kv f16] [--csv out.csv]
"""
import argparse
import collections
import csv
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la
from llamacog_amd import gguf_synth


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="llama3-8b-q4km")
    ap.add_argument("--tokens", type=int, default=16)
    ap.add_argument("--depth", type=int, default=0)
    ap.add_argument("--csv", default="gpurun_out/ktrace.csv")
    ap.add_argument("--kv", default="f16", help="KV cache type (f16, q8_0, q4_0)")
    a = ap.parse_args()
    path = gguf_synth.ensure(a.config)
    m = la.Model(path, gpu=True, n_ctx=max(512, a.depth + a.tokens + 64), kv_type=a.kv)
    plugin = la.plugin_lib()
    plugin.ggml_backend_mi355x_ktrace_dump.argtypes = [ctypes.c_char_p]
    if a.depth:
        m.time_prompt(a.depth)
    plugin.ggml_backend_mi355x_set_ktrace(1)
    m.time_gen(4)          # captures under the traced signature
    plugin.ggml_backend_mi355x_ktrace_dump(b"/dev/null")
    m.time_gen(a.tokens)
    os.makedirs(os.path.dirname(os.path.abspath(a.csv)), exist_ok=True)
    n = plugin.ggml_backend_mi355x_ktrace_dump(a.csv.encode())
    plugin.ggml_backend_mi355x_set_ktrace(0)
    m.close()
    rows = list(csv.DictReader(open(a.csv)))
    graphs = collections.defaultdict(list)
    for r in rows:
        graphs[int(r["graph"])].append(r)
    stats = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0, 0.0, 0.0])   # n, dur, ramp, gap_before, nwg, wg0 end, wg life
    spans, busy = [], []
    for g, rs in graphs.items():
        rs.sort(key=lambda r: int(r["idx"]))
        prev_end = None
        b = 0.0
        for r in rs:
            t0, tl, t1 = float(r["start_ns"]), float(r["last_start_ns"]), float(r["end_ns"])
            s = stats[r["kernel"]]
            s[0] += 1
            s[1] += t1 - t0
            s[2] += tl - t0
            s[3] += (t0 - prev_end) if prev_end is not None else 0.0
            s[4] = int(r["nwg"])
            s[5] += float(r.get("wg0_end_ns", 0) or 0) - t0
            s[6] += float(r.get("wg_mean_ns", 0) or 0)
            b += t1 - t0
            prev_end = t1
        spans.append(float(rs[-1]["end_ns"]) - float(rs[0]["start_ns"]))
        busy.append(b)
    ng = len(graphs)
    print(f"{a.config}: {ng} graphs ({n} launch records), depth {a.depth}")
    print(f"{'launch':24s} {'per tok':>7s} {'nwg':>5s} {'mean us':>8s} {'ramp us':>8s} {'gap before us':>14s} {'wg0 end us':>10s} {'wg life us':>10s}")
    for k, (cnt, d, rp, gp, nwg, w0, wl) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:24s} {cnt / ng:7.1f} {nwg:5d} {d / cnt / 1e3:8.2f} {rp / cnt / 1e3:8.2f} {gp / cnt / 1e3:14.2f} "
              f"{w0 / cnt / 1e3:10.2f} {wl / cnt / 1e3:10.2f}")
    sp, bu = sum(spans) / ng / 1e3, sum(busy) / ng / 1e3
    print(f"per token: span {sp:.1f} us (first instrumented start -> last end), instrumented kernels {bu:.1f} us, "
          f"gaps + other kernels {sp - bu:.1f} us")


if __name__ == "__main__":
    main()
