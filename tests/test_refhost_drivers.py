"""The reference's own drivers, built unchanged from /root/reference by refhost/Makefile, run
the BASELINE.json configs[0] plumbing case (stories15M-shape Q8_0 on ggml-cpu through
llama-bench) and, with the plugin loaded through GGML_BACKEND_PATH, the same model on MI355X
(llama-bench -ngl 99, and llama-cli greedy text identical to the CPU backend's)."""
import json
import os
import subprocess

import pytest

import llamacog_amd as la
from llamacog_amd import gguf_synth as gs

BENCH = os.path.join(la.REFHOST, "llama-bench")
CLI = os.path.join(la.REFHOST, "llama-cli")


@pytest.fixture(scope="module")
def stories(tmp_path_factory):
    d = tmp_path_factory.mktemp("stories")
    return gs.write_gguf(gs.CONFIGS["stories15m-q8_0"], str(d / "stories15m-q8_0.gguf"), seed=0)


def _bench(model, extra, env):
    cmd = [BENCH, "-m", model, "-p", "64", "-n", "16", "-r", "1", "-t", "4", "-o", "json"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout)


def test_llama_bench_stories15m_cpu(stories):
    env = {k: v for k, v in os.environ.items() if k != "GGML_BACKEND_PATH"}
    rows = _bench(stories, [], env)
    assert {r["n_prompt"] for r in rows} == {64, 0} and all(r["avg_ts"] > 0 for r in rows)
    assert all("MI355X" not in r.get("backends", "") for r in rows)


def _cli(model, ngl, env):
    cmd = [CLI, "-m", model, "-p", "Once upon a time", "-n", "24", "--temp", "0", "-ngl", str(ngl), "-no-cnv",
           "--no-warmup", "-t", "4", "--seed", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, stdin=subprocess.DEVNULL)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout, r.stderr


def test_llama_cli_runs_on_cpu(stories):
    env = {k: v for k, v in os.environ.items() if k != "GGML_BACKEND_PATH"}
    out, _ = _cli(stories, 0, env)
    # the synthetic SPM vocab prints the prompt pieces, then one "t<id>" piece per generated token
    assert "time" in out.split()[0] and len(out.split()) >= 20, out


@pytest.mark.gpu
def test_llama_bench_stories15m_plugin(stories):
    rows = _bench(stories, ["-ngl", "99", "-fa", "1"], dict(os.environ, GGML_BACKEND_PATH=la.PLUGIN))
    assert all("MI355X" in r.get("backends", "") or "MI355X" in r.get("gpu_info", "") for r in rows), rows
    assert all(r["avg_ts"] > 0 for r in rows)


@pytest.mark.gpu
def test_llama_cli_greedy_text_matches_cpu(stories):
    cpu_env = {k: v for k, v in os.environ.items() if k != "GGML_BACKEND_PATH"}
    out_c, _ = _cli(stories, 0, cpu_env)
    out_g, err_g = _cli(stories, 99, dict(os.environ, GGML_BACKEND_PATH=la.PLUGIN))
    assert "MI355X" in err_g
    assert out_g == out_c
