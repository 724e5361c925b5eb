"""bench.py's multi-process contract on CPU (gloo, world_size 2, 127.0.0.1), as the driver
launches it: `torch.distributed.run --nproc-per-node N bench.py --gpus N`.  The harness runs
with --cpu (libllama's CPU backend, a tiny synthetic model), so what is tested is the rank
logic — barriers, the max over ranks, rank 0's single JSON line — and the split series:
  * value: one replica per rank (weak scaling, value = N x steps / the slowest rank's time);
  * split_series: rank 0's child process (no rank environment) runs the layer-split model and
    its object rides on the same line, at N = 2 and at N = 1."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def tiny_dir(tmp_path_factory):
    from llamacog_amd import gguf_synth as gs
    d = tmp_path_factory.mktemp("models")
    gs.write_gguf(gs.CONFIGS["tiny-q4km"], str(d / "tiny-q4km-s0.gguf"), seed=0)
    return str(d)


def _run(tiny_dir, gpus, nproc=2):
    bench = [os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--cpu", "--config", "tiny-q4km",
             "--steps", "4", "--warmup", "1", "--pp", "0", "--roofline-steps", "0", "--no-cpu-baseline",
             "--model-dir", tiny_dir, "--split-config", "tiny-q4km", "--split-steps", "3", "--split-warmup", "1", "--split-pp", "32"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    # the rendezvous port is picked free and then released; another process can take it before
    # torch.distributed.run binds it, so a multi-process run that failed on exactly that (an
    # address-in-use error) gets one retry on a fresh port; any other failure fails the test
    for attempt in range(2 if nproc > 1 else 1):
        if nproc > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                   "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + bench
        else:
            cmd = [sys.executable] + bench
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
        port_taken = "address already in use" in (out.stderr + out.stdout).lower() or "EADDRINUSE" in out.stderr
        if out.returncode == 0 or not port_taken:
            break
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout      # rank 0 only
    return json.loads(lines[0])


def test_replicas_two_ranks_with_split_series(tiny_dir):
    d = _run(tiny_dir, 2)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["global_batch"] == 2
    assert d["steps"] == 4 and d["value"] > 0
    # value is the whole job: two streams over the slowest rank's time
    assert abs(d["value"] - 2 * 4 / (d["ms_per_step"] * 4 / 1e3)) / d["value"] < 0.01
    assert "replicas x2" in d["config"]["parallelism"]
    sp = d["split_series"]
    assert sp and "error" not in sp, sp
    assert sp["model"] == "tiny-q4km" and sp["steps"] == 3 and sp["tg_tok_s"] > 0
    # pp at N and the roofline fraction ride on the series (BASELINE.json metric: pp and tg at N)
    assert sp["pp_tokens"] == 32 and sp["pp_tok_s"] > 0 and sp["tg_frac_of_8TBs"] > 0


def test_single_process_with_split_series(tiny_dir):
    d = _run(tiny_dir, 1, nproc=1)
    assert d["n_gpus"] == 1 and d["config"]["global_batch"] == 1 and d["value"] > 0
    sp = d["split_series"]
    assert sp and "error" not in sp and sp["tg_tok_s"] > 0, sp
