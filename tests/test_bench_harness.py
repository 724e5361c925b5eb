"""bench.py's multi-process contract on CPU (gloo, world_size 2, 127.0.0.1), as the driver
launches it: `torch.distributed.run --nproc-per-node N bench.py --gpus N`.  The harness runs
with --cpu (libllama's CPU backend, a tiny synthetic model), so what is tested is the rank
logic — barriers, the max over ranks, rank 0's single JSON line — for both modes:
  * --gpus 2: one stream split over two devices in rank 0's process (strong scaling; the
    other rank only joins the barriers and the max);
  * --gpus 1 under two ranks: replicas (weak scaling, value = 2 x steps / max time)."""
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


def _run(tiny_dir, gpus):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--cpu", "--config", "tiny-q4km",
           "--steps", "4", "--warmup", "1", "--pp", "0", "--roofline-steps", "0", "--no-cpu-baseline",
           "--model-dir", tiny_dir]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout      # rank 0 only
    return json.loads(lines[0])


def test_split_mode_two_ranks(tiny_dir):
    d = _run(tiny_dir, 2)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["global_batch"] == 1
    assert d["steps"] == 4 and d["value"] > 0
    assert abs(d["value"] - 4 / (d["ms_per_step"] * 4 / 1e3)) / d["value"] < 0.01
    assert "layer split over 2 GPUs" in d["config"]["parallelism"]


def test_replica_mode_two_ranks(tiny_dir):
    d = _run(tiny_dir, 1)
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["config"]["global_batch"] == 2
    # value is the whole job: two streams over the slowest rank's time
    assert abs(d["value"] - 2 * 4 / (d["ms_per_step"] * 4 / 1e3)) / d["value"] < 0.01
