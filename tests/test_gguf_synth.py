"""Synthetic GGUF writer: Q4_K_M type map, byte budget, and that the reference's
libllama (CPU backend) loads and runs the files."""
import numpy as np
import pytest

import llamacog_amd as la
from llamacog_amd import gguf_synth as gs


def test_q4km_type_map_matches_llama_quant():
    cfg = gs.CONFIGS["llama3-8b-q4km"]
    types = {n: t for n, _, t in gs.tensor_types(cfg)}
    assert types["output.weight"] == gs.Q6_K
    assert types["token_embd.weight"] == gs.Q4_K
    six = [i for i in range(32) if types[f"blk.{i}.ffn_down.weight"] == gs.Q6_K]
    # src/llama-quant.cpp:185-187 use_more_bits: i < 4, i >= 28, (i-4) % 3 == 2
    assert six == [0, 1, 2, 3, 6, 9, 12, 15, 18, 21, 24, 27, 28, 29, 30, 31]
    assert all(types[f"blk.{i}.attn_v.weight"] == types[f"blk.{i}.ffn_down.weight"] for i in range(32))


def test_decode_bytes_per_token_llama3_8b():
    # SURVEY.md finding 5 / BASELINE.md §2: 4.617 GB per token of weights
    b = gs.weight_bytes_per_token(gs.CONFIGS["llama3-8b-q4km"])
    assert abs(b / 1e9 - 4.617) < 0.01, b


def test_blocks_are_valid_and_zero_mean(tmp_path):
    rng = np.random.default_rng(0)
    import _oracle as O
    for t in (gs.Q4_K, gs.Q5_K, gs.Q6_K, gs.Q8_0, gs.Q4_0):
        blk, bs = gs.BLOCK[t]
        raw = gs.make_blocks(t, 64, rng).reshape(64, bs)
        w = O.dequantize_rows(t, raw.reshape(1, -1), 64 * blk)
        assert np.isfinite(w).all()
        assert abs(w.mean()) < 0.004 and 0.005 < w.std() < 0.06, (t, w.mean(), w.std())


def test_tiny_model_runs_on_reference_cpu(tmp_path):
    path = gs.write_gguf(gs.CONFIGS["tiny-q4km"], str(tmp_path / "tiny.gguf"), seed=3)
    m = la.Model(path, gpu=False, n_ctx=256)
    ids, logits = m.greedy([1, 300, 301], 3)
    assert logits.shape == (3, 4096) and np.isfinite(logits).all()
    m.close()
