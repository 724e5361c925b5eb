"""Prints every node the plugin dispatches and every stand-alone activation quantize
(GGML_MI355X_DEBUG_OPS) for one decode step of a 2-layer model, to see which graph nodes still
cost a launch of their own."""
import os
import sys

os.environ["GGML_MI355X_DEBUG_OPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la
from llamacog_amd import gguf_synth as gs

cfg = sys.argv[1] if len(sys.argv) > 1 else "mixtral-2l-q5km"
m = la.Model(gs.ensure(cfg), gpu=True, n_ctx=256)
m.greedy([1, 300, 301, 302], 2)
m.close()
