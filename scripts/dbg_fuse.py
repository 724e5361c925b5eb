"""Prints the plugin's fusion decisions (GGML_MI355X_DEBUG_FUSE) for a few decode steps of a
2-layer Llama-3-8B-shaped model: which mat-vecs carry which prologue / epilogue."""
import os
import sys

os.environ["GGML_MI355X_DEBUG_FUSE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la
from llamacog_amd import gguf_synth as gs

cfg = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b-2l-q4km"
m = la.Model(gs.ensure(cfg), gpu=True, n_ctx=256)
m.greedy([1, 300, 301, 302], 3)
m.close()
