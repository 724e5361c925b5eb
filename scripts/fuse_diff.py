"""Logits of a short greedy run on MI355X under the current fusion flags (env), saved to a
file for cross-process comparison (debug aid for fused-vs-unfused bit parity)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la
from llamacog_amd import gguf_synth as gs

cfg, out = sys.argv[1], sys.argv[2]
path = gs.ensure(cfg)
rng = np.random.default_rng(5)
prompt = [1] + rng.integers(300, gs.CONFIGS[cfg].n_vocab, 11).tolist()
m = la.Model(path, gpu=True, n_ctx=512)
ids, lg = m.greedy(prompt, 6)
np.save(out, lg)
print(cfg, os.environ.get("TAG", ""), ids.tolist())
