"""q8_0 / q4_0 KV-cache model runs on MI355X vs the CPU backend (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import llamacog_amd as la
from llamacog_amd import gguf_synth as gs

kv = sys.argv[1] if len(sys.argv) > 1 else "q8_0"
cfg = sys.argv[2] if len(sys.argv) > 2 else "tiny-q4km"
path = gs.ensure(cfg)
prompt = [1] + list(range(300, 315))
res = {}
for gpu in (True, False):
    m = la.Model(path, gpu=gpu, n_ctx=512, flash_attn=True, kv_type=kv, n_threads=16)
    res[gpu] = m.greedy(prompt, 16)
    m.close()
    print("gpu" if gpu else "cpu", res[gpu][0].tolist(), flush=True)
(ig, lg), (ic, lc) = res[True], res[False]
print("ids equal", bool((ig == ic).all()), "logits bit-equal", bool((lg.view(np.uint32) == lc.view(np.uint32)).all()),
      "max rel", float(np.abs(lg - lc).max() / np.abs(lc).max()))
