"""Node-by-node CPU vs MI355X comparison of one llama_decode through the eval callback
(the examples/eval-callback mechanism).  Prints the first nodes whose relative error is large."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import llamacog_amd as la
from llamacog_amd import gguf_synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "tiny-q4km"
ntok = int(sys.argv[2]) if len(sys.argv) > 2 else 8
fa = int(sys.argv[3]) if len(sys.argv) > 3 else 1
path = gguf_synth.ensure(cfg)
prompt = [1] + [300 + 37 * i for i in range(ntok - 1)]
res = {}
for gpu in (False, True):
    m = la.Model(path, gpu=gpu, n_ctx=512, dump=True, flash_attn=bool(fa))
    ids, lg = m.greedy(prompt, 2)
    res[gpu] = (m.dumps(), lg)
    m.close()
c, g = res[False][0], res[True][0]
print(f"nodes cpu={len(c)} gpu={len(g)}")
shown = 0
for (nc, oc, ac), (ng, og, ag) in zip(c, g):
    if nc != ng or ac.shape != ag.shape:
        print("MISMATCH", nc, ng, ac.shape, ag.shape); break
    den = np.max(np.abs(ac)) + 1e-12
    err = np.max(np.abs(ac - ag)) / den
    flag = " <<<" if err > 1e-3 else ""
    if flag or shown < 400:
        print(f"{nc:28s} op={oc:3d} n={ac.size:8d} maxabs={den:9.3e} relerr={err:9.2e}{flag}")
        shown += 1
lc, lg_ = res[False][1], res[True][1]
print("logits rel err per step:", [float(np.max(np.abs(lc[i]-lg_[i]))/np.max(np.abs(lc[i]))) for i in range(len(lc))])
