import sys, os, ctypes
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import _oracle as O
from llamacog_amd import kernels as K
L = K.lib()
L.mi355x_fa_scores_d128.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
O.lib().orc_fa_scores.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
rng = np.random.default_rng(3)
n = 4096
q = rng.standard_normal(128).astype(np.float32)
k = rng.standard_normal((n, 128)).astype(np.float16)
dq, dk, ds = K.Dev(q), K.Dev(k), K.Dev(nbytes=4 * n)
L.mi355x_fa_scores_d128(dq.ptr, dk.ptr, n, ds.ptr, None)
g = ds.get(np.float32, (n,))
c = np.zeros(n, dtype=np.float32)
O.lib().orc_fa_scores(O.ptr(q), O.ptr(k), n, 128, O.ptr(c))
bad = np.argwhere(g.view(np.uint32) != c.view(np.uint32)).ravel()
print("score mismatches", len(bad), "of", n, [(int(b), float(g[b]), float(c[b])) for b in bad[:5]])
