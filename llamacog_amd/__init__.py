"""llamacog_amd — MI355X-native ggml backend for the reference's (OpenCoq/llamacog,
a llama.cpp fork) quantized LLaMA forward path.

The product is ``libggml-mi355x.so`` (C++/HIP, gfx950), a ggml backend plugin loaded by
the reference's own unchanged host stack (libllama, llama-bench, test-backend-ops) through
``GGML_BACKEND_PATH`` / ``ggml_backend_load``.  This Python package only locates the built
artefacts and wraps the small C driver ``libllb.so`` (tools/llb.cpp) that bench.py, the
tests and ``__graft_entry__.smoke()`` use to drive libllama.
"""
from __future__ import annotations

import ctypes
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "llamacog_amd")
# MI355X_PLUGIN: an A/B build of the plugin (scripts/gpu_iter.sh variants); default the in-tree one
PLUGIN = os.environ.get("MI355X_PLUGIN") or os.path.join(PKG, "libggml-mi355x.so")
LLB = os.path.join(PKG, "libllb.so")
REFHOST = os.path.join(REPO, "refhost", "build")

# ggml_type ids used for KV-cache types
GGML_TYPE = {"f32": 0, "f16": 1, "q4_0": 2, "q8_0": 8}


class BackendMissing(RuntimeError):
    pass


def _require(path: str, what: str) -> str:
    if not os.path.exists(path):
        raise BackendMissing(f"{what} not built: {path} is missing (run __graft_entry__.build())")
    return path


def plugin_lib() -> ctypes.CDLL:
    """The MI355X plugin as a ctypes library (same dlopen handle libllama uses)."""
    base = os.path.join(REFHOST, "libggml-base.so")
    if os.path.exists(base):   # an A/B build outside the tree has no rpath to it
        ctypes.CDLL(base, mode=ctypes.RTLD_GLOBAL)
    lib = ctypes.CDLL(_require(PLUGIN, "MI355X backend plugin"), mode=ctypes.RTLD_GLOBAL)
    lib.ggml_backend_mi355x_get_timing.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long)]
    lib.ggml_backend_mi355x_set_timing.argtypes = [ctypes.c_int]
    lib.ggml_backend_score.restype = ctypes.c_int
    lib.ggml_backend_mi355x_get_device_count.restype = ctypes.c_int
    return lib


def set_flags(no_fuse: bool = False, no_graph: bool = False) -> None:
    """Run-time switches of the plugin (ggml_backend_mi355x_set_flags): one kernel per ggml
    node (no_fuse) and / or no hipGraph replay (no_graph)."""
    plugin_lib().ggml_backend_mi355x_set_flags(1 if no_fuse else 0, 1 if no_graph else 0)


def graph_stats() -> tuple[int, int]:
    """(hipGraphs captured, hipGraph replays) since the plugin was loaded."""
    c, r = ctypes.c_long(), ctypes.c_long()
    plugin_lib().ggml_backend_mi355x_graph_stats(ctypes.byref(c), ctypes.byref(r))
    return c.value, r.value


def p2p_stats() -> tuple[int, int]:
    """(stage hand-offs sent over RCCL send/recv, sent as hipMemcpyPeerAsync) since load."""
    r, p = ctypes.c_long(), ctypes.c_long()
    plugin_lib().ggml_backend_mi355x_p2p_stats(ctypes.byref(r), ctypes.byref(p))
    return r.value, p.value


def handoff_stats() -> tuple[int, int, int]:
    """(stage hand-offs over RCCL, as hipMemcpyPeerAsync, as a same-GPU async copy) since load."""
    r, p, d = ctypes.c_long(), ctypes.c_long(), ctypes.c_long()
    plugin_lib().ggml_backend_mi355x_handoff_stats(ctypes.byref(r), ctypes.byref(p), ctypes.byref(d))
    return r.value, p.value, d.value


def split_stats() -> tuple[int, int]:
    """(row-split mat-muls executed, slices of them computed on another GPU) since load."""
    m, f = ctypes.c_long(), ctypes.c_long()
    plugin_lib().ggml_backend_mi355x_split_stats(ctypes.byref(m), ctypes.byref(f))
    return m.value, f.value


def hbm_read_gbs(device: int = 0) -> float:
    """Measured HBM read ceiling of a device, GB/s (k_stream.hip)."""
    lib = plugin_lib()
    lib.ggml_backend_mi355x_hbm_read_gbs.restype = ctypes.c_double
    lib.ggml_backend_mi355x_hbm_read_gbs.argtypes = [ctypes.c_int]
    return float(lib.ggml_backend_mi355x_hbm_read_gbs(device))


def kernel_timing(lib: ctypes.CDLL, kind: int) -> tuple[float, float, int]:
    ms, by, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_long()
    lib.ggml_backend_mi355x_get_timing(kind, ctypes.byref(ms), ctypes.byref(by), ctypes.byref(n))
    return ms.value, by.value, n.value


_llb = None


def llb(echo_log: bool = False, with_plugin: bool = True) -> ctypes.CDLL:
    """Load libllb (and through it libllama, the CPU backend and — unless with_plugin is
    False — the MI355X plugin).  Backends are registered once per process."""
    global _llb
    if _llb is not None:
        return _llb
    lib = ctypes.CDLL(_require(LLB, "libllb driver"), mode=ctypes.RTLD_GLOBAL)
    lib.llb_load_backends.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
    lib.llb_dev_name.restype = ctypes.c_char_p
    lib.llb_open.restype = ctypes.c_void_p
    lib.llb_open.argtypes = [ctypes.c_char_p, ctypes.c_ulonglong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int]
    lib.llb_dump_n.argtypes = [ctypes.c_void_p]
    lib.llb_dump_name.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.llb_dump_name.restype = ctypes.c_char_p
    lib.llb_dump_op.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.llb_dump_size.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.llb_dump_size.restype = ctypes.c_longlong
    lib.llb_dump_data.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
    lib.llb_dump_clear.argtypes = [ctypes.c_void_p]
    lib.llb_close.argtypes = [ctypes.c_void_p]
    lib.llb_clear.argtypes = [ctypes.c_void_p]
    lib.llb_n_vocab.argtypes = [ctypes.c_void_p]
    lib.llb_decode.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
    lib.llb_logits.argtypes = [ctypes.c_void_p]
    lib.llb_logits.restype = ctypes.POINTER(ctypes.c_float)
    lib.llb_time_prompt.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.llb_time_prompt.restype = ctypes.c_double
    lib.llb_time_gen.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.llb_time_gen.restype = ctypes.c_double
    lib.llb_time_gen_split.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_double)]
    lib.llb_time_gen_split.restype = ctypes.c_double
    lib.llb_greedy.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float)]
    lib.llb_log.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.llb_greedy_threads.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int,
                                       ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float)]
    plugin = _require(PLUGIN, "MI355X backend plugin").encode() if with_plugin else None
    n = lib.llb_load_backends(REFHOST.encode(), plugin, 1 if echo_log else 0)
    # n < 0: the plugin did not register (ggml_backend_score() == 0, i.e. no gfx950 GPU
    # visible).  CPU-only use stays possible; Model(gpu=True) then fails loudly.
    lib.plugin_loaded = n >= 0
    _llb = lib
    return lib


def devices(lib: ctypes.CDLL) -> list[tuple[int, str, int]]:
    return [(i, lib.llb_dev_name(i).decode(), lib.llb_dev_type(i)) for i in range(lib.llb_dev_count())]


def gpu_mask(lib: ctypes.CDLL, n: int | None = None) -> int:
    """Bit mask of MI355X devices in the ggml registry (type 1 = GGML_BACKEND_DEVICE_TYPE_GPU)."""
    idx = [i for i, name, t in devices(lib) if t == 1 and name.startswith("MI355X")]
    if n is not None:
        idx = idx[:n]
    m = 0
    for i in idx:
        m |= 1 << i
    return m


def log_tail(lib: ctypes.CDLL, cap: int = 1 << 16) -> str:
    buf = ctypes.create_string_buffer(cap)
    lib.llb_log(buf, cap)
    return buf.value.decode(errors="replace")


class Model:
    """A libllama model + context (llama_model_load_from_file / llama_init_from_model)."""

    def __init__(self, path: str, gpu: bool = True, n_ctx: int = 1024, flash_attn: bool = True, n_batch: int = 2048,
                 n_ubatch: int = 512, kv_type: str = "f16", n_threads: int = 8, n_gpus: int | None = None,
                 n_gpu_layers: int = 999, split_mode: int = 1, dump: bool = False):
        self.lib = llb()
        mask = gpu_mask(self.lib, n_gpus) if gpu else 0
        if gpu and mask == 0:
            raise BackendMissing("no MI355X device registered: the plugin did not load "
                                 f"(plugin_loaded={self.lib.plugin_loaded}); refusing to fall back to the CPU")
        kt = GGML_TYPE[kv_type]
        self.h = self.lib.llb_open(path.encode(), mask, n_gpu_layers, 1 if flash_attn else 0, n_ctx, n_batch, n_ubatch,
                                   kt, kt, n_threads, split_mode, 1 if dump else 0)
        if not self.h:
            raise RuntimeError(f"llama failed to load {path}:\n{log_tail(self.lib)}")
        self.n_vocab = self.lib.llb_n_vocab(self.h)

    def close(self):
        if self.h:
            self.lib.llb_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def clear(self):
        self.lib.llb_clear(self.h)

    def time_gen(self, n: int) -> float:
        t = self.lib.llb_time_gen(self.h, n)
        if t < 0:
            raise RuntimeError("llama_decode failed")
        return t

    def time_gen_split(self, n: int) -> tuple[float, float, float]:
        """test_gen with the host time split: (wall, inside llama_decode, inside llama_synchronize)."""
        td, ts = ctypes.c_double(), ctypes.c_double()
        t = self.lib.llb_time_gen_split(self.h, n, ctypes.byref(td), ctypes.byref(ts))
        if t < 0:
            raise RuntimeError("llama_decode failed")
        return t, td.value, ts.value

    def time_prompt(self, n: int) -> float:
        t = self.lib.llb_time_prompt(self.h, n)
        if t < 0:
            raise RuntimeError("llama_decode failed")
        return t

    def dumps(self):
        """[(name, op, f32 array)] of every node observed by the eval callback (dump=True)."""
        import numpy as np
        out = []
        for i in range(self.lib.llb_dump_n(self.h)):
            a = np.zeros(self.lib.llb_dump_size(self.h, i), dtype=np.float32)
            self.lib.llb_dump_data(self.h, i, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
            out.append((self.lib.llb_dump_name(self.h, i).decode(), self.lib.llb_dump_op(self.h, i), a))
        self.lib.llb_dump_clear(self.h)
        return out

    def decode(self, tokens: list[int]):
        """llama_decode of one batch; returns a copy of the last token's logits."""
        import numpy as np
        p = (ctypes.c_int32 * len(tokens))(*tokens)
        if self.lib.llb_decode(self.h, p, len(tokens)) != 0:
            raise RuntimeError("llama_decode failed")
        return np.ctypeslib.as_array(self.lib.llb_logits(self.h), shape=(self.n_vocab,)).copy()

    def greedy_threads(self, n_contexts: int, prompt: list[int], n_gen: int):
        """n_contexts extra contexts of this model greedy-decode `prompt` concurrently, one thread
        each (tests/test-thread-safety.cpp's pattern); returns ids [c][n_gen], logits [c][n_gen][V]"""
        import numpy as np
        p = (ctypes.c_int32 * len(prompt))(*prompt)
        ids = np.zeros((n_contexts, n_gen), dtype=np.int32)
        logits = np.zeros((n_contexts, n_gen, self.n_vocab), dtype=np.float32)
        r = self.lib.llb_greedy_threads(self.h, n_contexts, p, len(prompt), n_gen,
                                        ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                        logits.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        if r != 0:
            raise RuntimeError(f"threaded greedy decode failed ({r})")
        return ids, logits

    def greedy(self, prompt: list[int], n_gen: int, want_logits: bool = True):
        import numpy as np
        p = (ctypes.c_int32 * len(prompt))(*prompt)
        ids = np.zeros(n_gen, dtype=np.int32)
        logits = np.zeros((n_gen, self.n_vocab), dtype=np.float32) if want_logits else None
        r = self.lib.llb_greedy(self.h, p, len(prompt), n_gen, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                logits.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if want_logits else None)
        if r != 0:
            raise RuntimeError(f"greedy decode failed ({r})")
        return ids, logits
