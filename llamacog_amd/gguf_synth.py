"""Seeded synthetic GGUF models with the exact tensor shapes and quant mix of the
BASELINE.json configs (no network, no checkpoints: SURVEY.md §8(d) "Inputs").

The writer follows the GGUF v3 layout read by the reference loader
(ggml/src/gguf.cpp:319-480: magic, version, tensor/kv counts, KV pairs, tensor infos,
32-byte aligned data) and the LLaMA metadata keys of src/llama-arch.cpp.  Quant blocks
are written directly as random-but-valid blocks (fp16 super-block scales chosen so the
weights are ~N(0, 0.02^2) and zero-mean), which is what makes an 8B/70B model cheap to
create on the GPU box.  The quant type map reproduces llama_tensor_get_type for
LLAMA_FTYPE_MOSTLY_Q4_K_M / Q5_K_M / Q8_0 (src/llama-quant.cpp:178-420): attn_v and
ffn_down use Q6_K on the use_more_bits layers, output.weight is Q6_K.

The vocabulary is a synthetic SentencePiece ("llama") vocab: <unk>, <s>, </s>, the 256
byte tokens <0x00>..<0xFF> and filler pieces, padded to n_vocab.
"""
from __future__ import annotations

import argparse
import os
import struct
import sys
from dataclasses import dataclass, field

import numpy as np

GGUF_MAGIC = 0x46554747
GGUF_VERSION = 3
ALIGN = 32

# ggml_type ids (ggml/include/ggml.h:351-392)
F32, F16, Q4_0, Q8_0, Q4_K, Q5_K, Q6_K = 0, 1, 2, 8, 12, 13, 14
BLOCK = {F32: (1, 4), F16: (1, 2), Q4_0: (32, 18), Q8_0: (32, 34), Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210)}
TYPE_NAME = {F32: "f32", F16: "f16", Q4_0: "q4_0", Q8_0: "q8_0", Q4_K: "q4_K", Q5_K: "q5_K", Q6_K: "q6_K"}

# gguf value types
T_U8, T_I8, T_U16, T_I16, T_U32, T_I32, T_F32, T_BOOL, T_STR, T_ARR, T_U64, T_I64, T_F64 = range(13)

# llama_ftype (include/llama.h)
FTYPE = {"q8_0": 7, "q4_k_m": 15, "q5_k_m": 17, "q4_0": 2}


@dataclass
class ModelConfig:
    name: str
    n_embd: int
    n_layer: int
    n_head: int
    n_head_kv: int
    n_ff: int
    n_vocab: int
    ftype: str
    n_ctx_train: int = 8192
    rope_base: float = 500000.0
    rms_eps: float = 1e-5
    n_expert: int = 0
    n_expert_used: int = 0
    size_label: str = ""  # llama model type inference uses n_layer; kept for docs
    # the 70B rule of llama_tensor_get_type (src/llama-quant.cpp: LLM_TYPE_70B, 8 heads share each
    # attn_v: Q4_K -> Q5_K); a real 70B is recognised by its 80 layers, the 2-layer parity model
    # of the same shapes sets it explicitly
    v_q5k_70b: bool = False
    # router rows 2i + 1 equal to rows 2i (ffn_gate_inp): every token's expert probabilities come in
    # equal pairs, so the top-k ARGSORT meets ties (its exchange order decides which slot each
    # tied expert takes)
    router_ties: bool = False

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head


CONFIGS = {
    # BASELINE.json configs[0]: stories15M-shape, Q8_0 (CPU plumbing)
    "stories15m-q8_0": ModelConfig("stories15M-synthetic", 288, 6, 6, 6, 768, 32000, "q8_0", n_ctx_train=256,
                                   rope_base=10000.0),
    # configs[1], configs[2]: Llama-3-8B Q4_K_M
    "llama3-8b-q4km": ModelConfig("Llama-3-8B-synthetic", 4096, 32, 32, 8, 14336, 128256, "q4_k_m"),
    # configs[3]: Llama-3-70B Q4_K_M
    "llama3-70b-q4km": ModelConfig("Llama-3-70B-synthetic", 8192, 80, 64, 8, 28672, 128256, "q4_k_m", v_q5k_70b=True),
    # fast parity model: full Llama-3-70B layer shapes (8192 / 28672, 64 / 8 heads, Q5_K / Q6_K
    # attn_v), 2 layers: layer 0 the Q4_K / Q5_K mix, layer 1 the use_more_bits Q6_K one
    "llama3-70b-2l-q4km": ModelConfig("Llama-3-70B-2layer-synthetic", 8192, 2, 64, 8, 28672, 128256, "q4_k_m",
                                      v_q5k_70b=True),
    # configs[4]: Mixtral-8x7B Q5_K_M
    "mixtral-8x7b-q5km": ModelConfig("Mixtral-8x7B-synthetic", 4096, 32, 32, 8, 14336, 32000, "q5_k_m",
                                     n_ctx_train=32768, rope_base=1000000.0, n_expert=8, n_expert_used=2),
    # fast parity model: full Mixtral-8x7B layer shapes (4096 / 14336, 32 / 8 heads, 8 experts,
    # top-2, Q5_K_M with the Q8_0 attn_k / attn_v of llama-quant.cpp:300-311), 2 layers: layer 0
    # Q5_K experts, layer 1 the use_more_bits Q6_K ffn_down
    "mixtral-2l-q5km": ModelConfig("Mixtral-8x7B-2layer-synthetic", 4096, 2, 32, 8, 14336, 32000, "q5_k_m",
                                   n_ctx_train=32768, rope_base=1000000.0, n_expert=8, n_expert_used=2),
    # the same with tied router rows (the router's tie path)
    "mixtral-2l-ties-q5km": ModelConfig("Mixtral-8x7B-2layer-ties-synthetic", 4096, 2, 32, 8, 14336, 32000, "q5_k_m",
                                        n_ctx_train=32768, rope_base=1000000.0, n_expert=8, n_expert_used=2,
                                        router_ties=True),
    # fast parity models: full Llama-3-8B layer shapes, 2 layers
    "llama3-8b-2l-q4km": ModelConfig("Llama-3-8B-2layer-synthetic", 4096, 2, 32, 8, 14336, 128256, "q4_k_m"),
    "llama3-8b-2l-q8_0": ModelConfig("Llama-3-8B-2layer-q8-synthetic", 4096, 2, 32, 8, 14336, 128256, "q8_0"),
    # small fast model with every weight type exercised (CPU tests)
    "tiny-q4km": ModelConfig("tiny-synthetic", 512, 4, 8, 2, 1024, 4096, "q4_k_m", n_ctx_train=2048),
    "tiny-q8_0": ModelConfig("tiny-q8-synthetic", 512, 4, 8, 2, 1024, 4096, "q8_0", n_ctx_train=2048),
    # small Mixtral-style MoE (4 experts, top-2), Q5_K_M
    "tiny-moe-q5km": ModelConfig("tiny-moe-synthetic", 512, 4, 8, 2, 1024, 4096, "q5_k_m", n_ctx_train=2048,
                                 n_expert=4, n_expert_used=2),
    "tiny-moe-ties-q5km": ModelConfig("tiny-moe-ties-synthetic", 512, 4, 8, 2, 1024, 4096, "q5_k_m", n_ctx_train=2048,
                                      n_expert=4, n_expert_used=2, router_ties=True),
}


def use_more_bits(i: int, n: int) -> bool:
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def tensor_types(cfg: ModelConfig) -> list[tuple[str, list[int], int]]:
    """(name, ne, type) in load order; mirrors llama_tensor_get_type for the ftype."""
    E, F, V, L = cfg.n_embd, cfg.n_ff, cfg.n_vocab, cfg.n_layer
    kv = cfg.head_dim * cfg.n_head_kv
    ft = cfg.ftype
    if ft == "q8_0":
        base, out_t, emb_t = Q8_0, Q8_0, Q8_0
    elif ft == "q4_0":
        base, out_t, emb_t = Q4_0, Q6_K, Q4_0
    elif ft == "q4_k_m":
        base, out_t, emb_t = Q4_K, Q6_K, Q4_K
    elif ft == "q5_k_m":
        base, out_t, emb_t = Q5_K, Q6_K, Q5_K
    else:
        raise ValueError(ft)
    if E % 256 != 0 and base in (Q4_K, Q5_K, Q6_K):
        base, out_t, emb_t = Q8_0, Q8_0, Q8_0
    out = [("token_embd.weight", [E, V], emb_t), ("output_norm.weight", [E], F32), ("output.weight", [E, V], out_t)]
    is70b = L == 80 or cfg.v_q5k_70b
    for i in range(L):
        more = use_more_bits(i, L)
        if ft in ("q4_k_m", "q5_k_m"):
            v_t = Q6_K if more else base
            d_t = Q6_K if more else base
            if is70b and v_t in (Q4_K,):
                v_t = Q5_K
        else:
            v_t, d_t = base, base
        k_t = base
        if cfg.n_expert == 8 and ft != "q8_0":
            v_t, k_t = Q8_0, Q8_0  # Mixtral attn_k/attn_v (llama-quant.cpp:300-311)
        p = f"blk.{i}."
        out += [
            (p + "attn_norm.weight", [E], F32),
            (p + "attn_q.weight", [E, E], base),
            (p + "attn_k.weight", [E, kv], k_t),
            (p + "attn_v.weight", [E, kv], v_t),
            (p + "attn_output.weight", [E, E], base),
            (p + "ffn_norm.weight", [E], F32),
        ]
        if cfg.n_expert:
            X = cfg.n_expert
            out += [
                (p + "ffn_gate_inp.weight", [E, X], F32),
                (p + "ffn_gate_exps.weight", [E, F, X], base),
                (p + "ffn_down_exps.weight", [F, E, X], d_t),
                (p + "ffn_up_exps.weight", [E, F, X], base),
            ]
        else:
            out += [
                (p + "ffn_gate.weight", [E, F], base),
                (p + "ffn_down.weight", [F, E], d_t),
                (p + "ffn_up.weight", [E, F], base),
            ]
    return out


def nbytes(ne: list[int], t: int) -> int:
    blk, bs = BLOCK[t]
    n = int(np.prod(ne))
    assert ne[0] % blk == 0
    return n // blk * bs


# ---- random-but-valid quant blocks -----------------------------------------------------------
def _f16(rng, n, base):
    return (base * rng.uniform(0.75, 1.25, n)).astype(np.float16)


def _pack_k4_scales(sc: np.ndarray, m: np.ndarray) -> np.ndarray:
    """Inverse of get_scale_min_k4 (ggml-quants.c:625): 8 (scale, min) 6-bit pairs -> 12 bytes."""
    n = sc.shape[0]
    q = np.zeros((n, 12), dtype=np.uint8)
    sc = sc.astype(np.uint8)
    m = m.astype(np.uint8)
    q[:, 0:4] = (sc[:, 0:4] & 63) | ((sc[:, 4:8] >> 4) << 6)
    q[:, 4:8] = (m[:, 0:4] & 63) | ((m[:, 4:8] >> 4) << 6)
    q[:, 8:12] = (sc[:, 4:8] & 0xF) | ((m[:, 4:8] & 0xF) << 4)
    return q


def make_blocks(t: int, nblk: int, rng: np.random.Generator) -> np.ndarray:
    blk, bs = BLOCK[t]
    raw = rng.integers(0, 256, size=nblk * bs, dtype=np.uint8).reshape(nblk, bs)
    if t == Q4_0:
        raw[:, 0:2] = _f16(rng, nblk, 4.3e-3).view(np.uint8).reshape(nblk, 2)
    elif t == Q8_0:
        raw[:, 0:2] = _f16(rng, nblk, 2.7e-4).view(np.uint8).reshape(nblk, 2)
        qs = raw[:, 2:].view(np.int8)
        qs[qs == -128] = -127
    elif t in (Q4_K, Q5_K):
        d = _f16(rng, nblk, 8.5e-4 if t == Q4_K else 8.0e-4)
        raw[:, 0:2] = d.view(np.uint8).reshape(nblk, 2)
        raw[:, 2:4] = d.view(np.uint8).reshape(nblk, 2)  # dmin = d -> zero-mean weights
        hi = 9 if t == Q4_K else 5
        mid = 7.5 if t == Q4_K else 15.5
        sc = rng.integers(1, hi, size=(nblk, 8))
        m = np.minimum(np.rint(sc * mid), 63).astype(np.int64)
        raw[:, 4:16] = _pack_k4_scales(sc, m)
    elif t == Q6_K:
        sc = rng.integers(-16, 17, size=(nblk, 16)).astype(np.int8)
        sc[sc == 0] = 1
        raw[:, 192:208] = sc.view(np.uint8)
        raw[:, 208:210] = _f16(rng, nblk, 1.1e-4).view(np.uint8).reshape(nblk, 2)
    elif t == F32:
        raise ValueError("f32 handled separately")
    return raw.reshape(-1)


def tensor_data(name: str, ne: list[int], t: int, rng: np.random.Generator) -> np.ndarray:
    if t == F32:
        n = int(np.prod(ne))
        if name.endswith("norm.weight"):
            return (1.0 + 0.05 * rng.standard_normal(n)).astype(np.float32).view(np.uint8)
        return (0.02 * rng.standard_normal(n)).astype(np.float32).view(np.uint8)
    blk, _ = BLOCK[t]
    return make_blocks(t, int(np.prod(ne)) // blk, rng)


# ---- GGUF serialisation -------------------------------------------------------------------------
def _s(x: str) -> bytes:
    b = x.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def _kv(key: str, vtype: int, val) -> bytes:
    out = _s(key) + struct.pack("<I", vtype)
    if vtype == T_STR:
        out += _s(val)
    elif vtype == T_U32:
        out += struct.pack("<I", val)
    elif vtype == T_I32:
        out += struct.pack("<i", val)
    elif vtype == T_F32:
        out += struct.pack("<f", val)
    elif vtype == T_BOOL:
        out += struct.pack("<?", val)
    elif vtype == T_ARR:
        etype, items = val
        out += struct.pack("<IQ", etype, len(items))
        if etype == T_STR:
            out += b"".join(_s(x) for x in items)
        elif etype == T_F32:
            out += np.asarray(items, dtype=np.float32).tobytes()
        elif etype == T_I32:
            out += np.asarray(items, dtype=np.int32).tobytes()
        else:
            raise ValueError(etype)
    else:
        raise ValueError(vtype)
    return out


def vocab(n_vocab: int):
    toks = ["<unk>", "<s>", "</s>"] + [f"<0x{i:02X}>" for i in range(256)]
    types = [2, 3, 3] + [6] * 256
    i = 0
    while len(toks) < n_vocab:
        toks.append(f"▁t{i}")
        types.append(1)
        i += 1
    scores = [0.0] * 259 + [-float(k) for k in range(n_vocab - 259)]
    return toks[:n_vocab], scores[:n_vocab], types[:n_vocab]


def metadata(cfg: ModelConfig) -> list[bytes]:
    a = "llama"
    kvs = [
        _kv("general.architecture", T_STR, a),
        _kv("general.name", T_STR, cfg.name),
        _kv("general.file_type", T_U32, FTYPE[cfg.ftype]),
        _kv("general.alignment", T_U32, ALIGN),
        _kv(f"{a}.context_length", T_U32, cfg.n_ctx_train),
        _kv(f"{a}.embedding_length", T_U32, cfg.n_embd),
        _kv(f"{a}.block_count", T_U32, cfg.n_layer),
        _kv(f"{a}.feed_forward_length", T_U32, cfg.n_ff),
        _kv(f"{a}.attention.head_count", T_U32, cfg.n_head),
        _kv(f"{a}.attention.head_count_kv", T_U32, cfg.n_head_kv),
        _kv(f"{a}.rope.freq_base", T_F32, cfg.rope_base),
        _kv(f"{a}.attention.layer_norm_rms_epsilon", T_F32, cfg.rms_eps),
        _kv(f"{a}.rope.dimension_count", T_U32, cfg.head_dim),
        _kv(f"{a}.vocab_size", T_U32, cfg.n_vocab),
    ]
    if cfg.n_expert:
        kvs += [_kv(f"{a}.expert_count", T_U32, cfg.n_expert), _kv(f"{a}.expert_used_count", T_U32, cfg.n_expert_used)]
    toks, scores, types = vocab(cfg.n_vocab)
    kvs += [
        _kv("tokenizer.ggml.model", T_STR, "llama"),
        _kv("tokenizer.ggml.tokens", T_ARR, (T_STR, toks)),
        _kv("tokenizer.ggml.scores", T_ARR, (T_F32, scores)),
        _kv("tokenizer.ggml.token_type", T_ARR, (T_I32, types)),
        _kv("tokenizer.ggml.bos_token_id", T_U32, 1),
        _kv("tokenizer.ggml.eos_token_id", T_U32, 2),
        _kv("tokenizer.ggml.unknown_token_id", T_U32, 0),
        _kv("tokenizer.ggml.add_bos_token", T_BOOL, True),
    ]
    return kvs


def write_gguf(cfg: ModelConfig, path: str, seed: int = 0, n_layer: int | None = None, verbose: bool = False) -> str:
    if n_layer is not None:
        cfg = ModelConfig(**{**cfg.__dict__, "n_layer": n_layer})
    tensors = tensor_types(cfg)
    kvs = metadata(cfg)
    infos = []
    off = 0
    for name, ne, t in tensors:
        infos.append(_s(name) + struct.pack("<I", len(ne)) + struct.pack(f"<{len(ne)}Q", *ne) + struct.pack("<IQ", t, off))
        off += (nbytes(ne, t) + ALIGN - 1) // ALIGN * ALIGN
    header = struct.pack("<IIQQ", GGUF_MAGIC, GGUF_VERSION, len(tensors), len(kvs)) + b"".join(kvs) + b"".join(infos)
    pad = (-len(header)) % ALIGN
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(tmp, "wb") as f:
        f.write(header + b"\0" * pad)
        for idx, (name, ne, t) in enumerate(tensors):
            # per-tensor seed: files are identical regardless of which tensors were generated
            rng = np.random.default_rng([seed, idx])
            data = tensor_data(name, ne, t, rng)
            if cfg.router_ties and name.endswith("ffn_gate_inp.weight"):
                rows = data.view(np.float32).reshape(ne[1], ne[0])
                rows[1::2] = rows[0::2]
            assert data.nbytes == nbytes(ne, t), (name, data.nbytes, nbytes(ne, t))
            f.write(data.tobytes())
            f.write(b"\0" * ((-data.nbytes) % ALIGN))
            if verbose:
                print(f"  {name:32s} {TYPE_NAME[t]:5s} {ne}", file=sys.stderr)
    os.replace(tmp, path)
    return path


def weight_bytes_per_token(cfg: ModelConfig) -> int:
    """Algorithmic weight bytes streamed by one decode step: every layer matmul plus the
    output head; the token embedding GET_ROWS runs on the CPU (src/llama-model.cpp:1572)."""
    tot = 0
    for name, ne, t in tensor_types(cfg):
        if name == "token_embd.weight" or t == F32:
            continue
        if "_exps." in name:
            tot += nbytes(ne, t) * cfg.n_expert_used // cfg.n_expert
        else:
            tot += nbytes(ne, t)
    return tot


def model_path(config: str, seed: int = 0, n_layer: int | None = None) -> str:
    """Where ensure() keeps the synthetic GGUF of a config (LLAMACOG_MODEL_DIR, default /tmp)."""
    root = os.environ.get("LLAMACOG_MODEL_DIR", "/tmp/llamacog_amd_models")
    suffix = f"-{n_layer}l" if n_layer else ""
    return os.path.join(root, f"{config}{suffix}-s{seed}.gguf")


def ensure(config: str, path: str | None = None, seed: int = 0, n_layer: int | None = None) -> str:
    cfg = CONFIGS[config]
    if path is None:
        path = model_path(config, seed, n_layer)
    if not os.path.exists(path):
        write_gguf(cfg, path, seed=seed, n_layer=n_layer)
    return path


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config", default="llama3-8b-q4km", choices=sorted(CONFIGS))
    ap.add_argument("--out", required=True)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    write_gguf(CONFIGS[a.config], a.out, seed=a.seed, n_layer=a.layers, verbose=a.verbose)
    print(a.out)


if __name__ == "__main__":
    main()
