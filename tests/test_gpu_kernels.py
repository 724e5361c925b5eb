"""GPU parity of the HIP kernels through the C ABI (include/ggml-mi355x.h) against the
golden vectors of the reference CPU backend and the oracle restatement.

Tolerances (all stated here):
  * activation quantizers, mul_mat (mat-vec, batched mat-vec, MFMA prefill), mul_mat_id,
    rms_norm, rope, SiLU: BIT-EXACT — the kernels reproduce the x86-64-v4 CPU backend's integer
    sums and its fp32 combination order as libllama runs it (repacked Q4_K / Q4_0, vec_dot
    class chains, tinyBLAS; qtypes.h), and glibc's expf / sinf / cosf (libm_exact.h);
  * f16 flash-attention (exact kernel): bit-exact;
  * q8_0 flash-attention (split-K f32 kernel): < 1e-5 relative.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import _oracle as O


@pytest.fixture(scope="module")
def K():
    from llamacog_amd import kernels
    kernels.lib()
    return kernels


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


@pytest.mark.parametrize("vdt", [O.Q8_K, O.Q8_0])
def test_activation_quantizers_bit_exact(K, golden_dir, vdt):
    g = load(golden_dir, "quant_act.npz")
    x = g["x"]
    qs, d, s = K.quantize_rows(vdt, x)
    rq, rd, rs = O.split_q8(vdt, g["q8_K" if vdt == O.Q8_K else "q8_0"], x.shape[1])
    assert (qs == rq).all()
    assert (d.view(np.uint32) == rd.view(np.uint32)).all()
    assert (s == rs).all()


@pytest.mark.parametrize("vdt", [O.Q8_K, O.Q8_0])
def test_activation_quantizers_large_random(K, vdt):
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((33, 14336)) * rng.uniform(1e-3, 50, (33, 1))).astype(np.float32)
    x[3, :512] = 0.0
    qs, d, s = K.quantize_rows(vdt, x)
    rq, rd, rs = O.split_q8(vdt, O.quantize_rows(vdt, x), x.shape[1])
    assert (qs == rq).all() and (d.view(np.uint32) == rd.view(np.uint32)).all() and (s == rs).all()


def bits_equal(a, b):
    return (np.ascontiguousarray(a).view(np.uint32) == np.ascontiguousarray(b).view(np.uint32))


def assert_bits(y, ref, what):
    eq = bits_equal(y, ref)
    if not eq.all():
        bad = np.argwhere(~eq)
        i = tuple(bad[0])
        raise AssertionError(f"{what}: {len(bad)} of {eq.size} outputs differ; first {i}: {y[i]!r} vs {ref[i]!r}, "
                             f"max rel {np.abs(y - ref).max() / (np.abs(ref).max() + 1e-30):.2e}")


CPU_TYPES = {"q4_K": O.Q4_K, "q6_K": O.Q6_K, "q5_K": O.Q5_K, "q8_0": O.Q8_0, "q4_0": O.Q4_0, "f32": O.F32}


@pytest.mark.parametrize("name", sorted(CPU_TYPES))
def test_mul_mat_cpu_golden_bit_exact(K, golden_dir, name):
    """mul_mat vs the reference CPU backend as libllama runs it (tests/golden/mul_mat_cpu.npz:
    repacked Q4_K / Q4_0 gemv + gemm, vec_dot class chains, tinyBLAS f32): bit for bit."""
    g = load(golden_dir, "mul_mat_cpu.npz")
    wq = g[f"wq_{name}"]
    for T in (1, 3, 4, 9):
        x, ref = g[f"x_{name}_{T}"], g[f"y_{name}_{T}"]
        y = K.mul_mat(CPU_TYPES[name], wq, x.shape[1], ref.shape[1], x)
        assert_bits(y, ref, f"{name} T={T}")


@pytest.mark.parametrize("name,Kd,M", [("q4_K", 4096, 1024), ("q6_K", 14336, 256), ("q4_K", 14336, 256),
                                        ("q5_K", 4096, 512), ("q8_0", 4096, 512), ("q4_0", 4096, 512),
                                        ("q6_K", 4096, 4096), ("q4_K", 4096, 1020), ("q4_0", 2048, 300),
                                        ("q8_0", 8192, 96)])
def test_mul_mat_llama_shapes_bit_exact(K, name, Kd, M):
    """Full Llama-3-8B row lengths (K 4096 / 14336) with random-but-valid blocks, decode and
    small batches, M % 8 != 0 (not repacked: vec_dot order) included: bit-exact vs the oracle."""
    from llamacog_amd import gguf_synth as gs
    t = CPU_TYPES[name]
    rng = np.random.default_rng(11)
    blk, bs = gs.BLOCK[t]
    wq = gs.make_blocks(t, M * Kd // blk, rng).reshape(M, -1)
    for T in (1, 3, 4, 8, 17):
        x = rng.standard_normal((T, Kd)).astype(np.float32)
        assert_bits(K.mul_mat(t, wq, Kd, M, x), O.mul_mat_cpu(t, wq, Kd, M, x), f"{name} {Kd}x{M} T={T}")


def test_rms_norm_and_fused_mul(K, golden_dir):
    g = load(golden_dir, "rms_norm.npz")
    y = K.rms_norm(g["x"], float(g["eps"]))
    assert_bits(y, g["y"], "rms_norm")
    w = np.linspace(0.5, 1.5, g["x"].shape[1]).astype(np.float32)
    y2, ym = K.rms_norm(g["x"], float(g["eps"]), w)
    assert (y2.view(np.uint32) == y.view(np.uint32)).all()
    assert (ym.view(np.uint32) == (y * w).astype(np.float32).view(np.uint32)).all()


def test_rope_golden(K, golden_dir):
    g = load(golden_dir, "rope.npz")
    for i in range(len(g["modes"])):
        y = K.rope(g["x"], g["pos"], 128, int(g["modes"][i]), float(g["bases"][i]),
                   ff=g["ff"] if g["use_ff"][i] else None)
        # glibc cosf / sinf restated bit for bit (libm_exact.h)
        assert_bits(y, g["y"][i], f"rope case {i}")


def test_soft_max_golden(K, golden_dir):
    g = load(golden_dir, "soft_max.npz")
    y = K.soft_max(g["x"], g["mask"], float(g["scale"]))
    assert (y.view(np.uint32) == g["y"].view(np.uint32)).mean() > 0.999
    assert np.abs(y - g["y"]).max() < 1e-7


def test_silu_matches_avx512_restatement(K):
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((4, 14336 + 7)) * 4).astype(np.float32)
    x[0, :8] = [0.0, -0.0, 88.0, -88.0, 1e-30, -104.0, 30.0, -30.0]
    y = K.silu(x)
    ref = O.silu(x)
    # ggml_v_silu on 16-element chunks, glibc expf (libm_exact.h) on the tail: bit-exact
    assert_bits(y, ref, "silu")


@pytest.mark.parametrize("n_q", [1, 7])
def test_flash_attn_f16_golden(K, golden_dir, n_q):
    g = load(golden_dir, "flash_attn.npz")
    D, H, Hkv, n_kv = int(g["D"]), int(g["H"]), int(g["Hkv"]), int(g["n_kv"])
    out = K.flash_attn(g[f"q_{n_q}"], g[f"k_f16_{n_q}"], g[f"v_f16_{n_q}"], g[f"mask_{n_q}"], O.F16, D, H, Hkv, n_kv,
                       1.0 / np.sqrt(D))
    assert_bits(out, g[f"out_f16_{n_q}"], f"flash_attn f16 n_q={n_q}")


@pytest.mark.parametrize("n_q", [1, 7])
def test_flash_attn_q8_0_golden(K, golden_dir, n_q):
    """q8_0 KV cache: Q quantized to q8_0, vec_dot_q8_0_q8_0 class chains, f32 VKQ: bit-exact."""
    g = load(golden_dir, "flash_attn.npz")
    D, H, Hkv, n_kv = int(g["D"]), int(g["H"]), int(g["Hkv"]), int(g["n_kv"])
    out = K.flash_attn(g[f"q_{n_q}"], g[f"k_q8_0_{n_q}"], g[f"v_q8_0_{n_q}"], g[f"mask_{n_q}"], O.Q8_0, D, H, Hkv, n_kv,
                       1.0 / np.sqrt(D))
    assert_bits(out, g[f"out_q8_0_{n_q}"], f"flash_attn q8_0 n_q={n_q}")


@pytest.mark.parametrize("tag", ["1", "7", "long"])
@pytest.mark.parametrize("kv", ["f16", "q8_0", "q4_0"])
def test_flash_attn_golden_all_kv(K, golden_dir, tag, kv):
    """Every KV type against the reference CPU backend's own outputs, including a depth-1300 decode
    (the long-context pair: scores grid + per-head chain, one KV head so its rows are contiguous)."""
    g = load(golden_dir, "flash_attn.npz")
    sfx = "_long" if tag == "long" else ""
    D, H, Hkv, n_kv = int(g["D"]), int(g["H" + sfx]), int(g["Hkv" + sfx]), int(g["n_kv" + sfx])
    kvt = {"f16": O.F16, "q8_0": O.Q8_0, "q4_0": O.Q4_0}[kv]
    out = K.flash_attn(g[f"q_{tag}"], g[f"k_{kv}_{tag}"], g[f"v_{kv}_{tag}"], g[f"mask_{tag}"], kvt, D, H, Hkv, n_kv,
                       1.0 / np.sqrt(D))
    assert_bits(out, g[f"out_{kv}_{tag}"], f"flash_attn {kv} {tag}")


@pytest.mark.parametrize("kv,n_kv,Hkv,G,pattern", [("q8_0", 2500, 8, 4, "holes"), ("q4_0", 1300, 8, 4, "causal"),
                                                   ("q4_0", 4100, 2, 8, "sparse"), ("q8_0", 1024, 1, 8, "causal"),
                                                   ("q8_0", 8192, 8, 4, "causal"), ("q4_0", 600, 8, 4, "holes")])
def test_flash_attn_quant_long_vs_oracle(K, kv, n_kv, Hkv, G, pattern):
    """Quantized caches at depth through the long-context pair: interleaved heads (the llama cache
    view: rows a dword a lane into LDS) and a single KV head (contiguous rows), ragged last chunk,
    the longest cache the chain takes (8192), and a short one past the quantized threshold (384)."""
    rng = np.random.default_rng(n_kv + Hkv)
    D, H = 128, Hkv * G
    kvt = O.Q8_0 if kv == "q8_0" else O.Q4_0
    q = (rng.standard_normal((1, H, D)) * 2).astype(np.float32)
    k = O.quantize_rows(kvt, rng.standard_normal((n_kv * Hkv, D)).astype(np.float32)).reshape(n_kv, -1)
    v = O.quantize_rows(kvt, rng.standard_normal((n_kv * Hkv, D)).astype(np.float32)).reshape(n_kv, -1)
    m = np.zeros((1, n_kv), dtype=np.float16)
    if pattern == "holes":
        m[0, rng.random(n_kv) < 0.3] = -np.inf
    elif pattern == "sparse":
        m[0, rng.random(n_kv) < 0.9] = -np.inf
        m[0, -1] = 0
    out = K.flash_attn(q, k, v, m.view(np.uint16), kvt, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    ref = O.flash_attn(q, k, v, m.view(np.uint16), kvt, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    assert_bits(out, ref, f"flash_attn {kv} n_kv={n_kv} Hkv={Hkv} {pattern}")


@pytest.mark.parametrize("n_kv,n_q", [(256, 1), (1024, 1), (700, 9), (512, 64)])
def test_flash_attn_q8_0_llama_shapes_bit_exact(K, n_kv, n_q):
    """q8_0 cache at Llama-3-8B head layout (D 128, 32 / 8 heads), causal mask, vs the oracle."""
    rng = np.random.default_rng(n_kv + 3 * n_q)
    D, H, Hkv = 128, 32, 8
    q = rng.standard_normal((n_q, H, D)).astype(np.float32)
    kf = rng.standard_normal((n_kv * Hkv, D)).astype(np.float32)
    vf = rng.standard_normal((n_kv * Hkv, D)).astype(np.float32)
    k = O.quantize_rows(O.Q8_0, kf).reshape(n_kv, -1)
    v = O.quantize_rows(O.Q8_0, vf).reshape(n_kv, -1)
    m = np.zeros((n_q, n_kv), dtype=np.float16)
    for r in range(n_q):
        m[r, n_kv - n_q + r + 1:] = -np.inf
    out = K.flash_attn(q, k, v, m.view(np.uint16), O.Q8_0, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    ref = O.flash_attn(q, k, v, m.view(np.uint16), O.Q8_0, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    assert_bits(out, ref, f"flash_attn q8_0 n_kv={n_kv} n_q={n_q}")


@pytest.mark.parametrize("n_kv,n_q,Hkv,G", [(256, 1, 8, 4), (1024, 1, 8, 4), (4096, 1, 8, 8), (512, 32, 8, 4),
                                           (300, 5, 2, 1)])
def test_flash_attn_f16_llama_shapes_vs_oracle(K, n_kv, n_q, Hkv, G):
    rng = np.random.default_rng(n_kv + n_q)
    D, H = 128, Hkv * G
    q = rng.standard_normal((n_q, H, D)).astype(np.float32)
    k = rng.standard_normal((n_kv, Hkv, D)).astype(np.float16)
    v = rng.standard_normal((n_kv, Hkv, D)).astype(np.float16)
    m = np.zeros((n_q, n_kv), dtype=np.float16)
    for r in range(n_q):
        m[r, n_kv - n_q + r + 1:] = -np.inf   # causal tail like llama's KQ mask
    out = K.flash_attn(q, k.view(np.uint8), v.view(np.uint8), m.view(np.uint16), O.F16, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    ref = O.flash_attn(q, k.view(np.uint8), v.view(np.uint8), m.view(np.uint16), O.F16, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    assert_bits(out, ref, f"flash_attn f16 n_kv={n_kv} n_q={n_q}")


def test_buffer_from_host_ptr_matvec_bit_exact():
    """The device's buffer_from_host_ptr (hipHostRegister'd, mapped host memory): the decode
    mat-vec reads q4_K weights in place over the host link and returns the same bits as with the
    weights in HBM."""
    import ctypes
    import llamacog_amd as la
    from llamacog_amd import gguf_synth as gs
    rng = np.random.default_rng(3)
    K, M = 4096, 256
    blk, bs = gs.BLOCK[CPU_TYPES["q4_K"]]
    w = gs.make_blocks(CPU_TYPES["q4_K"], M * K // blk, rng)
    x = rng.standard_normal(K).astype(np.float32)
    lib = la.plugin_lib()
    f = lib.mi355x_check_host_ptr_matvec
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p]
    wb = np.ascontiguousarray(w)
    assert f(wb.ctypes.data, K, M, x.ctypes.data) == 0


@pytest.mark.parametrize("n_kv,Hkv,G,pattern", [(300, 4, 1, "holes"), (1000, 8, 2, "first_chunk_dead"),
                                                  (256, 8, 4, "single"), (129, 2, 4, "holes"), (4352, 8, 4, "sparse"),
                                                  (2000, 8, 2, "first_chunk_dead"), (1300, 2, 4, "single"),
                                                  (5000, 8, 4, "holes"), (8192, 8, 4, "sparse"), (800, 8, 4, "holes"),
                                                  (520, 8, 4, "holes")])
def test_flash_attn_f16_decode_masks_vs_oracle(K, n_kv, Hkv, G, pattern):
    """Decode (one query row) over masks the causal tail does not exercise: dead positions inside
    a batch, a whole dead chunk, a single live position, one position past a chunk boundary, and
    a sparse mask at depth; heads without GQA sharing (G = 1: two KV heads per head pair)."""
    rng = np.random.default_rng(n_kv * 7 + G)
    D, H = 128, Hkv * G
    q = (rng.standard_normal((1, H, D)) * 2).astype(np.float32)
    k = rng.standard_normal((n_kv, Hkv, D)).astype(np.float16)
    v = rng.standard_normal((n_kv, Hkv, D)).astype(np.float16)
    m = np.zeros((1, n_kv), dtype=np.float16)
    if pattern == "holes":
        m[0, rng.random(n_kv) < 0.3] = -np.inf
    elif pattern == "first_chunk_dead":
        m[0, :128] = -np.inf
        m[0, 500:517] = -np.inf
    elif pattern == "single":
        m[0, :] = -np.inf
        m[0, 77] = 0
    else:
        m[0, rng.random(n_kv) < 0.9] = -np.inf
        m[0, -1] = 0
    out = K.flash_attn(q, k.view(np.uint8), v.view(np.uint8), m.view(np.uint16), O.F16, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    ref = O.flash_attn(q, k.view(np.uint8), v.view(np.uint8), m.view(np.uint16), O.F16, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    assert_bits(out, ref, f"flash_attn f16 decode {pattern} n_kv={n_kv} G={G}")


@pytest.mark.parametrize("n_kv,live,pattern", [(256, 9, "tail"), (256, 136, "tail"), (256, 129, "holes"),
                                               (256, 256, "increasing"), (128, 100, "tail"), (64, 64, "increasing"),
                                               (200, 137, "holes"), (1, 1, "tail"), (7, 3, "single"), (256, 250, "sparse")])
def test_flash_attn_f16_decode_short_vs_oracle(K, n_kv, live, pattern):
    """The short-context decode kernel (k_fattn_dsh: at most 256 cached positions, tg128's depths):
    libllama's padded cache (live positions then -inf up to n_kv, a multiple of 256 in the graph),
    holes and a lone live position inside batches, a single-position cache, and scores rising at
    every position so the running max updates on every step (every batch takes the general step)."""
    rng = np.random.default_rng(n_kv * 13 + live)
    D, Hkv, G = 128, 8, 4
    H = Hkv * G
    q = (rng.standard_normal((1, H, D)) * 2).astype(np.float32)
    kf = rng.standard_normal((n_kv, Hkv, D)).astype(np.float32)
    if pattern == "increasing":
        # K row j leans on the group's first query head more and more: its score rises with j
        for hk in range(Hkv):
            qd = q[0, hk * G] / np.linalg.norm(q[0, hk * G])
            kf[:, hk, :] = 0.005 * kf[:, hk, :] + np.arange(n_kv, dtype=np.float32)[:, None] * 0.05 * qd[None, :]
    k = kf.astype(np.float16)
    v = rng.standard_normal((n_kv, Hkv, D)).astype(np.float16)
    m = np.zeros((1, n_kv), dtype=np.float16)
    m[0, live:] = -np.inf
    if pattern == "holes":
        m[0, :live][rng.random(live) < 0.3] = -np.inf
        m[0, live - 1] = 0
    elif pattern == "single":
        m[0, :] = -np.inf
        m[0, live - 1] = 0
    elif pattern == "sparse":
        m[0, :live][rng.random(live) < 0.9] = -np.inf
        m[0, 0] = 0
    out = K.flash_attn(q, k.view(np.uint8), v.view(np.uint8), m.view(np.uint16), O.F16, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    ref = O.flash_attn(q, k.view(np.uint8), v.view(np.uint8), m.view(np.uint16), O.F16, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    assert_bits(out, ref, f"flash_attn f16 short decode {pattern} n_kv={n_kv} live={live}")


@pytest.mark.parametrize("n_kv,n_q,Hkv,G,pattern", [(300, 37, 2, 4, "holes"), (200, 16, 4, 1, "causal"),
                                                    (130, 23, 2, 2, "sparse"), (1000, 64, 8, 8, "causal"),
                                                    (64, 40, 1, 16, "dead_prefix"), (97, 33, 2, 4, "increasing"),
                                                    (515, 48, 8, 4, "holes")])
def test_flash_attn_f16_prefill_masks_vs_oracle(K, n_kv, n_q, Hkv, G, pattern):
    """The prefill tile (k_fattn_pf, a batch of >= 16 query rows: 32-position chunks, two pairs per
    scoring quad and per coefficient pass): every GQA group size, row counts that leave a partial
    workgroup, cache lengths off the chunk grid, and masks beyond the causal tail — holes, a sparse
    mask, a dead prefix, and scores rising with the position (a running-max update at every step)."""
    rng = np.random.default_rng(n_kv * 31 + n_q * 7 + G)
    D, H = 128, Hkv * G
    q = (rng.standard_normal((n_q, H, D)) * 2).astype(np.float32)
    kf = rng.standard_normal((n_kv, Hkv, D)).astype(np.float32)
    if pattern == "increasing":
        for hk in range(Hkv):
            qd = q[0, hk * G] / np.linalg.norm(q[0, hk * G])
            kf[:, hk, :] = 0.005 * kf[:, hk, :] + np.arange(n_kv, dtype=np.float32)[:, None] * 0.05 * qd[None, :]
    k = kf.astype(np.float16)
    v = rng.standard_normal((n_kv, Hkv, D)).astype(np.float16)
    m = np.zeros((n_q, n_kv), dtype=np.float16)
    for r in range(n_q):
        last = n_kv - n_q + r
        m[r, last + 1:] = -np.inf
        if pattern == "holes":
            m[r, :last][rng.random(last) < 0.3] = -np.inf
        elif pattern == "sparse":
            m[r, :last][rng.random(last) < 0.9] = -np.inf
        elif pattern == "dead_prefix":
            m[r, :min(40, last)] = -np.inf
    out = K.flash_attn(q, k.view(np.uint8), v.view(np.uint8), m.view(np.uint16), O.F16, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    ref = O.flash_attn(q, k.view(np.uint8), v.view(np.uint8), m.view(np.uint16), O.F16, D, H, Hkv, n_kv, 1 / np.sqrt(D))
    assert_bits(out, ref, f"flash_attn f16 prefill {pattern} n_kv={n_kv} n_q={n_q} G={G}")


@pytest.mark.parametrize("name,Kd,M", [("q4_K", 4096, 256), ("q5_K", 4096, 200), ("q6_K", 4096, 136),
                                        ("q4_K", 14336, 128), ("q6_K", 14336, 64), ("q4_K", 4096, 100)])
def test_mul_mat_prefill_bit_exact(K, name, Kd, M):
    """Batched MUL_MAT (T >= 16: the MFMA tile for repacked Q4_K, gemm order for whole groups of
    four tokens and gemv order for the rest; the exact mat-vec for the other types): bit-exact."""
    from llamacog_amd import gguf_synth as gs
    t = CPU_TYPES[name]
    rng = np.random.default_rng(21)
    blk, bs = gs.BLOCK[t]
    wq = gs.make_blocks(t, M * Kd // blk, rng).reshape(M, -1)
    for T in (16, 64, 101, 512):
        if T == 512 and Kd * M > 4096 * 256:
            continue
        x = rng.standard_normal((T, Kd)).astype(np.float32)
        assert_bits(K.mul_mat(t, wq, Kd, M, x), O.mul_mat_cpu(t, wq, Kd, M, x), f"{name} {Kd}x{M} T={T}")


@pytest.mark.parametrize("name,Kd,M", [("q4_K", 4096, 14336), ("q6_K", 14336, 4096), ("q4_K", 14336, 4096),
                                        ("q4_K", 8192, 28672), ("q6_K", 28672, 8192)])
def test_mul_mat_prefill_full_llama_shapes_t512(K, name, Kd, M):
    """pp512's own launches at full Llama-3-8B / 70B matrix sizes (FFN gate/up 4096 x 14336, down
    14336 x 4096 in Q4_K and Q6_K, the 70B 8192 x 28672 and 28672 x 8192): the GPU computes every
    row for T = 512; the oracle checks the first 64, the last 64 and 16 groups of 8 spread between
    (rows are independent, so a row's bits do not depend on which others are computed)."""
    from llamacog_amd import gguf_synth as gs
    t = CPU_TYPES[name]
    rng = np.random.default_rng(Kd + M)
    blk, bs = gs.BLOCK[t]
    wq = gs.make_blocks(t, M * Kd // blk, rng).reshape(M, -1)
    T = 512
    x = rng.standard_normal((T, Kd)).astype(np.float32)
    y = K.mul_mat(t, wq, Kd, M, x)
    rows = np.unique(np.concatenate([np.arange(64), np.arange(M - 64, M), rng.choice(M, 16, replace=False)]))
    # the repacked-Q4_K order needs whole groups of 8 rows: check the 8-row groups holding them
    rows = np.unique((rows[:, None] // 8 * 8 + np.arange(8)[None, :]).reshape(-1))
    ref = O.mul_mat_cpu(t, np.ascontiguousarray(wq[rows]), Kd, len(rows), x)
    assert_bits(np.ascontiguousarray(y[:, rows]), ref, f"{name} {Kd}x{M} T={T} (rows {len(rows)})")


MOE_TYPES = {"q4_K": O.Q4_K, "q5_K": O.Q5_K, "q6_K": O.Q6_K, "q8_0": O.Q8_0, "q4_0": O.Q4_0}


@pytest.mark.parametrize("name", ["q4_K", "q4_K_m60", "q5_K", "q6_K", "q8_0", "q4_0"])
def test_mul_mat_id_cpu_golden_bit_exact(K, golden_dir, name):
    """MUL_MAT_ID vs the reference CPU backend as libllama runs it (tests/golden/moe_cpu.npz):
    decode (one mat-vec per routed pair, experts read on the device) and T = 9 (the
    expert-sorted path), ne11 = 1 and n_used; bit for bit."""
    g = load(golden_dir, "moe_cpu.npz")
    t = {"q4_K_m60": O.Q4_K, **MOE_TYPES}[name]
    n_as, n_used, M = int(g["n_as"]), int(g["n_used"]), int(g[f"M_{name}"])
    for T, ne11 in ((1, 1), (1, n_used), (9, 1), (9, n_used)):
        key = f"{name}_{T}_{ne11}"
        x = g[f"x_{key}"]
        y = K.mul_mat_id(t, g[f"wq_{name}"], x.shape[2], M, n_as, g[f"ids_{key}"], n_used, x)
        assert_bits(y, g[f"y_{key}"], key)


@pytest.mark.parametrize("name,Kd,M,n_as,n_used,T", [("q5_K", 4096, 1024, 8, 2, 1), ("q6_K", 14336, 256, 8, 2, 1),
                                                     ("q5_K", 4096, 512, 8, 2, 64), ("q8_0", 4096, 256, 4, 1, 33),
                                                     ("q4_K", 1024, 128, 32, 4, 129), ("q4_K", 4096, 256, 8, 2, 70)])
def test_mul_mat_id_mixtral_shapes_bit_exact(K, name, Kd, M, n_as, n_used, T):
    """Mixtral-like expert shapes (K 4096 / 14336, 8 experts, top-2) and batch routing with a
    view of a wider ids row (test-backend-ops builds ids as [n_mats, n] viewed to n_used)."""
    from llamacog_amd import gguf_synth as gs
    t = MOE_TYPES[name]
    rng = np.random.default_rng(21)
    blk, bs = gs.BLOCK[t]
    wq = gs.make_blocks(t, n_as * M * Kd // blk, rng).reshape(n_as * M, -1)
    ids = np.stack([rng.permutation(n_as) for _ in range(T)]).astype(np.int32)   # row of n_as, first n_used used
    for ne11 in (1, n_used):
        x = rng.standard_normal((T, ne11, Kd)).astype(np.float32)
        y = K.mul_mat_id(t, wq, Kd, M, n_as, ids, n_used, x)
        assert_bits(y, O.mul_mat_id_cpu(t, wq, Kd, M, n_as, ids, n_used, x), f"{name} T={T} ne11={ne11}")


def test_argsort_and_sum_rows_golden(K, golden_dir):
    """ARGSORT (ggml_top_k of the router): the CPU's exchange order, ties included, bit-exact;
    SUM_ROWS: the CPU's sequential double sum, bit-exact."""
    g = load(golden_dir, "moe.npz")
    for nm in ("s", "l"):
        for order in (0, 1):
            assert (K.argsort(g[f"argsort_{nm}_x"], order) == g[f"argsort_{nm}_{order}"]).all(), (nm, order)
    for nm in ("a", "b"):
        assert (K.sum_rows(g[f"sum_rows_{nm}_x"]).view(np.uint32) == g[f"sum_rows_{nm}_y"].view(np.uint32)).all()
