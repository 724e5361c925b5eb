"""GPU parity of the HIP kernels through the C ABI (include/ggml-mi355x.h) against the
golden vectors of the reference CPU backend and the oracle restatement.

Tolerances (all stated here):
  * integer / byte work (activation quantizers): bit-exact;
  * mat-vec results: the integer block sums are exact, only the fp32 combination order
    differs -> max |err| / max |ref| < 2e-6;
  * rms_norm, rope, soft_max, SiLU, f16 flash-attention: the kernels reproduce the
    x86-64-v4 CPU backend's operation order -> bit-exact except rare last-ulp differences
    of transcendental functions (fraction of differing elements bounded per test);
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


@pytest.mark.parametrize("name", ["q4_0", "q8_0", "q4_K", "q5_K", "q6_K"])
def test_mul_mat_golden(K, golden_dir, name):
    g = load(golden_dir, f"mul_mat_{name}.npz")
    t = int(g["type"])
    M, Kd = g["w"].shape
    for T, ref in ((1, g["y1"]), (8, g["y"])):
        y = K.mul_mat(t, g["wq"], Kd, M, g["x"][:T])
        err = np.abs(y - ref).max() / np.abs(ref).max()
        assert err < 2e-6, (name, T, err)


@pytest.mark.parametrize("name,Kd,M", [("q4_K", 4096, 1024), ("q6_K", 14336, 256), ("q4_K", 14336, 256),
                                        ("q5_K", 4096, 512), ("q8_0", 4096, 512), ("q4_0", 4096, 512),
                                        ("q6_K", 4096, 4096)])
def test_mul_mat_llama_shapes_vs_oracle(K, name, Kd, M):
    """Full Llama-3-8B row lengths (K 4096 / 14336) with random-but-valid blocks."""
    from llamacog_amd import gguf_synth as gs
    t = {"q4_0": O.Q4_0, "q8_0": O.Q8_0, "q4_K": O.Q4_K, "q5_K": O.Q5_K, "q6_K": O.Q6_K}[name]
    rng = np.random.default_rng(11)
    blk, bs = gs.BLOCK[t]
    wq = gs.make_blocks(t, M * Kd // blk, rng).reshape(M, -1)
    for T in (1, 3, 8, 17):
        x = rng.standard_normal((T, Kd)).astype(np.float32)
        y = K.mul_mat(t, wq, Kd, M, x)
        ref = O.mul_mat(t, wq, Kd, M, x)
        err = np.abs(y - ref).max() / np.abs(ref).max()
        assert err < 2e-6, (name, T, err)


def test_rms_norm_and_fused_mul(K, golden_dir):
    g = load(golden_dir, "rms_norm.npz")
    y = K.rms_norm(g["x"], float(g["eps"]))
    assert (y.view(np.uint32) == g["y"].view(np.uint32)).mean() > 0.999
    assert np.abs(y - g["y"]).max() <= 1e-6 * np.abs(g["y"]).max()
    w = np.linspace(0.5, 1.5, g["x"].shape[1]).astype(np.float32)
    y2, ym = K.rms_norm(g["x"], float(g["eps"]), w)
    assert (y2.view(np.uint32) == y.view(np.uint32)).all()
    assert (ym.view(np.uint32) == (y * w).astype(np.float32).view(np.uint32)).all()


def test_rope_golden(K, golden_dir):
    g = load(golden_dir, "rope.npz")
    for i in range(len(g["modes"])):
        y = K.rope(g["x"], g["pos"], 128, int(g["modes"][i]), float(g["bases"][i]),
                   ff=g["ff"] if g["use_ff"][i] else None)
        ref = g["y"][i]
        same = (y.view(np.uint32) == ref.view(np.uint32)).mean()
        # cos/sin are taken in double and rounded once; glibc's cosf/sinf are not always
        # correctly rounded, so ~1% of elements differ by one ulp
        assert same > 0.97 and np.abs(y - ref).max() < 1e-6, (i, same, np.abs(y - ref).max())


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
    body = (x.shape[1] // 16) * 16   # ggml_v_silu part: bit-exact; tail: libm expf vs exp(double)
    bad = np.argwhere(y[:, :body].view(np.uint32) != ref[:, :body].view(np.uint32))
    info = [(tuple(b), float(x[tuple(b)]), float(y[tuple(b)]), float(ref[tuple(b)])) for b in bad[:8]]
    assert len(bad) == 0, (len(bad), info)
    assert np.abs(y[:, body:] - ref[:, body:]).max() <= 1e-6 * np.abs(ref[:, body:]).max()


@pytest.mark.parametrize("n_q", [1, 7])
def test_flash_attn_f16_golden(K, golden_dir, n_q):
    g = load(golden_dir, "flash_attn.npz")
    D, H, Hkv, n_kv = int(g["D"]), int(g["H"]), int(g["Hkv"]), int(g["n_kv"])
    out = K.flash_attn(g[f"q_{n_q}"], g[f"k_f16_{n_q}"], g[f"v_f16_{n_q}"], g[f"mask_{n_q}"], O.F16, D, H, Hkv, n_kv,
                       1.0 / np.sqrt(D))
    ref = g[f"out_f16_{n_q}"]
    same = (out.view(np.uint32) == ref.view(np.uint32)).mean()
    err = np.abs(out - ref).max() / np.abs(ref).max()
    assert same > 0.995 and err < 1e-3, (same, err)


@pytest.mark.parametrize("n_q", [1, 7])
def test_flash_attn_q8_0_golden(K, golden_dir, n_q):
    g = load(golden_dir, "flash_attn.npz")
    D, H, Hkv, n_kv = int(g["D"]), int(g["H"]), int(g["Hkv"]), int(g["n_kv"])
    out = K.flash_attn(g[f"q_{n_q}"], g[f"k_q8_0_{n_q}"], g[f"v_q8_0_{n_q}"], g[f"mask_{n_q}"], O.Q8_0, D, H, Hkv, n_kv,
                       1.0 / np.sqrt(D))
    ref = g[f"out_q8_0_{n_q}"]
    assert np.abs(out - ref).max() / np.abs(ref).max() < 1e-5


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
    same = (out.view(np.uint32) == ref.view(np.uint32)).mean()
    assert same > 0.99 and np.abs(out - ref).max() / np.abs(ref).max() < 2e-3, same


@pytest.mark.parametrize("name,Kd,M", [("q4_K", 4096, 256), ("q5_K", 4096, 200), ("q6_K", 4096, 136),
                                        ("q4_K", 14336, 128), ("q6_K", 14336, 64)])
def test_mul_mat_prefill_mfma_vs_oracle(K, name, Kd, M):
    """Batched MUL_MAT (T >= 16) on the MFMA int8 path (k_mmq.hip): exact integer sub-block
    dots, fp32 block combination -> max |err| / max |ref| < 2e-6 like the mat-vec path."""
    from llamacog_amd import gguf_synth as gs
    t = {"q4_K": O.Q4_K, "q5_K": O.Q5_K, "q6_K": O.Q6_K}[name]
    rng = np.random.default_rng(21)
    blk, bs = gs.BLOCK[t]
    wq = gs.make_blocks(t, M * Kd // blk, rng).reshape(M, -1)
    for T in (16, 64, 100):
        x = rng.standard_normal((T, Kd)).astype(np.float32)
        y = K.mul_mat(t, wq, Kd, M, x)
        ref = O.mul_mat(t, wq, Kd, M, x)
        err = np.abs(y - ref).max() / np.abs(ref).max()
        assert err < 2e-6, (name, T, err)


MOE_TYPES = {"q4_K": O.Q4_K, "q5_K": O.Q5_K, "q6_K": O.Q6_K, "q8_0": O.Q8_0, "q4_0": O.Q4_0}


@pytest.mark.parametrize("name", sorted(MOE_TYPES))
def test_mul_mat_id_golden(K, golden_dir, name):
    """MUL_MAT_ID vs the reference CPU backend: decode (one GEMV per routed pair, experts read
    on the device) and T = 9 (the expert-sorted path); integer sums exact, fp32 combination
    order differs -> 2e-6 of the range, like mul_mat."""
    g = load(golden_dir, "moe.npz")
    n_as, M, Kd, n_used = (int(g[k]) for k in ("n_as", "M", "K", "n_used"))
    for T, ne11 in ((1, 1), (1, n_used), (9, 1), (9, n_used)):
        key = f"{name}_{T}_{ne11}"
        y = K.mul_mat_id(MOE_TYPES[name], g[f"wq_{name}"], Kd, M, n_as, g[f"ids_{key}"], n_used, g[f"x_{key}"])
        ref = g[f"y_{key}"]
        err = np.abs(y - ref).max() / np.abs(ref).max()
        assert err < 2e-6, (key, err)


@pytest.mark.parametrize("name,Kd,M,n_as,n_used,T", [("q5_K", 4096, 1024, 8, 2, 1), ("q6_K", 14336, 256, 8, 2, 1),
                                                     ("q5_K", 4096, 512, 8, 2, 64), ("q8_0", 4096, 256, 4, 1, 33),
                                                     ("q4_K", 1024, 128, 32, 4, 129)])
def test_mul_mat_id_mixtral_shapes_vs_oracle(K, name, Kd, M, n_as, n_used, T):
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
        ref = O.mul_mat_id(t, wq, Kd, M, n_as, ids, n_used, x)
        err = np.abs(y - ref).max() / np.abs(ref).max()
        assert err < 2e-6, (name, T, ne11, err)


def test_argsort_and_sum_rows_golden(K, golden_dir):
    """ARGSORT (ggml_top_k of the router): the CPU's exchange order, ties included, bit-exact;
    SUM_ROWS: the CPU's sequential double sum, bit-exact."""
    g = load(golden_dir, "moe.npz")
    for nm in ("s", "l"):
        for order in (0, 1):
            assert (K.argsort(g[f"argsort_{nm}_x"], order) == g[f"argsort_{nm}_{order}"]).all(), (nm, order)
    for nm in ("a", "b"):
        assert (K.sum_rows(g[f"sum_rows_{nm}_x"]).view(np.uint32) == g[f"sum_rows_{nm}_y"].view(np.uint32)).all()
