"""Pin the CPU restatement (oracle/ggml_oracle.c) against golden vectors produced by the
reference's own ggml CPU backend (oracle/make_golden.py -> tests/golden/*.npz).

Integer/byte work must be bit-exact: the Q8_K / Q8_0 activation quantizers, weight
dequantization and the integer block sums.  Float outputs must match to the tolerance
stated per test (the restatement follows the scalar operation order; SIMD summation order
in the reference only moves the last bits).
"""
import os

import numpy as np
import pytest

import _oracle as O


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def test_fp16_roundtrip_matches_numpy():
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.standard_normal(20000) * s for s in (1e-8, 1e-5, 1e-2, 1, 100, 6e4)]).astype(np.float32)
    vals = np.concatenate([vals, np.array([0.0, -0.0, 65504.0, 65520.0, 1e9, -1e9, 5.96e-8, 2.98e-8], dtype=np.float32)])
    L = O.lib()
    got = np.array([L.orc_fp32_to_fp16(float(v)) for v in vals], dtype=np.uint16)
    ref = vals.astype(np.float16).view(np.uint16)
    assert (got == ref).all()
    back = np.array([L.orc_fp16_to_fp32(int(h)) for h in ref[:2000]], dtype=np.float32)
    assert (back == ref[:2000].view(np.float16).astype(np.float32)).all()


def test_q8_K_activation_quantizer_bit_exact(golden_dir):
    g = load(golden_dir, "quant_act.npz")
    got = O.quantize_rows(O.Q8_K, g["x"])
    assert got.shape == g["q8_K"].shape
    assert (got == g["q8_K"]).all(), "Q8_K blocks differ from quantize_row_q8_K_ref"


def test_q8_0_activation_quantizer_bit_exact(golden_dir):
    g = load(golden_dir, "quant_act.npz")
    got = O.quantize_rows(O.Q8_0, g["x"])
    assert (got == g["q8_0"]).all(), "Q8_0 blocks differ from the x86 quantize_row_q8_0"


def test_q4_0_quantizer_bit_exact(golden_dir):
    """quantize_row_q4_0_ref (a q4_0 KV cache's from_float) vs the reference's own q4_0 blocks"""
    g = load(golden_dir, "mul_mat_q4_0.npz")
    got = O.quantize_rows(O.Q4_0, g["w"])
    assert (got == g["wq"]).all(), "Q4_0 blocks differ from quantize_row_q4_0_ref"


@pytest.mark.parametrize("name", ["q4_0", "q8_0", "q4_K", "q5_K", "q6_K"])
def test_dequantize_bit_exact(golden_dir, name):
    g = load(golden_dir, f"mul_mat_{name}.npz")
    t = int(g["type"])
    got = O.dequantize_rows(t, g["wq"], g["w"].shape[1])
    assert (got.view(np.uint32) == g["wd"].view(np.uint32)).all()


@pytest.mark.parametrize("name", ["q4_0", "q8_0", "q4_K", "q5_K", "q6_K"])
def test_activation_quantization_of_mul_mat_inputs(golden_dir, name):
    g = load(golden_dir, f"mul_mat_{name}.npz")
    t = int(g["type"])
    vdt = O.Q8_K if t in (O.Q4_K, O.Q5_K, O.Q6_K) else O.Q8_0
    assert (O.quantize_rows(vdt, g["x"]) == g["xq"]).all()


@pytest.mark.parametrize("name", ["q4_0", "q8_0", "q4_K", "q5_K", "q6_K"])
def test_vec_dot_matches_reference(golden_dir, name):
    """Integer block sums are exact; the float combination order of the reference's SIMD
    vec_dot differs from the generic one, so the result agrees to a few ulps."""
    g = load(golden_dir, f"mul_mat_{name}.npz")
    t = int(g["type"])
    K = g["w"].shape[1]
    vd = g["vec_dot"]
    got = np.zeros_like(vd)
    for a in range(vd.shape[0]):
        for m in range(vd.shape[1]):
            got[a, m], isum, _ = O.vec_dot(t, K, g["wq"][m], g["xq"][a])
    scale = np.abs(vd).max() + 1e-30
    assert np.abs(got - vd).max() / scale < 2e-6


@pytest.mark.parametrize("name", ["q4_0", "q8_0", "q4_K", "q5_K", "q6_K"])
def test_mul_mat_matches_reference(golden_dir, name):
    g = load(golden_dir, f"mul_mat_{name}.npz")
    t = int(g["type"])
    M, K = g["w"].shape
    y = O.mul_mat(t, g["wq"], K, M, g["x"])
    ref = g["y"]
    assert np.abs(y - ref).max() / (np.abs(ref).max() + 1e-30) < 2e-6
    # against the float weights the quantized product is only approximate
    assert np.abs(y - g["x"] @ g["wd"].T).max() / np.abs(ref).max() < 0.05


def test_rms_norm(golden_dir):
    g = load(golden_dir, "rms_norm.npz")
    y = O.rms_norm(g["x"], float(g["eps"]))
    assert (y.view(np.uint32) == g["y"].view(np.uint32)).mean() > 0.999
    assert np.abs(y - g["y"]).max() <= 1e-6 * np.abs(g["y"]).max()


def test_rope(golden_dir):
    g = load(golden_dir, "rope.npz")
    for i in range(len(g["modes"])):
        y = O.rope(g["x"], g["pos"], 128, int(g["modes"][i]), float(g["bases"][i]),
                   ff=g["ff"] if g["use_ff"][i] else None)
        ref = g["y"][i]
        err = np.abs(y - ref).max() / np.abs(ref).max()
        assert err < 2e-6, (i, err)


def test_soft_max(golden_dir):
    g = load(golden_dir, "soft_max.npz")
    y = O.soft_max(g["x"], g["mask"], float(g["scale"]))
    assert np.abs(y - g["y"]).max() < 2e-6
    assert np.allclose(y.sum(axis=1), 1.0, atol=1e-5)


FA_KV = {"f16": O.F16, "q8_0": O.Q8_0, "q4_0": O.Q4_0}


@pytest.mark.parametrize("tag", ["1", "7", "long"])
@pytest.mark.parametrize("kv", sorted(FA_KV))
def test_flash_attn(golden_dir, tag, kv):
    """flash_attn_ext as the reference CPU backend computes it (oracle/make_golden.py gg_flash_attn):
    prefill / decode rows over 256 positions, and a depth-1300 decode with holes and a dead tail."""
    g = load(golden_dir, "flash_attn.npz")
    sfx = "_long" if tag == "long" else ""
    D, H, Hkv, n_kv = int(g["D"]), int(g["H" + sfx]), int(g["Hkv" + sfx]), int(g["n_kv" + sfx])
    out = O.flash_attn(g[f"q_{tag}"], g[f"k_{kv}_{tag}"], g[f"v_{kv}_{tag}"], g[f"mask_{tag}"], FA_KV[kv], D, H, Hkv, n_kv,
                       1.0 / np.sqrt(D))
    ref = g[f"out_{kv}_{tag}"]
    # bit-exact: K.Q in the CPU's vec_dot order (AVX-512 f16 / q8_0 / q4_0 class chains), libm expf,
    # the FMA of ggml_vec_mad_f16 / _f32, the unfused S*ms + vs
    assert (out.view(np.uint32) == ref.view(np.uint32)).all(), np.abs(out - ref).max() / np.abs(ref).max()


MOE_TYPES = {"q4_K": O.Q4_K, "q5_K": O.Q5_K, "q6_K": O.Q6_K, "q8_0": O.Q8_0, "q4_0": O.Q4_0}


@pytest.mark.parametrize("name", sorted(MOE_TYPES))
def test_mul_mat_id_restatement(golden_dir, name):
    """MUL_MAT_ID (ggml-cpu.c:1466) per routed (slot, token): decode and a batch with repeated
    experts, the activation broadcast (ne11 = 1) or per slot (ne11 = n_used).  Same per-row
    arithmetic as mul_mat, so the same bound."""
    g = load(golden_dir, "moe.npz")
    n_as, M, K, n_used = (int(g[k]) for k in ("n_as", "M", "K", "n_used"))
    for T, ne11 in ((1, 1), (1, n_used), (9, 1), (9, n_used)):
        key = f"{name}_{T}_{ne11}"
        y = O.mul_mat_id(MOE_TYPES[name], g[f"wq_{name}"], K, M, n_as, g[f"ids_{key}"], n_used, g[f"x_{key}"])
        ref = g[f"y_{key}"]
        assert np.abs(y - ref).max() <= 1e-5 * np.abs(ref).max(), (key, np.abs(y - ref).max())


def test_argsort_restatement_bit_exact(golden_dir):
    """ARGSORT (ops.cpp:6956): the exchange sort, ties included (router rows of equal probability)."""
    g = load(golden_dir, "moe.npz")
    for nm in ("s", "l"):
        for order in (0, 1):
            assert (O.argsort(g[f"argsort_{nm}_x"], order) == g[f"argsort_{nm}_{order}"]).all(), (nm, order)


def test_sum_rows_restatement_bit_exact(golden_dir):
    g = load(golden_dir, "moe.npz")
    for nm in ("a", "b"):
        assert (O.sum_rows(g[f"sum_rows_{nm}_x"]).view(np.uint32) == g[f"sum_rows_{nm}_y"].view(np.uint32)).all()


@pytest.mark.parametrize("name", ["q4_K", "q6_K", "q5_K", "q8_0", "q4_0", "f32"])
@pytest.mark.parametrize("T", [1, 3, 4, 9])
def test_mul_mat_cpu_order_bit_exact(golden_dir, name, T):
    """orc_mul_mat_cpu reproduces the CPU backend's mul_mat BIT FOR BIT as libllama runs it:
    repacked Q4_K gemv (T % 4 rows) and gemm (groups of 4), the AVX2 vec_dot class chains of
    Q6_K / Q5_K / Q8_0, repacked Q4_0, and vec_dot_f32 / tinyBLAS for the f32 router
    (goldens: gg_mul_mat_backend, the reference's own ggml_backend_graph_compute)."""
    g = load(golden_dir, "mul_mat_cpu.npz")
    t = {"q4_K": O.Q4_K, "q6_K": O.Q6_K, "q5_K": O.Q5_K, "q8_0": O.Q8_0, "q4_0": O.Q4_0, "f32": O.F32}[name]
    wq = g[f"wq_{name}"]
    x = g[f"x_{name}_{T}"]
    y = g[f"y_{name}_{T}"]
    got = O.mul_mat_cpu(t, wq, x.shape[1], y.shape[1], x)
    assert (got.view(np.uint32) == y.view(np.uint32)).all(), \
        f"{int((got.view(np.uint32) != y.view(np.uint32)).sum())} of {y.size} outputs differ"


@pytest.mark.parametrize("name", ["q4_K", "q4_K_m60", "q5_K", "q6_K", "q8_0", "q4_0"])
def test_mul_mat_id_cpu_order_bit_exact(golden_dir, name):
    """orc_mul_mat_id_cpu reproduces the CPU backend's mul_mat_id BIT FOR BIT as libllama runs it:
    repacked forward_mul_mat_id gemv for Q4_K / Q4_0 stacks with M % 8 == 0, vec_dot otherwise
    (goldens: gg_mul_mat_id_backend through the CPU_REPACK extra buffer)."""
    g = load(golden_dir, "moe_cpu.npz")
    t = {"q4_K": O.Q4_K, "q4_K_m60": O.Q4_K, "q5_K": O.Q5_K, "q6_K": O.Q6_K, "q8_0": O.Q8_0, "q4_0": O.Q4_0}[name]
    n_as, n_used, M = int(g["n_as"]), int(g["n_used"]), int(g[f"M_{name}"])
    for T, ne11 in ((1, 1), (1, n_used), (9, 1), (9, n_used)):
        key = f"{name}_{T}_{ne11}"
        x, ref = g[f"x_{key}"], g[f"y_{key}"]
        got = O.mul_mat_id_cpu(t, g[f"wq_{name}"], x.shape[2], M, n_as, g[f"ids_{key}"], n_used, x)
        assert (got.view(np.uint32) == ref.view(np.uint32)).all(), \
            f"{key}: {int((got.view(np.uint32) != ref.view(np.uint32)).sum())} of {ref.size} differ"
