#!/usr/bin/env python3
"""make_golden.py — write tests/golden/*.npz from the REFERENCE's own ggml.

TEST INFRASTRUCTURE.  Calls oracle/_ref/libgolden.so (oracle/gen_golden.c linked against
libggml-base + the x86-64-v4 ggml-cpu built from /root/reference sources by refhost/) to
produce golden input/output vectors for the hot path:
  * activation quantizers (the CPU backend's from_float for Q8_K and Q8_0),
  * model-file quantized weights (ggml_quantize_chunk) + their dequantization,
  * per-row vec_dot results and CPU mul_mat outputs for Q4_0/Q8_0/Q4_K/Q5_K/Q6_K,
  * rms_norm, rope (NORM/NEOX, Llama-3 base 500000), soft_max, flash_attn_ext (f16, q8_0 and q4_0 KV; a depth-1300 decode case).
Inputs follow tests/test-quantize-fns.cpp:31-35 (0.1 + 2*cos(i + offset)) plus seeded
random data and hand-made edge cases.  Run here (where /root/reference exists):
    python oracle/make_golden.py
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")

F32, F16, Q4_0, Q8_0, Q4_K, Q5_K, Q6_K, Q8_K = 0, 1, 2, 8, 12, 13, 14, 15
BLK = {Q4_0: (32, 18), Q8_0: (32, 34), Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210), Q8_K: (256, 292),
       F16: (1, 2), F32: (1, 4)}
NAMES = {Q4_0: "q4_0", Q8_0: "q8_0", Q4_K: "q4_K", Q5_K: "q5_K", Q6_K: "q6_K"}

P = ctypes.c_void_p
I64 = ctypes.c_int64


def fptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def load():
    lib = ctypes.CDLL(os.path.join(HERE, "_ref", "libgolden.so"))
    lib.gg_quantize.argtypes = [ctypes.c_int, P, P, I64, I64]
    lib.gg_quantize.restype = ctypes.c_size_t
    lib.gg_from_float.argtypes = [ctypes.c_int, P, P, I64]
    lib.gg_to_float.argtypes = [ctypes.c_int, P, P, I64]
    lib.gg_vec_dot.argtypes = [ctypes.c_int, I64, P, P]
    lib.gg_vec_dot.restype = ctypes.c_float
    lib.gg_mul_mat.argtypes = [ctypes.c_int, P, I64, I64, P, I64, P, ctypes.c_int]
    lib.gg_rms_norm.argtypes = [P, I64, I64, ctypes.c_float, P]
    lib.gg_rope.argtypes = [P, I64, I64, I64, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                            ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, P, P]
    lib.gg_soft_max.argtypes = [P, I64, I64, P, I64, ctypes.c_float, P]
    lib.gg_flash_attn.argtypes = [P, P, P, P, ctypes.c_int, I64, I64, I64, I64, I64, ctypes.c_float, ctypes.c_float, P,
                                  ctypes.c_int]
    lib.gg_mul_mat_id.argtypes = [ctypes.c_int, P, I64, I64, I64, P, I64, P, I64, I64, P, ctypes.c_int]
    lib.gg_argsort.argtypes = [P, I64, I64, ctypes.c_int, P]
    lib.gg_sum_rows.argtypes = [P, I64, I64, P]
    lib.gg_mul_mat_backend.argtypes = [ctypes.c_int, P, I64, I64, P, I64, P, ctypes.c_int, ctypes.c_int]
    lib.gg_mul_mat_backend.restype = ctypes.c_int
    lib.gg_mul_mat_id_backend.argtypes = [ctypes.c_int, P, I64, I64, I64, P, I64, P, I64, I64, P, ctypes.c_int, ctypes.c_int]
    lib.gg_mul_mat_id_backend.restype = ctypes.c_int
    lib.gg_init()
    return lib


def nbytes(t, n):
    b, s = BLK[t]
    return n // b * s


def quantize(lib, t, w):
    rows, k = w.shape
    out = np.zeros(rows * nbytes(t, k), dtype=np.uint8)
    lib.gg_quantize(t, fptr(w), fptr(out), rows, k)
    return out.reshape(rows, -1)


def from_float(lib, t, x):
    rows, k = x.shape
    out = np.zeros((rows, nbytes(t, k)), dtype=np.uint8)
    for r in range(rows):
        lib.gg_from_float(t, fptr(x[r]), fptr(out[r]), k)
    return out


def to_float(lib, t, q, k):
    rows = q.shape[0]
    out = np.zeros((rows, k), dtype=np.float32)
    for r in range(rows):
        lib.gg_to_float(t, fptr(q[r]), fptr(out[r]), k)
    return out


def act_cases(k, rng):
    i = np.arange(k, dtype=np.float32)
    rows = [
        (0.1 + 2 * np.cos(i + 0.0)).astype(np.float32),           # test-quantize-fns data
        (0.1 + 2 * np.cos(i + 1.0)).astype(np.float32),
        rng.standard_normal(k).astype(np.float32),
        (rng.standard_normal(k) * 1e-3).astype(np.float32),
        (rng.standard_normal(k) * 300).astype(np.float32),
        np.zeros(k, dtype=np.float32),                               # all-zero blocks (d = 0)
    ]
    tie = rng.standard_normal(k).astype(np.float32) * 0.5
    tie[::256] = -3.0                                                # equal |max| of both signs:
    tie[5::256] = 3.0                                                # first index must win
    rows.append(tie)
    half = np.round(rng.standard_normal(k) * 40).astype(np.float32) / 127.0 * 0.5
    rows.append(half.astype(np.float32))                             # many x*iscale near .5
    return np.stack(rows)


def moe(lib):
    """MoE routing ops (build_moe_ffn, src/llama-graph.cpp:642-787): MUL_MAT_ID per expert type
    (decode T = 1 and a batch with repeated experts, ne11 = 1 broadcast and ne11 = n_used),
    ARGSORT with ties (ggml_top_k), SUM_ROWS."""
    rng = np.random.default_rng(4321)
    g = {}
    n_as, M, K, n_used = 4, 64, 512, 2
    for t, name in ((Q4_K, "q4_K"), (Q5_K, "q5_K"), (Q6_K, "q6_K"), (Q8_0, "q8_0"), (Q4_0, "q4_0")):
        w = (rng.standard_normal((n_as * M, K)) * 0.05).astype(np.float32)
        wq = quantize(lib, t, w)
        g[f"wq_{name}"] = wq
        for T, ne11 in ((1, 1), (1, n_used), (9, 1), (9, n_used)):
            ids = np.stack([rng.permutation(n_as)[:n_used] for _ in range(T)]).astype(np.int32)
            if T > 1:
                ids[1] = ids[0]            # repeated routing across tokens
            x = np.concatenate([act_cases(K, rng)[:2], rng.standard_normal((T * ne11, K)).astype(np.float32)])[:T * ne11]
            x = x.reshape(T, ne11, K)
            y = np.zeros((T, n_used, M), dtype=np.float32)
            lib.gg_mul_mat_id(t, fptr(wq), K, M, n_as, fptr(ids), n_used, fptr(x), ne11, T, fptr(y), 1)
            g[f"ids_{name}_{T}_{ne11}"] = ids
            g[f"x_{name}_{T}_{ne11}"] = x
            g[f"y_{name}_{T}_{ne11}"] = y
    # router-like rows with ties (equal probabilities must order as the CPU's exchange sort)
    xs = rng.standard_normal((12, 8)).astype(np.float32)
    xs[0] = [0.5, 0.1, 0.5, 0.3, 0.5, 0.1, 0.2, 0.5]
    xs[1] = 0.25
    xs[2, ::2] = xs[2, 1::2]
    xl = rng.integers(-4, 4, (3, 60)).astype(np.float32)   # wide rows, many ties
    for nm, arr in (("s", xs), ("l", xl)):
        for order in (0, 1):
            out = np.zeros(arr.shape, dtype=np.int32)
            lib.gg_argsort(fptr(arr), arr.shape[1], arr.shape[0], order, fptr(out))
            g[f"argsort_{nm}_{order}"] = out
        g[f"argsort_{nm}_x"] = arr
    xr = np.concatenate([rng.standard_normal((5, 2)), rng.standard_normal((5, 2)) * 1e6,
                         rng.standard_normal((2, 2)) * 1e-8]).astype(np.float32)
    xr2 = (rng.standard_normal((4, 1000)) * 100).astype(np.float32)
    for nm, arr in (("a", xr), ("b", xr2)):
        y = np.zeros(arr.shape[0], dtype=np.float32)
        lib.gg_sum_rows(fptr(arr), arr.shape[1], arr.shape[0], fptr(y))
        g[f"sum_rows_{nm}_x"] = arr
        g[f"sum_rows_{nm}_y"] = y
    np.savez_compressed(os.path.join(OUT, "moe.npz"), n_as=n_as, M=M, K=K, n_used=n_used, **g)
    print(f"moe.npz {os.path.getsize(os.path.join(OUT, 'moe.npz'))} B")


def cpu_orders(lib):
    """mul_mat exactly as libllama runs it on the CPU backend (gg_mul_mat_backend): Q4_K / Q4_0
    weights in the CPU_REPACK extra buffer (8x8 gemv for T % 4 rows, gemm for groups of 4),
    the other types through the vec_dot / llamafile kernels; F32 (the MoE router) through
    vec_dot_f32 at T = 1 and tinyBLAS at T >= 2.  These pin the float combination order that
    oracle/ggml_oracle.c orc_mul_mat_cpu restates and the GPU kernels must reproduce."""
    rng = np.random.default_rng(777)
    g = {}
    for t, name, M, K in ((Q4_K, "q4_K", 64, 2048), (Q6_K, "q6_K", 64, 2048), (Q5_K, "q5_K", 64, 1024),
                          (Q8_0, "q8_0", 64, 1024), (Q4_0, "q4_0", 64, 1024), (F32, "f32", 8, 1024)):
        w = (rng.standard_normal((M, K)) * 0.05).astype(np.float32)
        w[: M // 4] = (0.1 + 2 * np.cos(np.arange(M // 4 * K, dtype=np.float32).reshape(M // 4, K) + 0.5)) * 0.05
        wq = w if t == F32 else quantize(lib, t, w)
        g[f"wq_{name}"] = wq
        extra = 1 if t in (Q4_K, Q4_0) else 0
        for T in (1, 3, 4, 9):
            x = rng.standard_normal((T, K)).astype(np.float32)
            if T >= 3:
                x[1] = (0.1 + 2 * np.cos(np.arange(K, dtype=np.float32) + 1.0)).astype(np.float32)
            y = np.zeros((T, M), dtype=np.float32)
            st = lib.gg_mul_mat_backend(t, fptr(wq), K, M, fptr(x), T, fptr(y), 4, extra)
            assert st == 0, st
            g[f"x_{name}_{T}"] = x
            g[f"y_{name}_{T}"] = y
    np.savez_compressed(os.path.join(OUT, "mul_mat_cpu.npz"), **g)
    print(f"mul_mat_cpu.npz {os.path.getsize(os.path.join(OUT, 'mul_mat_cpu.npz'))} B")


def moe_cpu_orders(lib):
    """mul_mat_id exactly as libllama runs it on the CPU backend (gg_mul_mat_id_backend with the
    CPU_REPACK extra buffer): Q4_K / Q4_0 stacks with M % 8 == 0 through forward_mul_mat_id's
    repacked gemv, the others through the vec_dot order; decode and batched routing."""
    rng = np.random.default_rng(8642)
    g = {}
    n_as, n_used = 4, 2
    for t, name, M, K in ((Q4_K, "q4_K", 64, 1024), (Q4_K, "q4_K_m60", 60, 512), (Q5_K, "q5_K", 64, 512),
                          (Q6_K, "q6_K", 32, 1024), (Q8_0, "q8_0", 64, 512), (Q4_0, "q4_0", 64, 512)):
        w = (rng.standard_normal((n_as * M, K)) * 0.05).astype(np.float32)
        wq = quantize(lib, t, w)
        g[f"wq_{name}"] = wq
        g[f"M_{name}"] = M
        for T, ne11 in ((1, 1), (1, n_used), (9, 1), (9, n_used)):
            ids = np.stack([rng.permutation(n_as)[:n_used] for _ in range(T)]).astype(np.int32)
            x = rng.standard_normal((T, ne11, K)).astype(np.float32)
            y = np.zeros((T, n_used, M), dtype=np.float32)
            # libllama only places repackable stacks in CPU_REPACK (its supports_op declines the rest)
            extra = 1 if t in (Q4_K, Q4_0) and M % 8 == 0 else 0
            st = lib.gg_mul_mat_id_backend(t, fptr(wq), K, M, n_as, fptr(ids), n_used, fptr(x), ne11, T, fptr(y), 4, extra)
            assert st == 0, st
            g[f"ids_{name}_{T}_{ne11}"] = ids
            g[f"x_{name}_{T}_{ne11}"] = x
            g[f"y_{name}_{T}_{ne11}"] = y
    np.savez_compressed(os.path.join(OUT, "moe_cpu.npz"), n_as=n_as, n_used=n_used, **g)
    print(f"moe_cpu.npz {os.path.getsize(os.path.join(OUT, 'moe_cpu.npz'))} B")


def fa_case(lib, fa, tag, q, kf, vf, m, kvt, kvname, D, H, Hkv, n_kv):
    """one flash_attn_ext case through the reference CPU backend (gg_flash_attn), stored under tag"""
    if kvt == F16:
        kb, vb = kf.astype(np.float16).view(np.uint8), vf.astype(np.float16).view(np.uint8)
    else:
        kb = quantize(lib, kvt, kf.reshape(-1, D)).reshape(-1)
        vb = quantize(lib, kvt, vf.reshape(-1, D)).reshape(-1)
    n_q = q.shape[0]
    out = np.zeros((n_q, H, D), dtype=np.float32)
    lib.gg_flash_attn(fptr(q), fptr(np.ascontiguousarray(kb)), fptr(np.ascontiguousarray(vb)),
                      fptr(m.view(np.uint16)), kvt, D, n_q, H, n_kv, Hkv, 1.0 / np.sqrt(D), 0.0, fptr(out), 1)
    fa[f"q_{tag}"] = q
    fa[f"k_{kvname}_{tag}"] = np.ascontiguousarray(kb)
    fa[f"v_{kvname}_{tag}"] = np.ascontiguousarray(vb)
    fa[f"mask_{tag}"] = m.view(np.uint16)
    fa[f"out_{kvname}_{tag}"] = out


def main():
    os.makedirs(OUT, exist_ok=True)
    lib = load()
    if "moe" in sys.argv[1:]:   # only the MoE fixture (the others stay as committed)
        return moe(lib)
    if "cpu_orders" in sys.argv[1:]:
        return cpu_orders(lib)
    if "moe_cpu" in sys.argv[1:]:
        return moe_cpu_orders(lib)
    rng = np.random.default_rng(1234)

    # ---- activation quantizers ------------------------------------------------------------
    K = 1024
    x = act_cases(K, rng)
    np.savez_compressed(os.path.join(OUT, "quant_act.npz"), x=x, q8_K=from_float(lib, Q8_K, x), q8_0=from_float(lib, Q8_0, x))

    # ---- weights, dequant, vec_dot, mul_mat ------------------------------------------------
    M, K, T = 64, 512, 8
    for t, name in NAMES.items():
        i = np.arange(M * K, dtype=np.float32).reshape(M, K)
        w = (0.1 + 2 * np.cos(i + 0.5)).astype(np.float32) * 0.05
        w[M // 2:] = (rng.standard_normal((M - M // 2, K)) * 0.02).astype(np.float32)
        wq = quantize(lib, t, w)
        wd = to_float(lib, t, wq, K)
        xs = np.concatenate([act_cases(K, rng)[:T - 2], rng.standard_normal((2, K)).astype(np.float32)])
        vdt = Q8_K if t in (Q4_K, Q5_K, Q6_K) else Q8_0
        xq = from_float(lib, vdt, xs)
        vd = np.zeros((T, M), dtype=np.float32)
        for a in range(T):
            for m in range(M):
                vd[a, m] = lib.gg_vec_dot(t, K, fptr(wq[m]), fptr(xq[a]))
        y = np.zeros((T, M), dtype=np.float32)
        lib.gg_mul_mat(t, fptr(wq), K, M, fptr(xs), T, fptr(y), 1)
        y1 = np.zeros((1, M), dtype=np.float32)
        lib.gg_mul_mat(t, fptr(wq), K, M, fptr(xs[:1]), 1, fptr(y1), 1)
        np.savez_compressed(os.path.join(OUT, f"mul_mat_{name}.npz"), type=t, w=w, wq=wq, wd=wd, x=xs, xq=xq, vec_dot=vd,
                            y=y, y1=y1)

    # ---- rms_norm ----------------------------------------------------------------------------
    x = np.concatenate([act_cases(4096, rng)[:5], rng.standard_normal((3, 4096)).astype(np.float32)])
    y = np.zeros_like(x)
    lib.gg_rms_norm(fptr(x), 4096, x.shape[0], 1e-5, fptr(y))
    np.savez_compressed(os.path.join(OUT, "rms_norm.npz"), x=x, y=y, eps=np.float32(1e-5))

    # ---- rope: Llama-3 (NORM, base 500000) and NEOX, with/without freq factors --------------
    ne0, nh, ntok = 128, 4, 6
    pos = np.array([0, 1, 7, 255, 511, 4095], dtype=np.int32)
    xr = rng.standard_normal((ntok, nh, ne0)).astype(np.float32)
    ff = (1.0 + np.arange(ne0 // 2, dtype=np.float32) / 32).astype(np.float32)
    cases = []
    for mode in (0, 2):
        for base, use_ff in ((500000.0, False), (10000.0, True)):
            y = np.zeros_like(xr)
            lib.gg_rope(fptr(xr), ne0, nh, ntok, fptr(pos), ne0, mode, 8192, base, 1.0, 0.0, 1.0, 32.0, 1.0,
                        fptr(ff) if use_ff else None, fptr(y))
            cases.append((mode, base, use_ff, y))
    np.savez_compressed(os.path.join(OUT, "rope.npz"), x=xr, pos=pos, ff=ff,
                        modes=np.array([c[0] for c in cases]), bases=np.array([c[1] for c in cases], dtype=np.float32),
                        use_ff=np.array([c[2] for c in cases]), y=np.stack([c[3] for c in cases]))

    # ---- soft_max with a causal-style mask ---------------------------------------------------
    nc, nr = 200, 12
    xs = (rng.standard_normal((nr, nc)) * 3).astype(np.float32)
    mask = np.zeros((4, nc), dtype=np.float32)
    for r in range(4):
        mask[r, 150 + 10 * r:] = -np.inf
    y = np.zeros_like(xs)
    lib.gg_soft_max(fptr(xs), nc, nr, fptr(mask), 4, 0.125, fptr(y))
    np.savez_compressed(os.path.join(OUT, "soft_max.npz"), x=xs, mask=mask, scale=np.float32(0.125), y=y)

    # ---- flash attention: D 128, GQA 4, f16 and q8_0 KV ------------------------------------
    D, H, Hkv, n_kv = 128, 8, 2, 256
    fa = {}
    for n_q in (1, 7):
        q = rng.standard_normal((n_q, H, D)).astype(np.float32)
        kf = rng.standard_normal((n_kv, Hkv, D)).astype(np.float32)
        vf = rng.standard_normal((n_kv, Hkv, D)).astype(np.float32)
        m = np.zeros((n_q, n_kv), dtype=np.float16)
        valid = 200
        for r in range(n_q):
            m[r, valid + r:] = -np.inf
        m[:, 3] = -np.inf
        for kvt, kvname in ((F16, "f16"), (Q8_0, "q8_0"), (Q4_0, "q4_0")):
            fa_case(lib, fa, f"{n_q}", q, kf, vf, m, kvt, kvname, D, H, Hkv, n_kv)
    # decode at depth (the long-context pair: scores grid + per-head chain), one KV head (its rows
    # back to back in the cache) and a mask with holes and a dead tail
    n_kv_l, H_l, Hkv_l = 1300, 4, 1
    q = rng.standard_normal((1, H_l, D)).astype(np.float32) * 2
    kf = rng.standard_normal((n_kv_l, Hkv_l, D)).astype(np.float32)
    vf = rng.standard_normal((n_kv_l, Hkv_l, D)).astype(np.float32)
    m = np.zeros((1, n_kv_l), dtype=np.float16)
    m[0, rng.random(n_kv_l) < 0.25] = -np.inf
    m[0, 1290:] = -np.inf
    for kvt, kvname in ((F16, "f16"), (Q8_0, "q8_0"), (Q4_0, "q4_0")):
        fa_case(lib, fa, "long", q, kf, vf, m, kvt, kvname, D, H_l, Hkv_l, n_kv_l)
    np.savez_compressed(os.path.join(OUT, "flash_attn.npz"), D=D, H=H, Hkv=Hkv, n_kv=n_kv, H_long=H_l, Hkv_long=Hkv_l,
                        n_kv_long=n_kv_l, **fa)
    moe(lib)
    cpu_orders(lib)
    moe_cpu_orders(lib)
    for f in sorted(os.listdir(OUT)):
        print(f"{f:28s} {os.path.getsize(os.path.join(OUT, f)):9d} B")


if __name__ == "__main__":
    sys.exit(main())
