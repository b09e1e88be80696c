"""Per-op cases whose expected outputs come from the REFERENCE's own CPU build (oracle/_ref/libref.so,
``make -C oracle ref``): shared by tests/golden/make_ref_golden.py (writes ref_ops.npz with the reference
as the backend) and tests/test_oracle.py / tests/test_gpu_ops.py (recompute with the oracle or the HIP path
and compare).

Inputs are regenerated from the committed synthetic generator (include/sli_synth.h through
``oracle.synth_fill``, itself pinned by tests/test_oracle.py against an independent pure-Python
restatement); ``ref_ops.npz`` also stores a float64 checksum of every input so generator drift is caught
separately from an arithmetic mismatch. Outputs up to ``FULL_MAX`` values are stored whole; larger ones
as the SHA-256 of their bytes plus the first 256 values.

Shapes: the C0 op shapes, the 7B row shapes (GEMV 4096 / 11008 wide, RoPE tables at
hd 128 / T 2048 / θ 1e4, 1e5, 5e5), attention at hd 128 for MHA (32/32), GQA-4 (32/8) and GQA-8 (32/4) at
positions 0 / 777 / 2047, plus the reference's edge cases (argmax ties, ±0, NaN; softmax of one element).
"""
from __future__ import annotations

import hashlib

import numpy as np

SEED = 2026
FULL_MAX = 16384


def gen(O, n, stream, std=1.0, offset=0.0):
    return O.synth_fill(int(n), SEED, stream, O.synth_c(std), offset)


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()


def _matmul(rows, cols, layer_scale=True):
    def run(B, O):
        x = gen(O, cols, 1)
        w = gen(O, rows * cols, 2, 1.0 / np.sqrt(cols)).reshape(rows, cols)
        return {"x": x, "w": w}, {"y": B.matmul(x, w)}
    return run


def _rmsnorm(dim):
    def run(B, O):
        x = gen(O, dim, 3)
        w = gen(O, dim, 4, 0.1, 1.0)
        return {"x": x, "w": w}, {"y": B.rmsnorm(x, w, 1e-5)}
    return run


def _rope_cache(hd, T, theta):
    def run(B, O):
        s, c = B.rope_cache(hd, T, theta)
        return {}, {"sin": s, "cos": c}
    return run


def _rope(dim, kv, hd, pos):
    def run(B, O):
        s, c = O.rope_cache(hd, 2048, 10000.0)  # the table itself is pinned by the rope_cache cases
        q = gen(O, dim, 5)
        k = gen(O, kv, 6)
        qo, ko = B.rope(q, k, pos, s, c, hd)
        return {"q": q, "k": k}, {"q": qo, "k": ko}
    return run


def _softmax(n):
    def run(B, O):
        x = gen(O, n, 7, 3.0)
        return {"x": x}, {"y": B.softmax(x)}
    return run


def _mha(T, hd, H, Hkv, layer, pos, n_layers):
    def run(B, O):
        kv = Hkv * hd
        q = gen(O, H * hd, 8)
        kc = gen(O, n_layers * T * kv, 9).reshape(n_layers, T, kv)
        vc = gen(O, n_layers * T * kv, 10).reshape(n_layers, T, kv)
        return {"q": q, "k": kc, "v": vc}, {"o": B.mha(q, kc, vc, layer, pos, T, hd, H, Hkv)}
    return run


def _swiglu(n):
    def run(B, O):
        up = gen(O, n, 11)
        gate = gen(O, n, 12, 4.0)
        return {"up": up, "gate": gate}, {"y": B.swiglu(up, gate)}
    return run


def _embedding(vocab, dim, token):
    def run(B, O):
        tab = gen(O, vocab * dim, 13, 0.02).reshape(vocab, dim)
        return {"table": tab}, {"y": B.embedding(token, tab)}
    return run


def _argmax_inputs(O):
    big = gen(O, 32000, 14)
    tie = big.copy()
    tie[[100, 25000]] = np.float32(big.max() + 1)
    nan_mid = big.copy()
    nan_mid[7] = np.nan
    return {
        "rand32000": big,
        "tie": tie,
        "pm0": np.array([-0.0, 0.0, -1.0], np.float32),
        "mp0": np.array([0.0, -0.0, -1.0], np.float32),
        "nan_first": np.array([np.nan, 1.0, 5.0, 2.0], np.float32),
        "nan_mid": nan_mid,
        "all_equal": np.full(17, 0.25, np.float32),
        "neg": -np.abs(gen(O, 1000, 15)),
    }


def _argmax(kind):
    def run(B, O):
        x = _argmax_inputs(O)[kind]
        return {"x": x}, {"i": np.int32(B.argmax(x))}
    return run


CASES = {}
for r, c in ((48, 256), (64, 4096), (7, 1000), (1, 11008), (3, 14336)):
    CASES[f"matmul_{r}x{c}"] = _matmul(r, c)
for d in (256, 1000, 4096):
    CASES[f"rmsnorm_{d}"] = _rmsnorm(d)
CASES["rope_cache_64_64_10000"] = _rope_cache(64, 64, 10000.0)
for th in (10000.0, 100000.0, 500000.0):
    CASES[f"rope_cache_128_2048_{int(th)}"] = _rope_cache(128, 2048, th)
for d, kv, hd, p in ((256, 128, 64, 37), (4096, 4096, 128, 2047), (4096, 1024, 128, 777), (4096, 512, 128, 0)):
    CASES[f"rope_{d}_{kv}_{hd}_{p}"] = _rope(d, kv, hd, p)
for n in (1, 36, 300, 2048):
    CASES[f"softmax_{n}"] = _softmax(n)
CASES["mha_c0_4_2_l1_p35"] = _mha(64, 64, 4, 2, 1, 35, 2)
CASES["mha_c0_4_4_l0_p63"] = _mha(64, 64, 4, 4, 0, 63, 2)
for H, Hkv in ((32, 32), (32, 8), (32, 4)):
    for p in (0, 777, 2047):
        CASES[f"mha_{H}_{Hkv}_p{p}"] = _mha(2048, 128, H, Hkv, 0, p, 1)
for n in (768, 11008, 14336):
    CASES[f"swiglu_{n}"] = _swiglu(n)
for t in (0, 7, 511):
    CASES[f"embedding_512x256_t{t}"] = _embedding(512, 256, t)
for k in ("rand32000", "tie", "pm0", "mp0", "nan_first", "nan_mid", "all_equal", "neg"):
    CASES[f"argmax_{k}"] = _argmax(k)


def pack(name: str, inputs: dict, outputs: dict) -> dict:
    """npz entries for one case: input checksums, outputs whole or as digest + head."""
    f = {}
    for k, v in inputs.items():
        f[f"{name}/in/{k}/sum64"] = np.float64(np.asarray(v, np.float64).sum())
    for k, v in outputs.items():
        v = np.asarray(v)
        if v.size <= FULL_MAX:
            f[f"{name}/out/{k}"] = v
        else:
            f[f"{name}/out/{k}/sha256"] = np.array(digest(v))
            f[f"{name}/out/{k}/head"] = v.ravel()[:256].copy()
    return f


def check(name: str, gold, inputs: dict, outputs: dict):
    """Bit-exact comparison of recomputed outputs with the committed reference vectors."""
    for k, v in inputs.items():
        want = float(gold[f"{name}/in/{k}/sum64"])
        got = float(np.asarray(v, np.float64).sum())
        assert got == want or (np.isnan(got) and np.isnan(want)), f"{name}: input {k} drifted ({got} vs {want})"
    for k, v in outputs.items():
        v = np.asarray(v)
        key = f"{name}/out/{k}"
        if key in gold:
            w = gold[key]
            if v.dtype == np.float32:
                assert np.array_equal(v.view(np.uint32), w.view(np.uint32)), \
                    f"{name}/{k}: max |d| {np.nanmax(np.abs(v.astype(np.float64) - w)):.3e}"
            else:
                assert np.array_equal(v, w), f"{name}/{k}: {v} vs {w}"
        else:
            head = gold[key + "/head"]
            assert np.array_equal(v.ravel()[:256].view(np.uint32), head.view(np.uint32)), f"{name}/{k}: head differs"
            assert digest(v) == str(gold[key + "/sha256"]), f"{name}/{k}: sha256 differs"


# ---- model-level fixtures: the reference's op layers composed as model.cpp:40-187 ----------------------
PROMPT = [1, 17, 42, 99]
TINY = dict(vocab=512, dim=256, n_heads=4, head_dim=64, ffn=768, n_layers=2, max_len=64, eps=1e-5, theta=10000.0)
# 2-layer models with the 7B row shapes (the 32-layer models do not fit the reference's fp32 CPU path in a
# CPU-suite budget): Llama-2-7B MHA (θ 1e4) and a Llama-3-8B-shaped GQA-4 (θ 5e5; vocab cut to 32000)
L7B2 = dict(vocab=32000, dim=4096, n_heads=32, head_dim=128, ffn=11008, n_layers=2, max_len=64, eps=1e-5,
            theta=10000.0)
L8B2 = dict(vocab=32000, dim=4096, n_heads=32, head_dim=128, ffn=14336, n_layers=2, max_len=64, eps=1e-5,
            theta=500000.0)
MODELS = {
    "ref_c0_mha": (TINY, 4, 36, 0),
    "ref_c0_gqa": (TINY, 2, 36, 0),
    "ref_7b2l_mha": (L7B2, 32, 6, 1),
    "ref_8b2l_gqa": (L8B2, 8, 6, 1),
}
