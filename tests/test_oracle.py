"""CPU tests of the oracle (oracle/sli_oracle.c).

Pinned against the REFERENCE itself: tests/golden/ref_ops.npz and ref_{c0,7b2l,8b2l}_*.npz were written by
the reference's own CPU kernels and op layers, compiled in place from /root/reference (oracle/Makefile
`ref`, oracle/ref_harness.cpp, tests/golden/make_ref_golden.py); the oracle must reproduce them BIT FOR BIT.
Where /root/reference is present the reference build is also run live against the oracle on fresh inputs.
Also cross-checked against an independent float64 restatement (tests/refmath.py) and the reference's edge
cases. See DESIGN.md §2.
"""
import os

import numpy as np
import pytest

from tests import refmath

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TINY = dict(vocab=512, dim=256, n_heads=4, head_dim=64, ffn=768, n_layers=2, max_len=64, eps=1e-5, theta=10000.0)


def _weights(O, m, cfg):
    W = {"emb": m.weight(O.T_EMB).copy(), "norm": [m.weight(O.T_NORM, i).copy() for i in range(2 * cfg.n_layers + 1)]}
    for k, kind in (("wq", O.T_WQ), ("wk", O.T_WK), ("wv", O.T_WV), ("wo", O.T_WO), ("up", O.T_UP),
                    ("gate", O.T_GATE), ("down", O.T_DOWN)):
        W[k] = [m.weight(kind, l).copy() for l in range(cfg.n_layers)]
    return W


@pytest.mark.parametrize("name,n_kv", [("c0_mha.npz", 4), ("c0_gqa.npz", 2)])
def test_oracle_reproduces_golden_model_fixture(oracle, name, n_kv):
    g = np.load(os.path.join(GOLD, name))
    m = oracle.Model(oracle.Config(n_kv_heads=n_kv, **TINY), seed=0)
    toks, logits = m.predict(g["prompt"], 36)
    assert np.array_equal(toks, g["tokens"])
    assert np.array_equal(logits.view(np.uint32), g["logits"].view(np.uint32))  # deterministic C: bit-exact


@pytest.mark.parametrize("n_kv", [4, 2])
def test_oracle_matches_independent_float64_restatement(oracle, n_kv):
    cfg = oracle.Config(n_kv_heads=n_kv, **TINY)
    m = oracle.Model(cfg, seed=0)
    toks, logits = m.predict([1, 17, 42, 99], 36)
    ref = refmath.Model64(cfg, _weights(oracle, m, cfg))
    for p, t in enumerate(toks):
        l64 = ref.forward(int(t), p)
        assert np.abs(l64 - logits[p]).max() < 1e-5
        top2 = np.sort(l64)[-2:]
        if top2[1] - top2[0] > 1e-5:
            assert int(np.argmax(l64)) == int(np.argmax(logits[p]))
        if p >= 3:  # greedy steps: the token fed next is the oracle argmax
            if p + 1 < len(toks):
                assert toks[p + 1] == int(np.argmax(logits[p]))


def test_oracle_kv_f16_matches_float64_with_f16_cache(oracle):
    cfg = oracle.Config(n_kv_heads=2, **TINY)
    m = oracle.Model(cfg, seed=0, kv_f16=True)
    toks, logits = m.predict([1, 17, 42, 99], 20)
    ref = refmath.Model64(cfg, _weights(oracle, m, cfg), kv_f16=True)
    for p, t in enumerate(toks):
        assert np.abs(ref.forward(int(t), p) - logits[p]).max() < 5e-4


def test_per_op_fixtures(oracle):
    f = np.load(os.path.join(GOLD, "ops.npz"))
    eq = lambda a, b: np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))
    assert eq(oracle.matmul(f["matmul_x"], f["matmul_w"]), f["matmul_y"])
    assert eq(oracle.rmsnorm(f["matmul_x"], f["rms_w"], 1e-5), f["rms_y"])
    for th in (10000, 100000, 500000):
        s, c = oracle.rope_cache(64, 64, float(th))
        assert eq(s, f[f"rope_sin_{th}"]) and eq(c, f[f"rope_cos_{th}"])
    s, c = f["rope_sin_10000"], f["rope_cos_10000"]
    q, k = oracle.rope(f["rope_q"], f["rope_k"], 37, s, c, 64)
    assert eq(q, f["rope_q_out"]) and eq(k, f["rope_k_out"])
    for pos in (0, 17, 63):
        assert eq(oracle.mha(f["mha_q"], f["mha_k"], f["mha_v"], 1, pos, 64, 64, 4, 2), f[f"mha_gqa_out_{pos}"])
    assert eq(oracle.mha(f["mha_mq"], f["mha_k"], f["mha_v"], 0, 40, 64, 64, 2, 2), f["mha_mha_out_40"])
    assert eq(oracle.softmax(f["softmax_in"]), f["softmax_out"])
    assert eq(oracle.swiglu(f["swiglu_up"], f["swiglu_gate"]), f["swiglu_out"])
    assert eq(oracle.add(f["swiglu_up"], f["swiglu_gate"]), f["add_out"])
    assert eq(oracle.embedding(7, f["emb_table"]), f["emb_out_7"])
    assert oracle.argmax(f["argmax_in"]) == int(f["argmax_out"]) == 100


def test_per_op_against_float64(oracle):
    f = np.load(os.path.join(GOLD, "ops.npz"))
    x, w = f["matmul_x"].astype(np.float64), f["matmul_w"].astype(np.float64)
    np.testing.assert_allclose(f["matmul_y"], w @ x, rtol=0, atol=1e-5)
    np.testing.assert_allclose(f["rms_y"], refmath.rmsnorm(x, f["rms_w"], 1e-5), rtol=1e-6, atol=1e-6)
    s64, c64 = refmath.rope_tables(64, 64, 10000.0)
    np.testing.assert_allclose(f["rope_sin_10000"], s64, atol=2e-6)  # libm sinf vs float64 sin of the same arg
    np.testing.assert_allclose(f["rope_q_out"], refmath.rope(f["rope_q"], 37, s64, c64, 64), atol=1e-5)
    np.testing.assert_allclose(f["rope_k_out"], refmath.rope(f["rope_k"], 37, s64, c64, 64), atol=1e-5)
    for pos in (0, 17, 63):
        want = refmath.mha(f["mha_q"].astype(np.float64), f["mha_k"][1], f["mha_v"][1], pos, 64, 4, 2)
        np.testing.assert_allclose(f[f"mha_gqa_out_{pos}"], want, atol=1e-5)
    sm = f["softmax_in"].astype(np.float64)
    e = np.exp(sm - sm.max())
    np.testing.assert_allclose(f["softmax_out"], e / e.sum(), rtol=1e-5)
    np.testing.assert_allclose(f["swiglu_out"], refmath.swiglu(f["swiglu_up"], f["swiglu_gate"]), rtol=1e-5,
                               atol=1e-7)


def _hash32(x):
    x ^= x >> 16
    x = (x * 0x7feb352d) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846ca68b) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def _rng_u32(seed, stream, idx):
    h = _hash32(((seed * 0x9e3779b9) & 0xFFFFFFFF) ^ _hash32((stream + 0x632be5ab) & 0xFFFFFFFF))
    h = _hash32(h ^ (idx & 0xFFFFFFFF))
    return _hash32(h ^ (idx >> 32) ^ 0x85ebca6b)


def test_synthetic_generator_independent_python_restatement(oracle):
    """include/sli_synth.h re-implemented in pure Python: the C generator (shared with the HIP
    placement kernels) must produce exactly these values."""
    f = np.load(os.path.join(GOLD, "ops.npz"))
    for kind, idx, std in ((oracle.T_EMB, 0, 0.02), (oracle.T_WQ, 3, 1 / 64), (oracle.T_DOWN, 31, 1 / 105)):
        stream = oracle.stream_id(kind, idx)
        c = np.float32(oracle.synth_c(std))
        vals = []
        for i in range(64):
            a, b = _rng_u32(1, stream, 2 * i), _rng_u32(1, stream, 2 * i + 1)
            s = (a & 0xFFFF) + (a >> 16) + (b & 0xFFFF) + (b >> 16) - 2 * 65535
            vals.append(np.float32(s) * c)
        assert np.array_equal(np.array(vals, np.float32), f[f"synth_{kind}_{idx}"])
    # ~N(0, std): moments of a large draw
    big = oracle.synth_fill(200000, 5, oracle.stream_id(oracle.T_WK, 0), oracle.synth_c(1.0))
    assert abs(big.mean()) < 0.01 and abs(big.std() - 1.0) < 0.01


def test_f16_rounding_matches_numpy(oracle):
    r = np.random.default_rng(0)
    xs = (r.standard_normal(20000) * 10.0 ** r.integers(-9, 6, 20000)).astype(np.float32)
    xs = np.concatenate([xs, np.array([65504, 65520, 65519.99, 6e-8, 2.98e-8, 0.0, -0.0, np.inf], np.float32)])
    with np.errstate(over="ignore"):
        want = xs.astype(np.float16).astype(np.float32)
    assert np.array_equal(oracle.round_f16(xs).view(np.uint32), want.view(np.uint32))


def test_int8_row_quantisation(oracle):
    r = np.random.default_rng(1)
    row = r.standard_normal(4096).astype(np.float32)
    q, s = oracle.quant_row_i8(row)
    assert np.abs(q.astype(np.int32)).max() == 127
    assert np.float32(s) == np.float32(np.abs(row).max() / np.float32(127.0))
    assert np.abs(q * np.float32(s) - row).max() <= s / 2 + 1e-7
    q0, s0 = oracle.quant_row_i8(np.zeros(16, np.float32))
    assert s0 == 0.0 and not q0.any()


def test_reference_edge_cases(oracle):
    tab = np.arange(12, dtype=np.float32).reshape(4, 3)
    with pytest.raises(IndexError):
        oracle.embedding(4, tab)  # emb_kernel.cpp:10 (the reference would read one row past; we reject)
    assert oracle.argmax(np.array([1, 3, 3, 2], np.float32)) == 1  # std::max_element: first max
    assert np.array_equal(oracle.softmax(np.array([5.0], np.float32)), np.array([1.0], np.float32))
    # GQA RoPE: k (KV long) is rotated over its own length only (rope_kernel.cpp:27 runs to D)
    s, c = oracle.rope_cache(64, 8, 10000.0)
    q = np.ones(256, np.float32)
    k = np.ones(128, np.float32)
    q2, k2 = oracle.rope(q, k, 3, s, c, 64)
    assert np.array_equal(q2[:128], k2)
    # swiglu is the reference variant sigmoid(gate)*up, not SiLU
    assert np.isclose(oracle.swiglu(np.array([2.0], np.float32), np.array([0.0], np.float32))[0], 1.0)


def _max_element(x):
    """std::max_element (argmax.cpp:11) restated: keep the best unless `best < x[i]`."""
    best = 0
    for i in range(1, len(x)):
        if x[best] < x[i]:
            best = i
    return best


def test_argmax_special_values_follow_max_element(oracle):
    """The oracle's argmax on ±0 and NaN is std::max_element's `<` scan (the GPU key must match it)."""
    nan = np.float32("nan")
    cases = [[-0.0, 0.0], [0.0, -0.0], [nan, 1.0, 5.0], [1.0, nan, 5.0, nan], [-np.inf, nan, -np.inf],
             [nan, nan], [3.0, nan, 3.0, np.inf, nan, np.inf]]
    for c in cases:
        x = np.array(c, np.float32)
        assert oracle.argmax(x) == _max_element(x), c


def test_lazy_layers_match_eager(oracle):
    """orc_model_create_lazy (one layer of weights held, each layer regenerated inside the forward, over host
    threads) gives the eager model's logits bit for bit: f32 / f16 / int8 weights, MHA and GQA, two steps."""
    import numpy as np
    for (d, h, kvh, ffn), wm in [((64, 4, 4, 96), oracle.W_F32), ((64, 4, 2, 96), oracle.W_F16),
                                 ((128, 4, 1, 160), oracle.W_I8)]:
        cfg = oracle.Config(300, d, h, kvh, d // h, ffn, 3, 32, 1e-5, 10000.0)
        outs = []
        for lazy in (False, True):
            m = oracle.Model(cfg, seed=5, wmode=wm, kv_f16=True, lazy=lazy)
            m.fill_kv_synthetic(3, 20)
            outs.append([m.forward(7, 20), m.forward(11, 21)])
            m.close()
        for a, b in zip(*outs):
            assert np.array_equal(a, b)


# ---- pinned against the reference's own CPU build -----------------------------------------------------
from tests.golden import ref_cases as RC  # noqa: E402


@pytest.fixture(scope="module")
def ref_ops_gold():
    return np.load(os.path.join(GOLD, "ref_ops.npz"))


@pytest.mark.parametrize("name", sorted(RC.CASES))
def test_oracle_bit_exact_with_reference_build_ops(oracle, ref_ops_gold, name):
    inputs, outputs = RC.CASES[name](oracle, oracle)
    RC.check(name, ref_ops_gold, inputs, outputs)


def _check_model_fixture(g, toks, logits):
    assert np.array_equal(toks, g["tokens"]), (toks, g["tokens"])
    if "logits" in g:
        assert np.array_equal(logits.view(np.uint32), g["logits"].view(np.uint32))
    else:
        assert [RC.digest(r) for r in logits] == list(g["logits_sha256"])


@pytest.mark.parametrize("name", sorted(RC.MODELS))
def test_oracle_model_bit_exact_with_reference_op_layers(oracle, name):
    """model.cpp:40-187 composed over the reference's own op layers (weights through its flat-file loader)
    vs the oracle's orc_model_predict: same tokens, bit-identical logits at every step."""
    shape, n_kv, steps, seed = RC.MODELS[name]
    g = np.load(os.path.join(GOLD, name + ".npz"))
    m = oracle.Model(oracle.Config(n_kv_heads=n_kv, **shape), seed=seed)
    toks, logits = m.predict(RC.PROMPT, steps)
    m.close()
    _check_model_fixture(g, toks, logits)


def test_own_golden_fixtures_equal_reference_fixtures():
    """The round-1 fixtures (oracle outputs) are the reference's outputs too."""
    for own, ref in (("c0_mha.npz", "ref_c0_mha.npz"), ("c0_gqa.npz", "ref_c0_gqa.npz")):
        a, b = np.load(os.path.join(GOLD, own)), np.load(os.path.join(GOLD, ref))
        assert np.array_equal(a["tokens"], b["tokens"])
        assert np.array_equal(a["logits"].view(np.uint32), b["logits"].view(np.uint32))


def _ref_or_skip():
    import oracle.ref as R
    if not R.source_present():
        pytest.skip("/root/reference absent (GPU box): the committed reference vectors pin the oracle there")
    R.build()
    return R


def test_reference_build_live_random_ops(oracle):
    """Fresh random inputs (not the fixture seeds) through the live reference build and the oracle."""
    R = _ref_or_skip()
    r = np.random.default_rng(1234)
    for rows, cols in ((5, 4096), (33, 777), (1, 1)):
        x = r.standard_normal(cols).astype(np.float32)
        w = r.standard_normal((rows, cols)).astype(np.float32)
        assert np.array_equal(oracle.matmul(x, w), R.matmul(x, w))
        nw = r.standard_normal(cols).astype(np.float32)
        assert np.array_equal(oracle.rmsnorm(x, nw, 1e-6), R.rmsnorm(x, nw, 1e-6))
    for H, Hkv, hd, T, pos in ((8, 2, 64, 100, 99), (6, 3, 32, 50, 17), (16, 16, 128, 300, 0)):
        q = r.standard_normal(H * hd).astype(np.float32)
        kc = r.standard_normal((3, T, Hkv * hd)).astype(np.float32)
        vc = r.standard_normal((3, T, Hkv * hd)).astype(np.float32)
        assert np.array_equal(oracle.mha(q, kc, vc, 2, pos, T, hd, H, Hkv), R.mha(q, kc, vc, 2, pos, T, hd, H, Hkv))
        s, c = oracle.rope_cache(hd, T, 123456.0)
        s2, c2 = R.rope_cache(hd, T, 123456.0)
        assert np.array_equal(s, s2) and np.array_equal(c, c2)
        k = r.standard_normal(Hkv * hd).astype(np.float32)
        a, b = oracle.rope(q, k, pos, s, c, hd), R.rope(q, k, pos, s, c, hd)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    g = (5 * r.standard_normal(999)).astype(np.float32)
    assert np.array_equal(oracle.swiglu(g, g[::-1].copy()), R.swiglu(g, g[::-1].copy()))
    assert np.array_equal(oracle.softmax(g), R.softmax(g))
    for v in (g, np.array([np.nan, 2.0], np.float32), np.array([1.0, np.nan, 3.0], np.float32)):
        assert oracle.argmax(v) == R.argmax(v)


def test_reference_build_live_model(oracle, tmp_path):
    """A model shape the fixtures do not cover (3 layers, GQA-3, hd 32, θ 1e5), live through the
    reference's op layers vs the oracle."""
    R = _ref_or_skip()
    cfg = oracle.Config(vocab=300, dim=192, n_heads=6, n_kv_heads=2, head_dim=32, ffn=500, n_layers=3, max_len=40,
                        eps=1e-6, theta=100000.0)
    m = oracle.Model(cfg, seed=9)
    path = str(tmp_path / "w.bin")
    m.write_flat(path)
    ot, ol = m.predict([5, 6, 7], 30)
    m.close()
    rm = R.Model(cfg, path)
    rt, rl = rm.predict([5, 6, 7], 30)
    rm.close()
    assert np.array_equal(ot, rt)
    assert np.array_equal(ol.view(np.uint32), rl.view(np.uint32))
