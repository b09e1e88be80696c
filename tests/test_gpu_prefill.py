"""Prompt prefill (sli_model_prefill): the prompt's positions 0..n-2 run through the
layers in chunks of up to 256 positions — every projection one MFMA GEMM over the chunk, attention
block-causal over the cache — then decoding continues from the last prompt token. The reference
teacher-forces the prompt one token per forward (model.cpp:157-165); the oracle's predict does the same, so
the bar is the oracle's predict: greedy token ids bit-exact, logits of every computed position within 1e-3,
and the K/V rows the prefill writes within the fp16 cache rounding.

Chunk sizes 32 / 64 / 128 / 256 (prefill.h kPfMaxChunk): the prompt lengths below cover every chunk size,
one and two chunks, a ragged last chunk and the padding rows of a chunk.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ocfg(oracle, cfg):
    return oracle.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                         cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                         cfg.rms_norm_eps, cfg.rope_theta)


def _wmode(oracle, w):
    return {"f32": oracle.W_F32, "f16": oracle.W_F16, "i8": oracle.W_I8}[w]


def _pair(oracle, name, w="f16", kv="f16", seed=0, **over):
    from simplellminference_amd.model import LlamaModel, preset
    cfg = preset(name, **over)
    om = oracle.Model(_ocfg(oracle, cfg), seed=seed, wmode=_wmode(oracle, w), kv_f16=(kv == "f16"))
    gm = LlamaModel(config=cfg, w_dtype=w, kv_dtype=kv, seed=seed).init()
    return cfg, om, gm


def _prompt(n, vocab, seed=3):
    return [int(t) for t in np.random.default_rng(seed + n).integers(0, vocab, n)]


def _check(gtok, glog, otok, olog, n, tol=1e-3):
    assert np.array_equal(gtok, otok), (gtok, otok)
    assert np.isnan(glog[:n - 1]).all()
    err = np.abs(glog[n - 1:] - olog[n - 1:]).max()
    assert err <= tol, err


@pytest.mark.parametrize("name", ["tiny", "tiny-gqa"])
@pytest.mark.parametrize("n", [1, 2, 9, 33, 63])
def test_prefill_predict_matches_oracle(gpu, oracle, name, n):
    """Short prompts (n - 1 prefilled positions = 0, 1, 8, 32, 62: chunk sizes 32 and 64, padding rows),
    then greedy up to the context end."""
    cfg, om, gm = _pair(oracle, name)
    prompt = _prompt(n, cfg.vocab_size)
    steps = 64
    otok, olog = om.predict(prompt, steps)
    gtok, glog = gm.predict_prefill(prompt, steps, want_logits=True)
    gm.close()
    om.close()
    _check(gtok, glog, otok, olog, n)


@pytest.mark.parametrize("n", [129, 200, 257, 300])
def test_prefill_long_prompts(gpu, oracle, n):
    """Prompts of 129..300 tokens: one chunk of 128 / 256 rows, two chunks (256 + 0 / 43 rows), GQA."""
    cfg, om, gm = _pair(oracle, "tiny-gqa", max_length=320)
    prompt = _prompt(n, cfg.vocab_size)
    steps = n + 12
    otok, olog = om.predict(prompt, steps)
    gtok, glog = gm.predict_prefill(prompt, steps, want_logits=True)
    gm.close()
    om.close()
    _check(gtok, glog, otok, olog, n)


@pytest.mark.parametrize("n", [21, 150])
def test_prefill_kv_rows_match_oracle(gpu, oracle, n):
    cfg, om, gm = _pair(oracle, "tiny-gqa", max_length=160)
    prompt = _prompt(n, cfg.vocab_size)
    om.predict(prompt, n)
    gm.prefill(prompt)
    st = gm.state()
    assert st["pos"] == n - 1 and st["token"] == prompt[-1]
    assert np.array_equal(gm.history(0, n), prompt)
    ok, ov = om.kv_cache()
    for layer in range(cfg.num_hidden_layers):  # rows 0..n-2 come from the prefill (row n-1 from the step)
        np.testing.assert_allclose(gm.kv(layer, 0, n - 1), ok[layer, :n - 1], rtol=0, atol=2e-3)
        np.testing.assert_allclose(gm.kv(layer, 1, n - 1), ov[layer, :n - 1], rtol=0, atol=2e-3)
    gm.close()
    om.close()


def test_prefill_llama7b_shape(gpu, oracle):
    """Llama-2-7B layer shapes (2 layers, full vocab): a 40-token prompt prefilled on MFMA, then 4 greedy
    steps, against the oracle's token-by-token predict."""
    cfg, om, gm = _pair(oracle, "llama2-7b", seed=1, num_hidden_layers=2, max_length=64)
    prompt = _prompt(40, cfg.vocab_size)
    otok, olog = om.predict(prompt, 44)
    gtok, glog = gm.predict_prefill(prompt, 44, want_logits=True)
    gm.close()
    om.close()
    _check(gtok, glog, otok, olog, 40)


@pytest.mark.timeout(400)
def test_prefill_llama7b_shape_long(gpu, oracle):
    """Llama-2-7B layer shapes (2 layers; vocab cut to 512 so the CPU oracle stays in budget), a 140-token
    prompt: one 256-row chunk with 117 padding rows, hd 128, 4096 x 11008 projections."""
    cfg, om, gm = _pair(oracle, "llama2-7b", seed=1, num_hidden_layers=2, max_length=160, vocab_size=512)
    prompt = _prompt(140, cfg.vocab_size)
    otok, olog = om.predict(prompt, 144)
    gtok, glog = gm.predict_prefill(prompt, 144, want_logits=True)
    gm.close()
    om.close()
    _check(gtok, glog, otok, olog, 140)


@pytest.mark.parametrize("kv", ["f16", "f32"])
@pytest.mark.parametrize("n", [13, 150])
def test_prefill_int8(gpu, oracle, kv, n):
    """int8 weights: the GEMM converts each int8 weight image to fp16 in registers (exact) and applies the
    per-row scales in the epilogue."""
    cfg, om, gm = _pair(oracle, "tiny-gqa", w="i8", kv=kv, max_length=160)
    prompt = _prompt(n, cfg.vocab_size)
    otok, olog = om.predict(prompt, n + 10)
    gtok, glog = gm.predict_prefill(prompt, n + 10, want_logits=True)
    gm.close()
    om.close()
    _check(gtok, glog, otok, olog, n)


@pytest.mark.parametrize("over", [dict(intermediate_size=704), dict(hidden_size=320, num_attention_heads=5,
                                                                      num_key_value_heads=5, kv_hidden_size=320)])
def test_prefill_int8_half_last_stage(gpu, oracle, over):
    """int8 GEMM depths that are 64 mod 128 (the int8 pgemm stage is 128 deep): the last stage is a half stage
    (prefill.h). Llama-2-7B int8 at TP 4 has such a down projection (2752 = 21.5 x 128); here the FFN width
    704 (down) and a hidden size of 320 (q/k/v, gate/up and wo)."""
    cfg, om, gm = _pair(oracle, "tiny", w="i8", kv="f16", max_length=160, **over)
    assert gm.prefill_path() == "mfma"
    prompt = _prompt(150, cfg.vocab_size)
    otok, olog = om.predict(prompt, 160)
    gtok, glog = gm.predict_prefill(prompt, 160, want_logits=True)
    gm.close()
    om.close()
    _check(gtok, glog, otok, olog, 150)


def test_prefill_f32_weights_teacher_forces(gpu, oracle):
    """fp32 weights have no MFMA projection: the prompt runs through the decode step (same tokens)."""
    cfg, om, gm = _pair(oracle, "tiny-gqa", w="f32", kv="f32")
    assert gm.prefill_path() == "decode"
    prompt = _prompt(13, cfg.vocab_size)
    otok, olog = om.predict(prompt, 30)
    gtok, glog = gm.predict_prefill(prompt, 30, want_logits=True)
    gm.close()
    om.close()
    _check(gtok, glog, otok, olog, 13, tol=1e-4)


def test_prefill_twice_reuses_graphs(gpu, oracle):
    """A second prompt on the same model (graphs already captured, other chunk sizes) gives the oracle's
    tokens too: the chunk position and count come from device memory, not from the capture."""
    cfg, om, gm = _pair(oracle, "tiny-gqa", max_length=320)
    for n in (70, 260, 5):
        prompt = _prompt(n, cfg.vocab_size, seed=11)
        otok, olog = om.predict(prompt, n + 6)
        gtok, glog = gm.predict_prefill(prompt, n + 6, want_logits=True)
        _check(gtok, glog, otok, olog, n)
    gm.close()
    om.close()


@pytest.mark.parametrize("name,tp,w,over", [("tiny-h8", 2, "f16", {}), ("tiny-h8", 8, "f16", {}),
                                            ("tiny-gqa-h16", 4, "i8", {}),
                                            ("tiny-gqa-h16", 4, "i8", dict(intermediate_size=2816))])
def test_prefill_tp_group(gpu, oracle, name, tp, w, over):
    """The sharded prefill (sli_tp_group_prefill): every rank's chunk GEMMs on its shard, the residual rows
    summed over the ranks after every wo and down GEMM; against the unsharded oracle. FFN 2816 at TP 4: each
    rank's int8 down projection is 704 deep, a half last stage (the Llama-2-7B int8 TP-4 case)."""
    from simplellminference_amd.model import TPGroup, preset
    cfg = preset(name, max_length=160, **over)
    g = TPGroup(cfg, tp, w_dtype=w, kv_dtype="f16", seed=2).init()
    om = oracle.Model(_ocfg(oracle, cfg), seed=2, wmode=_wmode(oracle, w), kv_f16=True)
    prompt = _prompt(140, cfg.vocab_size)
    otok, olog = om.predict(prompt, 150)
    gtok, glog = g.predict_prefill(prompt, 150, want_logits=True)
    states = [m.state() for m in g.ranks]
    g.close()
    om.close()
    assert all(s == states[0] for s in states), states
    _check(gtok, glog, otok, olog, 140)
