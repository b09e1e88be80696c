"""Prompt prefill (sli_model_prefill): the prompt's positions 0..n-2 run through the
layers 8 at a time with the projections on MFMA, then decoding continues from the last prompt token. The
reference teacher-forces the prompt one token per forward (model.cpp:157-165); the oracle's predict does
the same, so the bar is the oracle's predict: greedy token ids bit-exact, logits of every computed
position within 1e-3, and the K/V rows the prefill writes within the fp16 cache rounding.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(oracle, name, w="f16", kv="f16", seed=0, **over):
    from simplellminference_amd.model import LlamaModel, preset
    cfg = preset(name, **over)
    ocfg = oracle.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                         cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                         cfg.rms_norm_eps, cfg.rope_theta)
    wmode = {"f32": oracle.W_F32, "f16": oracle.W_F16, "i8": oracle.W_I8}[w]
    om = oracle.Model(ocfg, seed=seed, wmode=wmode, kv_f16=(kv == "f16"))
    gm = LlamaModel(config=cfg, w_dtype=w, kv_dtype=kv, seed=seed).init()
    return cfg, om, gm


def _prompt(n, vocab, seed=3):
    return [int(t) for t in np.random.default_rng(seed + n).integers(0, vocab, n)]


@pytest.mark.parametrize("name", ["tiny", "tiny-gqa"])
@pytest.mark.parametrize("n", [1, 2, 8, 9, 17, 33])
def test_prefill_predict_matches_oracle(gpu, oracle, name, n):
    """Ragged chunking (n - 1 prefilled positions = 0, 1, 7, 8, 16, 32 lanes), then greedy to 40 positions."""
    cfg, om, gm = _pair(oracle, name)
    prompt = _prompt(n, cfg.vocab_size)
    steps = 40
    otok, olog = om.predict(prompt, steps)
    gtok, glog = gm.predict_prefill(prompt, steps, want_logits=True)
    gm.close()
    om.close()
    assert np.array_equal(gtok, otok), (gtok, otok)
    assert np.isnan(glog[:n - 1]).all()
    err = np.abs(glog[n - 1:] - olog[n - 1:]).max()
    assert err <= 1e-3, err


def test_prefill_kv_rows_match_oracle(gpu, oracle):
    cfg, om, gm = _pair(oracle, "tiny-gqa")
    prompt = _prompt(21, cfg.vocab_size)
    om.predict(prompt, 21)
    gm.prefill(prompt)
    st = gm.state()
    assert st["pos"] == 20 and st["token"] == prompt[-1]
    assert np.array_equal(gm.history(0, 21), prompt)
    ok, ov = om.kv_cache()
    for layer in range(cfg.num_hidden_layers):  # rows 0..19 come from the prefill (row 20 from the step)
        np.testing.assert_allclose(gm.kv(layer, 0, 20), ok[layer, :20], rtol=0, atol=2e-3)
        np.testing.assert_allclose(gm.kv(layer, 1, 20), ov[layer, :20], rtol=0, atol=2e-3)
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
    assert np.array_equal(gtok, otok)
    assert np.abs(glog[39:] - olog[39:]).max() <= 1e-3


@pytest.mark.parametrize("w,kv", [("f32", "f32"), ("i8", "f16")])
def test_prefill_without_mfma_teacher_forces(gpu, oracle, w, kv):
    """fp32 / int8 weights have no MFMA projection: the prompt runs through the decode step (same tokens)."""
    cfg, om, gm = _pair(oracle, "tiny-gqa", w=w, kv=kv)
    prompt = _prompt(13, cfg.vocab_size)
    otok, olog = om.predict(prompt, 30)
    gtok, glog = gm.predict_prefill(prompt, 30, want_logits=True)
    gm.close()
    om.close()
    assert np.array_equal(gtok, otok)
    tol = 1e-4 if w == "f32" else 1e-3
    assert np.abs(glog[12:] - olog[12:]).max() <= tol


def test_prefill_then_persistent_decode(gpu, oracle):
    cfg, om, gm = _pair(oracle, "tiny")
    gm.set_exec("persistent")
    prompt = _prompt(19, cfg.vocab_size)
    otok, _ = om.predict(prompt, 36)
    gtok = gm.predict_prefill(prompt, 36)
    gm.close()
    om.close()
    assert np.array_equal(gtok, otok)
