"""SPELayer (simplellminference_amd/encode.py) — the reference's tokenizer layer, source/op/encode.cpp:5-27 — and
``LlamaModel.predict`` on text (model.cpp:142-187).

No sentencepiece model ships with the reference (no checkpoint or tokenizer file), so the tests
train a small BPE model offline with the same library and check the layer's contract: encode/decode round trip,
piece count, the load error, and the text the reference's predict loop prints. The GPU test runs the text path
through libsli.so and pins it to the C oracle's greedy tokens.
"""
import io
import random

import numpy as np
import pytest

spm = pytest.importorskip("sentencepiece")

WORDS = ("the quick brown fox jumps over a lazy dog while every wave streams its tile of weights from memory "
         "and the last arriver merges the partial sums").split()


@pytest.fixture(scope="module")
def spm_model(tmp_path_factory):
    rng = random.Random(0)
    lines = [" ".join(rng.choice(WORDS) for _ in range(14)) for _ in range(600)]
    buf = io.BytesIO()
    spm.SentencePieceTrainer.train(sentence_iterator=iter(lines), model_writer=buf, vocab_size=160,
                                   model_type="bpe", minloglevel=2)
    path = tmp_path_factory.mktemp("spm") / "tok.model"
    path.write_bytes(buf.getvalue())
    return str(path)


def reference_predict_text(layer, prompt_ids, max_length, argmax_after):
    """model.cpp:142-187 restated: print the first prompt token, then after each forward the next prompt token
    while the prompt lasts, else the argmax (``argmax_after(pos)`` = argmax of the forward at pos)."""
    out = layer.decode([prompt_ids[0]]) + " "
    pos = 0
    while pos < max_length:
        if pos < len(prompt_ids) - 1:
            nxt = prompt_ids[pos + 1]
        else:
            nxt = argmax_after(pos)
        pos += 1
        out += layer.decode([nxt]) + " "
    return out + "\n"


def test_encode_decode_round_trip(spm_model):
    from simplellminference_amd.encode import SPELayer
    layer = SPELayer(spm_model)
    assert layer.GetVocabularySize() == 160
    text = "the quick brown fox merges the partial sums"
    ids = layer.encode(text)
    assert ids and all(isinstance(i, int) and 0 <= i < 160 for i in ids)
    assert layer.decode(ids) == text
    assert layer.encode("") == [] and layer.decode([]) == ""
    # the in-memory form loads the same processor
    with open(spm_model, "rb") as f:
        assert SPELayer(model_proto=f.read()).encode(text) == ids


def test_load_failure_raises_runtime_error(tmp_path):
    from simplellminference_amd.encode import SPELayer
    with pytest.raises(RuntimeError):
        SPELayer(str(tmp_path / "missing.model"))  # encode.cpp:8-10
    bad = tmp_path / "bad.model"
    bad.write_bytes(b"not a model")
    with pytest.raises(RuntimeError):
        SPELayer(str(bad))


def test_init_loads_tokenizer_before_the_device(tmp_path):
    # create_nonparam_layers (model.cpp:328) throws from SPELayer's constructor: no engine is created
    from simplellminference_amd.model import LlamaModel, preset
    m = LlamaModel(tokenizer_path=str(tmp_path / "missing.model"), config=preset("tiny"), seed=0)
    with pytest.raises(RuntimeError):
        m.init()
    assert m._h is None


@pytest.mark.parametrize("max_length", [0, 1, 3, 4, 9])
def test_render_matches_reference_loop(spm_model, max_length):
    from simplellminference_amd.encode import SPELayer, render_predict
    layer = SPELayer(spm_model)
    prompt = layer.encode("the lazy dog streams its tile")
    assert len(prompt) >= 4

    def argmax_after(pos):
        return (7 * pos + 3) % 160

    want = reference_predict_text(layer, prompt, max_length, argmax_after)
    # the engine's view of the same run: the token fed at each position, and the token after the last forward
    fed = [prompt[0]]
    for pos in range(max_length):
        fed.append(prompt[pos + 1] if pos < len(prompt) - 1 else argmax_after(pos))
    assert render_predict(layer, fed[:max_length], fed[max_length]) == want


@pytest.mark.gpu
def test_predict_text_matches_oracle(gpu, oracle, spm_model, capsys):
    from simplellminference_amd.encode import SPELayer, render_predict
    from simplellminference_amd.model import LlamaModel, preset
    cfg = preset("tiny-gqa", vocab_size=160)  # the tokenizer's vocabulary, as a real checkpoint pairs them
    layer = SPELayer(spm_model)
    prompt = "the quick brown fox jumps"
    ids = layer.encode(prompt)
    steps = 20
    ocfg = oracle.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                         cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                         cfg.rms_norm_eps, cfg.rope_theta)
    om = oracle.Model(ocfg, seed=0, wmode=oracle.W_F16, kv_f16=True)
    otok, olog = om.predict(ids, steps)
    want = render_predict(layer, otok, int(np.argmax(olog[-1])))
    gm = LlamaModel(tokenizer_path=spm_model, config=cfg, w_dtype="f16", kv_dtype="f16", seed=0).init()
    got = gm.predict(prompt, steps)
    gm.close()
    assert got == want
    assert capsys.readouterr().out == want  # printed like the reference (std::cout, model.cpp:155-186)
