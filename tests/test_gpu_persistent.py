"""The persistent step (persist.h: the whole batch-1 decode step as ONE launch, grid barriers between the
phases, sc1 hand-offs) against the C oracle, and against the launch path of the same engine.

Bar (north_star): greedy token ids bit-exact, logits within 1e-3 (fp32-weight runs 1e-4); the fp16/int8
oracle runs in fp32 on the identically rounded / quantised weights and the same fp16 K/V rounding.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PROMPT = [1, 17, 42, 99]


def _models(oracle, name, w, kv, seed=0, **over):
    from simplellminference_amd.model import LlamaModel, preset
    cfg = preset(name, **over)
    ocfg = oracle.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                         cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                         cfg.rms_norm_eps, cfg.rope_theta)
    wmode = {"f32": oracle.W_F32, "f16": oracle.W_F16, "i8": oracle.W_I8}[w]
    om = oracle.Model(ocfg, seed=seed, wmode=wmode, kv_f16=(kv == "f16"))
    gm = LlamaModel(config=cfg, w_dtype=w, kv_dtype=kv, seed=seed).init().set_exec("persistent")
    return om, gm


@pytest.mark.parametrize("name", ["tiny", "tiny-gqa"])
@pytest.mark.parametrize("w,kv,tol", [("f32", "f32", 1e-4), ("f16", "f16", 1e-3), ("i8", "f16", 1e-3),
                                      ("f32", "f16", 1e-3), ("f16", "f32", 1e-3)])
def test_persistent_tiny_predict_parity(gpu, oracle, name, w, kv, tol):
    """BASELINE configs[0]: 4 prompt + 32 greedy tokens, the state advancing inside the one launch."""
    om, gm = _models(oracle, name, w, kv)
    assert gm.exec_mode() == "persistent"
    otok, olog = om.predict(PROMPT, 36)
    gtok, glog = gm.predict(PROMPT, 36, want_logits=True)
    assert gm.state()["error"] == 0
    gm.close()
    om.close()
    assert np.array_equal(gtok, otok), (gtok, otok)
    assert np.abs(glog - olog).max() <= tol, np.abs(glog - olog).max()


@pytest.mark.parametrize("w", ["f16", "i8"])
def test_persistent_llama7b_shape_two_layers(gpu, oracle, w):
    """Llama-2-7B layer shapes at ctx 2048 (KV filled to 2046, step at 2047): 7 attention splits per head,
    the full 32000-row LM head, against the oracle."""
    om, gm = _models(oracle, "llama2-7b", w, "f16", seed=1, num_hidden_layers=2)
    om.fill_kv_synthetic(7, 2047)
    gm.fill_kv_synthetic(7, 2047)
    want = om.forward(1234, 2047)
    got = gm.forward(1234, 2047)
    assert gm.state()["error"] == 0
    gm.close()
    om.close()
    assert np.abs(got - want).max() <= 1e-3
    assert int(np.argmax(got)) == int(np.argmax(want))


def test_persistent_short_context_many_heads(gpu, oracle):
    om, gm = _models(oracle, "llama2-7b", "f16", "f16", seed=2, num_hidden_layers=2, max_length=64)
    otok, olog = om.predict(PROMPT, 8)
    gtok, glog = gm.predict(PROMPT, 8, want_logits=True)
    gm.close()
    om.close()
    assert np.array_equal(gtok, otok)
    assert np.abs(glog - olog).max() <= 1e-3


@pytest.mark.parametrize("w", ["f16", "i8"])
def test_persistent_matches_launches_full_7b(gpu, w):
    """The full 32-layer bench workload: the one-launch step and the launch graph of the same engine agree
    (same kernels' arithmetic up to the RMS reduction order), the step is deterministic and idempotent, and
    the launch and persistent modes switch on one model without losing the decode state."""
    from simplellminference_amd.model import LlamaModel, preset
    gm = LlamaModel(config=preset("llama2-7b"), w_dtype=w, kv_dtype="f16", seed=1).init()
    gm.fill_kv_synthetic(7, 2047)
    ref = gm.forward(1234, 2047)
    gm.set_exec("persistent")
    a = gm.forward(1234, 2047)
    b = gm.forward(1234, 2047)
    assert gm.state()["error"] == 0
    assert np.array_equal(a, b)
    assert np.abs(a - ref).max() <= 1e-4 * max(1.0, float(np.abs(ref).max()))
    assert int(np.argmax(a)) == int(np.argmax(ref))
    # a greedy run in persistent mode continues exactly where a launch-mode run would
    gm.set_exec("launches")
    gm.set_state(1234, 2000, advance=True)
    for _ in range(8):
        gm.step()
    want = gm.history(0, 2009)[2000:2009]
    gm.set_exec("persistent")
    gm.set_state(1234, 2000, advance=True)
    for _ in range(8):
        gm.step()
    got = gm.history(0, 2009)[2000:2009]
    gm.close()
    assert np.array_equal(got, want)


def test_persistent_unsupported_configs_refused(gpu):
    from simplellminference_amd import SliError
    from simplellminference_amd.model import LlamaModel, preset
    m = LlamaModel(config=preset("tiny-gqa"), w_dtype="f16", kv_dtype="f16", seed=0, batch=2).init()
    with pytest.raises(SliError):
        m.set_exec("persistent")  # batch > 1 runs the MFMA launches
    assert m.exec_mode() == "launches"
    m.close()
