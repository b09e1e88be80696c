"""The stream engine (stream_engine.h: the whole batch-1 decode step as ONE launch, a loader wave per CU
streaming every weight / K-V byte through an LDS ring while consumer waves wait for each op's input) against
the C oracle, and against the launch path of the same engine.

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
    gm = LlamaModel(config=cfg, w_dtype=w, kv_dtype=kv, seed=seed).init().set_exec("stream")
    return om, gm


GQA4 = {"num_key_value_heads": 1, "kv_hidden_size": 64}  # tiny with 4 q heads per kv head


@pytest.mark.parametrize("name,over", [("tiny", {}), ("tiny-gqa", {}), ("tiny", GQA4)],
                         ids=["mha", "gqa2", "gqa4"])
@pytest.mark.parametrize("w,kv,tol", [("f32", "f32", 1e-4), ("f16", "f16", 1e-3), ("i8", "f16", 1e-3),
                                      ("f32", "f16", 1e-3), ("f16", "f32", 1e-3)])
def test_stream_tiny_predict_parity(gpu, oracle, name, over, w, kv, tol):
    """BASELINE configs[0]: 4 prompt + 32 greedy tokens, the state advancing inside the one launch."""
    om, gm = _models(oracle, name, w, kv, **over)
    assert gm.exec_mode() == "stream"
    otok, olog = om.predict(PROMPT, 36)
    gtok, glog = gm.predict(PROMPT, 36, want_logits=True)
    assert gm.state()["error"] == 0
    gm.close()
    om.close()
    assert np.array_equal(gtok, otok), (gtok, otok)
    assert np.abs(glog - olog).max() <= tol, np.abs(glog - olog).max()


@pytest.mark.parametrize("w", ["f16", "i8"])
def test_stream_llama7b_shape_two_layers(gpu, oracle, w):
    """Llama-2-7B layer shapes at ctx 2048 (KV filled to 2046, step at 2047): 8 attention jobs per head on 256
    CUs, the full 32000-row LM head, against the oracle."""
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


@pytest.mark.parametrize("pos", [0, 1, 63, 64, 255, 256, 1000])
def test_stream_llama7b_shape_positions(gpu, oracle, pos):
    """Ragged live contexts: the last attention job partially filled, jobs past the context idle."""
    om, gm = _models(oracle, "llama2-7b", "f16", "f16", seed=3, num_hidden_layers=1, max_length=1024)
    if pos:
        om.fill_kv_synthetic(5, pos)
        gm.fill_kv_synthetic(5, pos)
    want = om.forward(77, pos)
    got = gm.forward(77, pos)
    assert gm.state()["error"] == 0
    gm.close()
    om.close()
    assert np.abs(got - want).max() <= 1e-3
    assert int(np.argmax(got)) == int(np.argmax(want))


def test_stream_llama3_shape_gqa4(gpu, oracle):
    """Llama-3-8B layer shapes at batch 1 (GQA-4, I = 14336, the 128256-row head) at ctx 4096."""
    om, gm = _models(oracle, "llama3-8b", "f16", "f16", seed=1, num_hidden_layers=1)
    om.fill_kv_synthetic(9, 3000)
    gm.fill_kv_synthetic(9, 3000)
    want = om.forward(4321, 3000)
    got = gm.forward(4321, 3000)
    assert gm.state()["error"] == 0
    gm.close()
    om.close()
    assert np.abs(got - want).max() <= 1e-3
    assert int(np.argmax(got)) == int(np.argmax(want))


def test_stream_short_context_many_heads(gpu, oracle):
    om, gm = _models(oracle, "llama2-7b", "f16", "f16", seed=2, num_hidden_layers=2, max_length=64)
    otok, olog = om.predict(PROMPT, 8)
    gtok, glog = gm.predict(PROMPT, 8, want_logits=True)
    gm.close()
    om.close()
    assert np.array_equal(gtok, otok)
    assert np.abs(glog - olog).max() <= 1e-3


@pytest.mark.parametrize("w", ["f16", "i8"])
def test_stream_matches_launches_full_7b(gpu, w):
    """The full 32-layer bench workload: the stream step and the launch graph of the same engine agree, the
    stream step is deterministic and idempotent, and switching modes keeps the decode state."""
    from simplellminference_amd.model import LlamaModel, preset
    gm = LlamaModel(config=preset("llama2-7b"), w_dtype=w, kv_dtype="f16", seed=1).init()
    gm.set_exec("launches")
    gm.fill_kv_synthetic(7, 2047)
    ref = gm.forward(1234, 2047)
    gm.set_exec("stream")
    a = gm.forward(1234, 2047)
    b = gm.forward(1234, 2047)
    assert gm.state()["error"] == 0
    assert np.array_equal(a, b)
    assert np.abs(a - ref).max() <= 1e-3 * max(1.0, float(np.abs(ref).max()))
    assert int(np.argmax(a)) == int(np.argmax(ref))
    gm.set_exec("launches")
    gm.set_state(1234, 2000, advance=True)
    for _ in range(8):
        gm.step()
    want = gm.history(0, 2009)[2000:2009]
    gm.set_exec("stream")
    gm.set_state(1234, 2000, advance=True)
    for _ in range(8):
        gm.step()
    got = gm.history(0, 2009)[2000:2009]
    gm.close()
    assert np.array_equal(got, want)


def test_stream_unsupported_configs_refused(gpu):
    from simplellminference_amd import SliError
    from simplellminference_amd.model import LlamaModel, preset
    m = LlamaModel(config=preset("tiny-gqa"), w_dtype="f16", kv_dtype="f16", seed=0, batch=2).init()
    with pytest.raises(SliError):
        m.set_exec("stream")  # batch > 1 runs the MFMA launches
    m.close()
