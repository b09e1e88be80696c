"""The batch-1 wo GEMV split over its input columns (engine.hip wo_ksplit, gemv.h EpiKPart / XStageSum /
EpiStoreSum; SLI_WO_KSPLIT=2|4): each workgroup block streams one column block of wo and merges only those heads'
attention split partials; the gate/up GEMV stages x + the partial row sums, and the down GEMV adds the same sum
as its residual. Same bar as tests/test_gpu_model.py: greedy tokens bit-exact, logits within 1e-3 of the
oracle (fp32 weights 1e-4)."""
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
    gm = LlamaModel(config=cfg, w_dtype=w, kv_dtype=kv, seed=seed).init()
    return om, gm


@pytest.mark.parametrize("ks", ["2", "4"])
@pytest.mark.parametrize("name", ["tiny", "tiny-gqa"])
@pytest.mark.parametrize("w,kv,tol", [("f32", "f32", 1e-4), ("f16", "f16", 1e-3), ("i8", "f16", 1e-3)])
def test_tiny_predict_wo_ksplit(gpu, oracle, monkeypatch, ks, name, w, kv, tol):
    monkeypatch.setenv("SLI_WO_KSPLIT", ks)
    om, gm = _models(oracle, name, w, kv)
    otok, olog = om.predict(PROMPT, 36)
    gtok, glog = gm.predict(PROMPT, 36, want_logits=True)
    gm.close()
    om.close()
    assert np.array_equal(gtok, otok), (gtok, otok)
    assert np.abs(glog - olog).max() <= tol


@pytest.mark.parametrize("ks", ["1", "2", "4"])
@pytest.mark.parametrize("w", ["f16", "i8"])
def test_llama7b_two_layers_wo_ksplit(gpu, oracle, monkeypatch, ks, w):
    """Llama-2-7B layer shapes at ctx 2048 (8 attention splits per head), step at position 2047."""
    monkeypatch.setenv("SLI_WO_KSPLIT", ks)
    om, gm = _models(oracle, "llama2-7b", w, "f16", seed=1, num_hidden_layers=2)
    om.fill_kv_synthetic(7, 2047)
    gm.fill_kv_synthetic(7, 2047)
    want = om.forward(1234, 2047)
    got = gm.forward(1234, 2047)
    gm.close()
    om.close()
    assert np.abs(got - want).max() <= 1e-3
    assert int(np.argmax(got)) == int(np.argmax(want))


@pytest.mark.parametrize("merge,ks", [("0", "1"), ("1", "1"), ("1", "2"), ("1", "4")])
def test_ctx4096_sixteen_splits_wo_ksplit(gpu, oracle, monkeypatch, merge, ks):
    """ctx 4096 (16 splits per head), GQA-4 Llama-3-8B shapes (batch 1: run as GQA-2 groups), 2 layers: the
    default (merge 0: the attention's last arriver merges, wo stages a plain input) and the wo-side merges
    (the NS = 16 batch), unsplit and K-split."""
    monkeypatch.setenv("SLI_WO_MERGE", merge)
    monkeypatch.setenv("SLI_WO_KSPLIT", ks)
    om, gm = _models(oracle, "llama3-8b", "f16", "f16", seed=1, num_hidden_layers=2, vocab_size=32000)
    om.fill_kv_synthetic(7, 4095)
    gm.fill_kv_synthetic(7, 4095)
    want = om.forward(77, 4095)
    got = gm.forward(77, 4095)
    gm.close()
    om.close()
    assert np.abs(got - want).max() <= 1e-3


@pytest.mark.parametrize("ks", ["2", "4"])
def test_wo_ksplit_greedy_and_prefill(gpu, oracle, monkeypatch, ks):
    """Prefill (chunked MFMA GEMMs, not split) then K-split decode steps."""
    monkeypatch.setenv("SLI_WO_KSPLIT", ks)
    om, gm = _models(oracle, "tiny-gqa", "f16", "f16", max_length=160)
    prompt = [int(t) for t in np.random.default_rng(5).integers(0, 512, 70)]
    otok, olog = om.predict(prompt, 100)
    gtok, glog = gm.predict_prefill(prompt, 100, want_logits=True)
    assert np.array_equal(gtok, otok)
    assert np.abs(glog[69:] - olog[69:]).max() <= 1e-3
    gm.close()
    om.close()

