"""The tensor-parallel engine at TP 2 / 4 / 8 on one GPU (sli_tp_group, the SURVEY.md §4 item-5 "fake
communicator"): N rank engines, each holding its sli_tp_plan shard (heads, kv heads, FFN columns, vocab
rows), step in lockstep; the all-reduces of the multi-GPU step are device-side reductions in rank order.
Every rank runs the multi-GPU kernels (partials into xpart, residual on rank 0, vocab-sharded LM head,
global first-max argmax), so this is the sharded engine itself against the UNSHARDED oracle.

Bar (north_star): greedy token ids bit-exact, logits within 1e-3 (fp16 / int8 weights: the oracle runs
in fp32 on the identically rounded / quantised weights and the same fp16 K/V rounding).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PROMPT = [1, 17, 42, 99]
PROMPTS = [[1, 17, 42, 99], [5, 6], [300, 2, 77, 8, 9], [11]]


def _ocfg(oracle, cfg):
    return oracle.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                         cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                         cfg.rms_norm_eps, cfg.rope_theta)


WMODE = {"f32": "W_F32", "f16": "W_F16", "i8": "W_I8"}


def _oracle_predict(oracle, cfg, w, kv, prompt, steps, seed=0):
    om = oracle.Model(_ocfg(oracle, cfg), seed=seed, wmode=getattr(oracle, WMODE[w]), kv_f16=(kv == "f16"))
    toks, logits = om.predict(prompt, steps)
    om.close()
    return toks, logits


@pytest.mark.parametrize("name,world,w,kv", [
    ("tiny", 2, "f16", "f16"), ("tiny", 4, "f16", "f16"), ("tiny", 4, "f32", "f32"), ("tiny", 2, "i8", "f16"),
    ("tiny-gqa", 2, "f16", "f16"), ("tiny-gqa", 2, "i8", "f16"),
    ("tiny-h8", 2, "f16", "f16"), ("tiny-h8", 4, "f16", "f16"), ("tiny-h8", 8, "f16", "f16"),
    ("tiny-h8", 8, "i8", "f16"), ("tiny-h8", 8, "f32", "f16"),
    ("tiny-gqa-h16", 2, "f16", "f16"), ("tiny-gqa-h16", 4, "f16", "f16"), ("tiny-gqa-h16", 8, "f16", "f16"),
])
def test_group_predict_36_steps(gpu, oracle, name, world, w, kv):
    """BASELINE configs[0] (4 prompt + 32 greedy tokens) through the sharded engine at TP = world."""
    from simplellminference_amd.model import TPGroup, preset
    cfg = preset(name)
    g = TPGroup(cfg, world, w_dtype=w, kv_dtype=kv, seed=0).init()
    toks, logits = g.predict(PROMPT, 36, want_logits=True)
    g.close()
    otoks, ologits = _oracle_predict(oracle, cfg, w, kv, PROMPT, 36)
    assert np.array_equal(toks, otoks), (toks, otoks)
    tol = 1e-4 if (w, kv) == ("f32", "f32") else 1e-3
    assert np.abs(logits - ologits).max() <= tol, np.abs(logits - ologits).max()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_group_batch_predict_ragged(gpu, oracle, world):
    """Batch 4 with ragged prompts, GQA 16/8, TP = world: per-sequence tokens and logits."""
    from simplellminference_amd.model import TPGroup, preset
    cfg = preset("tiny-gqa-h16")
    g = TPGroup(cfg, world, w_dtype="f16", kv_dtype="f16", seed=0, batch=len(PROMPTS)).init()
    toks, logits = g.predict_batch(PROMPTS, 24, want_logits=True)
    for b in range(len(PROMPTS)):  # every rank ends in the same decode state
        states = [m.state(b) for m in g.ranks]
        assert all(s == states[0] for s in states), states
    g.close()
    for b, p in enumerate(PROMPTS):
        otok, olog = _oracle_predict(oracle, cfg, "f16", "f16", p, 24)
        assert np.array_equal(toks[b], otok), (b, toks[b], otok)
        assert np.abs(logits[b] - olog).max() <= 1e-3


def test_group_argmax_across_vocab_shards(gpu, oracle):
    """Greedy tokens come from the global first max over the ranks' vocab shards: every rank's fed-token
    history equals the oracle's, whichever shard held the winner."""
    from simplellminference_amd.model import TPGroup, preset
    cfg = preset("tiny-h8")
    g = TPGroup(cfg, 8, w_dtype="f16", kv_dtype="f16", seed=5).init()
    toks = g.predict(PROMPT, 30)
    hists = [m.history(0, 30) for m in g.ranks]
    g.close()
    otoks, ologits = _oracle_predict(oracle, cfg, "f16", "f16", PROMPT, 30, seed=5)
    assert np.array_equal(toks, otoks)
    for h in hists:
        assert np.array_equal(h, otoks)
    shards = {int(np.argmax(ologits[p])) // (cfg.vocab_size // 8) for p in range(3, 29)}
    assert len(shards) >= 2, shards  # the winners really come from more than one rank's shard


@pytest.fixture(scope="module")
def c2_oracle(oracle):
    """Oracle logits of a 2-layer Llama-2-7B (configs[2] layer shapes) at pos 2047, f16 and i8 weights."""
    from simplellminference_amd.model import preset
    cfg = preset("llama2-7b", num_hidden_layers=2)
    out = {}
    for w in ("f16", "i8"):
        om = oracle.Model(_ocfg(oracle, cfg), seed=1, wmode=getattr(oracle, WMODE[w]), kv_f16=True)
        om.fill_kv_synthetic(7, 2047)
        out[w] = om.forward(1234, 2047)
        om.close()
    return cfg, out


@pytest.mark.parametrize("w", ["f16", "i8"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_group_c2_shard_shapes(gpu, c2_oracle, w, world):
    """BASELINE configs[2] shard shapes (TP 8: qkv 1536x4096, wo 4096x512, gate/up 2752x4096, down
    4096x1376, LM head 4000x4096, 4 heads of attention per rank), two layers, ctx 2048, one step at
    position 2047 against the unsharded oracle."""
    from simplellminference_amd.model import TPGroup
    cfg, want = c2_oracle
    g = TPGroup(cfg, world, w_dtype=w, kv_dtype="f16", seed=1).init()
    g.fill_kv_synthetic(7, 2047)
    got = g.forward(1234, 2047)
    again = g.forward(1234, 2047)
    g.close()
    assert np.array_equal(got, again)  # deterministic, idempotent
    assert np.abs(got - want[w]).max() <= 1e-3, np.abs(got - want[w]).max()
    assert int(np.argmax(got)) == int(np.argmax(want[w]))


@pytest.mark.timeout(600)
def test_group_c2_full_model_tp8(gpu, oracle):
    """BASELINE configs[2] end to end on one GPU: the whole 32-layer Llama-2-7B fp16 step (ctx 2048, pos 2047)
    sharded over 8 in-process ranks (rank-order sums in place of the all-reduces), against the unsharded
    lazy oracle (each layer's weights regenerated in turn)."""
    from simplellminference_amd.model import TPGroup, preset
    cfg = preset("llama2-7b")
    g = TPGroup(cfg, 8, w_dtype="f16", kv_dtype="f16", seed=1).init()
    g.fill_kv_synthetic(7, 2047)
    got = g.forward(1234, 2047)
    g.close()
    om = oracle.Model(_ocfg(oracle, cfg), seed=1, wmode=oracle.W_F16, kv_f16=True, lazy=True)
    om.fill_kv_synthetic(7, 2047)
    want = om.forward(1234, 2047)
    om.close()
    assert np.abs(got - want).max() <= 1e-3, np.abs(got - want).max()
    assert int(np.argmax(got)) == int(np.argmax(want))


C4_TOKENS = [1234 + 9001 * b for b in range(8)]
C4_POS = [4095, 4095, 100, 2047, 4000, 1, 3333, 4095]


@pytest.fixture(scope="module")
def c4_oracle(oracle):
    """Oracle logits of a 2-layer Llama-3-8B (configs[4] layer shapes), 8 sequences at ragged positions."""
    from simplellminference_amd.model import preset
    cfg = preset("llama3-8b", num_hidden_layers=2)
    om = oracle.Model(_ocfg(oracle, cfg), seed=1, wmode=oracle.W_F16, kv_f16=True)
    want = []
    for b in range(8):
        om.fill_kv_synthetic(7 + b, 4095)
        want.append(om.forward(C4_TOKENS[b], C4_POS[b]))
    om.close()
    return cfg, np.stack(want)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_group_c4_shard_shapes_batch8(gpu, c4_oracle, world):
    """BASELINE configs[4] at its TP (8: one kv head, FFN 1792, vocab 16032 rows per rank), batch 8 on the
    MFMA projections, two layers, ctx 4096, ragged positions: one step against the oracle per sequence."""
    from simplellminference_amd.model import TPGroup
    cfg, want = c4_oracle
    g = TPGroup(cfg, world, w_dtype="f16", kv_dtype="f16", seed=1, batch=8).init()
    g.fill_kv_synthetic(7, 4095)
    got = g.forward_batch(C4_TOKENS, C4_POS)
    g.close()
    for b in range(8):
        assert np.abs(got[b] - want[b]).max() <= 1e-3, (b, np.abs(got[b] - want[b]).max())
        assert int(np.argmax(got[b])) == int(np.argmax(want[b]))


def test_group_rank_handles_are_borrowed(gpu):
    """A rank handle cannot step or be destroyed on its own (the group's graph owns the lockstep)."""
    from simplellminference_amd import SliError
    from simplellminference_amd.model import TPGroup, preset
    g = TPGroup(preset("tiny"), 2, seed=0).init()
    with pytest.raises(SliError):
        g.ranks[1].step()
    g.close()
