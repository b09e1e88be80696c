"""The fused q/k/v + attention launch (csrc/qkv_attn.h) against the two-launch step it replaces, and against the
oracle.

The fused launch's q/k/v units are the same row sums as the separate GEMV, and its attention is attention.h's
register-staged split kernel. At every shape below the two-launch step's attention is that same kernel too: its
split merge is deferred to the wo GEMV (at most 8 splits per head: tiny max_length 64, Llama-2-7B ctx 2048 at 256
positions per split), and the MFMA kernel (attn_mfma.h) never takes a deferred merge (ops.hip attn_mfma_ok). So the
two must agree BIT FOR BIT (the guard that catches ordering or hand-off bugs in qkv_attn.h): each case runs in two
child processes, SLI_QKV_ATTN=1 and SLI_QKV_ATTN=0 (the switch is read once per process). Cases: the
tiny presets at TP 1 (MHA and GQA-2, head_dim 64, fp16 / int8 weights, a greedy run of 24 tokens, also held
DIRECTLY to the oracle's predict: tokens equal, logits within 1e-3), and one rank of Llama-2-7B's TP-4 / TP-8
shards (2 layers, ctx 2048, head_dim 128, 8 splits per head; SLI_DEBUG_NOCOMM: the rank's own step, no exchange)
at positions on and around the split and wave boundaries, each step run twice (the counters the launch leaves at
zero must serve the next launch). The shards' fused steps are held to the oracle through the multi-process TP tests
(test_gpu_tp.py, +qa, including Llama-2-7B's TP-4 shards), which compare whole TP steps with the exchange."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROMPT = [1, 17, 42, 99]
POSITIONS = [0, 1, 3, 4, 255, 256, 257, 511, 1000, 2047]


def _child(name, w, tp, out):
    sys.path.insert(0, ROOT)
    from simplellminference_amd.model import LlamaModel, preset
    base, _, layers = name.partition(":")
    cfg = preset(base, num_hidden_layers=int(layers)) if layers else preset(base)
    m = LlamaModel(config=cfg, w_dtype=w, kv_dtype="f16", seed=3, tp_rank=tp - 1, tp_size=tp).init()
    res = {"fused": m.fused_qkv_attn()}
    if tp == 1:
        toks, logits = m.predict(PROMPT, 24, want_logits=True)
        res["toks"] = np.asarray(toks).tolist()
        np.save(out + ".npy", np.asarray(logits, dtype=np.float32))
    else:
        m.fill_kv_synthetic(7, cfg.max_length - 1)
        rows = []
        for p in POSITIONS:
            a = m.forward(100 + p % 300, p)
            b = m.forward(100 + p % 300, p)
            assert np.array_equal(a, b), f"step at {p} not idempotent"
            rows.append(a)
        np.save(out + ".npy", np.stack(rows).astype(np.float32))
    res["error"] = int(m.state()["error"])
    m.close()
    with open(out + ".json", "w") as f:
        json.dump(res, f)


def _run(tmp_path, name, w, tp, qa):
    env = dict(os.environ, SLI_QKV_ATTN=str(qa))
    if tp > 1:
        env["SLI_DEBUG_NOCOMM"] = "1"
    out = str(tmp_path / f"{name.replace(':', '_')}_{w}_{tp}_{qa}")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), name, w, str(tp), out], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    with open(out + ".json") as f:
        res = json.load(f)
    return res, np.load(out + ".npy")


@pytest.mark.parametrize("name,w,tp", [("tiny", "f16", 1), ("tiny-gqa", "f16", 1), ("tiny", "i8", 1),
                                       ("tiny-gqa", "i8", 1), ("llama2-7b:2", "f16", 8), ("llama2-7b:2", "i8", 8),
                                       ("llama2-7b:2", "f16", 4)])
def test_fused_qkv_attention_matches_two_launches(gpu, oracle, tmp_path, name, w, tp):
    fused, a = _run(tmp_path, name, w, tp, 1)
    plain, b = _run(tmp_path, name, w, tp, 0)
    assert fused["fused"] == 1 and plain["fused"] == 0
    assert fused["error"] == 0 and plain["error"] == 0
    assert np.isfinite(a).all()
    assert np.array_equal(a, b), float(np.abs(a - b).max())
    if tp == 1:
        assert fused["toks"] == plain["toks"]
        import oracle as O
        from simplellminference_amd.model import preset
        cfg = preset(name)
        om = O.Model(O.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                              cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                              cfg.rms_norm_eps, cfg.rope_theta), seed=3, wmode=O.W_F16 if w == "f16" else O.W_I8,
                     kv_f16=True)
        otoks, ologits = om.predict(PROMPT, 24)
        om.close()
        assert fused["toks"] == np.asarray(otoks).tolist()
        assert float(np.abs(a - ologits).max()) <= 1e-3


if __name__ == "__main__":
    _child(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4])
