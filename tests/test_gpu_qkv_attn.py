"""The fused q/k/v + attention launch (csrc/qkv_attn.h) against the two-launch step it replaces.

The launch computes the same sums in the same order (the q/k/v units' row sums, the attention splits and their
merge), so its results are compared BIT-exactly with the two launches on the same weights and K/V: each case
runs in two child processes, SLI_QKV_ATTN=1 and SLI_QKV_ATTN=0 (the switch is read once per process). Cases:
the tiny presets at TP 1 (MHA and GQA-2, head_dim 64, fp16 / int8 weights, a greedy run of 24 tokens), and one
rank of Llama-2-7B's TP-4 / TP-8 shards (2 layers, ctx 2048, head_dim 128, 8 splits per head; SLI_DEBUG_NOCOMM:
the rank's own step, no exchange; also as the chain, wo in the same launch) at positions on and around the split
and wave boundaries, each step run twice
(the counters the launch leaves at zero must serve the next launch). The tiny runs are also held to the oracle
through the TP-1 tests that run the default path (test_gpu_model.py)."""
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


def _run(tmp_path, name, w, tp, qa, chain=False):
    env = dict(os.environ, SLI_QKV_ATTN=str(qa))
    if chain:
        env["SLI_QKV_CHAIN"] = "1"
    if tp > 1:
        env["SLI_DEBUG_NOCOMM"] = "1"
    out = str(tmp_path / f"{name.replace(':', '_')}_{w}_{tp}_{qa}_{int(chain)}")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), name, w, str(tp), out], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    with open(out + ".json") as f:
        res = json.load(f)
    return res, np.load(out + ".npy")


@pytest.mark.parametrize("name,w,tp,chain", [("tiny", "f16", 1, False), ("tiny-gqa", "f16", 1, False),
                                             ("tiny", "i8", 1, False), ("tiny-gqa", "i8", 1, False),
                                             ("llama2-7b:2", "f16", 8, False), ("llama2-7b:2", "i8", 8, False),
                                             ("llama2-7b:2", "f16", 4, False), ("llama2-7b:2", "f16", 8, True),
                                             ("llama2-7b:2", "f16", 4, True)])
def test_fused_qkv_attention_matches_two_launches(gpu, tmp_path, name, w, tp, chain):
    """chain: wo in the same launch too (SLI_QKV_CHAIN=1, sli_model_fused_qkv_attn == 2)."""
    fused, a = _run(tmp_path, name, w, tp, 1, chain)
    plain, b = _run(tmp_path, name, w, tp, 0)
    assert fused["fused"] == (2 if chain else 1) and plain["fused"] == 0
    assert fused["error"] == 0 and plain["error"] == 0
    if tp == 1:
        assert fused["toks"] == plain["toks"]
    assert np.isfinite(a).all()
    assert np.array_equal(a, b), float(np.abs(a - b).max())


if __name__ == "__main__":
    _child(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4])
