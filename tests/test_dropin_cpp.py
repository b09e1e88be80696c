"""The C++ drop-in API (include/op, include/memory, include/model) used the way the reference's
model.cpp uses it: tests/cpp/dropin_llama.cpp builds the model op by op from the reference's flat
fp32 weight file and also runs model::LlamaModel (fused engine). Both must reproduce the oracle:
greedy tokens exact, logits within 1e-4 (fp32 weights, fp32 KV — the reference's numerics)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "dropin_llama.cpp")
BIN = os.path.join(ROOT, "tests", "cpp", "_build", "dropin_llama")
PROMPT = [1, 17, 42, 99]


def _compile():
    from simplellminference_amd import build
    build.build()
    if os.path.exists(BIN) and os.path.getmtime(BIN) >= max(os.path.getmtime(SRC), os.path.getmtime(build.LIB)):
        return BIN
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    inc = [f"-I{os.path.join(ROOT, 'include', d)}" for d in ("", "base", "memory", "op", "model", "kernel")]
    cmd = ["hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", *inc, SRC, "-o", BIN,
           f"-L{os.path.join(ROOT, 'simplellminference_amd')}", "-lsli",
           "-Wl,-rpath,$ORIGIN/../../../simplellminference_amd"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return BIN


def _read(path):
    raw = open(path, "rb").read()
    n = int(np.frombuffer(raw[:4], np.int32)[0])
    toks = np.frombuffer(raw[4:4 + 4 * n], np.int32)
    logits = np.frombuffer(raw[4 + 4 * n:], np.float32).reshape(n, -1)
    return toks, logits


def test_dropin_client_compiles():
    assert os.path.exists(_compile())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny", "tiny-gqa"])
def test_dropin_op_path_and_model_match_oracle(gpu, oracle, tmp_path, name):
    from simplellminference_amd.model import preset
    binary = _compile()
    c = preset(name)
    om = oracle.Model(oracle.Config(c.vocab_size, c.hidden_size, c.num_attention_heads, c.num_key_value_heads,
                                    c.head_dim, c.intermediate_size, c.num_hidden_layers, c.max_length,
                                    c.rms_norm_eps, c.rope_theta), seed=0)
    wpath = str(tmp_path / "w.bin")
    om.write_flat(wpath)
    steps = 36
    otoks, ologits = om.predict(PROMPT, steps)
    out = str(tmp_path / "run")
    args = [binary, wpath, out, str(steps), str(c.vocab_size), str(c.hidden_size), str(c.num_attention_heads),
            str(c.num_key_value_heads), str(c.head_dim), str(c.intermediate_size), str(c.num_hidden_layers),
            str(c.max_length), str(c.rope_theta)] + [str(t) for t in PROMPT]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    for suffix in (".ops.bin", ".engine.bin"):
        toks, logits = _read(out + suffix)
        assert np.array_equal(toks, otoks), suffix
        assert np.abs(logits - ologits).max() <= 1e-4, suffix
