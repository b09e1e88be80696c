#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/ from the C oracle (oracle/sli_oracle.c).

    python tests/golden/make_golden.py

The reference cannot be built in this image and ships no fixtures, so these vectors
are oracle outputs: they pin the oracle (and through it every parity test) against regressions, and
tests/test_oracle.py cross-checks the oracle itself against an independent float64 restatement.
Inputs are seeded (numpy default_rng / the sli_synth.h generator), sizes are CPU-seconds small.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle as O  # noqa: E402

PROMPT = np.array([1, 17, 42, 99], np.int32)
TINY = dict(vocab=512, dim=256, n_heads=4, head_dim=64, ffn=768, n_layers=2, max_len=64, eps=1e-5, theta=10000.0)


def model_fixture(n_kv_heads, name):
    cfg = O.Config(n_kv_heads=n_kv_heads, **TINY)
    m = O.Model(cfg, seed=0, wmode=O.W_F32)
    toks, logits = m.predict(PROMPT, 36)  # BASELINE.json configs[0]: 4 prompt + 32 greedy tokens
    np.savez_compressed(os.path.join(HERE, name), tokens=toks, logits=logits, prompt=PROMPT,
                        n_kv_heads=np.int32(n_kv_heads))
    m.close()


def op_fixtures():
    r = np.random.default_rng(2025)
    f = {}
    x = r.standard_normal(256).astype(np.float32)
    w = (r.standard_normal((48, 256)) / 16).astype(np.float32)
    f["matmul_x"], f["matmul_w"], f["matmul_y"] = x, w, O.matmul(x, w)
    nw = (1 + 0.1 * r.standard_normal(256)).astype(np.float32)
    f["rms_w"], f["rms_y"] = nw, O.rmsnorm(x, nw, 1e-5)
    for th in (10000.0, 100000.0, 500000.0):
        s, c = O.rope_cache(64, 64, th)
        f[f"rope_sin_{int(th)}"], f[f"rope_cos_{int(th)}"] = s, c
    s, c = O.rope_cache(64, 64, 10000.0)
    q = r.standard_normal(256).astype(np.float32)
    k = r.standard_normal(128).astype(np.float32)
    f["rope_q"], f["rope_k"] = q, k
    f["rope_q_out"], f["rope_k_out"] = O.rope(q, k, 37, s, c, 64)
    kc = r.standard_normal((2, 64, 128)).astype(np.float32)
    vc = r.standard_normal((2, 64, 128)).astype(np.float32)
    f["mha_q"], f["mha_k"], f["mha_v"] = q, kc, vc
    for pos in (0, 17, 63):
        f[f"mha_gqa_out_{pos}"] = O.mha(q, kc, vc, 1, pos, 64, 64, 4, 2)
    qm = r.standard_normal(128).astype(np.float32)
    f["mha_mq"] = qm
    f["mha_mha_out_40"] = O.mha(qm, kc, vc, 0, 40, 64, 64, 2, 2)
    sm = (3 * r.standard_normal(100)).astype(np.float32)
    f["softmax_in"], f["softmax_out"] = sm, O.softmax(sm)
    u = r.standard_normal(768).astype(np.float32)
    g = (4 * r.standard_normal(768)).astype(np.float32)
    f["swiglu_up"], f["swiglu_gate"], f["swiglu_out"] = u, g, O.swiglu(u, g)
    f["add_out"] = O.add(u, g)
    tab = r.standard_normal((32, 16)).astype(np.float32)
    f["emb_table"], f["emb_out_7"] = tab, O.embedding(7, tab)
    am = r.standard_normal(1000).astype(np.float32)
    am[[100, 500]] = am.max() + 1.0  # tie: first index wins (argmax.cpp:11)
    f["argmax_in"], f["argmax_out"] = am, np.int32(O.argmax(am))
    # the synthetic-weight generator contract (include/sli_synth.h)
    for kind, idx, std in ((O.T_EMB, 0, 0.02), (O.T_WQ, 3, 1 / 64), (O.T_DOWN, 31, 1 / 105)):
        f[f"synth_{kind}_{idx}"] = O.synth_fill(64, 1, O.stream_id(kind, idx), O.synth_c(std))
    f["synth_norm"] = O.synth_fill(64, 0, O.stream_id(O.T_NORM, 2), O.synth_c(0.1), 1.0)
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **f)


if __name__ == "__main__":
    O.build()
    model_fixture(4, "c0_mha.npz")
    model_fixture(2, "c0_gqa.npz")
    op_fixtures()
    print("wrote", sorted(p for p in os.listdir(HERE) if p.endswith(".npz")))
