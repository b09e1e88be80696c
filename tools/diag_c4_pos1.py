"""Diagnostic: the C4 full model (Llama-3-8B fp16, 32 layers) at a short context, batched (bgemm) vs batch-1
(GEMV) vs the lazy oracle: which path carries the error at position 1."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from simplellminference_amd.model import LlamaModel, preset  # noqa: E402

cfg = preset("llama3-8b")
tok = 1234 + 9001 * 5
pos_list = [1, 2, 5, 100]
om = oracle.Model(oracle.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                                cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                                cfg.rms_norm_eps, cfg.rope_theta), seed=1, wmode=oracle.W_F16, kv_f16=True, lazy=True)
om.fill_kv_synthetic(12, 4095)
want = {p: om.forward(tok, p) for p in pos_list}
om.close()
g1 = LlamaModel(config=cfg, w_dtype="f16", kv_dtype="f16", seed=1).init()
g1.fill_kv_synthetic(12, 4095)
for p in pos_list:
    got = g1.forward(tok, p)
    print(f"batch-1 GEMV pos {p}: max|dlogit| {np.abs(got - want[p]).max():.3e}  |logit|max {np.abs(want[p]).max():.2f} "
          f"argmax ok {int(np.argmax(got)) == int(np.argmax(want[p]))}", flush=True)
g1.close()
gb = LlamaModel(config=cfg, w_dtype="f16", kv_dtype="f16", seed=1, batch=8).init()
gb.fill_kv_synthetic(7, 4095)  # sequence b: seed 7 + b -> sequence 5 = seed 12
for p in pos_list:
    got = gb.forward_batch([tok] * 8, [p] * 8)[5]
    print(f"batch-8 bgemm pos {p}: max|dlogit| {np.abs(got - want[p]).max():.3e}", flush=True)
gb.close()
