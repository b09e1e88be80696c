"""What an fp16 all-reduce payload would cost in accuracy (SURVEY §8(e) sizes the exchange at
8 KiB = D fp16 values per message). The in-process TP group (rank-order sums in place of the exchange) runs the
whole 32-layer Llama-2-7B fp16 step at TP 8 (BASELINE configs[2], ctx 2048, position 2047) twice: with the fp32
payload the engine ships, and with SLI_DEBUG_AR_F16=1 — every rank's contribution rounded to fp16 before the
sum (the residual kept in fp32 and added once), i.e. exactly what an fp16 exchange would deliver. Both against
the unsharded lazy oracle, at the north star's 1e-3 bar.
    python tools/ar_payload_error.py            (GPU; ~2 min, most of it the oracle)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402  (test infrastructure: the checker)
from simplellminference_amd.model import TPGroup, preset  # noqa: E402


def ocfg(cfg):
    return oracle.Config(cfg.vocab_size, cfg.hidden_size, cfg.num_attention_heads, cfg.num_key_value_heads,
                         cfg.head_dim, cfg.intermediate_size, cfg.num_hidden_layers, cfg.max_length,
                         cfg.rms_norm_eps, cfg.rope_theta)


def main():
    cfg = preset("llama2-7b")
    cases = [(1234, 2047), (777, 1000), (31999, 5)]
    t0 = time.time()
    om = oracle.Model(ocfg(cfg), seed=1, wmode=oracle.W_F16, kv_f16=True, lazy=True)
    om.set_threads(16)  # GEMV rows over host threads: bit-identical to one thread
    om.fill_kv_synthetic(7, 2047)
    want = [om.forward(tok, pos) for tok, pos in cases]
    om.close()
    print(f"oracle: {time.time() - t0:.0f} s", flush=True)
    for mode in ("fp32", "fp16"):
        if mode == "fp16":
            os.environ["SLI_DEBUG_AR_F16"] = "1"
        g = TPGroup(cfg, 8, w_dtype="f16", kv_dtype="f16", seed=1).init()
        g.fill_kv_synthetic(7, 2047)
        for (tok, pos), w in zip(cases, want):
            got = g.forward(tok, pos)
            err = float(np.abs(got - w).max())
            print(f"TP 8, {mode} payload, token {tok} pos {pos}: max|logit - oracle| {err:.3e} "
                  f"({'within' if err <= 1e-3 else 'OVER'} the 1e-3 bar), argmax {'equal' if int(np.argmax(got)) == int(np.argmax(w)) else 'DIFFERS'}",
                  flush=True)
        g.close()
        os.environ.pop("SLI_DEBUG_AR_F16", None)


if __name__ == "__main__":
    main()
