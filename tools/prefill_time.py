"""Prefill timing probe: Llama-2-7B (random init), prompts of the given lengths, prefill wall time per prompt
(sli_model_prefill, after one warm-up that captures the chunk graphs).

    python tools/prefill_time.py [--w f16|i8] [--tokens 512 2048] [--reps 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w", default="f16")
    ap.add_argument("--kv", default="f16")
    ap.add_argument("--tokens", type=int, nargs="+", default=[512])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--layers", type=int, default=32)
    a = ap.parse_args()
    from simplellminference_amd.model import LlamaModel, preset
    cfg = preset("llama2-7b", num_hidden_layers=a.layers)
    m = LlamaModel(config=cfg, w_dtype=a.w, kv_dtype=a.kv, seed=1).init()
    params = a.layers * (4 * 4096 * 4096 + 3 * 4096 * 11008)
    for n in a.tokens:
        ids = [(1 + 7919 * i) % cfg.vocab_size for i in range(n)]
        m.prefill(ids)
        t = time.perf_counter()
        for _ in range(a.reps):
            m.prefill(ids)
        t = (time.perf_counter() - t) / a.reps
        tf = 2.0 * params * (n - 1) / t / 1e12
        print(f"w={a.w} kv={a.kv} n={n}: {t * 1e3:.2f} ms  {(n - 1) / t:.0f} tok/s  projections {tf:.1f} TFLOP/s",
              flush=True)
    m.close()


if __name__ == "__main__":
    main()
