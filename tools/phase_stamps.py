"""Per-phase timing of the persistent decode step (workgroup 0's view), from SLI_DEBUG_STAMPS.

    SLI_DEBUG_STAMPS=1 python tools/phase_stamps.py [--preset llama2-7b] [--layers 32]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SLI_DEBUG_STAMPS", "1")

from simplellminference_amd import _lib  # noqa: E402
from simplellminference_amd.model import LlamaModel, preset  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--preset", default="llama2-7b")
ap.add_argument("--layers", type=int, default=32)
a = ap.parse_args()
cfg = preset(a.preset, num_hidden_layers=a.layers)
m = LlamaModel(config=cfg, w_dtype="f16", kv_dtype="f16", seed=1).init()
m.fill_kv_synthetic(7, cfg.max_length - 1)
m.set_state(1234, cfg.max_length - 1, advance=False)
for _ in range(5):
    m.step()
m.sync()
n = 3 * (cfg.num_hidden_layers * 5 + 1)
buf = np.zeros(n, np.uint64)
got = _lib.load().sli_model_debug_stamps(m._h, buf.ctypes.data_as(ctypes.c_void_p), n)
assert got == n, got
t = buf.astype(np.float64) / 100.0  # 100 MHz -> us
names = ["QKV", "ATTN", "WO", "GU", "DOWN"]
work, wait = {k: [] for k in names}, {k: [] for k in names}
for p in range(cfg.num_hidden_layers * 5):
    k = names[p % 5]
    work[k].append(t[3 * p + 1] - t[3 * p])
    wait[k].append(t[3 * p + 2] - t[3 * p + 1])
print(f"{'phase':6s} {'work_us':>9s} {'barrier_us':>11s}")
for k in names:
    print(f"{k:6s} {np.median(work[k]):9.2f} {np.median(wait[k]):11.2f}")
total = t[3 * (cfg.num_hidden_layers * 5) + 1] - t[0]
print(f"step (WG0, start of QKV0 -> end of LM): {total:.1f} us")
