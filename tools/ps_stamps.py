"""Phase breakdown of the persistent step (persist.h) from its in-kernel s_memrealtime stamps.

    python tools/ps_stamps.py [--w-dtype f16] [--ctx 2048] [--layers 32]

Runs the bench workload (Llama-2-7B shapes, KV filled to ctx-1, step at ctx-1), warms the persistent step,
then one stamped launch. Per phase type prints medians over workgroups and layers (µs):
  wait   = barrier passed - entry  (the barrier's latency as this workgroup sees it)
  stage  = input staged - barrier passed (control wave: sc1 loads + RMS into LDS)
  comp   = compute done - input staged (the weight stream / attention after the input landed)
  tail   = arrival - compute done (epilogue stores, drain, arrival add)
  span   = phase-end(max over workgroups) - previous phase-end(max): the phase's share of the step
  lat    = barrier passed - the previous phase's last arrival (the barrier's own latency)
  skew   = last - first arrival of the phase
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--w-dtype", default="f16")
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--preset", default="llama2-7b")
    a = ap.parse_args()
    import torch  # noqa: F401  (device init)
    from simplellminference_amd._lib import call
    from simplellminference_amd.model import LlamaModel, preset
    cfg = preset(a.preset, max_length=a.ctx, num_hidden_layers=a.layers)
    m = LlamaModel(config=cfg, w_dtype=a.w_dtype, kv_dtype="f16", seed=1).init().set_exec("persistent")
    m.fill_kv_synthetic(7, a.ctx - 1)
    m.set_state(1234, a.ctx - 1, advance=False)
    for _ in range(10):
        m.step()
    m.sync()
    L = cfg.num_hidden_layers
    nph = 2 + 5 * L
    import simplellminference_amd._lib as lib
    grid = ctypes.c_int32()
    n = nph * 256 * 5
    buf = np.zeros(n, np.uint64)
    rc = lib.load().sli_model_ps_stamps(m._h, buf.ctypes.data_as(ctypes.c_void_p), n, ctypes.byref(grid))
    if rc != 0:  # grid is not 256: retry with the device's size
        g = grid.value
        n = nph * g * 5
        buf = np.zeros(n, np.uint64)
        call("sli_model_ps_stamps", m._h, buf.ctypes.data_as(ctypes.c_void_p), n, ctypes.byref(grid))
    g = grid.value
    st = buf.reshape(nph, g, 5).astype(np.float64) * 0.01  # 100 MHz -> µs
    t0 = st[0, :, 0].min()
    st -= t0
    names = ["qkv", "attention", "wo", "gate_up", "down"]
    ends = st[:, :, 4].max(axis=1)
    spans = np.diff(np.concatenate([[0.0], ends]))
    rows = {k: [] for k in names + ["lm_head"]}
    for p in range(1, nph):
        name = "lm_head" if p == nph - 1 else names[(p - 1) % 5]
        s = st[p]
        last_prev = st[p - 1, :, 4].max()  # the barrier's last arrival
        rows[name].append((np.median(s[:, 1] - s[:, 0]), np.median(s[:, 1] - last_prev), np.median(s[:, 2] - s[:, 1]),
                           np.median(s[:, 3] - s[:, 2]), np.median(s[:, 4] - s[:, 3]), spans[p],
                           np.max(s[:, 4]) - np.min(s[:, 4])))
    step = ends[-1] - st[1, :, 0].min()
    print(f"{a.preset} {a.w_dtype} ctx {a.ctx} L {L}: step (qkv(0) entry -> LM-head last arrival) {step:.1f} us, grid {g}")
    print(f"{'phase':10s} {'wait':>7s} {'lat':>7s} {'stage':>7s} {'comp':>7s} {'tail':>7s} {'span':>7s} {'skew':>7s}"
          f"  (median us; lat = barrier pass - the barrier's last arrival)")
    for k, v in rows.items():
        v = np.array(v)
        med = np.median(v, axis=0)
        tot = v[:, 5].sum()
        print(f"{k:10s} {med[0]:7.2f} {med[1]:7.2f} {med[2]:7.2f} {med[3]:7.2f} {med[4]:7.2f} {med[5]:7.2f} {med[6]:7.2f}"
              f"  sum span {tot:8.1f}")
    m.close()


if __name__ == "__main__":
    main()
