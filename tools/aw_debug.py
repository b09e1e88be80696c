"""Diagnosis of the fused attention + wo launch (attn_wo.h): a 1- and 2-layer Llama-2-7B-shape model with the
launch off / on (SLI_DEBUG_AW variants), logits compared at positions 0, 300 and 2047."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simplellminference_amd.model import LlamaModel, preset  # noqa: E402


def run(aw, dbg, layers, pos):
    os.environ["SLI_ATTN_WO"] = aw
    os.environ["SLI_DEBUG_AW"] = dbg
    m = LlamaModel(config=preset("llama2-7b", num_hidden_layers=layers), w_dtype="f16", kv_dtype="f16", seed=1).init()
    fams = list(m.time_families(1))
    m.fill_kv_synthetic(7, 2047)
    out = m.forward(1234, pos)
    err = m.state()["error"]
    m.close()
    return out, err, fams


for layers in (1, 2):
    for pos in (0, 300, 2047):
        ref, _, _ = run("0", "0", layers, pos)
        for dbg in ("0", "1"):
            got, err, fams = run("1", dbg, layers, pos)
            print(f"layers {layers} pos {pos} dbg {dbg}: max|d| {np.abs(got - ref).max():.3e} err {err} "
                  f"fused {'wo' not in fams}", flush=True)
