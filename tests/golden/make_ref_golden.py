#!/usr/bin/env python3
"""Write tests/golden/ref_ops.npz and tests/golden/ref_*.npz from the REFERENCE's own CPU build.

    make -C oracle ref && python tests/golden/make_ref_golden.py

Runs only where /root/reference exists (this container): oracle/_ref/libref.so is the reference's
source/kernel/cpu, source/memory, source/op and weight_loader.cpp compiled in place (oracle/Makefile), and
the model fixtures compose its op layers as model.cpp:40-187 does (oracle/ref_harness.cpp). The weights are
the synthetic ones every test uses, written in the reference's flat fp32 layout by the oracle
(orc_model_write_flat, model.cpp:336-469 order) and read back through the reference's RawModelDataFp32.
The vectors are data; no reference source travels with them.
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle as O  # noqa: E402
import oracle.ref as R  # noqa: E402
from tests.golden import ref_cases as C  # noqa: E402


def ops():
    f = {}
    for name, run in C.CASES.items():
        inputs, outputs = run(R, O)
        f.update(C.pack(name, inputs, outputs))
    np.savez_compressed(os.path.join(HERE, "ref_ops.npz"), **f)
    print(f"ref_ops.npz: {len(C.CASES)} cases")


def models(names=None):
    for name, (shape, n_kv, steps, seed) in C.MODELS.items():
        if names and name not in names:
            continue
        cfg = O.Config(n_kv_heads=n_kv, **shape)
        m = O.Model(cfg, seed=seed, wmode=O.W_F32)
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "model.bin")
            m.write_flat(path)
            m.close()
            rm = R.Model(cfg, path)
            toks, logits = rm.predict(C.PROMPT, steps)
            rm.close()
        f = {"prompt": np.array(C.PROMPT, np.int32), "tokens": toks, "seed": np.int32(seed),
             "n_kv_heads": np.int32(n_kv)}
        if logits.size <= 4 * C.FULL_MAX * 8:
            f["logits"] = logits
        else:
            f["logits_sha256"] = np.array([C.digest(row) for row in logits])
            f["logits_head"] = logits[:, :512].copy()
            f["argmax"] = logits.argmax(1).astype(np.int32)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **f)
        print(f"{name}.npz: tokens {toks.tolist()}")


if __name__ == "__main__":
    O.build()
    R.build()
    which = sys.argv[1:]
    if not which or "ops" in which:
        ops()
    models([w for w in which if w != "ops"] or None)
