"""tools/pmc_traffic.py: per-family attribution of a rocprofv3 FETCH_SIZE pass.

Synthetic counter files in the rocprofv3 csv shape: one decode step (q/k/v, attention, wo, gate/up, down, LM head)
followed by the family-timing replays (sli_model_time_families: each family's launches back to back). The batched
wo and down share the BgEpiStore epilogue; the script must name them by the step context (the family dispatched
before them) and the replays by their (kernel, grid) shape — never by dispatch parity — and fail when a family
reads below 0.99x its algorithmic bytes or when one shape serves both families."""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "pmc_traffic.py")

QKV = "void sli::bgemm_kernel<sli::BgEpiQKV<__half>, true, 4>(__half const*, sli::BgIn, sli::BgEpiQKV<__half>)"
ATT = "void sli::attn_mfma_kernel<128, 4, 2>(sli::AttnArgs<__half>)"
WO = "void sli::bgemm_kernel<sli::BgEpiStore, false, 2>(__half const*, sli::BgIn, sli::BgEpiStore)"
GU = "void sli::bgemm_kernel<sli::BgEpiSwiGLU, true, 4>(__half const*, sli::BgIn, sli::BgEpiSwiGLU)"
DOWN = "void sli::bgemm_kernel<sli::BgEpiStore, false, 7>(__half const*, sli::BgIn, sli::BgEpiStore)"
LM = "void sli::bgemm_kernel<sli::BgEpiLogits, true, 4>(__half const*, sli::BgIn, sli::BgEpiLogits)"
FILL = "void sli::synth_fill_kernel(float*, unsigned long)"

# algorithmic bytes per launch, and the FETCH_SIZE (KiB, half the bytes on gfx950) the "hardware" reports
ALG = {"qkv": 50331648, "attention": 134217728, "wo": 33554432, "gate_up": 234881024, "down": 117440512,
       "lm_head": 1050673152}
OVER = {"qkv": 1.03, "attention": 1.01, "wo": 1.04, "gate_up": 1.006, "down": 1.015, "lm_head": 1.001}


def kib(fam, over=None):
    return ALG[fam] * (over or OVER[fam]) / 2 / 1024


def write_csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, (k, g, v) in enumerate(rows):
            w.writerow({"Dispatch_Id": d, "Kernel_Name": k, "Grid_Size": g, "Counter_Name": "FETCH_SIZE",
                        "Counter_Value": v})


def write_bench(path):
    line = {"roofline": {"families": {f: {"bytes_per_launch": b} for f, b in ALG.items()}}}
    with open(path, "w") as f:
        f.write("[bench] progress\n" + json.dumps(line) + "\n")


def step(layers=2, wo_grid=262144, down_grid=262144, down_over=None):
    rows = [(FILL, 1024, 1.0)]
    for _ in range(layers):
        rows += [(QKV, 196608, kib("qkv")), (ATT, 65536, kib("attention")), (WO, wo_grid, kib("wo")),
                 (GU, 262144, kib("gate_up")), (DOWN, down_grid, kib("down", down_over))]
    rows.append((LM, 262144, kib("lm_head")))
    return rows


def run(tmp_path, rows):
    c, b, o = tmp_path / "c.csv", tmp_path / "b.log", tmp_path / "o.json"
    write_csv(c, rows)
    write_bench(b)
    p = subprocess.run([sys.executable, TOOL, str(c), str(ALG["gate_up"]), str(o), "k", "gate_up", str(b)],
                       capture_output=True, text=True)
    return p, (json.load(open(o))["k"] if o.exists() else None)


def test_step_and_replays_attributed(tmp_path):
    # the step, then the replays: wo x3, down x3, each at its own (kernel, grid) shape from the step
    p, r = run(tmp_path, step(wo_grid=262144, down_grid=131072) + [(WO, 262144, kib("wo"))] * 3
               + [(DOWN, 131072, kib("down"))] * 3)
    assert p.returncode == 0, p.stderr
    ratio = r["per_family_hbm_over_algorithmic"]
    for f, want in OVER.items():
        assert ratio[f] == pytest.approx(want, abs=2e-4), (f, ratio)
    assert r["per_family_dispatches"]["wo"] == 2 + 3 and r["per_family_dispatches"]["down"] == 2 + 3


def test_parity_does_not_decide(tmp_path):
    # two wo replays then three down replays: a parity split would swap families; the shape vote must not
    p, r = run(tmp_path, step(wo_grid=262144, down_grid=131072) + [(WO, 262144, kib("wo"))] * 2
               + [(DOWN, 131072, kib("down"))] * 3)
    assert p.returncode == 0, p.stderr
    assert r["per_family_hbm_over_algorithmic"]["wo"] == pytest.approx(OVER["wo"], abs=2e-4)
    assert r["per_family_hbm_over_algorithmic"]["down"] == pytest.approx(OVER["down"], abs=2e-4)


def test_below_algorithmic_fails(tmp_path):
    p, _ = run(tmp_path, step(wo_grid=262144, down_grid=131072, down_over=0.93))
    assert p.returncode != 0 and "below 0.99x" in (p.stderr + p.stdout)


def test_one_shape_for_both_families_fails_on_replays(tmp_path):
    # wo and down with the same instantiation AND grid, plus replays: the replays cannot be named
    rows = step(wo_grid=262144, down_grid=262144)
    rows = [(DOWN if k == WO else k, g, v) for k, g, v in rows]  # same kernel name for both
    p, _ = run(tmp_path, rows + [(DOWN, 262144, kib("down"))] * 2)
    assert p.returncode != 0 and "serves both" in (p.stderr + p.stdout)
