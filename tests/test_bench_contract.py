"""The bench line contract (the task's bench.py section) on the committed round-5 bench lines (profiles/r5g_bench_*.json,
written by `python bench.py` on an MI355X): every required key, the roofline and cpu_baseline objects, the units and
the arithmetic that ties them together (value x ms_per_step = global batch; frac = achieved / peak; achieved = the
dominant family's algorithmic bytes / its launch time). CPU only: it reads JSON, runs nothing."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = sorted(glob.glob(os.path.join(ROOT, "profiles", "r5g_bench_c*.json")))
BASELINE = json.load(open(os.path.join(ROOT, "BASELINE.json")))


def _load(p):
    with open(p) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_lines_present():
    assert len(LINES) == 3, LINES


@pytest.mark.parametrize("path", LINES, ids=[os.path.basename(p) for p in LINES])
def test_bench_line_contract(path):
    d = _load(path)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in d, k
    assert d["metric"] == BASELINE["metric"]
    assert d["unit"] == "tokens/s" and d["higher_is_better"] is True and d["n_gpus"] == 1
    assert d["scaling"] in ("weak", "strong") and d["data"] == "synthetic"
    cfg = d["config"]
    assert "workload" in cfg and "model" not in cfg
    # tokens per step / seconds per step
    assert d["value"] * d["ms_per_step"] / 1e3 == pytest.approx(cfg["global_batch"], rel=2e-3)
    r = d["roofline"]
    assert r["bound"] in ("hbm", "mfma") and r["unit"] == ("GB/s" if r["bound"] == "hbm" else "TFLOP/s")
    assert r["peak"] == 8000.0
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    assert r["achieved"] == pytest.approx(r["algorithmic_bytes_per_launch"] / (r["avg_launch_us"] * 1e3), rel=1e-3)
    # traffic: HBM bytes per launch of the dominant kernel, at least its algorithmic bytes (tools/pmc_traffic.py's bar)
    assert r["traffic"] is None or r["traffic"] >= 0.99 * r["algorithmic_bytes_per_launch"]
    fams = r["families"]
    assert set(fams) == {"qkv", "attention", "wo", "gate_up", "down", "lm_head"}
    dom = max(fams, key=lambda f: fams[f]["avg_launch_us"] * fams[f]["launches_per_step"])
    assert fams[dom]["avg_launch_us"] == pytest.approx(r["avg_launch_us"], rel=1e-3)


@pytest.mark.parametrize("path", [p for p in LINES if not p.endswith("c3.json")],
                         ids=lambda p: os.path.basename(p))
def test_cpu_baseline(path):
    d = _load(path)
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("reference", "port") and c["cores"] >= 1 and c["value"] > 0
    assert c["unit"] == "tokens/s"
