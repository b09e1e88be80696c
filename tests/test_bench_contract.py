"""The bench line contract (the task's bench.py section) on the committed round-6 bench lines (profiles/r6*_bench_c*.json,
written by `python bench.py` on an MI355X): every required key, the roofline and cpu_baseline objects, the units and
the arithmetic that ties them together (value x ms_per_step = global batch; frac = achieved / peak; achieved = the
dominant family's algorithmic bytes / its launch time), and the step_ms block (SURVEY §5's p50 / p99: one HIP event
between consecutive graph replays of the timed window; its mean against the host clock, its p50 against the mean, the
timed window against the same process's 64-token greedy run). CPU only: it reads JSON, runs nothing."""
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = sorted(glob.glob(os.path.join(ROOT, "profiles", "r6*_bench_c*.json")))
BASELINE = json.load(open(os.path.join(ROOT, "BASELINE.json")))


def _load(p):
    with open(p) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def test_lines_present():
    names = {os.path.basename(p).split("_bench_")[1] for p in LINES}
    assert {"c1.json", "c3.json", "c4.json"} <= names, LINES


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


@pytest.mark.parametrize("path", LINES, ids=[os.path.basename(p) for p in LINES])
def test_step_ms_block(path):
    d = _load(path)
    s = d["step_ms"]
    for k in ("n", "p50", "p99", "min", "max", "mean", "first5_mean", "last5_mean", "host_clock_mean"):
        assert k in s, k
    assert s["n"] == d["steps"]
    assert s["min"] <= s["p50"] <= s["p99"] <= s["max"]
    assert s["min"] <= s["first5_mean"] <= s["max"] and s["min"] <= s["last5_mean"] <= s["max"]
    assert s["host_clock_mean"] == pytest.approx(d["ms_per_step"], rel=1e-3)
    # the events see the same window as the host clock; p50 within 1 % of the mean
    assert s["mean"] == pytest.approx(s["host_clock_mean"], rel=1e-2)
    assert s["p50"] == pytest.approx(s["mean"], rel=1e-2)
    if "greedy_64" in d and "timed_mean_over_greedy" in d["greedy_64"]:
        assert abs(d["greedy_64"]["timed_mean_over_greedy"] - 1.0) <= 0.01


@pytest.mark.parametrize("path", [p for p in LINES if p.endswith("_c1.json") or p.endswith("_c4.json")],
                         ids=lambda p: os.path.basename(p))
def test_cpu_baseline(path):
    d = _load(path)
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("reference", "port") and c["cores"] >= 1 and c["value"] > 0
    assert c["unit"] == "tokens/s"
