"""HBM traffic per GEMV launch from a rocprofv3 FETCH_SIZE pass (run tools/pmc_traffic.sh on the GPU box).

FETCH_SIZE is in KiB and, on gfx950, reads exactly half the bytes of a wide coalesced 16-B/lane stream
(cdna_hip_programming.md section 7; MI355X_MICROARCH.md HBM), so traffic = 2 * FETCH_SIZE * 1024. Only
the decode step's own GEMV dispatches are counted: the weight-placement and KV-fill kernels at model
build are skipped by name.
    python tools/pmc_traffic.py <counter_collection.csv> <dominant family's algorithmic bytes per launch> <out.json>
                                <key> [<dominant family>]
Top-level fields: the mean over EVERY weight-streaming launch of the step (all families together), then the
dominant family's own algorithmic bytes; per-family HBM bytes per launch are in per_family_hbm_bytes_per_launch.
"""
import csv
import json
import sys
from collections import defaultdict

path, alg, out, key = sys.argv[1], float(sys.argv[2]), sys.argv[3], sys.argv[4]
dom = sys.argv[5] if len(sys.argv) > 5 else None  # the bench line's dominant family (whose bytes alg are)
per = defaultdict(list)
rows = []  # (dispatch id, kernel, value) in dispatch order
for r in csv.DictReader(open(path)):
    if r.get("Counter_Name") != "FETCH_SIZE":
        continue
    per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    rows.append((int(r.get("Dispatch_Id") or len(rows)), r["Kernel_Name"], float(r["Counter_Value"])))
rows.sort()


def weight_kernel(k):  # the step's weight-streaming kernels: batch-1 GEMV or the batched MFMA projection
    return "gemv_kernel" in k or "gemv_merge_kernel" in k or "gemv_sum_kernel" in k or "bgemm_kernel" in k


gemv = [v for k, vs in per.items() if weight_kernel(k) for v in vs]
if not gemv:
    raise SystemExit("no gemv_kernel / bgemm_kernel dispatches with FETCH_SIZE in " + path)
kb = sum(gemv) / len(gemv)
res = {}
try:
    res = json.load(open(out))
except (OSError, ValueError):
    pass
res[key] = {
    "all_weight_kernels_mean_hbm_bytes_per_launch": round(2 * kb * 1024),
    "all_weight_kernels_mean_fetch_size_kib_raw": round(kb, 1),
    "correction": ("x2: gfx950 FETCH_SIZE counts half the bytes of a coalesced 16-B/lane stream"
                   + ("" if "bgemm" not in "".join(per) else "; bgemm streams its weights in the fragment layout "
                      "(one contiguous KiB per wave load), the same coalesced 16-B/lane pattern")),
    "dominant_family": dom,
    "dominant_family_algorithmic_bytes_per_launch": round(alg),
    "weight_kernel_dispatches": len(gemv),
    "per_kernel_mean_kib_raw": {k.split("(")[0][:90]: round(sum(v) / len(v), 1) for k, v in per.items()
                                if weight_kernel(k)},
}


def family(k):
    """Kernel family of a decode-step dispatch (the names bench.py's roofline uses), or None."""
    if "attn_partial_kernel" in k:
        return "attention"
    for tag, fam in (("EpiQKV", "qkv"), ("EpiSwiGLU", "gate_up"), ("EpiLogits", "lm_head")):
        if tag in k and weight_kernel(k):
            return fam
    if "gemv_merge_kernel" in k:  # wo: its input staged from the attention's split partials (EpiKPart: K-split)
        return "wo"
    if "gemv_kernel" in k and ("EpiStore<1>" in k or "EpiStoreSum<1" in k):  # the other single-row residual GEMV
        return "down"
    if "bgemm_kernel" in k and "BgEpiStore" in k:
        return "wo|down"  # one instantiation serves both batched row-parallel projections: split by order below
    return None


fam = defaultdict(list)
nth = 0  # batched row-parallel projections alternate wo, down in a step's dispatch order (engine record_phase)
for _, k, v in rows:
    f = family(k)
    if f == "wo|down":
        f = "wo" if nth % 2 == 0 else "down"
        nth += 1
    if f:
        fam[f].append(v)
res[key]["per_family_hbm_bytes_per_launch"] = {f: round(2 * 1024 * sum(v) / len(v)) for f, v in fam.items()}
if dom in res[key]["per_family_hbm_bytes_per_launch"]:
    res[key]["dominant_family_hbm_over_algorithmic"] = round(res[key]["per_family_hbm_bytes_per_launch"][dom] / alg, 4)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res[key], indent=1))
