"""HBM traffic per GEMV launch from a rocprofv3 FETCH_SIZE pass (run tools/pmc_traffic.sh on the GPU box).

FETCH_SIZE is in KiB and, on gfx950, reads exactly half the bytes of a wide coalesced 16-B/lane stream
(cdna_hip_programming.md section 7; MI355X_MICROARCH.md HBM), so traffic = 2 * FETCH_SIZE * 1024. Only
the decode step's own GEMV dispatches are counted: the weight-placement and KV-fill kernels at model
build are skipped by name.
    python tools/pmc_traffic.py <counter_collection.csv> <dominant family's algorithmic bytes per launch> <out.json>
                                <key> [<dominant family> [<bench log holding the run's JSON line>]]
With the bench log, every family's traffic is divided by its algorithmic bytes, and the script FAILS if any
family reads below 0.99x of them (an attribution or counter error: one pass must read every byte once).
Top-level fields: the mean over EVERY weight-streaming launch of the step (all families together), then the
dominant family's own algorithmic bytes; per-family HBM bytes per launch are in per_family_hbm_bytes_per_launch.
"""
import csv
import json
import sys
from collections import defaultdict

path, alg, out, key = sys.argv[1], float(sys.argv[2]), sys.argv[3], sys.argv[4]
dom = sys.argv[5] if len(sys.argv) > 5 else None  # the bench line's dominant family (whose bytes alg are)
# optional: the bench JSON line of the same run, for every family's algorithmic bytes per launch (the 0.99x check)
fam_alg = {}
if len(sys.argv) > 6:
    line = [l for l in open(sys.argv[6]) if l.startswith("{")][-1]
    fam_alg = {f: float(v["bytes_per_launch"]) for f, v in json.loads(line)["roofline"]["families"].items()}
per = defaultdict(list)
rows = []  # (dispatch id, kernel, value) in dispatch order
for r in csv.DictReader(open(path)):
    if r.get("Counter_Name") != "FETCH_SIZE":
        continue
    per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    rows.append((int(r.get("Dispatch_Id") or len(rows)), r["Kernel_Name"], float(r["Counter_Value"]),
                 r.get("Grid_Size", "")))
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
    if "attn_partial_kernel" in k or "attn_mfma_kernel" in k:  # register path / MFMA GQA path (merge in-launch)
        return "attention"
    for tag, fam in (("EpiQKV", "qkv"), ("EpiSwiGLU", "gate_up"), ("EpiLogits", "lm_head")):
        if tag in k and weight_kernel(k):
            return fam
    if "gemv_merge_kernel" in k:  # wo: its input staged from the attention's split partials (EpiKPart: K-split)
        return "wo"
    if "gemv_kernel" in k and ("EpiStore<1>" in k or "EpiStoreSum<1" in k):  # the other single-row residual GEMV
        return "down"
    if "bgemm_kernel" in k and "BgEpiStore" in k:
        return "wo|down"  # both batched row-parallel projections use BgEpiStore: resolved below
    return None


# The batched row-parallel projections (wo, down) share the BgEpiStore epilogue. Inside a captured step each
# is identified by the family dispatched before it (engine record_batched: ... attention [merge] -> wo,
# gate/up -> down). The family-timing replays (sli_model_time_families) run one family's launches back to back,
# so those dispatches take the label of their instantiation + grid (one matrix shape), learned from the step.
# Never by dispatch parity: the replays break any alternation.
def base(k):
    return k.split("(")[0]


ctx_label = {}  # dispatch id -> "wo" | "down" where the step context decides it
shape_votes = defaultdict(lambda: defaultdict(int))  # (kernel, grid) -> label -> count
prev = None
for d, k, v, g in rows:
    f = family(k)
    if f == "wo|down":
        lab = "down" if prev == "gate_up" else "wo" if prev in ("attention", "attn_merge", "qkv") else None
        if lab:
            ctx_label[d] = lab
            shape_votes[(base(k), g)][lab] += 1
    prev = f if f else ("attn_merge" if "attn_merge_kernel" in k else prev if "rocclr" in k else None)
shape_label = {}
for sk, votes in shape_votes.items():
    lab, n = max(votes.items(), key=lambda kv: kv[1])
    if n != sum(votes.values()):
        raise SystemExit(f"{sk}: one instantiation and grid serves both wo and down ({dict(votes)}); "
                         "the family replays cannot be attributed")
    shape_label[sk] = lab

fam = defaultdict(list)
for d, k, v, g in rows:
    f = family(k)
    if f == "wo|down":
        f = ctx_label.get(d) or shape_label.get((base(k), g))
        if f is None:
            raise SystemExit(f"dispatch {d} ({base(k)}, grid {g}): no step context names it wo or down")
    if f:
        fam[f].append(v)
res[key]["per_family_hbm_bytes_per_launch"] = {f: round(2 * 1024 * sum(v) / len(v)) for f, v in fam.items()}
res[key]["per_family_dispatches"] = {f: len(v) for f, v in fam.items()}
if dom in res[key]["per_family_hbm_bytes_per_launch"]:
    res[key]["dominant_family_hbm_over_algorithmic"] = round(res[key]["per_family_hbm_bytes_per_launch"][dom] / alg, 4)
bad = []
if fam_alg:
    res[key]["per_family_hbm_over_algorithmic"] = {
        f: round(b / fam_alg[f], 4) for f, b in res[key]["per_family_hbm_bytes_per_launch"].items() if f in fam_alg}
    # A single pass must read every weight (or K/V) byte once: a family BELOW its algorithmic bytes means the
    # counter pass or its attribution is wrong, not that the kernel is efficient.
    bad = [f for f, r in res[key]["per_family_hbm_over_algorithmic"].items() if r < 0.99]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res[key], indent=1))
if bad:
    raise SystemExit(f"traffic below 0.99x algorithmic for {bad}: attribution error")
