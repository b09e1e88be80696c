"""MFMA utilisation of the batched projections (bgemm_kernel) and the prefill from one rocprofv3 PMC pass
(tools/pmc_mfma.sh: SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F16, SQ_INSTS_VALU_MFMA_F16,
GRBM_GUI_ACTIVE in one pass; 3 SQ + 1 GRBM slots).

Per kernel family, means per dispatch of:
  flops      = SQ_INSTS_VALU_MFMA_MOPS_F16 * 512 (rocprofv3's MfmaFlopsF16 expression)
  mfma_insts = SQ_INSTS_VALU_MFMA_F16
  util       = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * SIMDs) (rocprofv3's MfmaUtil expression, SIMDs =
               4 x 256 CUs; GRBM_GUI_ACTIVE as reported, which MI355X_MICROARCH.md says sums the 8 XCDs, so
               the same ratio with GRBM_GUI_ACTIVE / 8 is reported too)
    python tools/pmc_mfma.py <counter_collection.csv> <out.json> <key>
"""
import csv
import json
import sys
from collections import defaultdict

path, out, key = sys.argv[1], sys.argv[2], sys.argv[3]
vals = defaultdict(lambda: defaultdict(float))  # dispatch id -> counter -> value
names = {}
for r in csv.DictReader(open(path)):
    d = r.get("Dispatch_Id") or r.get("Correlation_Id") or r.get("Index")
    vals[d][r["Counter_Name"]] += float(r["Counter_Value"])
    names[d] = r["Kernel_Name"]


def family(k):
    if "pgemm_kernel" in k:  # the prompt prefill's chunk GEMMs (prefill.h)
        for tag, fam in (("PgEpiQKV", "prefill_qkv"), ("PgEpiSwiGLU", "prefill_gate_up"), ("PgEpiResid", "prefill_wo+down")):
            if tag in k:
                return fam
        return "prefill_other"
    if "pf_attn_mfma_kernel" in k:
        return "prefill_attention"
    if "bgemm_kernel" not in k:
        return None
    for tag, fam in (("BgEpiQKV", "qkv"), ("BgEpiSwiGLU", "gate_up"), ("BgEpiLogits", "lm_head"),
                     ("BgEpiStore", "wo+down")):
        if tag in k:
            return fam
    return "other"


SIMDS = 4 * 256
fam = defaultdict(list)
for d, c in vals.items():
    f = family(names[d])
    if f:
        fam[f].append(c)
res = {}
try:
    res = json.load(open(out))
except (OSError, ValueError):
    pass
entry = {}
for f, cs in sorted(fam.items()):
    n = len(cs)
    mean = lambda name: sum(c.get(name, 0.0) for c in cs) / n
    busy, gui = mean("SQ_VALU_MFMA_BUSY_CYCLES"), mean("GRBM_GUI_ACTIVE")
    entry[f] = {
        "dispatches": n,
        "mfma_flops_per_dispatch": round(512 * mean("SQ_INSTS_VALU_MFMA_MOPS_F16")),
        "mfma_insts_per_dispatch": round(mean("SQ_INSTS_VALU_MFMA_F16")),
        "mfma_busy_cycles_per_dispatch": round(busy),
        "grbm_gui_active_per_dispatch": round(gui),
        "mfma_util_pct": round(100 * busy / (gui * SIMDS), 3) if gui else None,
        "mfma_util_pct_gui_over_8": round(100 * busy / (gui / 8 * SIMDS), 3) if gui else None,
    }
res[key] = entry
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(entry, indent=1))
