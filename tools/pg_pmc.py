"""Summarise a rocprofv3 --pmc counter_collection.csv of tools/pgemm_lab (tools/gpu_pg_pmc.sh): per GEMM tiling,
the mean of each SQ counter over its dispatches, and the shares the guide defines (MI355X_MICROARCH.md, PMC slots):
WAIT_ANY (parked on s_waitcnt / barrier), WAIT_INST_ANY (issue stall), ACTIVE_INST_ANY, all over WAVE_CYCLES; LDS
bank-conflict cycles over LDS-array cycles.   python tools/pg_pmc.py gpurun_out/pmc/<...>_counter_collection.csv
"""
import collections
import csv
import re
import sys


def main(path):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "")
        if "pgemm_kernel" not in name:
            continue
        m = re.search(r"PgCfg<([^>]*)>", name)
        cfg = m.group(1) if m else name[:60]
        acc[cfg][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for cfg, c in acc.items():
        mean = {k: sum(v) / len(v) for k, v in c.items()}
        wc = mean.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        print(f"PgCfg<{cfg}> ({len(next(iter(c.values())))} dispatches)")
        print("   " + "  ".join(f"{k} {v:.3g}" for k, v in sorted(mean.items())))
        print(f"   wait_any {mean.get('SQ_WAIT_ANY', 0) / wc:.2f}  wait_inst_any {mean.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}"
              f" (of which lds {mean.get('SQ_WAIT_INST_LDS', 0) / wc:.2f})  active_inst {mean.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}"
              f" | lds bank conflict / lds active {mean.get('SQ_LDS_BANK_CONFLICT', 0) / max(mean.get('SQ_LDS_IDX_ACTIVE', 1), 1):.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
