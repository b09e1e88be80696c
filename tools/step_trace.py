"""Decode-step kernel breakdown from a rocprofv3 kernel_trace.csv: every complete step (embedding to next
embedding) with the usual kernel count, per-kernel mean duration over those steps, and the median step time."""
import csv
import statistics
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "embedding" in r["Kernel_Name"]]
wins = [(a, b) for a, b in zip(idx, idx[1:])]
mode = Counter(b - a for a, b in wins).most_common(1)[0][0]
wins = [(a, b) for a, b in wins if b - a == mode]  # ordinary steps (not the per-family probes in between)
agg = {}
steps = []
for a, b in wins:
    steps.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1000)
    prev = None
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:70]
        d = agg.setdefault(name, [0, 0.0, 0.0])
        d[0] += 1
        d[1] += (e - s) / 1000
        d[2] += ((s - prev) / 1000) if prev else 0
        prev = e
ns = len(wins)
for k, (n, dur, gap) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:70s} n/step={n // ns:4d} avg={dur / n:7.2f} us  per step={dur / ns:8.1f} us  gaps/step={gap / ns:6.1f}")
print(f"steps {ns}: median {statistics.median(steps):.1f} us, min {min(steps):.1f}, max {max(steps):.1f}")
