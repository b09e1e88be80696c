"""Print one decode step's kernel sequence (durations, gaps) from a rocprofv3 kernel_trace.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "embedding" in r["Kernel_Name"]]
i0, i1 = idx[-3], idx[-2]
agg = {}
prev = None
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0][:70]
    d = agg.setdefault(name, [0, 0.0, 0.0])
    d[0] += 1
    d[1] += (e - s) / 1000
    d[2] += ((s - prev) / 1000) if prev else 0
    prev = e
tot = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1000
for k, (n, dur, gap) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:70s} n={n:4d} avg={dur / n:7.2f} us  total={dur:8.1f} us  gaps={gap:6.1f}")
print(f"step {tot:.1f} us")
