"""Kernel resource summary from hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin): name, VGPRs,
scratch bytes/lane, occupancy.   hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [filter]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = {}
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        if cur:
            rows.append(cur)
        cur = {"name": m.group(1)}
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
if cur:
    rows.append(cur)
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    if flt in n:
        print(f"vgpr {r.get('vgpr', '?'):>3} scratch {r.get('scratch', '?'):>4} occ {r.get('occ', '?')}  {n[:150]}")
