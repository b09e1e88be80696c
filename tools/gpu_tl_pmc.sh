#!/bin/bash
# instruction-cache counters of tools/tl_lab (one --pmc pass of its own, per the guide)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6_tlpmc}
mkdir -p $out
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $out -o pmc --output-format csv -- $GRAFT_REPO_ROOT/tools/tl_lab -m 1 -r 3 > $out/log.txt 2>&1
rc=$?
tail -3 $out/log.txt
find $out -name "*counter_collection*" | head -3
f=$(find $out -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(float)
for r in rows:
    if 'tp_layers' in r.get('Kernel_Name', ''):
        agg[r['Counter_Name']] += float(r['Counter_Value'])
n = sum(1 for r in rows if 'tp_layers' in r.get('Kernel_Name', '') and r['Counter_Name'] == 'SQC_ICACHE_REQ')
print({k: v / max(n, 1) for k, v in agg.items()}, 'launches', n)
PY
exit $rc
