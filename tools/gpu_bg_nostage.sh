#!/bin/bash
# The batched projection's activation staging, bounded: tools/bgemm_lab (AUTO plans, C4 shapes, fragment-layout
# weights) as built and with BG_LAB_NOSTAGE (no activation loads), interleaved twice.   tools/gpu_bg_nostage.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6b}
mkdir -p gpurun_out
out=gpurun_out/${tag}_bg_nostage.txt
: > $out
for r in 1 2; do
  for v in bgemm_lab bgemm_lab_nostage; do
    echo "## $v round $r" >> $out
    LAB_TILED=1 LAB_AUTO_ONLY=1 timeout -k 10 120 ./tools/$v 8 >> $out 2>&1 || { echo FAILED $v; tail -5 $out; exit 1; }
  done
done
grep -E "^##|AUTO" $out
