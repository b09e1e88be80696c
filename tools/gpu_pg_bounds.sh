#!/bin/bash
# Prefill GEMM bounds (tools/pgemm_lab LAB_QUICK builds with PG_LAB_SKIP / PG_LAB_MFMA): what limits the chunk GEMM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6b}
out=gpurun_out/${tag}_pg_bounds.txt
: > $out
for v in base nob noa noab hionly nomfma; do
  echo "## $v" >> $out
  LAB_QUICK=1 timeout -k 10 100 ./tools/pgemm_lab_$v >> $out 2>&1 || { echo FAILED $v; tail -3 $out; exit 1; }
done
cat $out
