#!/bin/bash
# tools/tl_lab on one box: the persistent layer stack at a C2 TP-8 rank's shapes, per-phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r6_tllab}
{ timeout -k 10 60 tools/tl_lab -m 1 && timeout -k 10 60 tools/tl_lab -m 2 && timeout -k 10 60 tools/tl_lab -m 0; } > gpurun_out/${tag}.txt 2>&1
rc=$?
cat gpurun_out/${tag}.txt
exit $rc
