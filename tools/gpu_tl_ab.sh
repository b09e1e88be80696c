#!/bin/bash
# A/B of tools/tl_lab builds (variants named on the command line), loopback exchange (-m 2) and one rank (-m 0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=$1; shift
for b in "$@"; do
  for m in 2 0; do
    timeout -k 10 60 tools/$b -m $m | head -1 | sed "s/^/$b: /" || exit 1
  done
done > gpurun_out/${tag}.txt 2>&1
rc=$?
cat gpurun_out/${tag}.txt
exit $rc
