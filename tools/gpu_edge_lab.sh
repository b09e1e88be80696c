#!/bin/bash
# edge_chain_lab on one box: the pure edge chain and the chain with each CU's weight share held in registers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r6_edge}
{ timeout -k 10 60 tools/edge_chain_lab -L 32 -r 20 && timeout -k 10 60 tools/edge_chain_lab -w -L 32 -r 20; } > gpurun_out/${tag}.txt 2>&1
rc=$?
cat gpurun_out/${tag}.txt
exit $rc
