#!/bin/bash
# Round 6: the whole GPU suite once (one process), summary into gpurun_out/<tag>_gpu_tests.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6}
mkdir -p gpurun_out
timeout -k 10 1080 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 900 --timeout-method thread -rs > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${tag}_gpu_tests.log | tail -8
exit $rc
