#!/bin/bash
# Round-end style check on the GPU box: gpu tests, the bench line (with CPU baseline), a rocprofv3 kernel
# trace + stats of the bench, and the FETCH_SIZE traffic pass. Usage: tools/gpu_check.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r02}
mkdir -p gpurun_out/prof
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
./tools/prof_step.sh "$tag" || exit 1
./tools/pmc_traffic.sh "$tag" || exit 1
echo done
