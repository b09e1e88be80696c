#!/bin/bash
# Prefill: the GPU prefill tests, then prompt timings (fp16 and int8, 128 / 512 / 2048 tokens).   tools/gpu_pf.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6b}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_prefill.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_pf_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${tag}_pf_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_pf_tests.log
timeout -k 10 300 python3 tools/prefill_time.py --tokens 128 512 2048 > gpurun_out/${tag}_pf_time.txt 2>&1 &&
timeout -k 10 300 python3 tools/prefill_time.py --w i8 --tokens 128 512 2048 >> gpurun_out/${tag}_pf_time.txt 2>&1 || { echo TIME FAILED; tail -20 gpurun_out/${tag}_pf_time.txt; exit 1; }
cat gpurun_out/${tag}_pf_time.txt
