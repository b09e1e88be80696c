#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tp.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tp_tests.log 2>&1 || { echo TP TESTS FAILED; tail -40 gpurun_out/tp_tests.log; exit 1; }
grep -E "passed|failed|skipped" gpurun_out/tp_tests.log | tail -3
for ar in "" oneshot fused; do TP_AR=$ar timeout -k 10 300 python3 tools/tp_rank_time.py 2 4 8 || exit 1; done > gpurun_out/tp_rank_time.txt 2>&1 || { cat gpurun_out/tp_rank_time.txt; exit 1; }
cat gpurun_out/tp_rank_time.txt
