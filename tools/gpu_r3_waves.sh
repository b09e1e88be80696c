#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/w_tests.log 2>&1 || { tail -30 gpurun_out/w_tests.log; exit 1; }
tail -1 gpurun_out/w_tests.log
tools/ab_env.sh 2 "SLI_GEMV_WAVES=0" "SLI_GEMV_WAVES=1" || exit 1
tools/ab_env.sh 2 "SLI_GEMV_WAVES=0" "SLI_GEMV_WAVES=1" -- --w-dtype i8
