#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
tools/ab_env.sh 2 "SLI_GEMV_BALANCE=0" "SLI_GEMV_BALANCE=1" > gpurun_out/bal_c1.txt || exit 1
tools/ab_env.sh 2 "SLI_GEMV_BALANCE=0" "SLI_GEMV_BALANCE=1" -- --w-dtype i8 > gpurun_out/bal_c3.txt || exit 1
cat gpurun_out/bal_c1.txt gpurun_out/bal_c3.txt
