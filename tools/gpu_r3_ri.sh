#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_prefill.py tests/test_gpu_persistent.py -x -q -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/ri_tests.log 2>&1 || { tail -30 gpurun_out/ri_tests.log; exit 1; }
tail -1 gpurun_out/ri_tests.log
tools/ab_env.sh 2 "SLI_QKV_RI=0" "SLI_QKV_RI=1" || exit 1
tools/ab_env.sh 2 "SLI_QKV_RI=0" "SLI_QKV_RI=1" -- --w-dtype i8
