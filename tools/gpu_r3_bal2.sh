#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SLI_QKV_GRID=192 SLI_GU_GRID=230 SLI_LM_GRID=250 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/bal_tests.log 2>&1 || { tail -30 gpurun_out/bal_tests.log; exit 1; }
tail -1 gpurun_out/bal_tests.log
tools/ab_env.sh 2 "SLI_GU_GRID=230" "SLI_GU_GRID=230 SLI_QKV_GRID=192" "SLI_GU_GRID=230 SLI_QKV_GRID=224" "SLI_GU_GRID=230 SLI_QKV_GRID=240" "SLI_GU_GRID=230 SLI_LM_GRID=250" || exit 1
tools/ab_env.sh 2 "SLI_X=0" "SLI_GU_GRID=230" "SLI_GU_GRID=230 SLI_QKV_GRID=192 SLI_LM_GRID=250" -- --w-dtype i8
