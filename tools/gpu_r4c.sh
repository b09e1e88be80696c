#!/bin/bash
# round 4: the fused attention + wo launch (SLI_ATTN_WO=1): parity, then A/B at C1 / C3 (K-split 2 default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_wo_ksplit.py -k "attn_wo" -x -v --timeout 400 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || { tail -40 gpurun_out/r4c_tests.log; exit 1; }
tail -3 gpurun_out/r4c_tests.log
bash tools/ab_env.sh 2 "SLI_ATTN_WO=0" "SLI_ATTN_WO=1" > gpurun_out/r4c_ab_c1.txt 2>&1 || { cat gpurun_out/r4c_ab_c1.txt; exit 1; }
cat gpurun_out/r4c_ab_c1.txt
bash tools/ab_env.sh 2 "SLI_ATTN_WO=0" "SLI_ATTN_WO=1" -- --w-dtype i8 > gpurun_out/r4c_ab_c3.txt 2>&1 || { cat gpurun_out/r4c_ab_c3.txt; exit 1; }
cat gpurun_out/r4c_ab_c3.txt
