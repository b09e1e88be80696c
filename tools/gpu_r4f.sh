#!/bin/bash
# round 4: where the batch-1 attention splits merge past 8 splits (SLI_WO_MERGE): parity, then A/B at ctx 4096
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_wo_ksplit.py tests/test_gpu_model.py tests/test_gpu_tp.py tests/test_gpu_tp_group.py -k "not full_32" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { tail -30 gpurun_out/r4f_tests.log; exit 1; }
tail -2 gpurun_out/r4f_tests.log
bash tools/ab_env.sh 2 "SLI_WO_MERGE=1 SLI_WO_KSPLIT=4" "SLI_WO_MERGE=0" -- --ctx 4096 && \
bash tools/ab_env.sh 2 "SLI_WO_MERGE=1 SLI_WO_KSPLIT=4" "SLI_WO_MERGE=0" -- --preset llama3-8b --ctx 4096
