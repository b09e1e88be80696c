#!/bin/bash
# round 4: context-dependent K-split (4 past 8 splits) and the batch-1 GQA split default: parity, then A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_wo_ksplit.py tests/test_gpu_model.py tests/test_gpu_batch.py -k "not full_batch8 and not full_32" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4e_tests.log 2>&1 || { tail -30 gpurun_out/r4e_tests.log; exit 1; }
tail -2 gpurun_out/r4e_tests.log
bash tools/ab_env.sh 1 "SLI_WO_KSPLIT=2 SLI_ATTN_GQA_SPLIT=1" "SLI_WO_KSPLIT=2" "SLI_WO_KSPLIT=4" "SLI_WO_KSPLIT=4 SLI_ATTN_GQA_SPLIT=1" -- --preset llama3-8b --ctx 4096 && \
bash tools/ab_env.sh 1 "SLI_WO_KSPLIT=2" "SLI_WO_KSPLIT=4" -- --ctx 4096 && \
bash tools/ab_env.sh 1 "SLI_WO_KSPLIT=1" "SLI_WO_KSPLIT=2" -- --ctx 2048
