#!/bin/bash
# SLI_ATTN_GQA_SPLIT=2|4 (a GQA-4 kv head as two GQA-2 groups or four MHA heads): parity, then A/B at C4 and Llama-3-8B B1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SLI_ATTN_GQA_SPLIT=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -k "not full_batch8" -x -q --timeout 300 --timeout-method thread > gpurun_out/gs_tests2.log 2>&1 || { tail -30 gpurun_out/gs_tests2.log; exit 1; }
SLI_ATTN_GQA_SPLIT=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_ops.py -k "not full_batch8" -x -q --timeout 300 --timeout-method thread > gpurun_out/gs_tests.log 2>&1 || { tail -30 gpurun_out/gs_tests.log; exit 1; }
tail -2 gpurun_out/gs_tests.log
bash tools/ab_env.sh 2 "SLI_ATTN_GQA_SPLIT=0" "SLI_ATTN_GQA_SPLIT=2" "SLI_ATTN_GQA_SPLIT=4" -- --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 && \
bash tools/ab_env.sh 1 "SLI_ATTN_GQA_SPLIT=0" "SLI_ATTN_GQA_SPLIT=2" "SLI_ATTN_GQA_SPLIT=4" -- --preset llama3-8b --ctx 4096
