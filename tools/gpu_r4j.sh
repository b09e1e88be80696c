#!/bin/bash
# round 4: fp16 exchange payload accuracy (in-process TP 8 group vs oracle), then where C4's attention splits merge
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ar_payload_error.py > gpurun_out/r4j_payload.txt 2>&1 || { tail -20 gpurun_out/r4j_payload.txt; exit 1; }
cat gpurun_out/r4j_payload.txt
bash tools/ab_env.sh 2 "SLI_ATTN_MERGE_LAUNCH=2" "SLI_ATTN_MERGE_LAUNCH=0" -- --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10
