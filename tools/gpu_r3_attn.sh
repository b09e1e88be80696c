#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tools/ab_env.sh 2 "SLI_ATTN_MERGE_LAUNCH=2" "SLI_ATTN_MERGE_LAUNCH=0" -- --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 || exit 1
tools/ab_variants.sh "base s32" --greedy-steps 2 --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10
