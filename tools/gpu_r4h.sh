#!/bin/bash
# round 4: A/B of producer sums of squares at C4 (parity run separately), then the TP shard anatomy
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/ab_env.sh 2 "SLI_BG_EXT_SS=0" "SLI_BG_EXT_SS=1" -- --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 > gpurun_out/r4h_ab.txt || { cat gpurun_out/r4h_ab.txt; exit 1; }
cat gpurun_out/r4h_ab.txt
bash tools/gpu_tp8.sh r4h
