#!/bin/bash
# timing anatomy of the fused attention + wo launch (SLI_DEBUG_AW bits, attn_wo.h; 4 / 8 give wrong results)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/ab_env.sh 1 "SLI_ATTN_WO=0" "SLI_ATTN_WO=1" "SLI_ATTN_WO=1 SLI_DEBUG_AW=1" "SLI_ATTN_WO=1 SLI_DEBUG_AW=4" "SLI_ATTN_WO=1 SLI_DEBUG_AW=8" "SLI_ATTN_WO=1 SLI_DEBUG_AW=12" "SLI_ATTN_WO=1 SLI_DEBUG_AW=13"
