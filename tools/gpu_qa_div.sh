#!/bin/bash
# TP-2 rank step (loopback, per-workgroup exchange): the fused q/k/v + attention launch at half the CUs for the
# attention (SLI_QKV_ATTN_DIV=2) against the two launches.   tools/gpu_qa_div.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-qadiv}
mkdir -p gpurun_out
for r in 1 2; do
  for qa in 0 1; do
    echo "== SLI_QKV_ATTN=$qa SLI_QKV_ATTN_DIV=2 round $r" >> gpurun_out/${tag}.txt
    SLI_QKV_ATTN=$qa SLI_QKV_ATTN_DIV=2 TP_AR=fused_wg timeout -k 10 300 python3 tools/tp_rank_time.py 2 >> gpurun_out/${tag}.txt 2>&1 || { tail -20 gpurun_out/${tag}.txt; exit 1; }
  done
done
SLI_QKV_ATTN_DIV=2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_qkv_attn.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread >> gpurun_out/${tag}.txt 2>&1 || { tail -30 gpurun_out/${tag}.txt; exit 1; }
cat gpurun_out/${tag}.txt
