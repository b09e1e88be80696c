#!/bin/bash
# rocprofv3 kernel traces of the last TP-8 rank's step in loopback (tools/tp_rank_time.py, the per-workgroup
# exchange): C2 (Llama-2-7B batch 1) and C4 (Llama-3-8B batch 8 ctx 4096) -> step traces.  tools/gpu_tp_trace.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r4}
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export TP_AR=fused_wg
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o "${tag}_c2_tp8" --output-format csv -- python3 tools/tp_rank_time.py 8 > gpurun_out/prof/${tag}_c2_tp8.log 2>&1 || { tail -20 gpurun_out/prof/${tag}_c2_tp8.log; exit 1; }
export TP_PRESET=llama3-8b TP_BATCH=8 TP_CTX=4096
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o "${tag}_c4_tp8" --output-format csv -- python3 tools/tp_rank_time.py 8 > gpurun_out/prof/${tag}_c4_tp8.log 2>&1 || { tail -20 gpurun_out/prof/${tag}_c4_tp8.log; exit 1; }
for c in c2_tp8 c4_tp8; do
  python3 tools/step_trace.py $(find gpurun_out/prof -name "${tag}_${c}_kernel_trace.csv" | head -1) > gpurun_out/prof/${tag}_${c}_step_trace.txt
  cat gpurun_out/prof/${tag}_${c}_step_trace.txt
done
find gpurun_out/prof -name '*_kernel_trace.csv' -delete
