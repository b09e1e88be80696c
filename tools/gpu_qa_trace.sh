#!/bin/bash
# Step trace of the TP-8 rank step (C2 shard, loopback per-workgroup exchange) with the fused q/k/v + attention
# launch: rocprofv3 kernel trace -> tools/step_trace.py.   tools/gpu_qa_trace.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-qatr}
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
SLI_QKV_ATTN=1 TP_AR=fused_wg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o "${tag}_rank7" --output-format csv -- python3 tools/tp_rank_time.py 8 > gpurun_out/prof/${tag}_rank7.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof/${tag}_rank7.log; exit 1; }
tail -1 gpurun_out/prof/${tag}_rank7.log
python3 tools/step_trace.py $(find gpurun_out/prof -name "${tag}_rank7_kernel_trace.csv" | head -1) > gpurun_out/prof/${tag}_rank7_step_trace.txt
cat gpurun_out/prof/${tag}_rank7_step_trace.txt
find gpurun_out/prof -name '*_kernel_trace.csv' -delete
