#!/bin/bash
# Kernel stats of the TP-8 rank step (loopback, per-workgroup exchange) with and without the fused q/k/v +
# attention launch.   tools/gpu_qa_prof.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-qap}
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for qa in 0 1; do
  SLI_QKV_ATTN=$qa TP_AR=fused_wg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o "${tag}_qa${qa}" --output-format csv -- python3 tools/tp_rank_time.py 8 > gpurun_out/prof/${tag}_qa${qa}.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof/${tag}_qa${qa}.log; exit 1; }
  tail -1 gpurun_out/prof/${tag}_qa${qa}.log
  python3 tools/kstats.py $(find gpurun_out/prof -name "${tag}_qa${qa}_kernel_stats.csv" | head -1) 12
done
find gpurun_out/prof -name '*_kernel_trace.csv' -delete
