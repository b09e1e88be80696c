#!/bin/bash
# TP shard anatomy on one GPU (loopback): per-family launch times vs stream floors at TP 1/8 (no exchange and
# fused), then a rocprofv3 kernel trace of the TP-8 rank step with the fused exchange -> step trace.
#   tools/gpu_tp8.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-tp8}
mkdir -p gpurun_out/prof
timeout -k 10 300 python3 tools/tp_families.py 1 8 > gpurun_out/${tag}_families.txt 2>&1 || { tail -20 gpurun_out/${tag}_families.txt; exit 1; }
TP_AR=fused timeout -k 10 300 python3 tools/tp_families.py 8 >> gpurun_out/${tag}_families.txt 2>&1 || { tail -20 gpurun_out/${tag}_families.txt; exit 1; }
cat gpurun_out/${tag}_families.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TP_AR=fused timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o "${tag}_rank7" --output-format csv -- python3 tools/tp_rank_time.py 8 > gpurun_out/prof/${tag}_rank7.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof/${tag}_rank7.log; exit 1; }
tail -1 gpurun_out/prof/${tag}_rank7.log
python3 tools/step_trace.py $(find gpurun_out/prof -name "${tag}_rank7_kernel_trace.csv" | head -1) > gpurun_out/prof/${tag}_rank7_step_trace.txt
cat gpurun_out/prof/${tag}_rank7_step_trace.txt
find gpurun_out/prof -name '*_kernel_trace.csv' -delete
