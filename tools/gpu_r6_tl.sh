#!/bin/bash
# Round 6: the persistent layer stack (csrc/tp_layers.h): its GPU tests, then the loopback TP-8 / TP-4 rank step
# against the launch graph. Usage: tools/gpu_r6_tl.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6_tl}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tp_layers.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|persist vs|print" gpurun_out/${tag}_tests.log | tail -30
[ $rc -ne 0 ] && { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
{
SLI_QKV_ATTN=1 timeout -k 10 120 python3 tools/tp_rank_time.py 8 4 &&
TP_EXEC=persist timeout -k 10 120 python3 tools/tp_rank_time.py 8 4 &&
SLI_QKV_ATTN=1 TP_AR=fused_wg timeout -k 10 120 python3 tools/tp_rank_time.py 8 4 &&
TP_AR=fused_wg TP_EXEC=persist timeout -k 10 120 python3 tools/tp_rank_time.py 8 4
} > gpurun_out/${tag}_rank_time.txt 2>&1
rc=$?
cat gpurun_out/${tag}_rank_time.txt
exit $rc
