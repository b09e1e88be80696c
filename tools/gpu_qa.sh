#!/bin/bash
# Fused q/k/v + attention launch (qkv_attn.h): its tests, the model / TP suites it touches, then the TP rank step
# in loopback with and without it (interleaved).   tools/gpu_qa.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-qa}
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python3 -u -m pytest tests/test_gpu_qkv_attn.py tests/test_gpu_model.py tests/test_gpu_tp.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for r in 1 2; do
  for qa in 0 1; do
    echo "== SLI_QKV_ATTN=$qa TP_AR=fused_wg round $r" >> gpurun_out/${tag}_ab.txt
    SLI_QKV_ATTN=$qa TP_AR=fused_wg $T 300 python3 tools/tp_rank_time.py 4 8 >> gpurun_out/${tag}_ab.txt 2>&1 || { tail -20 gpurun_out/${tag}_ab.txt; exit 1; }
  done
done
cat gpurun_out/${tag}_ab.txt
