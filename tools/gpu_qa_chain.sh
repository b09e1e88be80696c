#!/bin/bash
# The chain launch (q/k/v + attention + wo, SLI_QKV_CHAIN=1): its tests, then the TP rank step in loopback
# (per-workgroup exchange) two launches / q/k/v + attention / chain, interleaved.   tools/gpu_qa_chain.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-qac}
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python3 -u -m pytest tests/test_gpu_qkv_attn.py tests/test_gpu_tp.py -k "qkv or qa" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for r in 1 2; do
  for mode in "0 0" "1 0" "1 1"; do
    set -- $mode
    echo "== SLI_QKV_ATTN=$1 SLI_QKV_CHAIN=$2 round $r" >> gpurun_out/${tag}_ab.txt
    SLI_QKV_ATTN=$1 SLI_QKV_CHAIN=$2 TP_AR=fused_wg $T 300 python3 tools/tp_rank_time.py 4 8 >> gpurun_out/${tag}_ab.txt 2>&1 || { tail -20 gpurun_out/${tag}_ab.txt; exit 1; }
  done
done
cat gpurun_out/${tag}_ab.txt
