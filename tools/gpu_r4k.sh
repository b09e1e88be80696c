#!/bin/bash
# round 4: the wo launches' phase stamps (lab), the per-workgroup fused exchange (SLI_ALLREDUCE_FUSED_WG):
# two/four-process tests, then the loopback per-rank step against the launch-level fused exchange
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemv_lab wo > gpurun_out/r4_gemv_lab_wo.txt 2>&1 || { cat gpurun_out/r4_gemv_lab_wo.txt; exit 1; }
cat gpurun_out/r4_gemv_lab_wo.txt
timeout -k 10 700 python -u -m pytest tests/test_gpu_tp.py -k "oneshot" -x -v --timeout 300 --timeout-method thread > gpurun_out/r4k_tests.log 2>&1 || { tail -40 gpurun_out/r4k_tests.log; exit 1; }
tail -3 gpurun_out/r4k_tests.log
for r in 1 2; do
  TP_AR=fused timeout -k 10 200 python3 tools/tp_rank_time.py 2 4 8 || exit 1
  TP_AR=fused_wg timeout -k 10 200 python3 tools/tp_rank_time.py 2 4 8 || exit 1
done
