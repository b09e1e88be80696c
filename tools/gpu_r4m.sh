#!/bin/bash
# round 4: the per-workgroup exchange with relaxed flag store / poll (variant libsli_relaxed.so,
# SLI_OS_WG_FENCE=0): its two/four-process tests, then loopback per-rank steps against the fenced form
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SLI_LIB_VARIANT=relaxed timeout -k 10 600 python -u -m pytest tests/test_gpu_tp.py -k "fused_wg" -x -v --timeout 300 --timeout-method thread > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log; exit 1; }
tail -2 gpurun_out/r4m_tests.log
for r in 1 2; do
  TP_AR=fused_wg timeout -k 10 200 python3 tools/tp_rank_time.py 2 8 || exit 1
  SLI_LIB_VARIANT=relaxed TP_AR=fused_wg timeout -k 10 200 python3 tools/tp_rank_time.py 2 8 | sed 's/^/relaxed /' || exit 1
done
