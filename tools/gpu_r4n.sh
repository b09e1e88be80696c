#!/bin/bash
# round 4: relaxed flags for the separate one-shot launch and the launch-level fused exchange (variant
# libsli_osrelaxed.so, SLI_OS_FENCE=0): tests, then loopback per-rank steps at C2 (batch 1) and C4 (batch 8) shards
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SLI_LIB_VARIANT=osrelaxed timeout -k 10 600 python -u -m pytest tests/test_gpu_tp.py -k "oneshot" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1 || { tail -30 gpurun_out/r4n_tests.log; exit 1; }
tail -2 gpurun_out/r4n_tests.log
for r in 1 2; do
  for v in base osrelaxed; do
    if [ $v = base ]; then unset SLI_LIB_VARIANT; else export SLI_LIB_VARIANT=$v; fi
    TP_AR=oneshot timeout -k 10 200 python3 tools/tp_rank_time.py 8 | sed "s/^/$v /" || exit 1
    TP_AR=fused timeout -k 10 200 python3 tools/tp_rank_time.py 8 | sed "s/^/$v /" || exit 1
    TP_PRESET=llama3-8b TP_BATCH=8 TP_CTX=4096 TP_AR=oneshot timeout -k 10 200 python3 tools/tp_rank_time.py 8 | sed "s/^/$v /" || exit 1
  done
done
unset SLI_LIB_VARIANT
TP_PRESET=llama3-8b TP_BATCH=8 TP_CTX=4096 timeout -k 10 200 python3 tools/tp_rank_time.py 8 || exit 1
