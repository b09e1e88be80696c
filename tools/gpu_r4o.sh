#!/bin/bash
# round 4: the separate one-shot residual sum sliced over workgroups (oneshot_sliced_kernel): the two/four-process
# one-shot tests, then loopback per-rank steps at C4 (batch 8) and C2 (batch 1) TP-8 shards, sliced vs one workgroup
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tp.py tests/test_gpu_tp_group.py -k "oneshot or c4" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 || { tail -30 gpurun_out/r4o_tests.log; exit 1; }
tail -2 gpurun_out/r4o_tests.log
for r in 1 2; do
  for sl in 1 0; do
    SLI_ONESHOT_SLICED=$sl TP_PRESET=llama3-8b TP_BATCH=8 TP_CTX=4096 TP_AR=oneshot timeout -k 10 200 python3 tools/tp_rank_time.py 2 8 | sed "s/^/sliced=$sl /" || exit 1
    SLI_ONESHOT_SLICED=$sl TP_AR=oneshot timeout -k 10 200 python3 tools/tp_rank_time.py 8 | sed "s/^/sliced=$sl /" || exit 1
  done
done
