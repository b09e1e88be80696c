#!/bin/bash
# round 4: the batched per-group exchange inside the MFMA wo / down (BgEpiPush, fused_wg at batch > 1): the
# one-shot / fused tests, then loopback C4 shard rank steps against the sliced one-shot launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_tp.py -k "oneshot" -x -v --timeout 300 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1 || { tail -30 gpurun_out/r4p_tests.log; exit 1; }
tail -2 gpurun_out/r4p_tests.log
for r in 1 2; do
  for ar in oneshot fused_wg; do
    TP_PRESET=llama3-8b TP_BATCH=8 TP_CTX=4096 TP_AR=$ar timeout -k 10 200 python3 tools/tp_rank_time.py 2 8 || exit 1
  done
done
