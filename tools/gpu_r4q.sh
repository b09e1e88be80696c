#!/bin/bash
# round 4: split fused-RMS bgemm plans for small tile counts (C4 TP-8 q/k/v) and the GQA split on small deferred
# grids: batched / TP-group / op parity, then the C4 TP shard families and the C4 TP-1 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_tp_group.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4q_tests.log 2>&1 || { tail -30 gpurun_out/r4q_tests.log; exit 1; }
tail -2 gpurun_out/r4q_tests.log
TP_PRESET=llama3-8b TP_BATCH=8 TP_CTX=4096 timeout -k 10 300 python3 tools/tp_families.py 4 8 || exit 1
TP_PRESET=llama3-8b TP_BATCH=8 TP_CTX=4096 TP_AR=fused_wg timeout -k 10 200 python3 tools/tp_rank_time.py 8 || exit 1
bash tools/ab_env.sh 1 "SLI_X=0" -- --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10
