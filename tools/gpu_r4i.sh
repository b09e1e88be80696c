#!/bin/bash
# round 4: bgemm weights in the fragment layout (SLI_BG_TILED): batched parity, then A/B at C4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_tp_group.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1 || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -2 gpurun_out/r4i_tests.log
bash tools/ab_env.sh 2 "SLI_BG_TILED=0" "SLI_BG_TILED=1" -- --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10
