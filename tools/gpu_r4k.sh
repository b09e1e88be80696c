#!/bin/bash
# round 4: the wo launches' phase stamps (lab); the per-workgroup fused exchange (SLI_ALLREDUCE_FUSED_WG) and the
# batch-1 LM head with the key reduce + state update folded in (SLI_LM_FINALIZE): tests, then A/B and the
# loopback per-rank step against the launch-level fused exchange
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemv_lab wo > gpurun_out/r4_gemv_lab_wo.txt 2>&1 || { cat gpurun_out/r4_gemv_lab_wo.txt; exit 1; }
cat gpurun_out/r4_gemv_lab_wo.txt
timeout -k 10 1000 python -u -m pytest tests/test_gpu_tp.py tests/test_gpu_model.py tests/test_gpu_batch.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4k_tests.log 2>&1 || { tail -40 gpurun_out/r4k_tests.log; exit 1; }
tail -3 gpurun_out/r4k_tests.log
bash tools/ab_env.sh 2 "SLI_LM_FINALIZE=0" "SLI_LM_FINALIZE=1" || exit 1
bash tools/ab_env.sh 1 "SLI_LM_FINALIZE=0" "SLI_LM_FINALIZE=1" -- --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 || exit 1
for r in 1; do
  TP_AR=fused timeout -k 10 200 python3 tools/tp_rank_time.py 2 4 8 || exit 1
  TP_AR=fused_wg timeout -k 10 200 python3 tools/tp_rank_time.py 2 4 8 || exit 1
done
