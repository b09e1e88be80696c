#!/bin/bash
# round 4: parity (reference-build vectors, Level 2, prefill fixes, K-split wo), then the K-split wo A/B at C1 / C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_dropin_cpp.py tests/test_gpu_prefill.py tests/test_gpu_tp.py tests/test_gpu_wo_ksplit.py -k "reference_build or level2 or half_last_stage or prefill_tp_group or prefill_two_processes or teacher_forces or ksplit" -x -v --timeout 300 --timeout-method thread > gpurun_out/r4b_tests.log 2>&1 || { tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -3 gpurun_out/r4b_tests.log
bash tools/ab_env.sh 2 "SLI_WO_KSPLIT=1" "SLI_WO_KSPLIT=2" "SLI_WO_KSPLIT=4" > gpurun_out/r4b_ab_c1.txt 2>&1 || { cat gpurun_out/r4b_ab_c1.txt; exit 1; }
cat gpurun_out/r4b_ab_c1.txt
bash tools/ab_env.sh 2 "SLI_WO_KSPLIT=1" "SLI_WO_KSPLIT=2" "SLI_WO_KSPLIT=4" -- --w-dtype i8 > gpurun_out/r4b_ab_c3.txt 2>&1 || { cat gpurun_out/r4b_ab_c3.txt; exit 1; }
cat gpurun_out/r4b_ab_c3.txt
