#!/bin/bash
# round 4: GPU parity against the reference-build vectors, Level 2, the prefill fixes, then the GQA split knob
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_dropin_cpp.py tests/test_gpu_prefill.py tests/test_gpu_tp.py -k "reference_build or level2 or half_last_stage or prefill_tp_group or prefill_two_processes or teacher_forces" -x -v --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1 || { tail -40 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
bash tools/gpu_r3_gsplit.sh
