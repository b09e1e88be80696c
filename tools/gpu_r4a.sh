#!/bin/bash
# round 4: GPU parity against the reference-build vectors, then the GQA split knob (tests + A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -k reference_build -x -v --timeout 300 --timeout-method thread > gpurun_out/r4a_refvec.log 2>&1 || { tail -40 gpurun_out/r4a_refvec.log; exit 1; }
tail -3 gpurun_out/r4a_refvec.log
bash tools/gpu_r3_gsplit.sh
