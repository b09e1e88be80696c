#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_batch.py tests/test_gpu_model.py tests/test_gpu_tp_group.py -x -q -p no:cacheprovider --timeout 500 --timeout-method thread -k "not full" > gpurun_out/vlds_tests.log 2>&1 || { tail -30 gpurun_out/vlds_tests.log; exit 1; }
tail -1 gpurun_out/vlds_tests.log
tools/ab_variants.sh "base novlds" --greedy-steps 2 --preset llama3-8b --ctx 4096 --batch 8
