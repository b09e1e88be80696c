#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_tp_group.py tests/test_gpu_prefill.py -x -q -p no:cacheprovider --timeout 500 --timeout-method thread -k "not full" > gpurun_out/dup_tests.log 2>&1 || { tail -30 gpurun_out/dup_tests.log; exit 1; }
tail -1 gpurun_out/dup_tests.log
tools/ab_variants.sh "base dup" --greedy-steps 2 --w-dtype i8 || exit 1
tools/ab_variants.sh "base dup" --greedy-steps 2 || exit 1
KEY=llama2-7b/i8/tp1 ./tools/pmc_traffic.sh r3dummy --w-dtype i8 > /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/pmc/r3dummy_gemv_traffic.json')); print(d['llama2-7b/i8/tp1']['per_family_hbm_bytes_per_launch'])"
