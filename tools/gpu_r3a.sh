#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 60 --warmup 10 > gpurun_out/bench_c1.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log
timeout -k 10 200 python3 tools/prefill_time.py --tokens 512 2048 > gpurun_out/prefill.log 2>&1 || { echo PF FAILED; tail gpurun_out/prefill.log; exit 1; }
cat gpurun_out/prefill.log
