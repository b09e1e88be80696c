#!/bin/bash
# GPU box: the whole gpu test suite, then bench lines for C1 (default), C4 (llama3-8b batch 8 ctx 4096)
# and C3 (int8 weights). Usage: tools/gpu_round.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench_c1.log 2>&1 || { echo BENCH C1 FAILED; tail -20 gpurun_out/${tag}_bench_c1.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c1.log
timeout -k 10 400 python3 bench.py --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 > gpurun_out/${tag}_bench_c4.log 2>&1 || { echo BENCH C4 FAILED; tail -20 gpurun_out/${tag}_bench_c4.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c4.log
timeout -k 10 300 python3 bench.py --w-dtype i8 --no-cpu-baseline > gpurun_out/${tag}_bench_c3.log 2>&1 || { echo BENCH C3 FAILED; tail -20 gpurun_out/${tag}_bench_c3.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c3.log
echo done
