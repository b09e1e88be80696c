#!/bin/bash
# GPU box: the C1 / C3 / C4 bench lines only.   tools/gpu_bench3.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r4}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench_c1.log 2>&1 || { echo BENCH C1 FAILED; tail -20 gpurun_out/${tag}_bench_c1.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c1.log | cut -c1-300
timeout -k 10 400 python3 bench.py --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 > gpurun_out/${tag}_bench_c4.log 2>&1 || { echo BENCH C4 FAILED; tail -20 gpurun_out/${tag}_bench_c4.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c4.log | cut -c1-300
timeout -k 10 300 python3 bench.py --w-dtype i8 --no-cpu-baseline > gpurun_out/${tag}_bench_c3.log 2>&1 || { echo BENCH C3 FAILED; tail -20 gpurun_out/${tag}_bench_c3.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c3.log | cut -c1-300
echo done
