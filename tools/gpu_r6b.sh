#!/bin/bash
# Round 6 (second session), first box: the driver's default bench command, then the prefill GEMM lab and the
# library ceiling for the same shapes.   tools/gpu_r6b.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6b}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench_c1.log 2>&1 || { echo BENCH C1 FAILED; tail -20 gpurun_out/${tag}_bench_c1.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c1.log | cut -c1-400
timeout -k 10 240 ./tools/pgemm_lab > gpurun_out/${tag}_pgemm_lab.txt 2>&1 || { echo PGEMM LAB FAILED; tail -20 gpurun_out/${tag}_pgemm_lab.txt; exit 1; }
timeout -k 10 240 python3 tools/gemm_ceiling.py > gpurun_out/${tag}_gemm_ceiling.txt 2>&1 || { echo CEILING FAILED; tail -20 gpurun_out/${tag}_gemm_ceiling.txt; exit 1; }
cat gpurun_out/${tag}_gemm_ceiling.txt
echo done
