#!/bin/bash
# Round 6 bench lines on one box: C1 (the driver's default command), C4, C3, then the loopback TP rank steps
# (launch graph vs persistent layers, with and without the per-workgroup exchange).   tools/gpu_r6_bench.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench_c1.log 2>&1 || { echo BENCH C1 FAILED; tail -20 gpurun_out/${tag}_bench_c1.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c1.log | cut -c1-300
timeout -k 10 400 python3 bench.py --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 > gpurun_out/${tag}_bench_c4.log 2>&1 || { echo BENCH C4 FAILED; tail -20 gpurun_out/${tag}_bench_c4.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c4.log | cut -c1-300
timeout -k 10 300 python3 bench.py --w-dtype i8 --no-cpu-baseline > gpurun_out/${tag}_bench_c3.log 2>&1 || { echo BENCH C3 FAILED; tail -20 gpurun_out/${tag}_bench_c3.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c3.log | cut -c1-300
{
SLI_QKV_ATTN=1 timeout -k 10 120 python3 tools/tp_rank_time.py 1 2 4 8 &&
TP_EXEC=persist timeout -k 10 120 python3 tools/tp_rank_time.py 8 4 &&
SLI_QKV_ATTN=1 TP_AR=fused_wg timeout -k 10 120 python3 tools/tp_rank_time.py 2 4 8 &&
TP_AR=fused_wg TP_EXEC=persist timeout -k 10 120 python3 tools/tp_rank_time.py 8 4
} > gpurun_out/${tag}_tp_rank_time.txt 2>&1 || { echo TP RANK TIME FAILED; tail -20 gpurun_out/${tag}_tp_rank_time.txt; exit 1; }
cat gpurun_out/${tag}_tp_rank_time.txt
echo done
