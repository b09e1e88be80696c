#!/bin/bash
# Round 6, first box: the GPU suite, then the driver's own bench command with and without the settle phase
# (step_ms p50 / p99 and first-5 / last-5 means explain the window), then C4 and C3. Usage: tools/gpu_r6a.sh [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-r6a}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/${tag}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_gpu_tests.log
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --settle-ms 0 --no-cpu-baseline > gpurun_out/${tag}_bench_c1_nosettle.log 2>&1 || { echo BENCH C1 FAILED; tail -20 gpurun_out/${tag}_bench_c1_nosettle.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c1_nosettle.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('nosettle', d['value'], d['step_ms'], d['greedy_64'])"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${tag}_bench_c1.log 2>&1 || { echo BENCH C1 FAILED; tail -20 gpurun_out/${tag}_bench_c1.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('settle', d['value'], d['step_ms'], d['greedy_64'], d['settle'])"
timeout -k 10 400 python3 bench.py --preset llama3-8b --ctx 4096 --batch 8 --steps 50 --warmup 10 > gpurun_out/${tag}_bench_c4.log 2>&1 || { echo BENCH C4 FAILED; tail -20 gpurun_out/${tag}_bench_c4.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['step_ms'])"
timeout -k 10 300 python3 bench.py --w-dtype i8 --no-cpu-baseline > gpurun_out/${tag}_bench_c3.log 2>&1 || { echo BENCH C3 FAILED; tail -20 gpurun_out/${tag}_bench_c3.log; exit 1; }
tail -1 gpurun_out/${tag}_bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['step_ms'])"
echo done
